// Batched page coherence for gfx950 (SPEC §5): the per-page state machine that the reference
// only describes (resources/NUTSHELL.md:52-69, resources/IMPLEMENTATION.md:137-249) on the
// fields of its unused ApplicationMemory record (gallocy/include/gallocy/models.h:171-213).
//
// The sequential fold is recast as a scan over 32-bit transforms (SPEC §5a, state part only):
//   READ(R)  : copyset |= R; EXCLUSIVE -> SHARED if R is not inside the copyset   (bit 31 = 0)
//   CONST(s) : the state becomes s                                              (bit 31 = 1)
// A read by n is READ({n}); a write by n is CONST(EXCLUSIVE, owner n, copyset {n}, dirty);
// the first event of a page is seeded with CONST(page-table state). Composition is
// associative, so every event's incoming state is an exclusive scan, and each event's fault /
// invalidation / transfer follows from its incoming state alone.
//
// Kernels (no workgroup ever waits on another):
//   A coh_tail_kernel    one wave per 4096-event block: composes the block from its LAST
//                        segment head to its end (reads only that tail), records that head's
//                        page-table state so pass C never reads a word another block writes.
//   B coh_scan_kernel    one workgroup: exclusive scan of the block aggregates -> carry-in.
//   C coh_apply_kernel   per block: events staged in LDS, per-thread fold of 16 events,
//                        block scan with the carry-in, per-event faults, segmented sum of
//                        per-page faults, final states written at segment ends, block partials.
//   D coh_reduce_kernel  partial rows -> the 10 batch totals.
#include "gdsm_common.h"
#include "gdsm_launch.h"

namespace gdsm {

constexpr uint32_t kConst = 1u << 31;
constexpr uint32_t kCohK = 16;                 // events per thread
constexpr uint32_t kCohBlock = 256 * kCohK;    // events per block
constexpr uint32_t kNoHead = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t tcompose(uint32_t a, uint32_t b) {  // a, then b
  if (b & kConst) return b;
  const uint32_t R = b & 0xFFu;
  if (a & kConst) {
    const uint32_t cs = a & 0xFFu;
    uint32_t st = (a >> 16) & 3u;
    if ((R & ~cs) && st == 2u) st = 1u;
    return (a & ~(0xFFu | (3u << 16))) | (cs | R) | (st << 16);
  }
  return a | R;
}

__device__ __forceinline__ uint32_t ev_transform(uint64_t e) {
  const uint32_t node = (uint32_t)(e >> 1) & 7u;
  return (e & 1u) ? (kConst | (1u << node) | (node << 8) | (2u << 16) | (1u << 18)) : (1u << node);
}

__device__ __forceinline__ uint64_t ev_page(uint64_t e) { return e >> 4; }

// Ordered reduction over the wave: lane 0 gets v_0 ∘ v_1 ∘ … ∘ v_63.
__device__ __forceinline__ uint32_t wave_reduce_compose(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_down(v, d, 64);
    if (lane + d < 64u) v = tcompose(v, t);
  }
  return __shfl(v, 0, 64);
}

__device__ __forceinline__ uint32_t wave_incl_compose(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v = tcompose(t, v);
  }
  return v;
}

// Segmented sum: bit 31 = "a segment starts in here", low bits = count since the last start.
__device__ __forceinline__ uint32_t segsum(uint32_t a, uint32_t b) {
  return ((b & kConst) ? (b & ~kConst) : ((a & ~kConst) + (b & ~kConst))) | ((a | b) & kConst);
}
__device__ __forceinline__ uint32_t wave_incl_segsum(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v = segsum(t, v);
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// ---------------------------------------------------------------- init
__global__ __launch_bounds__(256) void coh_init_kernel(uint32_t* __restrict__ state,
                                                       uint32_t* __restrict__ faults, uint64_t n,
                                                       uint64_t per) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t home = (uint32_t)(p / per);
    state[p] = (1u << home) | (home << 8) | (2u << 16);
    faults[p] = 0;
  }
}

// ---------------------------------------------------------------- A: block tails
__global__ __launch_bounds__(256) void coh_tail_kernel(const uint32_t* __restrict__ state,
                                                       uint64_t n_pages,
                                                       const uint64_t* __restrict__ ev, uint64_t n,
                                                       uint64_t nb, uint32_t* __restrict__ agg,
                                                       uint32_t* __restrict__ last_head,
                                                       uint32_t* __restrict__ head_state) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const uint64_t lo = b * kCohBlock;
  const uint64_t hi = min(n, lo + kCohBlock);
  uint32_t acc = 0, lh = kNoHead, hs = 0;
  bool found = false;
  for (uint64_t top = hi; top > lo && !found; top = (top - lo > 64) ? top - 64 : lo) {
    const uint64_t wlo = (top - lo > 64) ? top - 64 : lo;
    const uint64_t idx = wlo + lane;
    const bool valid = idx < top;
    const uint64_t e = valid ? ev[idx] : 0;
    const uint64_t ep = (valid && idx > 0) ? ev[idx - 1] : 0;
    const bool head = valid && (idx == 0 || ev_page(e) != ev_page(ep));
    const uint64_t hm = __ballot(head);
    uint32_t hl = 0;
    if (hm) {
      found = true;
      hl = 63u - (uint32_t)__clzll(hm);
    }
    uint32_t te = (valid && (!found || lane >= hl)) ? ev_transform(e) : 0u;
    if (found && lane == hl) {
      const uint64_t p = ev_page(e);
      const uint32_t s0 = (p < n_pages) ? state[p] : 0u;
      te = tcompose(kConst | s0, te);
      lh = (uint32_t)(idx - lo);
      hs = s0;
    }
    acc = tcompose(wave_reduce_compose(te), acc);
  }
  if (found) {  // broadcast from the head lane
    const uint64_t hm = __ballot(lh != kNoHead);
    const uint32_t src = (uint32_t)__builtin_ctzll(hm);
    lh = __shfl(lh, src, 64);
    hs = __shfl(hs, src, 64);
  }
  if (lane == 0) {
    agg[b] = acc;
    last_head[b] = lh;
    head_state[b] = hs;
  }
}

// ---------------------------------------------------------------- B: scan of block aggregates
__global__ __launch_bounds__(1024) void coh_scan_kernel(const uint32_t* __restrict__ agg,
                                                        uint64_t nb,
                                                        uint32_t* __restrict__ carry) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t lo = min(nb, (uint64_t)t * per), hi = min(nb, lo + per);
  uint32_t s = 0;
  for (uint64_t b = lo; b < hi; ++b) s = tcompose(s, agg[b]);
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = (t >= d) ? part[t - d] : 0u;
    __syncthreads();
    part[t] = tcompose(v, part[t]);
    __syncthreads();
  }
  uint32_t run = (t > 0) ? part[t - 1] : 0u;
  for (uint64_t b = lo; b < hi; ++b) {
    carry[b] = run;
    run = tcompose(run, agg[b]);
  }
}

// ---------------------------------------------------------------- C: apply the batch
__device__ __forceinline__ uint32_t pad_idx(uint32_t x) { return x + ((x >> 4) << 1); }

__global__ __launch_bounds__(256) void coh_apply_kernel(
    uint32_t* __restrict__ state, uint32_t* __restrict__ faults, uint64_t n_pages,
    const uint64_t* __restrict__ ev, uint64_t n, const uint32_t* __restrict__ carry,
    const uint32_t* __restrict__ last_head, const uint32_t* __restrict__ head_state,
    uint32_t* __restrict__ partial, uint32_t* __restrict__ err) {
  __shared__ uint64_t sev[kCohBlock + kCohBlock / 8];
  __shared__ uint32_t wtot[4];
  __shared__ uint32_t red[4][10];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint64_t b = blockIdx.x;
  const uint64_t b0 = b * kCohBlock;
  const uint32_t cnt = (uint32_t)min((uint64_t)kCohBlock, n - b0);
  for (uint32_t x = t; x < kCohBlock; x += 256) sev[pad_idx(x)] = (x < cnt) ? ev[b0 + x] : 0ull;
  __syncthreads();

  const uint32_t first = t * kCohK;  // block-relative index of this thread's first event
  const uint32_t lh = last_head[b], lhs = head_state[b];
  uint64_t e[kCohK];
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) e[k] = sev[pad_idx(first + k)];
  const uint64_t eprev = (first > 0) ? sev[pad_idx(first - 1)] : (b0 > 0 ? ev[b0 - 1] : 0ull);
  const bool has_prev = (first > 0) || (b0 > 0);
  uint64_t enext = 0;
  bool has_next = false;
  if (first + kCohK < cnt) {
    enext = sev[pad_idx(first + kCohK)];
    has_next = true;
  } else if (first + kCohK == cnt && b0 + cnt < n) {
    enext = ev[b0 + cnt];
    has_next = true;
  }
  uint32_t bad = 0;

  // Per-event head / end flags (bit k).
  // Head states are read here, before the first barrier below; every page-table write of this
  // kernel comes after that barrier, so no thread reads a state another thread has rewritten.
  uint32_t hmask = 0, emask = 0;
  uint32_t hsv[kCohK];
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    hsv[k] = 0;
    if (first + k >= cnt) continue;
    const uint64_t pg = ev_page(e[k]);
    const bool hp = (k == 0) ? has_prev : true;
    const uint64_t pp = (k == 0) ? ev_page(eprev) : ev_page(e[k > 0 ? k - 1 : 0]);
    if (!hp || pg != pp) {
      hmask |= 1u << k;
      hsv[k] = (first + k == lh) ? lhs : (pg < n_pages ? state[pg] : 0u);
    }
    if (hp && pg < pp) bad = 1;
    if (pg >= n_pages) bad = 1;
    const bool hn = (k + 1 < kCohK && first + k + 1 < cnt) ? true : has_next;
    const uint64_t pn = (k + 1 < kCohK && first + k + 1 < cnt) ? ev_page(e[k + 1 < kCohK ? k + 1 : k])
                                                               : ev_page(enext);
    if (!hn || pn != pg) emask |= 1u << k;
  }

  // Thread aggregate.
  uint32_t a = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k >= cnt) continue;
    const uint32_t te = ev_transform(e[k]);
    if ((hmask >> k) & 1u) {
      a = tcompose(kConst | hsv[k], te);
    } else {
      a = tcompose(a, te);
    }
  }
  // Block exclusive scan of the aggregates, carry-in first.
  uint32_t inc = wave_incl_compose(a);
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  uint32_t pre = carry[b];
  for (uint32_t w = 0; w < wave; ++w) pre = tcompose(pre, wtot[w]);
  uint32_t ex = __shfl_up(inc, 1, 64);
  uint32_t cur = (lane == 0) ? pre : tcompose(pre, ex);
  __syncthreads();

  // Walk: incoming state of every event.
  uint64_t nf_lo = 0, nf_hi = 0;
  uint32_t inv = 0, xfer = 0, fmask = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k >= cnt) continue;
    const uint64_t pg = ev_page(e[k]);
    const uint32_t node = (uint32_t)(e[k] >> 1) & 7u;
    const bool wr = e[k] & 1u;
    uint32_t S;
    if ((hmask >> k) & 1u)
      S = kConst | hsv[k];
    else
      S = cur;
    if (!(S & kConst)) bad = 1;
    const uint32_t cs = S & 0xFFu, owner = (S >> 8) & 0xFFu, st = (S >> 16) & 3u;
    const uint32_t bit = 1u << node;
    uint32_t fault;
    if (!wr) {
      fault = (cs & bit) ? 0u : 1u;
    } else {
      fault = (st == 2u && owner == node) ? 0u : 1u;
      if (fault) {
        inv += (uint32_t)__popc(cs & ~bit);
        xfer += (owner != node) ? 1u : 0u;
      }
    }
    const uint64_t inc1 = (uint64_t)fault << (16 * (node & 3u));
    if (node < 4) nf_lo += inc1; else nf_hi += inc1;
    fmask |= fault << k;
    cur = tcompose(S, ev_transform(e[k]));
    if (((emask >> k) & 1u) && pg < n_pages) state[pg] = cur & ~kConst;
  }

  // Segmented sum of faults -> per-page fault counters.
  uint32_t sv = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k >= cnt) continue;
    sv = segsum(sv, (((hmask >> k) & 1u) ? kConst : 0u) | ((fmask >> k) & 1u));
  }
  uint32_t sinc = wave_incl_segsum(sv);
  if (lane == 63) wtot[wave] = sinc;
  __syncthreads();
  uint32_t spre = 0;
  for (uint32_t w = 0; w < wave; ++w) spre = segsum(spre, wtot[w]);
  const uint32_t sex = __shfl_up(sinc, 1, 64);
  uint32_t run_f = (lane == 0) ? spre : segsum(spre, sex);
  bool head_in_block = (run_f & kConst) != 0;
  uint32_t running = run_f & ~kConst;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k >= cnt) continue;
    if ((hmask >> k) & 1u) {
      running = 0;
      head_in_block = true;
    }
    running += (fmask >> k) & 1u;
    const bool seg_end = (emask >> k) & 1u;
    const bool blk_end = (first + k + 1 == cnt);
    if ((seg_end || blk_end) && running) {
      const uint64_t pg = ev_page(e[k]);
      if (pg < n_pages) {
        if (seg_end && head_in_block)
          faults[pg] += running;
        else
          atomicAdd(&faults[pg], running);
      }
    }
  }

  // Block partial row: inv, xfer, node faults 0..7.
  uint32_t vals[10];
  vals[0] = inv;
  vals[1] = xfer;
  const uint64_t slo = wave_sum64(nf_lo), shi = wave_sum64(nf_hi);
  const uint32_t sinv = (uint32_t)wave_sum64(inv), sxf = (uint32_t)wave_sum64(xfer);
  vals[0] = sinv;
  vals[1] = sxf;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    vals[2 + q] = (uint32_t)(slo >> (16 * q)) & 0xFFFFu;
    vals[6 + q] = (uint32_t)(shi >> (16 * q)) & 0xFFFFu;
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 10; ++q) red[wave][q] = vals[q];
  }
  const uint64_t anybad = __ballot(bad != 0);
  if (anybad && lane == 0) atomicOr(err, 2u);
  __syncthreads();
  if (t < 10) partial[b * 10 + t] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}

// ---------------------------------------------------------------- D: totals
__global__ __launch_bounds__(256) void coh_reduce_kernel(const uint32_t* __restrict__ partial,
                                                         uint64_t nb,
                                                         unsigned long long* __restrict__ totals) {
  __shared__ uint64_t red[4][10];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t acc[10];
#pragma unroll
  for (int q = 0; q < 10; ++q) acc[q] = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb;
       b += (uint64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int q = 0; q < 10; ++q) acc[q] += partial[b * 10 + q];
  }
#pragma unroll
  for (int q = 0; q < 10; ++q) acc[q] = wave_sum64(acc[q]);
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < 10; ++q) red[wave][q] = acc[q];
  __syncthreads();
  if (threadIdx.x < 10) {
    const uint64_t s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                       red[3][threadIdx.x];
    if (s) atomicAdd(&totals[threadIdx.x], (unsigned long long)s);
  }
}

// ---------------------------------------------------------------- events (SPEC §6)
__global__ __launch_bounds__(256) void gen_events_kernel(uint64_t* __restrict__ events,
                                                         const uint64_t* __restrict__ offsets,
                                                         uint64_t first_page, uint64_t n,
                                                         uint64_t seed, uint32_t n_nodes,
                                                         uint32_t write_pct) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n;
       i += (uint64_t)gridDim.x * 4) {
    const uint64_t p = first_page + i;
    const uint64_t o = offsets[i], c = offsets[i + 1] - o;
    for (uint64_t j = lane; j < c; j += 64) {
      const uint64_t node = hash3(seed ^ 0x40DEull, p, j) % n_nodes;
      const uint64_t rw = (hash3(seed ^ 0x3217Eull, p, j) % 100u) < write_pct;
      events[o + j] = (p << 4) | (node << 1) | rw;
    }
  }
}

// ---------------------------------------------------------------- launchers
static inline uint64_t coh_blocks(uint64_t n) { return (n + kCohBlock - 1) / kCohBlock; }

uint64_t coh_workspace_bytes(uint64_t n_events) {
  const uint64_t nb = coh_blocks(n_events);
  return nb * 4 * 4 + nb * 10 * 4 + 256;
}

hipError_t launch_coh_init(uint32_t* state, uint32_t* faults, uint64_t n_pages, uint32_t n_nodes,
                           hipStream_t s) {
  if (n_pages == 0) return hipSuccess;
  const uint64_t per = (n_pages + n_nodes - 1) / n_nodes;
  uint64_t g = (n_pages + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(coh_init_kernel, dim3((unsigned)g), dim3(256), 0, s, state, faults, n_pages,
                     per);
  return hipGetLastError();
}

hipError_t launch_coherence(uint32_t* state, uint32_t* faults, uint64_t n_pages,
                            const uint64_t* events, uint64_t n_events, uint64_t* totals,
                            uint8_t* ws, uint64_t ws_bytes, uint32_t* err, hipStream_t s,
                            Prof* prof) {
  hipError_t r = hipMemsetAsync(totals, 0, 10 * sizeof(uint64_t), s);
  if (r != hipSuccess || n_events == 0) return r;
  const uint64_t nb = coh_blocks(n_events);
  if (coh_workspace_bytes(n_events) > ws_bytes) return hipErrorInvalidValue;
  uint32_t* agg = reinterpret_cast<uint32_t*>(ws);
  uint32_t* lh = agg + nb;
  uint32_t* hs = lh + nb;
  uint32_t* carry = hs + nb;
  uint32_t* partial = carry + nb;
  {
    ProfScope ps(prof, 5, s);
    hipLaunchKernelGGL(coh_tail_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, state,
                       n_pages, events, n_events, nb, agg, lh, hs);
  }
  {
    ProfScope ps(prof, 6, s);
    hipLaunchKernelGGL(coh_scan_kernel, dim3(1), dim3(1024), 0, s, agg, nb, carry);
  }
  {
    ProfScope ps(prof, 7, s);
    hipLaunchKernelGGL(coh_apply_kernel, dim3((unsigned)nb), dim3(256), 0, s, state, faults,
                       n_pages, events, n_events, carry, lh, hs, partial, err);
  }
  uint64_t g = (nb + 255) / 256;
  if (g > 1024) g = 1024;
  {
    ProfScope ps(prof, 8, s);
    hipLaunchKernelGGL(coh_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, partial, nb,
                       reinterpret_cast<unsigned long long*>(totals));
  }
  return hipGetLastError();
}

hipError_t launch_gen_events(uint64_t* events, const uint64_t* offsets, uint64_t first_page,
                             uint64_t n, uint64_t seed, uint32_t n_nodes, uint32_t write_pct,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t g = (n + 3) / 4;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(gen_events_kernel, dim3((unsigned)g), dim3(256), 0, s, events, offsets,
                     first_page, n, seed, n_nodes, write_pct);
  return hipGetLastError();
}

}  // namespace gdsm
