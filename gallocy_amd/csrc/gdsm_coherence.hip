// Batched page coherence for gfx950 (SPEC §5): the per-page state machine that the reference
// only describes (resources/NUTSHELL.md:52-69, resources/IMPLEMENTATION.md:137-249) on the
// fields of its unused ApplicationMemory record (gallocy/include/gallocy/models.h:171-213).
//
// Page table in HBM: one u64 per page, `state | faults << 32` (SPEC §5 bit layout for state),
// so a segment head costs one 8-B load and a segment that closes inside a block one 8-B store.
//
// The sequential fold is recast as a scan over 32-bit transforms (SPEC §5a, state part only):
//   READ(R)  : copyset |= R; EXCLUSIVE -> SHARED if R is not inside the copyset   (bit 31 = 0)
//   CONST(s) : the state becomes s                                              (bit 31 = 1)
// A read by n is READ({n}); a write by n is CONST(EXCLUSIVE, owner n, copyset {n}, dirty);
// the first event of a page is seeded with CONST(page-table state). Composition is
// associative, so every event's incoming state is an exclusive scan, and each event's fault /
// invalidation / transfer follows from its incoming state alone. Per-page fault counts are a
// segmented sum seeded with the page's old count at its head.
//
// Kernels (no workgroup ever waits on another; events are blocked by kCohBlock = 2048):
//   A coh_tail_kernel   one wave per block: the block's aggregate transform. If the block's last
//                       64 events hold a segment head only that tail is read; otherwise (a hot
//                       page covering most of the block) the wave folds the whole block, 32
//                       events per lane. Records the last head's page-table word so pass C never
//                       reads a word another block writes.
//   B coh_group/_top/_rescan  exclusive scan of the block aggregates (groups of 1024 blocks).
//   C coh_apply_kernel  per block: events staged in LDS, 8 events per thread, block scan with
//                       the carry-in, per-event faults, segmented fault sums, final words
//                       written at segment ends (atomics only for segments split across
//                       blocks), one partial row of totals per block.
//   D coh_reduce_kernel partial rows -> the 10 batch totals.
#include "gdsm_common.h"
#include "gdsm_launch.h"

namespace gdsm {

constexpr uint32_t kConst = 1u << 31;
constexpr uint32_t kCohK = 8;                   // events per thread
constexpr uint32_t kCohBlock = 256 * kCohK;     // events per block
constexpr uint32_t kCohGroup = 1024;            // blocks per scan group
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

// Ordered reduction over the wave: every lane gets v_0 ∘ v_1 ∘ … ∘ v_63.
__device__ __forceinline__ uint32_t wave_reduce_compose(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_down(v, d, 64);
    if (lane + d < 64u) v = tcompose(v, t);
  }
  return lane_bcast(v, 0);
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

// Exclusive block-wide compose scan for 256 threads (4 waves); `carry` precedes thread 0.
__device__ __forceinline__ uint32_t block_excl_compose(uint32_t a, uint32_t carry,
                                                       uint32_t* wtot) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_compose(a);
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  uint32_t pre = carry;
  for (uint32_t w = 0; w < wave; ++w) pre = tcompose(pre, wtot[w]);
  const uint32_t ex = __shfl_up(inc, 1, 64);
  __syncthreads();
  return lane == 0 ? pre : tcompose(pre, ex);
}

// ---------------------------------------------------------------- init
__global__ __launch_bounds__(256) void coh_init_kernel(uint64_t* __restrict__ pt, uint64_t n,
                                                       uint64_t per) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t home = (uint32_t)(p / per);
    pt[p] = (uint64_t)((1u << home) | (home << 8) | (2u << 16));
  }
}

// ---------------------------------------------------------------- A: block aggregates
__global__ __launch_bounds__(256) void coh_tail_kernel(const uint64_t* __restrict__ pt,
                                                       uint64_t n_pages,
                                                       const uint64_t* __restrict__ ev, uint64_t n,
                                                       uint64_t nb, uint32_t* __restrict__ agg,
                                                       uint32_t* __restrict__ last_head,
                                                       uint64_t* __restrict__ head_pt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const uint64_t lo = b * kCohBlock;
  const uint64_t hi = min(n, lo + kCohBlock);
  // 1) the last 64 events: a head there means only the tail matters
  const uint64_t wlo = (hi - lo > 64) ? hi - 64 : lo;
  const uint64_t idx = wlo + lane;
  const bool valid = idx < hi;
  const uint64_t e = valid ? ev[idx] : 0;
  const uint64_t ep = (valid && idx > 0) ? ev[idx - 1] : 0;
  const bool head = valid && (idx == 0 || ev_page(e) != ev_page(ep));
  const uint64_t hm = __ballot(head);
  uint32_t acc, lh = kNoHead;
  uint64_t hp = 0;
  if (hm) {
    const uint32_t hl = 63u - (uint32_t)__clzll(hm);
    uint32_t te = (valid && lane >= hl) ? ev_transform(e) : 0u;
    if (lane == hl) {
      const uint64_t p = ev_page(e);
      hp = (p < n_pages) ? pt[p] : 0ull;
      te = tcompose(kConst | (uint32_t)hp, te);
    }
    acc = wave_reduce_compose(te);
    lh = (uint32_t)(wlo + hl - lo);
    hp = lane_bcast64(hp, (int)hl);
  } else {
    // 2) no head in the tail: fold the whole block, lane l takes a contiguous share
    const uint32_t cnt = (uint32_t)(hi - lo);
    const uint32_t per = (cnt + 63) / 64;
    const uint32_t a0 = min(cnt, lane * per), a1 = min(cnt, a0 + per);
    uint32_t f = 0, mylh = kNoHead;
    uint64_t myhp = 0;
    uint64_t prev = (lo + a0 > 0 && a0 < a1) ? ev[lo + a0 - 1] : 0;
    for (uint32_t x = a0; x < a1; ++x) {
      const uint64_t ex = ev[lo + x];
      const uint32_t te = ev_transform(ex);
      if (lo + x == 0 || ev_page(ex) != ev_page(prev)) {
        const uint64_t p = ev_page(ex);
        myhp = (p < n_pages) ? pt[p] : 0ull;
        mylh = x;
        f = tcompose(kConst | (uint32_t)myhp, te);
      } else {
        f = tcompose(f, te);
      }
      prev = ex;
    }
    acc = wave_reduce_compose(f);
    const uint64_t any = __ballot(mylh != kNoHead);
    if (any) {
      const uint32_t src = 63u - (uint32_t)__clzll(any);
      lh = lane_bcast(mylh, (int)src);
      hp = lane_bcast64(myhp, (int)src);
    }
  }
  if (lane == 0) {
    agg[b] = acc;
    last_head[b] = lh;
    head_pt[b] = hp;
  }
}

// ---------------------------------------------------------------- B: scan of block aggregates
// B1: one workgroup per group of kCohGroup blocks -> group aggregate.
__global__ __launch_bounds__(256) void coh_group_kernel(const uint32_t* __restrict__ agg,
                                                        uint64_t nb, uint32_t* __restrict__ gagg) {
  __shared__ uint32_t wtot[4];
  const uint64_t g0 = (uint64_t)blockIdx.x * kCohGroup + threadIdx.x * 4;
  uint32_t a = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (g0 + q < nb) a = tcompose(a, agg[g0 + q]);
  const uint32_t inc = wave_incl_compose(a);
  if ((threadIdx.x & 63) == 63) wtot[threadIdx.x >> 6] = inc;
  __syncthreads();
  if (threadIdx.x == 0)
    gagg[blockIdx.x] = tcompose(tcompose(wtot[0], wtot[1]), tcompose(wtot[2], wtot[3]));
}

// B2: one workgroup: exclusive scan of the group aggregates, in place.
__global__ __launch_bounds__(1024) void coh_top_kernel(uint32_t* __restrict__ g, uint64_t ng) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (ng + 1023) / 1024;
  const uint64_t lo = min(ng, (uint64_t)t * per), hi = min(ng, lo + per);
  uint32_t s = 0;
  for (uint64_t b = lo; b < hi; ++b) s = tcompose(s, g[b]);
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
    const uint32_t v = g[b];
    g[b] = run;
    run = tcompose(run, v);
  }
}

// B3: per group: exclusive scan of its blocks, seeded with the group's carry.
__global__ __launch_bounds__(256) void coh_rescan_kernel(const uint32_t* __restrict__ agg,
                                                         uint64_t nb,
                                                         const uint32_t* __restrict__ gcarry,
                                                         uint32_t* __restrict__ carry) {
  __shared__ uint32_t wtot[4];
  const uint64_t g0 = (uint64_t)blockIdx.x * kCohGroup + threadIdx.x * 4;
  uint32_t v[4];
  uint32_t a = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = (g0 + q < nb) ? agg[g0 + q] : 0u;
    a = tcompose(a, v[q]);
  }
  uint32_t run = block_excl_compose(a, gcarry[blockIdx.x], wtot);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (g0 + q < nb) carry[g0 + q] = run;
    run = tcompose(run, v[q]);
  }
}

// ---------------------------------------------------------------- C: apply the batch
__device__ __forceinline__ uint32_t pad_idx(uint32_t x) { return x + (x >> 3); }  // +8 B / 64 B

__global__ __launch_bounds__(256) void coh_apply_kernel(
    uint64_t* __restrict__ pt, uint64_t n_pages, const uint64_t* __restrict__ ev, uint64_t n,
    const uint32_t* __restrict__ carry, const uint32_t* __restrict__ last_head,
    const uint64_t* __restrict__ head_pt, uint32_t* __restrict__ partial,
    uint32_t* __restrict__ err) {
  __shared__ uint64_t sev[kCohBlock + kCohBlock / 8];
  __shared__ uint32_t wtot[4];
  __shared__ uint32_t red[4][10];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint64_t b = blockIdx.x;
  const uint64_t b0 = b * kCohBlock;
  const uint32_t cnt = (uint32_t)min((uint64_t)kCohBlock, n - b0);
  for (uint32_t x = t; x < kCohBlock; x += 256) sev[pad_idx(x)] = (x < cnt) ? ev[b0 + x] : 0ull;
  const uint64_t before = (b0 > 0) ? ev[b0 - 1] : 0ull;
  const bool has_after = b0 + cnt < n;
  const uint64_t after = has_after ? ev[b0 + cnt] : 0ull;
  __syncthreads();

  const uint32_t first = t * kCohK;
  const uint32_t lh = last_head[b];
  const uint64_t lhp = head_pt[b];
  uint32_t* pst = reinterpret_cast<uint32_t*>(pt);  // state words at even indices
  uint32_t* pfl = pst + 1;                          // fault words at odd indices

  // ---- flags, sortedness, head words (every page-table read is before the first barrier
  // below; every page-table write of this kernel is after it)
  uint64_t e[kCohK];
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) e[k] = sev[pad_idx(first + k)];
  const uint64_t eprev = (first > 0) ? sev[pad_idx(first - 1)] : before;
  const uint64_t enext = (first + kCohK < cnt) ? sev[pad_idx(first + kCohK)] : after;
  uint32_t hmask = 0, emask = 0, bad = 0;
  uint32_t hs[kCohK], hf[kCohK];
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    hs[k] = 0;
    hf[k] = 0;
    const uint32_t x = first + k;
    if (x < cnt) {
      const uint64_t pg = ev_page(e[k]);
      const bool hp = (k == 0) ? (b0 + x > 0) : true;
      const uint64_t pp = ev_page(k == 0 ? eprev : e[k > 0 ? k - 1 : 0]);
      if (!hp || pg != pp) {
        hmask |= 1u << k;
        uint64_t w = 0;
        if (x == lh) w = lhp;
        else if (pg < n_pages) w = pt[pg];
        hs[k] = (uint32_t)w;
        hf[k] = (uint32_t)(w >> 32);
      }
      if (hp && pg < pp) bad = 1;
      if (pg >= n_pages) bad = 1;
      const bool last_in_blk = (x + 1 == cnt);
      const bool hn = last_in_blk ? has_after : true;
      const uint64_t pn = ev_page((k + 1 < kCohK && !last_in_blk) ? e[k + 1 < kCohK ? k + 1 : k]
                                                                  : enext);
      if (!hn || pn != pg) emask |= 1u << k;
    }
  }

  // ---- thread aggregate -> exclusive scan with the carry-in
  uint32_t a = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k < cnt) {
      const uint32_t te = ev_transform(e[k]);
      a = ((hmask >> k) & 1u) ? tcompose(kConst | hs[k], te) : tcompose(a, te);
    }
  }
  uint32_t cur = block_excl_compose(a, carry[b], wtot);

  // ---- walk: incoming state of every event -> faults / invalidations / transfers
  uint64_t nf_lo = 0, nf_hi = 0;
  uint32_t inv = 0, xfer = 0, fmask = 0;
  uint32_t endst[kCohK];
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    endst[k] = 0;
    if (first + k < cnt) {
      const uint32_t node = (uint32_t)(e[k] >> 1) & 7u;
      const bool wr = e[k] & 1u;
      const uint32_t S = ((hmask >> k) & 1u) ? (kConst | hs[k]) : cur;
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
      endst[k] = cur & ~kConst;
    }
  }

  // ---- segmented fault sums, seeded at each head with the page's old count
  uint32_t sv = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (first + k < cnt) {
      const uint32_t f = (fmask >> k) & 1u;
      sv = segsum(sv, ((hmask >> k) & 1u) ? (kConst | (hf[k] + f)) : f);
    }
  }
  const uint32_t sinc = wave_incl_segsum(sv);
  if (lane == 63) wtot[wave] = sinc;
  __syncthreads();
  uint32_t spre = 0;
  for (uint32_t w = 0; w < wave; ++w) spre = segsum(spre, wtot[w]);
  const uint32_t sex = __shfl_up(sinc, 1, 64);
  const uint32_t run_f = (lane == 0) ? spre : segsum(spre, sex);
  bool head_in_block = (run_f & kConst) != 0;
  uint32_t running = run_f & ~kConst;
  const uint32_t lh_old = (uint32_t)(lhp >> 32);
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    const uint32_t x = first + k;
    if (x < cnt) {
      const uint32_t f = (fmask >> k) & 1u;
      if ((hmask >> k) & 1u) {
        running = hf[k] + f;
        head_in_block = true;
      } else {
        running += f;
      }
      const uint64_t pg = ev_page(e[k]);
      if (pg < n_pages) {
        if ((emask >> k) & 1u) {
          if (head_in_block) {
            pt[pg] = (uint64_t)endst[k] | ((uint64_t)running << 32);  // closed here
          } else {
            pst[2 * pg] = endst[k];                                   // opened earlier
            if (running) atomicAdd(&pfl[2 * pg], running);
          }
        } else if (x + 1 == cnt) {                                   // continues
          const uint32_t add = head_in_block ? running - lh_old : running;
          if (add) atomicAdd(&pfl[2 * pg], add);
        }
      }
    }
  }

  // ---- block partial row: inv, xfer, node faults 0..7
  const uint64_t slo = wave_sum64(nf_lo), shi = wave_sum64(nf_hi);
  const uint32_t sinv = (uint32_t)wave_sum64(inv), sxf = (uint32_t)wave_sum64(xfer);
  const uint64_t anybad = __ballot(bad != 0);
  if (lane == 0) {
    red[wave][0] = sinv;
    red[wave][1] = sxf;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      red[wave][2 + q] = (uint32_t)(slo >> (16 * q)) & 0xFFFFu;
      red[wave][6 + q] = (uint32_t)(shi >> (16 * q)) & 0xFFFFu;
    }
    if (anybad) atomicOr(err, 2u);
  }
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
static inline uint64_t coh_groups(uint64_t nb) { return (nb + kCohGroup - 1) / kCohGroup; }

uint64_t coh_workspace_bytes(uint64_t n_events) {
  const uint64_t nb = coh_blocks(n_events);
  // head_pt (u64) + agg, last_head, carry (u32 each) + partial rows (10 u32) + groups
  return nb * (8 + 4 * 3 + 40) + coh_groups(nb) * 4 + 512;
}

hipError_t launch_coh_init(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes, hipStream_t s) {
  if (n_pages == 0) return hipSuccess;
  const uint64_t per = (n_pages + n_nodes - 1) / n_nodes;
  uint64_t g = (n_pages + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(coh_init_kernel, dim3((unsigned)g), dim3(256), 0, s, pt, n_pages, per);
  return hipGetLastError();
}

hipError_t launch_coherence(uint64_t* pt, uint64_t n_pages, const uint64_t* events,
                            uint64_t n_events, uint64_t* totals, uint8_t* ws, uint64_t ws_bytes,
                            uint32_t* err, hipStream_t s, Prof* prof) {
  hipError_t r = hipMemsetAsync(totals, 0, 10 * sizeof(uint64_t), s);
  if (r != hipSuccess || n_events == 0) return r;
  const uint64_t nb = coh_blocks(n_events), ng = coh_groups(nb);
  if (coh_workspace_bytes(n_events) > ws_bytes) return hipErrorInvalidValue;
  uint64_t* head_pt = reinterpret_cast<uint64_t*>(ws);
  uint32_t* agg = reinterpret_cast<uint32_t*>(head_pt + nb);
  uint32_t* lh = agg + nb;
  uint32_t* carry = lh + nb;
  uint32_t* partial = carry + nb;
  uint32_t* groups = partial + nb * 10;
  {
    ProfScope ps(prof, 5, s);
    hipLaunchKernelGGL(coh_tail_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, pt,
                       n_pages, events, n_events, nb, agg, lh, head_pt);
  }
  {
    ProfScope ps(prof, 6, s);
    hipLaunchKernelGGL(coh_group_kernel, dim3((unsigned)ng), dim3(256), 0, s, agg, nb, groups);
    hipLaunchKernelGGL(coh_top_kernel, dim3(1), dim3(1024), 0, s, groups, ng);
    hipLaunchKernelGGL(coh_rescan_kernel, dim3((unsigned)ng), dim3(256), 0, s, agg, nb, groups,
                       carry);
  }
  {
    ProfScope ps(prof, 7, s);
    hipLaunchKernelGGL(coh_apply_kernel, dim3((unsigned)nb), dim3(256), 0, s, pt, n_pages,
                       events, n_events, carry, lh, head_pt, partial, err);
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
