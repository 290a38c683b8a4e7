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
//                       page covering most of the block) the wave folds the whole block in
//                       coalesced 64-event steps. Records the last head's page-table word so
//                       pass C never reads a word another block writes.
//   B coh_group/_top/_rescan  exclusive scan of the block aggregates (groups of 1024 blocks).
//   C coh_apply_block_kernel  one block per workgroup, 8 consecutive events per thread, each
//                       wave on its own 512 events (coh_wave): DPP scans, one barrier for the
//                       wave aggregates, per-event faults from a (last CONST, reads since)
//                       state, page-table words loaded / stored through a per-wave LDS head
//                       list by consecutive lanes, one partial row of totals per wave.
//   D coh_reduce_kernel partial rows -> the 10 batch totals.
#include "gdsm_common.h"
#include "gdsm_launch.h"

#include <stdlib.h>
#include <string.h>

namespace gdsm {

constexpr uint32_t kConst = 1u << 31;
constexpr uint32_t kCohK = 8;                   // events per thread
constexpr uint32_t kCohBlock = 256 * kCohK;     // events per block
constexpr uint32_t kSamp = kCohBlock / 64;       // pass A: sampling stride over a block
static_assert(kSamp <= 64, "pass A samples the block with one wave");
constexpr uint32_t kCohGroup = 1024;            // blocks per scan group
constexpr uint32_t kNoHead = 0xFFFFFFFFu;
constexpr uint64_t kNoHead64 = ~0ull;

#ifdef GDSM_COH_STAMPS
// Debug build only: per-wave phase time stamps (s_memtime) of every 64th block.
__device__ unsigned long long g_coh_stamps[8192 * 4 * 8];
#define COH_STAMP(i)                                                                         \
  do {                                                                                        \
    if ((blockIdx.x & 63) == 0 && blockIdx.x / 64 < 8192 && (threadIdx.x & 63) == 0)          \
      g_coh_stamps[((blockIdx.x / 64) * 4 + (threadIdx.x >> 6)) * 8 + (i)] =                  \
          __builtin_amdgcn_s_memtime();                                                       \
  } while (0)
#else
#define COH_STAMP(i) \
  do {               \
  } while (0)
#endif

// a, then b. Branch-free: for a READ b the copyset gains R, and a CONST(EXCLUSIVE) a turns
// SHARED (state bits 10 -> 01) when R holds a node outside its copyset.
__device__ __forceinline__ uint32_t tcompose(uint32_t a, uint32_t b) {
  const uint32_t R = b & 0xFFu;
  const bool excl = ((a >> 16) & 3u) == 2u;
  const bool flip = (a & kConst) && excl && (R & ~a & 0xFFu);
  const uint32_t rr = (a | R) ^ (flip ? 0x30000u : 0u);
  return (b & kConst) ? b : rr;
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

// The same two scans on DPP (no LDS traffic): 0 is the identity of tcompose and of segsum,
// and it is what an out-of-range or masked-off DPP source reads.
__device__ __forceinline__ uint32_t wave_incl_compose_dpp(uint32_t v) {
  v = tcompose(dpp0<0x111>(v), v);
  v = tcompose(dpp0<0x112>(v), v);
  v = tcompose(dpp0<0x114>(v), v);
  v = tcompose(dpp0<0x118>(v), v);
  v = tcompose(dpp0<0x142, 0xA>(v), v);
  v = tcompose(dpp0<0x143, 0xC>(v), v);
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_segsum_dpp(uint32_t v) {
  v = segsum(dpp0<0x111>(v), v);
  v = segsum(dpp0<0x112>(v), v);
  v = segsum(dpp0<0x114>(v), v);
  v = segsum(dpp0<0x118>(v), v);
  v = segsum(dpp0<0x142, 0xA>(v), v);
  v = segsum(dpp0<0x143, 0xC>(v), v);
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
  } else if (const uint64_t wm = __ballot(valid && (e & 1u))) {
    // 2) no head in the tail but a write in it: the aggregate only depends on the events from
    //    the tail's last write on. The block's last head (if any) is the first event of the
    //    tail's page: found by sampling every kSamp-th event, then the kSamp events before the
    //    hit.
    const uint32_t lw = 63u - (uint32_t)__clzll(wm);
    acc = wave_reduce_compose((valid && lane >= lw) ? ev_transform(e) : 0u);
    const uint64_t P = ev_page(lane_bcast64(e, 63));
    uint64_t h = kNoHead64;  // global index of the last head
    if (hi - lo <= 64) {
      // the whole block is the tail and holds no head
    } else if (ev_page(ev[lo]) == P) {
      // the block starts on P too: the batch is sorted, so the whole block is P's (a hot page
      // spanning blocks); its head, if any, is its first event
      if (lo == 0 || ev_page(ev[lo - 1]) != P) h = lo;
    } else {
      const uint64_t sidx = lo + (uint64_t)lane * kSamp;
      const bool in = sidx < wlo;
      const uint64_t sm = __ballot(in && ev_page(ev[sidx]) == P);
      const uint32_t j0 =
          sm ? (uint32_t)__builtin_ctzll(sm) : (uint32_t)((wlo - lo + kSamp - 1) / kSamp);
      if (j0 == 0) {  // the block starts inside P's segment
        if (lo == 0 || ev_page(ev[lo - 1]) != P) h = lo;
      } else {
        const uint64_t w0 = lo + (uint64_t)(j0 - 1) * kSamp + 1;  // after the last sample below P
        const uint64_t ix = w0 + lane;
        const uint64_t hm2 = __ballot(lane < kSamp && ix <= wlo && ev_page(ev[ix]) == P);
        h = w0 + (uint64_t)__builtin_ctzll(hm2);  // hm2 != 0: ev[wlo] has page P
      }
    }
    if (h != kNoHead64) {
      lh = (uint32_t)(h - lo);
      hp = (P < n_pages) ? pt[P] : 0ull;
      // a head inside the block seeds the fold: CONST(page-table state) before the last write
      // changes nothing (the write replaces it), so acc stands
    }
  } else {
    // 3) no head and no write in the tail: fold the whole block in 64-event steps of coalesced
    //    loads (8 steps in flight at a time), one ordered wave reduction per step.
    acc = 0;
    uint64_t carry_ev = (lo > 0) ? ev[lo - 1] : 0;  // event before the current step's lane 0
    for (uint64_t j0 = lo; j0 < hi; j0 += 512) {
      uint64_t x[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t ix = j0 + 64 * q + lane;
        x[q] = (ix < hi) ? ev[ix] : 0ull;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t ix = j0 + 64 * q + lane;
        const bool v = ix < hi;
        uint64_t pv = (uint64_t)from_prev_lane((uint32_t)x[q]) |
                      ((uint64_t)from_prev_lane((uint32_t)(x[q] >> 32)) << 32);
        if (lane == 0) pv = carry_ev;
        const bool hd = v && (ix == 0 || ev_page(x[q]) != ev_page(pv));
        uint32_t te = v ? ev_transform(x[q]) : 0u;
        uint64_t w = 0;
        if (hd) {
          const uint64_t p = ev_page(x[q]);
          w = (p < n_pages) ? pt[p] : 0ull;
          te = tcompose(kConst | (uint32_t)w, te);
        }
        acc = tcompose(acc, wave_reduce_compose(te));
        const uint64_t hb = __ballot(hd);
        if (hb) {
          const uint32_t src = 63u - (uint32_t)__clzll(hb);
          lh = (uint32_t)(j0 + 64 * q + src - lo);
          hp = lane_bcast64(w, (int)src);
        }
        carry_ev = lane_bcast64(x[q], 63);
      }
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
// Thread t of a block holds the block's events [8t, 8t+8) in registers (four 16-B loads);
// the workgroup loops over blocks (grid-stride) and loads the next block's events while it
// works on the current one.
template <bool kVec>
__device__ __forceinline__ void load_block_events(const uint64_t* __restrict__ ev, uint64_t n,
                                                  uint64_t i0, uint64_t (&E)[kCohK]) {
  if (kVec && i0 + kCohK <= n) {
#pragma unroll
    for (int q = 0; q < kCohK / 2; ++q) {
      const uint4 v = ld_nt16(ev + i0 + 2 * q);
      E[2 * q] = (uint64_t)v.x | ((uint64_t)v.y << 32);
      E[2 * q + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
  } else {
#pragma unroll
    for (int k = 0; k < (int)kCohK; ++k) E[k] = (i0 + k < n) ? ev[i0 + k] : 0ull;
  }
}


// ---------------------------------------------------------------- C': wave-sliced pass C
// Block / carry inputs from passes A and B, restated for a low instruction count per event:
//  * every wave works on its own 512 events (8 consecutive per lane); neighbours by DPP, the
//    wave edges read from memory; ONE barrier per block hands the four wave aggregates across
//    (double-buffered slots);
//  * pages are compared as 32-bit ids (SPEC §1: page ids are u32; any higher page bit marks the
//    batch invalid);
//  * inside a lane the state is kept as (C, R) = the last CONST word and the OR of the reads
//    since, so an event costs a few selects instead of a transform composition: a read by n
//    faults iff n is outside C.copyset | R; a write by n faults unless C is EXCLUSIVE, owned by
//    n and no read since brought in a node outside C.copyset; the lane aggregate for the scan
//    is CONST(C) then READ(R), or READ(R) when the lane saw no CONST;
//  * fault counts are segmented per wave (a segment that leaves the wave adds its count
//    atomically; its head's old count stays in memory); page-table words move through the wave's
//    LDS head list (below), so loads and stores are coalesced 8-B accesses.
struct CohAcc {
  uint32_t inv, xfer;
  uint64_t nf8;  // per-node faults of the block, one byte per node (<= 8 per thread)
};

__device__ __forceinline__ uint32_t page32(uint64_t e) { return (uint32_t)(e >> 4); }

// Page-table traffic of one wave goes through its LDS head list (wd / hpg, kCohHeads entries):
// the heads of the wave are ranked in event order; their page-table words are loaded by
// consecutive lanes (coalesced), and every segment that starts AND ends inside the wave leaves
// its final (state | faults << 32) word in its head's slot, stored by consecutive lanes as one
// 8-B write per page. Only the wave's first segment (opened before it) and its last (continued
// after it) touch the page table from the event's lane: one state store / fault atomic each.
constexpr uint32_t kCohHeads = 64 * kCohK;  // heads per wave, at most one per event
constexpr uint32_t kSent = 0xFFFFFFFFu;

// kMeasure (MEASUREMENT ONLY, output invalid): 1 = no page-table stores, 2 = no page-table
// loads or stores either.
template <bool kFull, int kMeasure = 0>
__device__ __forceinline__ void coh_wave(uint64_t* __restrict__ pt, uint64_t n_pages,
                                         const uint64_t* __restrict__ ev, uint64_t n,
                                         const uint64_t (&e)[kCohK], uint64_t b0, uint32_t cnt,
                                         uint32_t lh, uint64_t lhp, uint32_t cin,
                                         uint32_t* __restrict__ slot, uint64_t* __restrict__ wd,
                                         uint32_t* __restrict__ hpg, CohAcc& A, uint32_t& bad,
                                         uint32_t n_nodes) {
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t first = t * kCohK;  // block-relative index of e[0]
  uint32_t* pst = reinterpret_cast<uint32_t*>(pt);
  uint32_t* pfl = pst + 1;
  const uint64_t wfirst = b0 + (uint64_t)wave * 64 * kCohK;
  const uint32_t nvalid =
      kFull ? kCohK
            : (uint32_t)min((int64_t)kCohK, max((int64_t)0, (int64_t)cnt - (int64_t)first));
  uint32_t pprev = from_prev_lane(page32(e[kCohK - 1]));
  uint32_t pnext = from_next_lane(page32(e[0]));
  if (lane == 0 && wfirst > 0 && wfirst <= n) pprev = page32(ev[wfirst - 1]);
  if (lane == 63 && wfirst + 64 * kCohK < n) pnext = page32(ev[wfirst + 64 * kCohK]);
  const uint64_t g0 = b0 + first;  // global index of e[0]

  COH_STAMP(1);
  // ---- heads, segment ends and the lane aggregate (its last CONST: a write, or a head whose
  // page-table word is fetched below), one pass over the events
  uint32_t hmask = 0, emask = 0, hib = 0, lw = 0, ra = 0, lastc = 0;  // lastc: 0 none, 1 write, 2 head
  uint32_t nodes = 0;  // nodes named by the lane's events (checked against n_nodes once)
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (kFull || k < nvalid) {
      const uint32_t x = (uint32_t)e[k], node = (x >> 1) & 7u, bit = 1u << node;
      hib |= (uint32_t)(e[k] >> 32);
      nodes |= bit;
      const uint32_t pk = page32(e[k]);
      const uint32_t pp = k ? page32(e[k > 0 ? k - 1 : 0]) : pprev;
      if ((k == 0 && g0 == 0) || pk != pp) {
        hmask |= 1u << k;
        if ((k > 0 || g0 > 0) && pk < pp) bad = 1;
        if (pk >= n_pages) bad = 1;
        lastc = 2;
        ra = 0;
      }
      if (x & 1u) {
        lastc = 1;
        lw = (node << 8) | bit | 0x60000u;
        ra = 0;
      } else {
        ra |= bit;
      }
      const uint32_t pn = (k + 1 < kCohK) ? page32(e[k + 1 < kCohK ? k + 1 : k]) : pnext;
      if (g0 + k + 1 >= n || pn != pk) emask |= 1u << k;
    }
  }
  if (hib >> 4) bad = 1;         // page ids are u32 (SPEC §1)
  if (nodes >> n_nodes) bad = 1;  // a node outside the page table's n_nodes
  const uint32_t hc = (uint32_t)__popc(hmask);
  const uint32_t hinc = wave_incl_sum(hc);
  const uint32_t hb0 = hinc - hc, nh = lane_bcast(hinc, 63);

  COH_STAMP(2);
  // ---- head list: pages, then the page-table words by consecutive lanes (before the barrier)
  uint32_t hr = hb0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k)
    if ((hmask >> k) & 1u) {
      const uint32_t pk = page32(e[k]);
      if (first + k == lh) {  // the block's last head: pass A's snapshot
        hpg[hr] = kSent;
        wd[hr] = lhp;
      } else {
        hpg[hr] = pk < n_pages ? pk : kSent;
        wd[hr] = 0;
      }
      ++hr;
    }
  wave_lds_sync();
  for (uint32_t j = lane; j < nh; j += 64) {
    const uint32_t pg = hpg[j];
    if (pg != kSent) wd[j] = (kMeasure < 2) ? pt[pg] : (uint64_t)pg * 0x9E3779B9u;
    hpg[j] = kSent;
  }
  wave_lds_sync();

  COH_STAMP(3);
  // ---- lane aggregate CONST(last CONST) then READ(reads since), or READ(all reads); scan
  const uint32_t lc = (lastc == 2) ? (uint32_t)wd[hinc - 1] : lw;
  const uint32_t a = lastc ? tcompose(kConst | lc, ra) : ra;
  const uint32_t inc = wave_incl_compose_dpp(a);
  if (lane == 63) slot[wave] = inc;
  __syncthreads();
  COH_STAMP(4);
  uint32_t carry = cin;
  for (uint32_t w = 0; w < wave; ++w) carry = tcompose(carry, slot[w]);
  const uint32_t cur = tcompose(carry, from_prev_lane(inc));
  if (!(cur & kConst) && (hmask & 1u) == 0u && (kFull || nvalid > 0)) bad = 1;

  COH_STAMP(5);
  // ---- walk: faults, invalidations, transfers; final state of each segment end (parked in its
  // head's slot when the head is in this wave, else stored: the wave's first segment)
  uint32_t C = cur & ~kConst, R = 0, fmask = 0, run = 0;
  hr = hb0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (kFull || k < nvalid) {
      const uint32_t x = (uint32_t)e[k], node = (x >> 1) & 7u, bit = 1u << node;
      const uint32_t wr = x & 1u;
      if ((hmask >> k) & 1u) {
        C = (uint32_t)wd[hr++];
        R = 0;
        run = 0;
      }
      const uint32_t csr = (C | R) & 0xFFu;
      const uint32_t own = (((C >> 8) & 0xFFu) == node) ? 1u : 0u;
      const uint32_t excl = (((C >> 16) & 3u) == 2u && (R & ~C) == 0u) ? 1u : 0u;
      const uint32_t wf = wr & ~(excl & own);
      const uint32_t rf = ((csr >> node) & 1u) ^ 1u;
      const uint32_t f = wr ? wf : rf;
      A.inv += wf ? (uint32_t)__popc(csr & ~bit) : 0u;
      A.xfer += wf & (own ^ 1u);
      A.nf8 += (uint64_t)f << (8u * node);
      fmask |= f << k;
      run += f;
      if (wr) {
        C = (node << 8) | bit | 0x60000u;
        R = 0;
      } else {
        R |= bit;
      }
      if ((emask >> k) & 1u) {
        const uint32_t flip = (((C >> 16) & 3u) == 2u && (R & ~C) != 0u) ? 0x30000u : 0u;
        const uint32_t st = (C | R) ^ flip;
        const uint32_t pk = page32(e[k]);
        if (hr > 0)
          hpg[hr - 1] = st;  // segment inside the wave: parked in its head's slot
        else if (pk < n_pages && kMeasure == 0)
          pst[2 * (uint64_t)pk] = st;  // the wave's first segment, opened before it
        if (kMeasure && pk == kSent) bad |= st;
      }
    }
  }
  wave_lds_sync();

  COH_STAMP(6);
  // ---- fault counts since each head (segmented over the wave); the head's old count is added
  // for segments that end in the wave, and stays in memory for the two edge segments
  const uint32_t sex = from_prev_lane(wave_incl_segsum_dpp((hmask ? kConst : 0u) | run));
  uint32_t running = sex & ~kConst;
  hr = hb0;
#pragma unroll
  for (uint32_t k = 0; k < kCohK; ++k) {
    if (kFull || k < nvalid) {
      const uint32_t f = (fmask >> k) & 1u;
      if ((hmask >> k) & 1u) {
        running = f;
        ++hr;
      } else {
        running += f;
      }
      const uint32_t pk = page32(e[k]);
      if ((emask >> k) & 1u) {
        if (hr > 0) {
          // branch-free: the slot of an out-of-range page (a rejected batch) gets kSent, so the
          // state word parked in it is never taken for a page id; its wd is never stored. (The
          // branchy form of this guard ran pass C at 4.64 ms instead of 4.14, config 4 uniform.)
          const uint32_t st = hpg[hr - 1];
          const uint32_t fl = (uint32_t)(wd[hr - 1] >> 32) + running;
          wd[hr - 1] = (uint64_t)st | ((uint64_t)fl << 32);
          hpg[hr - 1] = pk < n_pages ? pk : kSent;
        } else if (running && pk < n_pages && kMeasure == 0) {
          atomicAdd(&pfl[2 * (uint64_t)pk], running);
        }
      } else if (k == kCohK - 1 && lane == 63 && running && pk < n_pages && kMeasure == 0) {
        atomicAdd(&pfl[2 * (uint64_t)pk], running);  // continues past this wave
      }
      if (kMeasure && pk == kSent) bad |= running;
    }
  }
  wave_lds_sync();
  COH_STAMP(7);
  // ---- segments closed inside the wave: one 8-B page-table word each, consecutive lanes
  for (uint32_t j = lane; j < nh; j += 64) {
    const uint32_t pg = hpg[j];
    if (pg != kSent && kMeasure == 0) pt[pg] = wd[j];
  }
  wave_lds_sync();
}

// C' kernel: one 2048-event block per workgroup, four coh_wave bodies (no persistent loop and
// no prefetch: at ~90 VGPRs five workgroups per CU hide the latency; persistent versions, with
// or without the next block in registers, were 1.2-1.3x slower), one partial row of totals per
// wave.
template <int kMeasure, bool kVec>
__global__ __launch_bounds__(256) void coh_apply_block_kernel(
    uint64_t* __restrict__ pt, uint64_t n_pages, const uint64_t* __restrict__ ev, uint64_t n,
    uint64_t nb, const uint32_t* __restrict__ carry, const uint32_t* __restrict__ last_head,
    const uint64_t* __restrict__ head_pt, uint32_t* __restrict__ partial,
    uint32_t* __restrict__ err, uint32_t n_nodes) {
  __shared__ uint32_t slots[4];
  __shared__ uint64_t wd[4][kCohHeads];
  __shared__ uint32_t hpg[4][kCohHeads];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint64_t b = blockIdx.x;
  uint32_t bad = 0;
  CohAcc A;
  A.inv = A.xfer = 0;
  A.nf8 = 0;
  const uint64_t b0 = b * kCohBlock;
  const uint32_t cnt = (uint32_t)min((uint64_t)kCohBlock, n - b0);
  COH_STAMP(0);
  uint64_t e[kCohK];
  load_block_events<kVec>(ev, n, b0 + t * kCohK, e);
  if (cnt == kCohBlock)
    coh_wave<true, kMeasure>(pt, n_pages, ev, n, e, b0, cnt, last_head[b], head_pt[b], carry[b],
                             slots, wd[wave], hpg[wave], A, bad, n_nodes);
  else
    coh_wave<false, kMeasure>(pt, n_pages, ev, n, e, b0, cnt, last_head[b], head_pt[b], carry[b],
                              slots, wd[wave], hpg[wave], A, bad, n_nodes);
  // per thread: inv <= 7 x 8, xfer <= 8, faults per node <= 8, so 16-bit fields hold a wave's
  // sums: five packed wave sums, one partial row per wave
  const uint32_t lo = (uint32_t)A.nf8, hi = (uint32_t)(A.nf8 >> 32);
  const uint32_t v[5] = {A.inv | (A.xfer << 16), (lo & 0xFFu) | ((lo & 0xFF00u) << 8),
                         ((lo >> 16) & 0xFFu) | ((lo >> 8) & 0xFF0000u),
                         (hi & 0xFFu) | ((hi & 0xFF00u) << 8),
                         ((hi >> 16) & 0xFFu) | ((hi >> 8) & 0xFF0000u)};
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint32_t s = wave_sum(v[q]);
    if (lane == 2u * q) mine = s & 0xFFFFu;
    if (lane == 2u * q + 1u) mine = s >> 16;
  }
  if (lane < 10) partial[(b * 4 + wave) * 10 + lane] = mine;
  if (__ballot(bad != 0) && lane == 0) atomicOr(err, 2u);
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
// Pass C variant (gdsm_tune "coh_variant" or GDSM_COH_VARIANT): 0 = coh_apply_block_kernel, the
// only product kernel (events that are not 16-B aligned take its scalar-load instance). Built
// with -DGDSM_MEASURE only: 1 / 2 = without page-table stores / without any page-table traffic
// (output invalid). (Rounds 1-2 also carried the round-1 block-scan kernel and a hit-mask
// restatement; both were slower and are in the history.)
#ifdef GDSM_MEASURE
constexpr int kCohVariants = 3;
#else
constexpr int kCohVariants = 1;
#endif
static int coh_variant_from_env() {
  const char* e = getenv("GDSM_COH_VARIANT");
  const int v = e ? atoi(e) : 0;
  return (v >= 0 && v < kCohVariants) ? v : 0;
}
static int g_coh_variant = coh_variant_from_env();
int coh_tune(const char* key, int64_t value) {
  if (!strcmp(key, "coh_variant") && value >= 0 && value < kCohVariants) {
    g_coh_variant = (int)value;
    return 0;
  }
  return -1;
}

static inline uint64_t coh_blocks(uint64_t n) { return (n + kCohBlock - 1) / kCohBlock; }
static inline uint64_t coh_groups(uint64_t nb) { return (nb + kCohGroup - 1) / kCohGroup; }

uint64_t coh_workspace_bytes(uint64_t n_events) {
  const uint64_t nb = coh_blocks(n_events);
  // head_pt (u64) + agg, last_head, carry (u32 each) + partial rows (10 u32, one per wave of
  // pass C: 4 per block) + groups
  return nb * (8 + 4 * 3 + 4 * 40) + coh_groups(nb) * 4 + 512;
}

hipError_t launch_coh_init(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes, hipStream_t s) {
  if (n_pages == 0) return hipSuccess;
  const uint64_t per = (n_pages + n_nodes - 1) / n_nodes;
  uint64_t g = (n_pages + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(coh_init_kernel, dim3((unsigned)g), dim3(256), 0, s, pt, n_pages, per);
  return hipGetLastError();
}

hipError_t launch_coherence(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                            const uint64_t* events, uint64_t n_events, uint64_t* totals,
                            uint8_t* ws, uint64_t ws_bytes, uint32_t* err, hipStream_t s,
                            Prof* prof) {
  hipError_t r = hipMemsetAsync(totals, 0, 10 * sizeof(uint64_t), s);
  if (r != hipSuccess || n_events == 0) return r;
  const uint64_t nb = coh_blocks(n_events), ng = coh_groups(nb);
  if (coh_workspace_bytes(n_events) > ws_bytes) return hipErrorInvalidValue;
  uint64_t* head_pt = reinterpret_cast<uint64_t*>(ws);
  uint32_t* agg = reinterpret_cast<uint32_t*>(head_pt + nb);
  uint32_t* lh = agg + nb;
  uint32_t* carry = lh + nb;
  uint32_t* partial = carry + nb;
  uint32_t* groups = partial + nb * 40;
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
    const bool vec = (reinterpret_cast<uintptr_t>(events) & 15) == 0;
#ifdef GDSM_MEASURE
    auto kern = !vec                 ? coh_apply_block_kernel<0, false>
                : g_coh_variant == 1 ? coh_apply_block_kernel<1, true>
                : g_coh_variant == 2 ? coh_apply_block_kernel<2, true>
                                     : coh_apply_block_kernel<0, true>;
#else
    auto kern = vec ? coh_apply_block_kernel<0, true> : coh_apply_block_kernel<0, false>;
#endif
    hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(256), 0, s, pt, n_pages, events, n_events,
                       nb, carry, lh, head_pt, partial, err, n_nodes);
  }
  const uint64_t rows = nb * 4;  // partial rows of totals: one per wave of pass C
  uint64_t g = (rows + 255) / 256;
  if (g > 1024) g = 1024;
  {
    ProfScope ps(prof, 8, s);
    hipLaunchKernelGGL(coh_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, partial, rows,
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

#ifdef GDSM_COH_STAMPS
extern "C" int gdsm_debug_coh_stamps(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gdsm::g_coh_stamps), bytes, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -1;
}
#endif
