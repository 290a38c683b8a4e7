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
// Kernels: coh_fold_kernel (one pass: a wave folds a block of 2048 events and finds its carry by
// decoupled look-back over the other waves' published aggregates, section F below), then
// coh_reduce_kernel (the blocks' partial rows -> the 10 batch totals).
#include "gdsm_common.h"
#include "gdsm_launch.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>

namespace gdsm {

constexpr uint32_t kConst = 1u << 31;
// Measurement builds only (-DGDSM_ROUNDS_STAMPS): per span of each gdsm_rounds round (spans < 32,
// rounds < 1024), lane 0's s_memtime at [0] entry, [1] aggregate published, [2] look-back done,
// [3] exit; read by gdsm_debug_fold_spans.
#ifdef GDSM_ROUNDS_STAMPS
__device__ unsigned long long g_fold_spans[1024][32][4];
#define GDSM_SSTAMP(r_, b_, i_)                                                   \
  do {                                                                           \
    if (lane == 0 && (r_) < 1024 && (b_) < 32)                                   \
      g_fold_spans[r_][b_][i_] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
#else
#define GDSM_SSTAMP(r_, b_, i_) \
  do {                          \
  } while (0)
#endif
#ifdef GDSM_COH_STAMPS
__device__ unsigned long long g_coh_stamps[8192 * 4 * 8];
// Fold kernel: every 16th block b (by ticket), lane 0: [0] entry, [1] events in LDS, [2] walk
// done, [3] look-back done, [4] end (s_memtime), [5] ordered | heads << 1 | look-back rounds << 16,
// [6] heads pass done, [7] the heads' page-table words landed (this build waits for them there)
#define COH_FSTAMP(i, v)                                                                     \
  do {                                                                                        \
    if ((b & 15) == 0 && b / 16 < 32768 && lane == 0) g_coh_stamps[(b / 16) * 8 + (i)] = (v); \
  } while (0)
#else
#define COH_FSTAMP(i, v) \
  do {                   \
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

// The compose scan on DPP (no LDS traffic): 0 is the identity of tcompose (and of segsum,
// gdsm_common.h), and it is what an out-of-range or masked-off DPP source reads.
__device__ __forceinline__ uint32_t wave_incl_compose_dpp(uint32_t v) {
  v = tcompose(dpp0<0x111>(v), v);
  v = tcompose(dpp0<0x112>(v), v);
  v = tcompose(dpp0<0x114>(v), v);
  v = tcompose(dpp0<0x118>(v), v);
  v = tcompose(dpp0<0x142, 0xA>(v), v);
  v = tcompose(dpp0<0x143, 0xC>(v), v);
  return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
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


// ---------------------------------------------------------------- F: single-pass fold
// One wave = one block of kFBlock events (kFK consecutive events per lane), no other pass before
// it: the block's carry comes from a decoupled look-back over the other waves' published
// aggregates (the diff kernel's protocol), so passes A and B and their head snapshots go away.
//
// The walk keeps, per lane, a HIT MASK instead of the state word: bit n = a read by node n hits
// (n in the copyset: bits 0-7 ARE the state word's copyset), bit 8 + n = a write by n hits
// (EXCLUSIVE, owned by n), kHE = EXCLUSIVE, kHW = a write since the segment's base. An event's
// bit index is node + 8 * rw, so "does it fault" is one bit-field extract, a read miss is
// (H | bit) & kKr and every write sets H = 0x101 << n | kHE | kHW. O = 2 * owner for transfers.
// The state word of a segment end is rebuilt from (H, O, base) only where a segment ends, and a
// head's hit mask is its word's copyset plus one write bit (no bit spreading: heads are frequent).
//
// Ordering without head snapshots: the only page-table word this wave loads that another wave
// may store is the one of its last head (that segment can end in a later wave). A wave whose
// first segment started before it looks back until a predecessor that holds a head (kFHead) or
// has published its inclusive prefix, and every wave publishes only after its loads landed, so
// the head's wave has read the word before anyone stores it. Page ids are taken from the low
// dword (n_pages <= 2^28; any high-dword bit rejects the batch).
// Events per lane: 32 (2048-event blocks). A -DGDSM_FOLD_K=16 build (1024-event blocks, 64 VGPRs
// and 16 KiB of LDS per workgroup: 8 waves/SIMD instead of 5) is bit-exact and measured slower,
// 3.18 / 3.03 ms against 2.42 / 2.43 (uniform / Zipf, same box): twice the blocks, twice the
// per-block prologue, look-back and tail.
#ifndef GDSM_FOLD_K
#define GDSM_FOLD_K 32
#endif
// Issue priority (GDSM_FOLD_PRIO, default 5): bit 0 raises a wave's priority (s_setprio 3) from
// its start until its block's event loads are issued and copied to LDS; bit 2 keeps it raised
// until the page-table words of the lanes' first and last heads are requested too; bit 1 raises
// it (2) from the look-back to the end. A wave that starts a block is the youngest on its SIMD,
// so without the raise its loads queue behind the older waves' walks, and its whole block
// starts late. Measured, same box, alternating (uniform / Zipf ms): 0: 2.41 / 2.42-2.43,
// 1: 2.29-2.32 / 2.41-2.43, 5: 2.30-2.31 / 2.42-2.43, 2: 2.40-2.41 / 2.42-2.44, 3: 2.29-2.30.
// GDSM_FOLD_PRE2 (default 1): the words of a lane's first GDSM_FOLD_PRE2 middle heads (its
// second, third head when it has more) are loaded with the first and last heads' words, before
// the walk, instead of inside it.
#ifndef GDSM_FOLD_PRE2
#define GDSM_FOLD_PRE2 1
#endif
#ifndef GDSM_FOLD_PRIO
#define GDSM_FOLD_PRIO 5
#endif
// GDSM_FOLD_REGHEADS (whole blocks): events loaded as 128q + lane and 128q + 64 + lane (8-B
// loads), their head flags taken in registers from the neighbouring lane's page, and two ballots
// per 128 events written into the head masks of walk lanes 4q .. 4q + 3 (v_writelane) — the
// heads pass over the LDS copy goes away. Bit-exact and slower, so off: without the heads pass the
// walk's allocation grows to 111 VGPRs (4 waves/SIMD; held to 5 it spills): 2.42 / 2.50 ms
// against 2.25 / 2.31 (uniform / Zipf, same box, alternating; profiles/r06_coh_regheads_ab.txt).
#ifndef GDSM_FOLD_REGHEADS
#define GDSM_FOLD_REGHEADS 0
#endif
// GDSM_FOLD_SPEC (whole blocks; 1: first and last heads, 2: the second head too): the heads'
// page-table words guessed from the lane's first and last events and gathered before the heads
// pass instead of after it (see the walk prologue). Bit-exact and slower, so off: the guesses
// are live through the heads pass, which takes the fold to 102-106 VGPRs (4 waves/SIMD), or to
// 96 with spills when held to 5 waves/SIMD; measured in that form (same box, alternating, 3
// rounds): 2.34 / 2.47-2.49 ms against 2.27-2.28 / 2.34-2.35 (uniform / Zipf),
// profiles/r06_coh_spec_ab.txt.
#ifndef GDSM_FOLD_SPEC
#define GDSM_FOLD_SPEC 0
#endif
constexpr uint32_t kFK = GDSM_FOLD_K;       // events per lane (16 or 32: hm is one 32-bit mask)
constexpr uint32_t kFH = 16;                // of them held in registers at a time
constexpr uint32_t kFBlock = 64 * kFK;
constexpr uint32_t kHE = 0x10000u, kHW = 0x20000u, kPRE = 0x40000u, kHRead = 0xFFu;
constexpr uint32_t kKr = kHRead | kHW | kPRE;  // kept by a read miss
constexpr uint64_t kFAgg = 1ull << 62, kFIncl = 2ull << 62, kFHead = 1ull << 61;
constexpr uint32_t kFoldCtrs = 8;                   // workgroup ticket counters
constexpr uint64_t kFoldStatus = kFoldCtrs * 32;    // u64 index of block 0's status granule

// v_writelane_b32 as the compiler's intrinsic (no __builtin in this clang; it owns M0)
extern "C" __device__ int coh_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint2 ld_nt8(const uint64_t* p) {
  const uint64_t v = __builtin_nontemporal_load(p);
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}

__device__ __forceinline__ uint32_t hit_seed(uint32_t w) {
  const uint32_t c = w & 0xFFu;
  const uint32_t owner = (w >> 8) & 0xFFu;
  const uint32_t wbit = owner < 8u ? (0x100u << owner) : 0u;
  return (((w >> 16) & 3u) == 2u) ? (c | kHE | wbit) : c;
}
__device__ __forceinline__ uint32_t hit_copyset(uint32_t h) { return h & kHRead; }
// The state word at a segment end: the base is the last writer's word when the lane wrote since
// the segment's base B (a head's word or the lane's incoming state), then the reads since.
__device__ __forceinline__ uint32_t seg_final(uint32_t h, uint32_t O, uint32_t B) {
  const uint32_t own = O >> 1;
  const uint32_t base = (h & kHW) ? ((own << 8) | (1u << own) | 0x60000u) : B;
  const bool flip = ((base >> 16) & 3u) == 2u && !(h & kHE);
  return (base | hit_copyset(h)) ^ (flip ? 0x30000u : 0u);
}
__device__ __forceinline__ uint32_t wr_word(uint32_t x) {  // CONST word of a write event
  const uint32_t node = (x >> 1) & 7u;
  return (node << 8) | (1u << node) | 0x60000u;
}
// v_s ∘ v_{s-1} ∘ … ∘ v_0 in lane 63 (higher lanes first): the scan with swapped operands.
__device__ __forceinline__ uint32_t wave_rev_compose_dpp(uint32_t v) {
  v = tcompose(v, dpp0<0x111>(v));
  v = tcompose(v, dpp0<0x112>(v));
  v = tcompose(v, dpp0<0x114>(v));
  v = tcompose(v, dpp0<0x118>(v));
  v = tcompose(v, dpp0<0x142, 0xA>(v));
  v = tcompose(v, dpp0<0x143, 0xC>(v));
  return lane_bcast(v, 63);
}

// 2v + (this lane's bit of `mask`): one v_addc with the lane mask as carry-in.
__device__ __forceinline__ uint32_t shl1_add(uint32_t v, uint64_t mask) {
  uint32_t r;
  uint64_t cout;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(cout) : "v"(v), "s"(mask));
  return r;
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {  // (a & m) | (b & ~m)
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// LDS slot of block event e (lo dword): an XOR swizzle of the 4-dword group (bits 2-5) by bits
// 6-9, so the coalesced b64 writes and the per-lane b128 reads of 4 consecutive events both spread
// over all 64 banks, without padding (8 KiB per wave keeps 5 workgroups per CU).
__device__ __forceinline__ uint32_t fold_slot(uint32_t e) { return e ^ (((e >> 6) & 15u) << 2); }

// 16 of the lane's events, [16h, 16h + 16), from the wave's LDS copy of its block.
__device__ __forceinline__ void fold_half(const uint32_t* __restrict__ tr, uint32_t lane,
                                          uint32_t h, uint32_t (&X)[kFH]) {
  asm volatile("" ::: "memory");  // not hoisted above the previous half's work
#pragma unroll
  for (uint32_t r = 0; r < kFH / 4; ++r) {
    const uint4 w = *reinterpret_cast<const uint4*>(tr + fold_slot(kFK * lane + kFH * h + 4 * r));
    X[4 * r] = w.x;
    X[4 * r + 1] = w.y;
    X[4 * r + 2] = w.z;
    X[4 * r + 3] = w.w;
  }
  // the walk recomputes every per-event value from X: without this the compiler keeps the
  // prologue's copies (pages, head flags) live through the walk
#pragma unroll
  for (uint32_t k = 0; k < kFH; ++k) asm volatile("" : "+v"(X[k]));
}

// kM (MEASUREMENT ONLY, -DGDSM_MEASURE builds, output invalid): 1 = no walk, 2 = no look-back,
// 3 = no ordered look-back (no wave waits for the block holding its first segment's head),
// 4 = events from a hot 64 MB window: block b loads the events of block b mod 4096 (kept in the
// Infinity Cache) with their pages shifted by (b / 4096) * n_pages / 128, so the walk, the
// page-table traffic and the look-back stay representative while the event loads hit in cache.
template <bool kVec, bool kFull, bool kNodes, int kM = 0>
__device__ __forceinline__ void coh_fold_wave(uint64_t* __restrict__ pt, uint64_t n_pages,
                                              const uint64_t* __restrict__ ev, uint64_t n,
                                              uint64_t b, uint64_t* __restrict__ status,
                                              uint32_t* __restrict__ partial,
                                              uint32_t* __restrict__ err, uint32_t n_nodes,
                                              uint32_t* __restrict__ tr) {
  const uint32_t lane = lane_id();
  const uint64_t lo = b * kFBlock;
  constexpr uint64_t kHotBlocks = 4096;
  const uint64_t lo_src = kM == 4 ? (b % kHotBlocks) * kFBlock : lo;  // where the events are read
  const uint32_t padd = kM == 4 ? (uint32_t)((b / kHotBlocks) * (n_pages >> 7)) << 4 : 0u;
  const uint64_t g0 = lo + (uint64_t)lane * kFK;  // global index of this lane's first event
  const uint32_t nv =
      kFull ? kFK : (uint32_t)min((uint64_t)kFK, g0 < n ? n - g0 : (uint64_t)0);
  COH_FSTAMP(0, __builtin_amdgcn_s_memtime());
  if (GDSM_FOLD_PRIO & 1) __builtin_amdgcn_s_setprio(3);
  // ---- events: low dwords (page << 4 | node << 1 | rw) into the wave's LDS copy of the block;
  // every high-dword bit is an error. Coalesced 16-B loads (load q: events [128q, 128q + 128),
  // two per lane); each lane then reads its 32 consecutive events 16 at a time. (Loading a
  // lane's events straight, at a 256-B lane stride, touched 64 lines per load instruction and
  // re-fetched every line from L2 once per instruction.)
  uint32_t hib = 0;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  uint32_t eagg = 0;
  bool early = false;
  uint32_t hm_r = 0, dec_r = 0;  // GDSM_FOLD_REGHEADS: this lane's head mask, a page decreased
  if (kVec && kFull && GDSM_FOLD_REGHEADS) {
    // the page of the event before the block (uniform)
    uint32_t pprev = (lo > 0 ? (uint32_t)ev[kM == 4 ? (lo_src ? lo_src - 1 : 0) : lo - 1] + padd : 0u) >> 4;
    uint32_t ea = 0, eb = 0;  // events 1920 + lane and 1984 + lane
    uint2 VA[kFBlock / 128], VB[kFBlock / 128];  // every load in flight at once
#pragma unroll
    for (uint32_t q = 0; q < kFBlock / 128; ++q) {
      VA[q] = ld_nt8(ev + lo_src + 128 * q + lane);
      VB[q] = ld_nt8(ev + lo_src + 128 * q + 64 + lane);
    }
#pragma unroll
    for (uint32_t q = 0; q < kFBlock / 128; ++q) {
      const uint2 va = VA[q], vb = VB[q];
      hib |= va.y | vb.y;
      const uint32_t xa = va.x + padd, xb = vb.x + padd;
      tr[fold_slot(128 * q + lane)] = xa;
      tr[fold_slot(128 * q + 64 + lane)] = xb;
      const uint32_t pa = xa >> 4, pb = xb >> 4;
      uint32_t qa = from_prev_lane(pa), qb = from_prev_lane(pb);
      if (lane == 0) {
        qa = pprev;
        qb = lane_bcast(pa, 63);
      }
      pprev = lane_bcast(pb, 63);
      const bool first = q == 0 && lo == 0 && lane == 0;  // the batch's first event
      dec_r |= ((!first && pa < qa) || pb < qb) ? 1u : 0u;
      asm volatile("" : "+v"(dec_r));  // now: sunk, it kept every chunk's pages live
      const uint64_t Ma = __ballot(first || pa != qa), Mb = __ballot(pb != qb);
      hm_r = (uint32_t)coh_writelane((int)(uint32_t)Ma, (int)(4 * q), (int)hm_r);
      hm_r = (uint32_t)coh_writelane((int)(uint32_t)(Ma >> 32), (int)(4 * q + 1), (int)hm_r);
      hm_r = (uint32_t)coh_writelane((int)(uint32_t)Mb, (int)(4 * q + 2), (int)hm_r);
      hm_r = (uint32_t)coh_writelane((int)(uint32_t)(Mb >> 32), (int)(4 * q + 3), (int)hm_r);
      if (q == kFBlock / 128 - 1) {
        ea = xa;
        eb = xb;
      }
    }
    // ---- early aggregate (as below, in this layout: a = event 1920 + lane, b = 1984 + lane)
    const uint64_t bwb = __ballot((eb & 1u) != 0), bwa = __ballot((ea & 1u) != 0);
    if (kM == 0 && b > 0 && (bwa | bwb)) {
      const bool inb = bwb != 0;
      const uint32_t Lw = 63u - (uint32_t)__builtin_clzll(inb ? bwb : bwa);
      const uint32_t xw = inb ? lane_bcast(eb, (int)Lw) : lane_bcast(ea, (int)Lw);
      const uint32_t wi = (inb ? 64u : 0u) + Lw;
      if ((xw >> 4) == (lane_bcast(eb, 63) >> 4)) {
        const uint32_t r = (lane > wi ? 1u << ((ea >> 1) & 7u) : 0u) |
                           (64u + lane > wi ? 1u << ((eb >> 1) & 7u) : 0u);
        uint32_t R = 0;
#pragma unroll
        for (uint32_t nd = 0; nd < 8; ++nd) R |= __ballot((r >> nd) & 1u) ? 1u << nd : 0u;
        eagg = tcompose(kConst | wr_word(xw), R);
        early = true;
      }
    }
  } else if (kVec && kFull) {
    uint32_t e0 = 0, e1 = 0;  // events 1920 + 2 * lane and the one after it
#pragma unroll
    for (uint32_t q = 0; q < kFBlock / 128; ++q) {
      const uint4 v = ld_nt16(ev + lo_src + 128 * q + 2 * lane);
      hib |= v.y | v.w;
      *reinterpret_cast<u32x2*>(tr + fold_slot(128 * q + 2 * lane)) = (u32x2){v.x + padd, v.z + padd};
      if (q == kFBlock / 128 - 1) {
        e0 = v.x + padd;
        e1 = v.z + padd;
      }
    }
    // ---- early aggregate: when the block's last 128 events hold a write W and no head follows
    // it (W's page is the block's last page), the block's transform is CONST(W) then READ(the
    // nodes that read after W). It is published before the walk (below), so successors do not
    // wait for this wave's walk; the walk's own aggregate is checked against it.
    const uint64_t bw = __ballot(((e0 | e1) & 1u) != 0);
    if (kM == 0 && b > 0 && bw) {
      const uint32_t Lw = 63u - (uint32_t)__builtin_clzll(bw);
      const uint32_t y1 = lane_bcast(e1, (int)Lw);
      const uint32_t xw = (y1 & 1u) ? y1 : lane_bcast(e0, (int)Lw);
      const uint32_t wi = 2u * Lw + (y1 & 1u);
      if ((xw >> 4) == (lane_bcast(e1, 63) >> 4)) {
        const uint32_t r = (2u * lane > wi ? 1u << ((e0 >> 1) & 7u) : 0u) |
                           (2u * lane + 1u > wi ? 1u << ((e1 >> 1) & 7u) : 0u);
        uint32_t R = 0;
#pragma unroll
        for (uint32_t nd = 0; nd < 8; ++nd) R |= __ballot((r >> nd) & 1u) ? 1u << nd : 0u;
        eagg = tcompose(kConst | wr_word(xw), R);
        early = true;
      }
    }
  } else {
#pragma unroll 8
    for (uint32_t k = 0; k < kFK; ++k) {
      const uint64_t e = (k < nv) ? ev[g0 + k] : 0ull;
      tr[fold_slot(kFK * lane + k)] = (uint32_t)e;
      hib |= (uint32_t)(e >> 32);
    }
  }
  wave_lds_sync();
  COH_FSTAMP(1, __builtin_amdgcn_s_memtime());
  if ((GDSM_FOLD_PRIO & 5) == 1) __builtin_amdgcn_s_setprio(0);
  const uint32_t xprev_w = lo > 0 ? (uint32_t)ev[kM == 4 ? (lo_src ? lo_src - 1 : 0) : lo - 1] + padd
                                  : 0u;  // uniform
  const bool has_next = lo + kFBlock < n;
  const uint32_t xnext_w =
      has_next ? (uint32_t)ev[kM == 4 ? lo_src + kFBlock : lo + kFBlock] + padd : 0u;  // uniform
  const uint32_t xlast = nv ? tr[fold_slot(kFK * lane + nv - 1)] : 0u;       // last valid event
  uint32_t xp = from_prev_lane(tr[fold_slot(kFK * lane + kFK - 1)]);
  if (lane == 0) xp = xprev_w;
  const bool batch_first = lo == 0 && lane == 0;
#if GDSM_FOLD_SPEC
  // ---- the page-table words of the lane's heads, guessed and gathered BEFORE the heads pass, so
  // their latency hides behind it: the lane's last head is the page of its last event (whenever
  // the lane has a head), its first head the page of its first event or, when that event
  // continues an earlier segment, the next page (right whenever the batch's pages are dense, as
  // config 4's are), its second head the page after the first. A wrong guess is loaded again
  // after the heads pass; a guessed word that is not one of the lane's heads is never used
  // (another wave may be storing it).
  uint64_t Wl_s = 0, Wf_s = 0, Ws_s = 0;
  uint32_t pf_s = 0;
  if (kFull) {
    const uint32_t pg0 = tr[fold_slot(kFK * lane)] >> 4;
    pf_s = (batch_first || pg0 != (xp >> 4)) ? pg0 : pg0 + 1u;
    const uint32_t pl_s = xlast >> 4;
    if (pl_s < n_pages) Wl_s = pt[pl_s];
    if (pf_s < pl_s && pf_s < n_pages) Wf_s = pt[pf_s];
#if GDSM_FOLD_SPEC > 1
    if (pf_s + 1u < pl_s && pf_s + 1u < n_pages) Ws_s = pt[pf_s + 1u];
#endif
  }
#endif

  // ---- heads (a new page), validity. (Sortedness inside a lane is checked where the walk meets
  // a head; the first / last head events are read back from LDS.)
  uint32_t X[kFH];
  uint32_t hm = 0;
  uint32_t bad = hib ? 1u : 0u;
  constexpr bool kRegHeads = kVec && kFull && GDSM_FOLD_REGHEADS;
  if (kRegHeads) {
    hm = hm_r;
    if (dec_r) bad = 1;
  }
#pragma unroll
  for (uint32_t h = 0; h < (kRegHeads ? 0u : kFK / kFH); ++h) {
    fold_half(tr, lane, h, X);
#pragma unroll
    for (uint32_t j = 0; j < kFH; ++j) {
      const uint32_t k = kFH * h + j;
      if (kFull || k < nv) {
        const uint32_t x = X[j], pv = j ? X[j ? j - 1 : 0] : xp;
        const uint32_t pg = x >> 4, pp = pv >> 4;
        const bool first = k == 0 && batch_first;
        const bool head = first || pg != pp;
        if (k == 0 && !first && pg < pp) bad = 1;
        if (kFull)
          hm = shl1_add(hm, __ballot(head));  // bit 31 - k, one v_addc per event
        else
          hm |= (head ? 1u : 0u) << k;
      }
    }
    xp = X[kFH - 1];
  }
  if (kFull && !kRegHeads) hm = __brev(hm) >> (32u - kFK);
  const uint32_t hc = (uint32_t)__popc(hm);
  uint32_t xf = 0, xl = 0;  // the lane's first and last head events
  if (hc) {
    xf = tr[fold_slot(kFK * lane + (uint32_t)__builtin_ctz(hm))];
    xl = tr[fold_slot(kFK * lane + 31u - (uint32_t)__builtin_clz(hm))];
  }
  // opaque from here on: the walk re-derives its per-event head flags from these words instead
  // of the compiler keeping the prologue's 32 masks live
  asm volatile("" : "+v"(hm), "+v"(xf), "+v"(xl));
  if (nv && (xlast >> 4) >= n_pages) bad = 1;
  // does the lane's last event end its segment? (the next lane's first event is a head, or the
  // next wave's, or the batch ends there)
  uint32_t nh0 = from_next_lane(hm & 1u);
  if (lane == 63) nh0 = has_next ? (((xnext_w >> 4) != (xlast >> 4)) ? 1u : 0u) : 1u;
  bool last_end = nh0 != 0;
  if (!kFull && nv > 0 && g0 + nv == n) last_end = true;

  COH_FSTAMP(6, __builtin_amdgcn_s_memtime());
  // ---- page-table words of the lane's last and first heads (one gathered load each)
  uint64_t Wl = 0, Wf = 0, Ws = 0, Wt = 0;  // last, first, second, third heads (others: walk)
#if GDSM_FOLD_SPEC
  if (kFull) {  // the guesses above, and a load where one missed
    const uint32_t pf = xf >> 4;
    Wl = Wl_s;  // (pages of the lane's last head and last event are equal)
    Wf = Wf_s;
    if (hc > 1 && pf != pf_s && pf < n_pages) Wf = pt[pf];
    if (GDSM_FOLD_PRE2 && hc > 2) {
      const uint32_t h2 = hm & (hm - 1u);
      const uint32_t p2 = tr[fold_slot(kFK * lane + (uint32_t)__builtin_ctz(h2))] >> 4;
      Ws = Ws_s;
      if ((GDSM_FOLD_SPEC < 2 || p2 != pf_s + 1u) && p2 < n_pages) Ws = pt[p2];
      if (GDSM_FOLD_PRE2 > 1 && hc > 3) {
        const uint32_t h3 = h2 & (h2 - 1u);
        const uint32_t p3 = tr[fold_slot(kFK * lane + (uint32_t)__builtin_ctz(h3))] >> 4;
        if (p3 < n_pages) Wt = pt[p3];
      }
    }
  } else
#endif
  {
    const uint32_t pl = xl >> 4, pf = xf >> 4;
    if (hc && pl < n_pages) Wl = pt[pl];
    if (hc > 1 && pf < n_pages) Wf = pt[pf];
    if (GDSM_FOLD_PRE2 && hc > 2) {  // a middle head: its page lies inside this lane
      const uint32_t h2 = hm & (hm - 1u);
      const uint32_t p2 = tr[fold_slot(kFK * lane + (uint32_t)__builtin_ctz(h2))] >> 4;
      if (p2 < n_pages) Ws = pt[p2];
      if (GDSM_FOLD_PRE2 > 1 && hc > 3) {
        const uint32_t h3 = h2 & (h2 - 1u);
        const uint32_t p3 = tr[fold_slot(kFK * lane + (uint32_t)__builtin_ctz(h3))] >> 4;
        if (p3 < n_pages) Wt = pt[p3];
      }
    }
  }
  const uint32_t Bl = (uint32_t)Wl & 0x7FFFFu, Bfl = (uint32_t)(Wl >> 32);
  const uint32_t Hl = hit_seed(Bl), Ol = ((Bl >> 8) & 0xFFu) << 1;
  if ((GDSM_FOLD_PRIO & 5) == 5) __builtin_amdgcn_s_setprio(0);
  asm volatile("" : "+v"(Wf), "+v"(Ws), "+v"(Wt));  // waited for here, not inside the walk
#ifdef GDSM_COH_STAMPS
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  COH_FSTAMP(7, __builtin_amdgcn_s_memtime());
#endif
  // Early publication (see above): the words of every lane's first and last heads have landed
  // (the wave's last head's word is the only one another wave may store), so the head flag goes
  // out with it and ordered successors need not wait for this walk either.
  if (early) {
    asm volatile("" ::"v"(Bl) : "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): only the loads above are in flight here
    if (lane == 0)
      __hip_atomic_store(status + b, kFAgg | (__ballot(hc != 0) ? kFHead : 0ull) | eagg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- the walk, from a PROBE state: the lane's incoming state is not known yet (it comes
  // from the look-back below, which this walk hides). Only the events before the lane's first
  // CONST (its first write or head) depend on it, and those are reads: the probe starts with an
  // empty copyset and no write hits (kPRE marks "still in that prefix"), so each prefix read
  // misses once per node and the first write (if it comes before any head) misses. Hc / Xc keep
  // the state after the prefix and the first CONST event; both outcomes are corrected once the
  // incoming state is known. Everything after the first CONST is exact.
  uint32_t H = kPRE, O = 0x1FEu, B = 0, Bfo = 0, c0 = 0, T = 0, hs = 0;
  uint32_t inv = 0, xfer = 0, F[4] = {0, 0, 0, 0}, Hc = kPRE, Xc = 0, pm = ~0u;
  uint32_t sH = 0, sO = 0, sB = 0, sBf = 0, sN = 0, sP = 0;  // pending local segment end
  uint32_t dHOT = 0;  // the lane's first segment end: H | O << 19 | T << 23 (read only when the
                      // lane wrote before it: then O <= 14 and T <= 32)
  bool local = false, hasS = false, hasD = false;
// (macros, not lambdas: captured flags end up in scratch memory)
#define COH_FLUSH_S()                                                                        \
  do {                                                                                       \
    if (sP < n_pages) pt[sP] = (uint64_t)seg_final(sH, sO, sB) | ((uint64_t)(sBf + sN) << 32); \
  } while (0)
#define COH_END_SEG(p_)        \
  do {                         \
    if (!local) {              \
      dHOT = H | ((O & 15u) << 19) | (T << 23); \
      hasD = true;             \
    } else {                   \
      if (hasS) COH_FLUSH_S(); \
      sH = H;                  \
      sO = O;                  \
      sB = B;                  \
      sBf = Bfo;               \
      sN = T - c0;             \
      sP = (p_);               \
      hasS = true;             \
    }                          \
  } while (0)
  uint32_t xprevh = 0;  // the event before X[0] in this lane (half 1)
#pragma unroll
  for (uint32_t h = 0; h < (kM == 1 ? 0u : kFK / kFH); ++h) {
    fold_half(tr, lane, h, X);
#pragma unroll
    for (uint32_t j = 0; j < kFH; ++j) {
      const uint32_t k = kFH * h + j;
      if (kFull || k < nv) {
        const uint32_t x = X[j];
        Xc = bfi(pm, x, Xc);  // the event, while still in the prefix
        if ((hm >> k) & 1u) {  // a head: the previous segment ends, this one's base is its word
          if (k > 0) {
            const uint32_t pp = (j ? X[j ? j - 1 : 0] : xprevh) >> 4;
            if ((x >> 4) < pp) bad = 1;  // pages must not decrease
            COH_END_SEG(pp);
          }
          if (hs + 1 == hc) {
            H = Hl;
            O = Ol;
            B = Bl;
            Bfo = Bfl;
          } else {
            // the first head's word was loaded (and waited for) with the last head's, before the
            // walk; a middle head (lanes with >= 3 heads) loads its word here. A word prefetched
            // one head ahead instead made every head step wait: the wave's one vmcnt counter also
            // counts the walk's stores, and some lane is at a head at most steps.
            if (GDSM_FOLD_PRE2 && hs == 1) {
              B = (uint32_t)Ws & 0x7FFFFu;
              Bfo = (uint32_t)(Ws >> 32);
            } else if (GDSM_FOLD_PRE2 > 1 && hs == 2) {
              B = (uint32_t)Wt & 0x7FFFFu;
              Bfo = (uint32_t)(Wt >> 32);
            } else if (hs != 0) {
              const uint32_t pg = x >> 4;  // a page >= n_pages fails the batch (clamped load)
              const uint64_t w = pt[pg < n_pages ? pg : 0u];
              B = (uint32_t)w & 0x7FFFFu;
              Bfo = (uint32_t)(w >> 32);
              asm volatile("" : "+v"(B), "+v"(Bfo));  // the wait stays on this path
            } else {
              B = (uint32_t)Wf & 0x7FFFFu;
              Bfo = (uint32_t)(Wf >> 32);
            }
            H = hit_seed(B);
            O = ((B >> 8) & 0xFFu) << 1;
          }
          c0 = T;
          local = true;
          ++hs;
        }
        const uint32_t xn2 = x & 14u, nd = xn2 >> 1, rw = x & 1u;
        const bool wr = rw != 0u;
        const uint32_t bi = nd + (rw << 3);
        const uint32_t hitv = __builtin_amdgcn_ubfe(H, bi, 1u);
        const bool hit = hitv != 0;
        const uint32_t miss = hitv ^ 1u;
        const uint32_t m = 1u << nd;
        const uint32_t sel = (wr && !hit) ? (H & kHRead & ~m) : 0u;
        asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(inv) : "v"(sel), "v"(inv));
        xfer += (wr && O != xn2) ? 1u : 0u;  // a write by a non-owner always faults
        const uint32_t Hr = hit ? H : ((H | m) & kKr);
        H = wr ? ((0x101u << nd) | (kHE | kHW)) : Hr;
        O = wr ? xn2 : O;
        asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(F[k / 8]) : "v"(miss), "v"(2u * xn2), "v"(F[k / 8]));
        T += miss;
        pm = (uint32_t)((int32_t)(H << 13) >> 31);  // still in the prefix after this event
        asm volatile("" : "+v"(pm));
        Hc = bfi(pm, H, Hc);
        // accumulate now: left alone, the compiler sinks these sums past the walk and keeps
        // every event's intermediate values live
        asm volatile("" : "+v"(inv), "+v"(xfer), "+v"(F[k / 8]), "+v"(Hc), "+v"(Xc));
      }
    }
    xprevh = X[kFH - 1];
  }
  if (nv && last_end) COH_END_SEG(xlast >> 4);
  if (hasS) COH_FLUSH_S();
  if (kNodes) {
    // a node outside the group fails the batch: checked from the LDS copy once the walk's
    // registers are free (taken in the heads pass, it kept the fold at 103 VGPRs, 4 waves/SIMD)
    uint32_t nodes = 0;
#pragma unroll
    for (uint32_t r = 0; r < kFK / 4; ++r) {
      const uint4 w = *reinterpret_cast<const uint4*>(tr + fold_slot(kFK * lane + 4 * r));
      nodes = max(nodes, max(max(w.x & 14u, w.y & 14u), max(w.z & 14u, w.w & 14u)));
    }
    // (slots past the block's end in a partial block hold the zero events written for them)
    if ((nodes >> 1) >= n_nodes) bad = 1;
  }
#undef COH_END_SEG
#undef COH_FLUSH_S

  // ---- lane aggregate (exact: the state after the lane's first CONST does not depend on the
  // incoming state; without a CONST the lane is READ(its reads)), scan, publish, look back
  COH_FSTAMP(2, __builtin_amdgcn_s_memtime());
  const bool has_c = !(H & kPRE);
  const uint32_t a = has_c ? (kConst | seg_final(H, O, B)) : hit_copyset(H);
  const uint32_t inc = wave_incl_compose_dpp(a);
  const uint32_t agg = lane_bcast(inc, 63);
  const bool whead = __ballot(hc != 0) != 0;
  if (early && agg != eagg) bad = 1;  // never expected
  // every load of this wave has landed before its status is visible (see above). (Waiting only
  // for the last head's word, not for the walk's stores, measured the same: the wave's tail then
  // waits for them instead.)
  if (!early) {  // (an early publication went out after its loads already)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  if (lane == 0 && !early)
    __hip_atomic_store(status + b, (b == 0 ? kFIncl : kFAgg) | (whead ? kFHead : 0ull) | agg,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // Only a wave that stores the state of a segment opened before it (its first segment ends
  // here) needs the head's wave to have loaded that page's word: it looks back to a block with a
  // head. Every other wave stops at the nearest CONST aggregate or inclusive prefix (CONST
  // absorbs everything before it), so the blocks of a hot page do not chain their look-backs.
  const bool ordered = kM != 3 &&
                       __ballot(hasD && (__ballot(hc != 0) & ((1ull << lane) - 1ull)) == 0) != 0;
  uint32_t carry = 0;
  if (GDSM_FOLD_PRIO & 2) __builtin_amdgcn_s_setprio(2);
#ifdef GDSM_COH_STAMPS
  uint32_t lb_rounds = 0;
#endif
  if (b > 0 && kM != 2) {
    int64_t pos = (int64_t)b - 1;
    for (;;) {
#ifdef GDSM_COH_STAMPS
      ++lb_rounds;
#endif
      const int64_t q = pos - (int64_t)lane;
      uint64_t st = q >= 0 ? __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : kFIncl;
      uint32_t s, spins = 0;
      for (;;) {
        const uint64_t pub = __ballot((st >> 62) != 0);
        const uint64_t stop =
            __ballot(ordered ? (st & kFHead) != 0
                             : ((st >> 62) == 2 || (st & kFHead) || (st & kConst)));
        const uint32_t u = ~pub ? (uint32_t)__builtin_ctzll(~pub) : 64u;
        s = (stop & pub) ? (uint32_t)__builtin_ctzll(stop & pub) : 64u;
        if (s < u || u == 64) break;
        if (++spins > (1u << 24)) {  // never expected: fail the batch rather than hang the GPU
          bad = 1;
          s = u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if ((st >> 62) == 0 && q >= 0)
          st = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint32_t part;
      if (s == 0)
        part = (uint32_t)lane_bcast64(st, 0);
      else
        part = wave_rev_compose_dpp(lane <= s ? (uint32_t)st : 0u);
      carry = tcompose(part, carry);
      if (s < 64) break;
      pos -= 64;
    }
    if (lane == 0)
      __hip_atomic_store(status + b, kFIncl | (whead ? kFHead : 0ull) | tcompose(carry, agg),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef GDSM_COH_STAMPS
  COH_FSTAMP(3, __builtin_amdgcn_s_memtime());
  const uint64_t st_heads = (uint64_t)__popcll(__ballot(hc != 0));
  COH_FSTAMP(5, (ordered ? 1ull : 0ull) | (st_heads << 1) | ((uint64_t)lb_rounds << 16));
#endif
  const uint32_t cur = tcompose(carry, from_prev_lane(inc));
  const bool cont = nv && !(hm & 1u);  // the lane's first event continues a segment
  if (cont && !(cur & kConst)) bad = 1;

  // ---- corrections of the probe prefix, now that the incoming state `cur` is known
  const uint32_t P8 = hit_copyset(Hc);      // nodes read before the first CONST
  const uint32_t cs = cur & 0xFFu;
  const uint32_t hitP = cont ? (P8 & cs) : 0u;  // prefix reads that hit after all
  const uint32_t s1 = tcompose(cur, P8);     // the state after the prefix (CONST)
  const bool wfirst = cont && has_c && !(hc && Xc == xf);  // the first CONST is a write
  int32_t dfirst = -(int32_t)__popc(hitP);   // correction of the lane's first segment count
  uint32_t wcorr = 0;                        // node whose probe write fault did not happen
  bool wnofault = false;
  if (wfirst) {
    const uint32_t w = (Xc >> 1) & 7u, wb = 1u << w;
    const bool f = !(((s1 >> 16) & 3u) == 2u && ((s1 >> 8) & 0xFFu) == w);
    inv = inv - (uint32_t)__popc(P8 & ~wb) + (f ? (uint32_t)__popc(s1 & 0xFFu & ~wb) : 0u);
    xfer = xfer - 1u + ((f && ((s1 >> 8) & 0xFFu) != w) ? 1u : 0u);
    if (!f) {
      wnofault = true;
      wcorr = w;
      dfirst -= 1;
    }
  }
  // the lane's first segment ends here: its state and count
  uint32_t Df = 0, Dc = 0;
  const uint32_t dP = tr[fold_slot(kFK * lane)] >> 4;  // the first segment's page
  if (hasD) {
    Df = wfirst ? seg_final(dHOT & 0x7FFFFu, (dHOT >> 19) & 15u, 0u) : (s1 & 0x7FFFFu);
    Dc = (uint32_t)((int32_t)(dHOT >> 23) + dfirst);
  }

  // ---- fault counts of segments that cross lanes (counts only: old counts are 32-bit)
  const uint32_t own = hc ? T - c0 : (uint32_t)((int32_t)T + dfirst);
  const uint32_t sin = wave_incl_segsum_dpp((hc ? kConst : 0u) | own);
  const uint32_t cnt_in = from_prev_lane(sin) & ~kConst;
  const uint64_t hb = __ballot(hc != 0);
  const uint64_t below = hb & ((1ull << lane) - 1ull);
  const uint32_t hl = below ? 63u - (uint32_t)__clzll(below) : 0u;
  const uint32_t oldf = (uint32_t)__shfl((int)Bfo, (int)hl, 64);
  uint32_t* pst = reinterpret_cast<uint32_t*>(pt);
  if (hasD && dP < n_pages) {
    const uint32_t c = cnt_in + Dc;
    if (below) {
      pt[dP] = (uint64_t)Df | ((uint64_t)(oldf + c) << 32);
    } else {  // the wave's first segment: opened before it
      pst[2 * (uint64_t)dP] = Df;
      if (c) atomicAdd(&pst[2 * (uint64_t)dP + 1], c);
    }
  }
  if (kFull && lane == 63 && !last_end) {  // the wave's last segment continues
    const uint32_t p = xlast >> 4, c = sin & ~kConst;
    if (c && p < n_pages) atomicAdd(&pst[2 * (uint64_t)p + 1], c);
  }

  // ---- totals: one partial row per wave (16-bit fields hold a wave's sums)
  uint32_t Fe = 0, Fo = 0;  // bytes: nodes 0, 2, 4, 6 / 1, 3, 5, 7
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    Fe += F[q] & 0x0F0F0F0Fu;
    Fo += (F[q] >> 4) & 0x0F0F0F0Fu;
  }
  {
    const uint32_t e = hitP & 0x55u, o = (hitP >> 1) & 0x55u;
    Fe -= (e & 1u) | ((e & 4u) << 6) | ((e & 16u) << 12) | ((e & 64u) << 18);
    Fo -= (o & 1u) | ((o & 4u) << 6) | ((o & 16u) << 12) | ((o & 64u) << 18);
    if (wnofault) {
      const uint32_t one = 1u << (8u * (wcorr >> 1));
      if (wcorr & 1u)
        Fo -= one;
      else
        Fe -= one;
    }
  }
  const uint32_t v[5] = {inv | (xfer << 16), (Fe & 0xFFu) | ((Fo & 0xFFu) << 16),
                         ((Fe >> 8) & 0xFFu) | (((Fo >> 8) & 0xFFu) << 16),
                         ((Fe >> 16) & 0xFFu) | (((Fo >> 16) & 0xFFu) << 16),
                         (Fe >> 24) | ((Fo >> 24) << 16)};
  uint32_t mine = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint32_t s = wave_sum(v[q]);
    if (lane == 2u * q) mine = s & 0xFFFFu;
    if (lane == 2u * q + 1u) mine = s >> 16;
  }
  if (lane < 10) partial[b * 10 + lane] = mine;
  if (kM == 0 && __ballot(bad != 0) && lane == 0) atomicOr(err, 2u);
  COH_FSTAMP(4, __builtin_amdgcn_s_memtime());
}

// Waves per workgroup (GDSM_FOLD_WAVES, 1, 2 or 4; default 4). LDS is held by a workgroup until
// its last wave ends, so a four-wave workgroup keeps its 32 KiB after its earlier waves' blocks are
// done; smaller workgroups free it sooner but measured slower (config 4, same box, alternating,
// 2 rounds: 1 wave 2.75-2.77 / 2.62 ms, 2 waves 2.51 / 2.40, 4 waves 2.27-2.28 / 2.34 uniform /
// Zipf; bit-exact, profiles/r06_coh_wg_ab.txt).
#ifndef GDSM_FOLD_WAVES
#define GDSM_FOLD_WAVES 4
#endif
constexpr uint32_t kFoldWaves = GDSM_FOLD_WAVES;
static_assert(kFoldWaves == 1 || kFoldWaves == 2 || kFoldWaves == 4, "fold workgroup");

// kFull: the batch's whole blocks, one ticket per workgroup (tickets are drawn in dispatch
// order, so a wave only ever waits for running waves); otherwise the single trailing partial
// block `nb - 1`, launched after them.
template <bool kVec, bool kFull, bool kNodes, int kM = 0>
__global__ __launch_bounds__(64 * kFoldWaves) void coh_fold_kernel(
    uint64_t* __restrict__ pt, uint64_t n_pages, const uint64_t* __restrict__ ev, uint64_t n,
    uint64_t nb, uint64_t* __restrict__ ws, uint32_t* __restrict__ partial,
    uint32_t* __restrict__ err, uint32_t n_nodes) {
  __shared__ __attribute__((aligned(16))) uint32_t tr_all[kFoldWaves][kFBlock];
  uint64_t b;
  if (kFull) {
    // kFoldCtrs ticket counters (one 256-B line each) keyed by blockIdx % kFoldCtrs: one counter
    // returns only ~88 atomics per us, which serialised 262144 workgroups (config 4) for 3 ms.
    // Workgroup w = ticket * kFoldCtrs + class is a permutation of blockIdx inside each class, and
    // every class draws its tickets in dispatch order, so the lowest block nobody has claimed is
    // always claimed once running blocks finish: no wave waits for a block that cannot run.
    // (the ticket passes through wave 0's event buffer: a separate LDS word would take the
    // workgroup past 32 KiB and cost a workgroup per CU)
    const uint32_t cls = blockIdx.x % kFoldCtrs;
    if (threadIdx.x == 0) tr_all[0][0] = atomicAdd(reinterpret_cast<uint32_t*>(ws + cls * 32), 1u);
    __syncthreads();
    const uint32_t ticket = __builtin_amdgcn_readfirstlane(tr_all[0][0]);
    __syncthreads();
    const uint64_t w = (uint64_t)ticket * kFoldCtrs + cls;
    b = w * kFoldWaves + (threadIdx.x >> 6);
    if (b >= nb) return;
  } else {
    if (threadIdx.x >= 64) return;
    b = nb - 1;
  }
  coh_fold_wave<kVec, kFull, kNodes, kM>(pt, n_pages, ev, n, b, ws + kFoldStatus, partial, err,
                                     n_nodes, tr_all[threadIdx.x >> 6]);
}

// ---------------------------------------------------------------- S: streaming fold
// One wave = one span of kSpan = 4096 events, walked as 64 chunks of 64 CONSECUTIVE events (lane
// l = event 64c + l of the span), with no LDS copy: the chunk's events come straight from a
// coalesced 8-B load issued kSD chunks ahead, and the page-table words of the chunk's heads from
// a gather issued kSG chunks ahead, so a wave never stops to load a block.
//
// Inside a chunk the fold is a segmented OR scan over the lanes (DPP): a lane's scan value is
// (F | base word) for a CONST event (a write, or a head: its page-table word, then the head's own
// read), or its reader bit in the R field for a read; a lane with F keeps its value, others OR in
// what precedes them. The exclusive value is the state the event meets: base word + the readers
// since it (s_state applies them: copyset |= R, EXCLUSIVE -> SHARED when R leaves the copyset).
// The last lane's inclusive value carries to the next chunk.
//
// The span's first segment (opened in an earlier span) starts from PROBE (no F, empty base): its
// reads before the first write (P8, the prefix) count one fault per node and its first write is
// left out; both are corrected after the decoupled look-back has given the incoming state, which
// is also when that segment's state word is stored (the low dword; its fault count is added to
// the high dword atomically, as is the count of a segment that continues past the span). A
// segment that starts and ends inside the span is stored whole (state | old count + faults).
// Status granules, tickets and ordering are the fold's (F above): a wave publishes after its
// loads landed; a wave that stores the state of a segment opened before it looks back to a span
// that holds a head.
// Chunks per span: 64 (4096 events) for whole-GPU batches (coh_variant 1), 4 (256 events) for
// small batches, where the number of waves in flight, not their efficiency, sets the time.
constexpr uint32_t kSCBig = 64, kSCSmall = 4;
constexpr uint32_t kSD = 6;               // event loads in flight (chunks ahead)
constexpr uint32_t kSG = 3;               // head-word gathers in flight (chunks ahead)
static_assert(kSD % kSG == 0 && kSG < kSD, "ring geometry");
constexpr uint32_t kSF = 1u << 31;        // scan value: a CONST at or before this lane
constexpr uint32_t kSProbe = 1u << 28;    // scan value: the span's incoming state (unknown)

// state word (bits 0-18) of base word `base` after the readers R since it
__device__ __forceinline__ uint32_t s_state(uint32_t v) {
  const uint32_t base = v & 0x7FFFFu, R = (v >> 20) & 0xFFu;
  const bool flip = ((base >> 16) & 3u) == 2u && (R & ~base & 0xFFu);
  return (base | R) ^ (flip ? 0x30000u : 0u);
}

// Segmented OR scan (inclusive) over the 64 lanes: a lane with kSF keeps its value. Per step one
// v_or_b32_dpp (the source lane's value OR this one; out-of-range sources read 0), then a v_bfi
// keyed by the lane's own kSF (arithmetic shift): 3 VALU, 4 for the row-masked broadcasts, which
// leave the rows they skip alone and so need the destination preset.
template <int kCtrl, int kRowMask, bool kBC>
__device__ __forceinline__ uint32_t sor_step(uint32_t v) {
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, kBC);
  return bfi((uint32_t)((int32_t)v >> 31), v, t | v);
}
__device__ __forceinline__ uint32_t sor_scan(uint32_t v) {
  v = sor_step<0x111, 0xF, true>(v);
  v = sor_step<0x112, 0xF, true>(v);
  v = sor_step<0x114, 0xF, true>(v);
  v = sor_step<0x118, 0xF, true>(v);
  v = sor_step<0x142, 0xA, false>(v);
  v = sor_step<0x143, 0xC, false>(v);
  return v;
}

__device__ __forceinline__ uint64_t le_mask(uint32_t lane) {  // lanes 0..lane
  return lane == 63 ? ~0ull : (2ull << lane) - 1ull;
}
__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }

// totals != nullptr (small batches): the span's totals are added to the batch totals directly
// (10 atomics per span) instead of a partial row for coh_reduce_kernel: one launch fewer.
// kChain (CohChain: a context's small batches without a zeroing launch): the status granules
// carry the launch's epoch (bits 32-60; a granule of an earlier launch reads as unpublished),
// and the caller's totals are zeroed by the wave of span 0 before it raises `flag` to the epoch;
// every wave adds its totals once it sees the flag (raised long before, at that wave's start).
// (An accumulator row in the chain copied out by the wave completing the last span, behind an
// acq_rel completion counter, measured 3.6-5.6 % fewer config-5 rounds/s: its three dependent
// round trips end the launch.)
struct CohChain {
  uint32_t epoch;    // 1 .. 2^29 - 1
  uint32_t* flag;    // == epoch once the caller's totals are zeroed
  uint32_t round;    // (gdsm_rounds, measurement stamps only)
};
// A span's events loaded ahead (gdsm_rounds: the next round's, while the barrier is waited out):
// its first chunks' events and the events before and after it.
struct SpanPre {
  uint64_t X[kSCSmall];
  uint32_t xprev, xnext;
};

// kWT (gdsm_rounds' persistent grid): page-table words stored write-through and gathered past
// L1 (st_wt / ld_wt), since the next round's waves on other XCDs read them after a fence-free
// barrier; kL2 (with kWT, a one-XCD team): stored plain and counted by L2 atomics instead, the
// team's gathers finding them in its L2. pre: the span's events already loaded (kSC <= kSCSmall),
// else loaded here.
template <uint32_t kSC, bool kFull, bool kChain = false, bool kWT = false, bool kL2 = false>
__device__ __forceinline__ void coh_stream_wave(uint64_t* __restrict__ pt, uint64_t n_pages,
                                                const uint64_t* __restrict__ ev, uint64_t n,
                                                uint64_t b, uint64_t* __restrict__ status,
                                                uint32_t* __restrict__ partial,
                                                uint32_t* __restrict__ err, uint32_t n_nodes,
                                                unsigned long long* __restrict__ totals,
                                                const CohChain ch = CohChain{},
                                                const bool use_pre = false,
                                                const SpanPre pre = SpanPre{},
                                                uint32_t* const tot_acc = nullptr) {
  const uint64_t tag = kChain ? (uint64_t)ch.epoch << 32 : 0ull;
  // a status granule as this launch sees it (kChain: an earlier launch's reads as unpublished)
  auto ld_status = [&](int64_t q) {
    const uint64_t x = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (kChain && ((x >> 32) & 0x1FFFFFFFull) != ch.epoch) ? 0ull : x;
  };
  constexpr uint32_t kSpan = 64 * kSC;
  constexpr bool kWTs = kWT && !kL2;  // write-through stores
  const uint32_t lane = lane_id();
  if (kWT) GDSM_SSTAMP(ch.round, b, 0);
  const uint64_t lo = b * kSpan;
  const uint64_t hi = lo + kSpan;
  const uint32_t nev = kFull ? kSpan : (uint32_t)min((uint64_t)kSpan, n - lo);
  const uint32_t nch = kFull ? kSC : (nev + 63u) / 64u;
  const uint64_t lem = le_mask(lane);
  // the event before the span and the one after it (uniform scalar loads)
  const bool has_next = hi < n;
  const uint32_t xprev = use_pre ? pre.xprev : (lo > 0 ? (uint32_t)ev[lo - 1] : 0u);
  const uint32_t xnext = use_pre ? pre.xnext : (has_next ? (uint32_t)ev[hi] : 0u);

  // gather depth: the write-through rounds path gathers every chunk's head words at once (its
  // spans fit one ring pass, kSC <= kSD), so the span waits out one gather round trip, not two
  constexpr uint32_t kSGw = (kWT && kSC <= kSD) ? kSC : kSG;
  static_assert(kSGw == kSG || kSC <= kSD, "ring geometry");
  uint64_t X[kSD];       // events of chunks c .. c + kSD - 1 (ring)
  uint64_t Wg[kSGw];     // page-table words of the heads of chunks c .. c + kSGw - 1 (ring)
  uint64_t Hg[kSGw];     // their head masks
#define GDSM_SLOAD(c_, slot_)                                                        \
  do {                                                                               \
    const uint64_t g_ = lo + 64ull * (c_) + lane;                                    \
    X[slot_] = ((c_) < nch && (kFull || g_ < n)) ? __builtin_nontemporal_load(ev + g_) \
                                                 : ~0ull;                            \
  } while (0)
  uint32_t bad = 0, pprev = xprev >> 4;  // page of the event before chunk (gathers' view)
  const bool batch_first = lo == 0;
  // heads of chunk c (events in X[slot]) and their words; pprev = page of the event before it
#define GDSM_SGATHER(c_, slot_, gslot_)                                              \
  do {                                                                               \
    const uint64_t x_ = X[slot_];                                                    \
    const bool v_ = (c_) < nch && (kFull || lo + 64ull * (c_) + lane < n);           \
    const uint32_t xl_ = (uint32_t)x_, p_ = xl_ >> 4;                                \
    uint32_t pp_ = (uint32_t)__builtin_amdgcn_update_dpp((int)pprev, (int)p_, 0x138, 0xF, 0xF, false); \
    const bool first_ = batch_first && (c_) == 0 && lane == 0;                       \
    const bool h_ = v_ && (first_ || p_ != pp_);                                     \
    bad |= (v_ && ((uint32_t)(x_ >> 32) != 0u || p_ >= n_pages || (!first_ && p_ < pp_) || \
                   ((xl_ >> 1) & 7u) >= n_nodes)) ? 1u : 0u;                         \
    Hg[gslot_] = __ballot(h_);                                                       \
    uint64_t w_ = 0;                                                                 \
    if (h_ && p_ < n_pages) w_ = kWT ? ld_wt(pt + p_) : pt[p_];                      \
    Wg[gslot_] = w_;                                                                 \
    pprev = (uint32_t)__builtin_amdgcn_readlane((int)p_, 63);                        \
  } while (0)

#pragma unroll
  for (uint32_t j = 0; j < kSD; ++j) {
    if (kSC <= kSCSmall && use_pre)
      X[j] = j < kSC ? pre.X[j < kSC ? j : 0] : ~0ull;
    else
      GDSM_SLOAD(j, j);
  }
#pragma unroll
  for (uint32_t j = 0; j < kSGw; ++j) GDSM_SGATHER(j, j, j);

  // the span's first event continues the page before it: its first segment starts from PROBE
  const uint32_t x0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)X[0]);
  const bool first_cont = !batch_first && nev > 0 && (x0 >> 4) == (xprev >> 4);
  uint32_t carry = kSProbe;                   // inclusive scan value after the previous chunk
  uint32_t inv = 0, xfer = 0;
  uint64_t F64 = 0;                           // per-node faults, 8 bits each
  bool prefix_done = false;                   // the span's first CONST has been seen
  uint32_t P8 = 0, pw_node = 0;
  bool pw = false;
  bool open_local = false;                    // the open segment started in this span
  uint32_t open_page = x0 >> 4, open_f0 = 0, open_cnt = 0;
  bool has_d = false;                         // the span's first segment ended inside it
  uint32_t d_state = 0, d_cnt = 0, d_page = 0;
  bool any_head = false;
  // kDefer (the write-through rounds path, short spans): the segment ends found in the chunks are
  // held in registers and stored after the span's aggregate is published, so the publication's
  // wait for the loads does not also wait for write-through store acknowledgements
  constexpr bool kDefer = kWT && kSC <= kSD;
  constexpr uint32_t kDN = kDefer ? kSC : 1;
  uint64_t dval[kDN], oval[kDN];  // chunk j: this lane's segment end / lane 0's open segment
  uint32_t dpg[kDN], opg[kDN];    // their pages (~0u: none)
#pragma unroll
  for (uint32_t j = 0; j < kDN; ++j) {
    dpg[j] = opg[j] = ~0u;
    dval[j] = oval[j] = 0;
  }
  uint32_t lpg = ~0u, apg = ~0u, acnt = 0;  // the span-end store / count add
  uint64_t lval = 0;

  for (uint32_t c0 = 0; c0 < nch; c0 += kSD) {
#pragma unroll
    for (uint32_t j = 0; j < kSD; ++j) {
      const uint32_t c = c0 + j;
      if (c >= nch) break;
      const uint64_t x = X[j];
      const uint64_t W = Wg[j % kSGw];
      const uint64_t Hd = Hg[j % kSGw];
      any_head |= Hd != 0;
      // the open segment closes at the previous chunk's end when this chunk starts a page
      if (c > 0 && (Hd & 1ull)) {
        if (open_local) {
          const uint64_t wv = (uint64_t)s_state(carry) | ((uint64_t)(open_f0 + open_cnt) << 32);
          if (kDefer) {  // (c == j: one pass of the outer loop when kSC <= kSD)
            if (lane == 0 && open_page < n_pages) {
              opg[j < kDN ? j : 0] = open_page;
              oval[j < kDN ? j : 0] = wv;
            }
          } else if (lane == 0 && open_page < n_pages) {
            st_<kWTs>(pt + open_page, wv);
          }
        } else {
          has_d = true;
          d_state = carry;
          d_cnt = open_cnt;
          d_page = open_page;
        }
      }
      const bool valid = kFull || lo + 64ull * c + lane < n;
      const uint32_t xl = (uint32_t)x;
      const bool head = (Hd >> lane) & 1ull;
      const uint32_t nd = (xl >> 1) & 7u, wr = xl & 1u, bit = 1u << nd;
      const uint32_t wl = kSF | ((uint32_t)W & 0x7FFFFu);  // a head's CONST: its word
      const uint32_t hmask = 0u - (head ? 1u : 0u);
      // write: CONST(EXCLUSIVE, owner nd, copyset {nd}, dirty); read: its reader bit (after the
      // head's word when it is a head). Selected branch-free (a divergent ?: became a branch)
      uint32_t v = bfi(0u - wr, kSF | 0x60000u | (nd << 8) | bit, (hmask & wl) | (bit << 20));
      if (!valid) v = 0;
      if (lane == 0) v = bfi((uint32_t)((int32_t)v >> 31), v, v | carry);
      const uint32_t incl = sor_scan(v);
      const uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)incl, 0x138, 0xF,
                                                                0xF, false);
      const uint32_t sin = bfi(hmask, wl, ex);   // the state this event meets
      const bool exact = (sin & kSF) != 0;
      const uint32_t st = s_state(sin);
      const uint32_t cs = st & 0xFFu, own = (st >> 8) & 0xFFu;
      const bool excl = ((st >> 16) & 3u) == 2u;
      const bool fault_w = !(excl && own == nd);
      const bool m = wr ? fault_w : !((cs >> nd) & 1u);
      const bool mm = valid && (exact || !wr) && m;
      const bool wx = valid && exact && wr;
      inv += (wx && fault_w) ? (uint32_t)__popc(cs & ~bit) : 0u;
      xfer += (wx && own != nd) ? 1u : 0u;
      F64 += (uint64_t)(mm ? 1u : 0u) << (8u * nd);
      const uint64_t M = __ballot(mm);
      // the span's prefix: readers before its first CONST, and that CONST if it is a write
      if (!prefix_done) {
        const uint64_t cm = __ballot(valid && (head || wr));
        if (cm) {
          const uint32_t l = (uint32_t)__builtin_ctzll(cm);
          P8 = ((uint32_t)__builtin_amdgcn_readlane((int)ex, (int)l) >> 20) & 0xFFu;
          pw = !((Hd >> l) & 1ull);
          pw_node = ((uint32_t)__builtin_amdgcn_readlane((int)xl, (int)l) >> 1) & 7u;
          prefix_done = true;
        }
      }
      // segments ending inside the chunk: lane i ends when lane i + 1 is a head
      const uint64_t Ein = Hd >> 1;
      if (Ein) {
        const bool end = (Ein >> lane) & 1ull;
        const uint64_t hb = Hd & lem;
        const bool inchunk = hb != 0;
        const uint32_t h = inchunk ? 63u - (uint32_t)__builtin_clzll(hb) : 0u;
        const uint32_t cnt = popc64(M & lem & ~((1ull << h) - 1ull));
        const uint32_t f0 = (uint32_t)__shfl((int)(uint32_t)(W >> 32), (int)h, 64);
        const uint32_t pg = xl >> 4;
        if (end && pg < n_pages && (inchunk || open_local)) {
          const uint64_t wv = (uint64_t)s_state(incl) |
                              ((uint64_t)(inchunk ? f0 + cnt : open_f0 + open_cnt + cnt) << 32);
          if (kDefer) {
            dpg[j < kDN ? j : 0] = pg;
            dval[j < kDN ? j : 0] = wv;
          } else {
            st_<kWTs>(pt + pg, wv);
          }
        }
        if (!open_local) {
          const uint64_t dm = __ballot(end && !inchunk);
          if (dm) {  // the span's first segment ends here (lowest end lane)
            const uint32_t l = (uint32_t)__builtin_ctzll(dm);
            has_d = true;
            d_state = (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)l);
            d_cnt = open_cnt + (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)l);
            d_page = (uint32_t)__builtin_amdgcn_readlane((int)pg, (int)l);
          }
        }
      }
      // the open segment after this chunk
      if (Hd) {
        const uint32_t hl = 63u - (uint32_t)__builtin_clzll(Hd);
        open_local = true;
        open_page = (uint32_t)__builtin_amdgcn_readlane((int)(xl >> 4), (int)hl);
        open_f0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(W >> 32), (int)hl);
        open_cnt = popc64(M & ~((1ull << hl) - 1ull));
      } else {
        open_cnt += popc64(M);
      }
      carry = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      // refill the rings: events kSD chunks ahead, head words kSG chunks ahead
      GDSM_SLOAD(c + kSD, j);
      GDSM_SGATHER(c + kSGw, (j + kSGw) % kSD, j % kSGw);
    }
  }
#undef GDSM_SLOAD
#undef GDSM_SGATHER
  if (!prefix_done) P8 = (carry >> 20) & 0xFFu;
  // the open segment at the span's end: closed when the next event starts a page
  const uint32_t last_page = open_page;
  const bool next_head = !has_next || ((xnext >> 4) != last_page);
  bool cont_first = false;   // the span's first segment runs past it
  if (next_head) {
    if (open_local) {
      const uint64_t wv = (uint64_t)s_state(carry) | ((uint64_t)(open_f0 + open_cnt) << 32);
      if (lane == 0 && last_page < n_pages) {
        if (kDefer) {
          lpg = last_page;
          lval = wv;
        } else {
          st_<kWTs>(pt + last_page, wv);
        }
      }
    } else {
      has_d = true;
      d_state = carry;
      d_cnt = open_cnt;
      d_page = last_page;
    }
  } else if (open_local) {
    if (lane == 0 && open_cnt && last_page < n_pages) {
      if (kDefer) {
        apg = last_page;
        acnt = open_cnt;
      } else {
        add_u32<kL2>(reinterpret_cast<uint32_t*>(pt) + 2 * (uint64_t)last_page + 1, open_cnt);
      }
    }
  } else {
    cont_first = true;
  }

  // ---- publish the span's aggregate once its loads landed, then look back
  const uint32_t agg = (carry & kSF) ? (kConst | s_state(carry)) : ((carry >> 20) & 0xFFu);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (kWT) GDSM_RSTAMP(1, ch.round, 2);
  if (kWT) GDSM_SSTAMP(ch.round, b, 1);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0)
    __hip_atomic_store(status + b, (b == 0 ? kFIncl : kFAgg) | (any_head ? kFHead : 0ull) | tag | agg,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (kDefer) {  // the held segment ends (pages inside this span: no other wave touches them)
#pragma unroll
    for (uint32_t j = 0; j < kDN; ++j) {
      if (opg[j] != ~0u) st_<kWTs>(pt + opg[j], oval[j]);
      if (dpg[j] != ~0u) st_<kWTs>(pt + dpg[j], dval[j]);
    }
    if (lpg != ~0u) st_<kWTs>(pt + lpg, lval);
    if (apg != ~0u) add_u32<kL2>(reinterpret_cast<uint32_t*>(pt) + 2 * (uint64_t)apg + 1, acnt);
  }
  const bool ordered = has_d;
  uint32_t cur = 0;
  if (b > 0) {
    int64_t pos = (int64_t)b - 1;
    for (;;) {
      const int64_t q = pos - (int64_t)lane;
      uint64_t stv = q >= 0 ? ld_status(q) : kFIncl;
      uint32_t sidx, spins = 0;
      for (;;) {
        const uint64_t pub = __ballot((stv >> 62) != 0);
        const uint64_t stop =
            __ballot(ordered ? (stv & kFHead) != 0
                             : ((stv >> 62) == 2 || (stv & kFHead) || (stv & kConst)));
        const uint32_t u = ~pub ? (uint32_t)__builtin_ctzll(~pub) : 64u;
        sidx = (stop & pub) ? (uint32_t)__builtin_ctzll(stop & pub) : 64u;
        if (sidx < u || u == 64) break;
        if (++spins > (1u << 24)) {  // never expected: fail the batch rather than hang the GPU
          bad = 1;
          sidx = u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if ((stv >> 62) == 0 && q >= 0) stv = ld_status(q);
      }
      uint32_t part;
      if (sidx == 0)
        part = (uint32_t)lane_bcast64(stv, 0);
      else
        part = wave_rev_compose_dpp(lane <= sidx ? (uint32_t)stv : 0u);
      cur = tcompose(part, cur);
      if (sidx < 64) break;
      pos -= 64;
    }
    if (lane == 0)
      __hip_atomic_store(status + b, kFIncl | (any_head ? kFHead : 0ull) | tag | tcompose(cur, agg),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  if (kWT) GDSM_RSTAMP(1, ch.round, 3);
  if (kWT) GDSM_SSTAMP(ch.round, b, 2);
  // ---- the span's first segment, now that its incoming state `cur` is known
  uint32_t dfc = 0;                 // correction of the first segment's fault count
  uint32_t Fcorr_node_minus = 0;    // nodes whose probe read fault did not happen
  uint32_t pw_fault = 0;
  if (first_cont) {
    if (!(cur & kConst)) bad = 1;   // a continuing segment always has a CONST before it
    const uint32_t cs_in = cur & 0xFFu;
    Fcorr_node_minus = P8 & cs_in;
    dfc = 0u - (uint32_t)__popc(Fcorr_node_minus);
    const uint32_t s1 = tcompose(cur, P8) & 0x7FFFFu;
    if (pw) {
      const uint32_t cs1 = s1 & 0xFFu, own1 = (s1 >> 8) & 0xFFu;
      const bool f = !(((s1 >> 16) & 3u) == 2u && own1 == pw_node);
      if (f) {
        pw_fault = 1;
        dfc += 1;
        inv += lane == 0 ? (uint32_t)__popc(cs1 & ~(1u << pw_node)) : 0u;
      }
      xfer += (lane == 0 && own1 != pw_node) ? 1u : 0u;
    }
    if (has_d) {
      const uint32_t word = (d_state & kSF) ? s_state(d_state) : (tcompose(cur, (d_state >> 20) & 0xFFu) & 0x7FFFFu);
      if (lane == 0 && d_page < n_pages) {
        uint32_t* pst = reinterpret_cast<uint32_t*>(pt) + 2 * (uint64_t)d_page;
        st_<kWTs>(pst, word);
        const uint32_t c = d_cnt + dfc;
        if (c) add_u32<kL2>(pst + 1, c);
      }
    } else if (cont_first) {
      const uint32_t c = open_cnt + dfc;
      if (lane == 0 && c && last_page < n_pages)
        add_u32<kL2>(reinterpret_cast<uint32_t*>(pt) + 2 * (uint64_t)last_page + 1, c);
    }
  } else if (has_d || cont_first) {
    // no prefix (the span starts a page): the first segment was counted exactly
    if (has_d && lane == 0 && d_page < n_pages) {
      uint32_t* pst = reinterpret_cast<uint32_t*>(pt) + 2 * (uint64_t)d_page;
      st_<kWTs>(pst, s_state(d_state));
      if (d_cnt) add_u32<kL2>(pst + 1, d_cnt);
    }
  }

  // ---- totals: one partial row per span
  uint32_t tot[10];
  tot[0] = wave_sum(inv);
  tot[1] = wave_sum(xfer);
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) tot[2 + q] = wave_sum((uint32_t)(F64 >> (8 * q)) & 0xFFu);
  if (first_cont) {
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) tot[2 + q] -= (Fcorr_node_minus >> q) & 1u;
    if (pw_fault) tot[2 + pw_node] += 1;
  }
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t q = 0; q < 10; ++q) mine = lane == q ? tot[q] : mine;
  if (kChain && ch.flag) {  // the caller's totals are zeroed once the flag holds the epoch
    while (__hip_atomic_load(ch.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ch.epoch)
      __builtin_amdgcn_s_sleep(1);
    // (kWT: the zeroes were stored write-through and drained before the flag, and the adds below
    // are atomics: no acquire)
    if (kWT)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  if (tot_acc) {  // (the caller adds them once its round's hand-offs are drained)
    *tot_acc += mine;
  } else if (totals) {
    if (lane < 10 && mine) atomicAdd(totals + lane, (unsigned long long)mine);
  } else if (lane < 10) {
    partial[b * 10 + lane] = mine;
  }
  if (__ballot(bad != 0) && lane == 0) atomicOr(err, 2u);
  if (kWT) GDSM_SSTAMP(ch.round, b, 3);
}

// Spans [0, nfull) are whole; a partial last span (nb > nfull) is walked by the wave that draws
// it, in the same launch (a separate tail launch was one more dependent launch per batch).
// The chained small-batch workspace (kChain): two sets of the kFoldCtrs ticket-counter lines
// (launch E draws from set E & 1; its workgroup 0 zeroes set (E + 1) & 1 for launch E + 1), the
// totals flag, then the epoch-tagged status granules.
constexpr uint64_t kCohChainFlag = 2 * kFoldStatus;        // u64 index of the totals flag
constexpr uint64_t kCohChainStatus = kCohChainFlag + 32;   // u64 index of span 0's granule
template <uint32_t kSC, bool kChain = false>
__global__ __launch_bounds__(256) void coh_stream_kernel(uint64_t* __restrict__ pt,
                                                         uint64_t n_pages,
                                                         const uint64_t* __restrict__ ev,
                                                         uint64_t n, uint64_t nb, uint64_t nfull,
                                                         uint64_t* __restrict__ ws,
                                                         uint32_t* __restrict__ partial,
                                                         uint32_t* __restrict__ err,
                                                         uint32_t n_nodes,
                                                         unsigned long long* __restrict__ totals,
                                                         uint32_t epoch = 0) {
  __shared__ uint32_t tk;
  // tickets as coh_fold_kernel
  const uint32_t cls = blockIdx.x % kFoldCtrs;
  const uint32_t set = kChain ? epoch & 1u : 0u;
  if (threadIdx.x == 0)
    tk = atomicAdd(reinterpret_cast<uint32_t*>(ws + (set * kFoldCtrs + cls) * 32), 1u);
  if (kChain && blockIdx.x == 0 && threadIdx.x < kFoldCtrs)  // launch E + 1's counters
    __hip_atomic_store(reinterpret_cast<uint32_t*>(ws + ((set ^ 1u) * kFoldCtrs + threadIdx.x) * 32),
                       0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t ticket = __builtin_amdgcn_readfirstlane(tk);
  const uint64_t w = (uint64_t)ticket * kFoldCtrs + cls;
  const uint64_t b = w * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  uint64_t* const status = ws + (kChain ? kCohChainStatus : kFoldStatus);
  const CohChain ch{epoch, reinterpret_cast<uint32_t*>(ws + kCohChainFlag)};
  if (kChain && b == 0) {  // span 0's wave: the caller's totals zeroed, then the flag raised
    const uint32_t lane = threadIdx.x & 63;
    if (lane < 10) totals[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0) __hip_atomic_store(ch.flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (b < nfull)
    coh_stream_wave<kSC, true, kChain>(pt, n_pages, ev, n, b, status, partial, err, n_nodes,
                                       totals, ch);
  else
    coh_stream_wave<kSC, false, kChain>(pt, n_pages, ev, n, b, status, partial, err, n_nodes,
                                        totals, ch);
}

// ---- DSM rounds on the device (gdsm_rounds, page-table side): one persistent launch folds
// every round's events in turn, a grid barrier between rounds (round r + 1 reads the words round
// r stored). Round r = events [eoff[r], eoff[r+1]), spans of 256 (coh_stream_wave, chained form:
// granules tagged with epoch epoch0 + r in CohChainState's ws), span s on wave s mod
// (4 x gridDim.x), each wave's spans in ascending order, so a look-back only waits for running
// waves. Totals: row r of `totals` (10 u64, zeroed by the launcher), a wave's spans summed in
// registers and added after the workgroup's arrival at the barrier (the next round never reads
// them, so the barrier's drain does not wait for those atomics). The page-table words one round
// hands the next are stored write-through and gathered past L1 (kWT), so the barrier between
// rounds needs no fence. kXcd: the rounds run on a one-XCD team (xcd_team, control words at
// bar + 32), the page-table words stored plain and counted in that XCD's L2.
template <bool kXcd>
__global__ __launch_bounds__(256) void rounds_fold_kernel(uint64_t* __restrict__ pt,
                                                          uint64_t n_pages,
                                                          const uint64_t* __restrict__ ev,
                                                          const int64_t* __restrict__ eoff,
                                                          uint32_t n_rounds,
                                                          uint64_t* __restrict__ ws,
                                                          uint32_t* __restrict__ err,
                                                          uint32_t n_nodes,
                                                          unsigned long long* __restrict__ totals,
                                                          uint32_t epoch0,
                                                          uint32_t* __restrict__ bar) {
  constexpr uint64_t kSpan = 64ull * kSCSmall;
  const XcdTeam team = kXcd ? xcd_team(bar + 32, err, kErrRoundsBarrier)
                            : XcdTeam{blockIdx.x, gridDim.x};
  if (team.idx == ~0u) return;  // (workgroup-uniform: not on the team's XCD)
  GDSM_RSTAMP_WG(team.idx == 0);
  const uint64_t nw = (uint64_t)team.n * 4, wv = (uint64_t)team.idx * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  uint64_t* const status = ws + kCohChainStatus;
  // the events of this wave's first span of round r, loaded before round r - 1's barrier
  // (events are never written in the launch: no hand-off)
  SpanPre pre;
  uint64_t ne0 = 0, nn = 0;  // round r's event bounds, loaded with its events
  auto prefetch = [&](uint32_t r) {
    const uint64_t e0 = (uint64_t)eoff[r], n = (uint64_t)eoff[r + 1] - e0;
    ne0 = e0;
    nn = n;
    const uint64_t lo = wv * kSpan;
    if (lo >= n) return false;
#pragma unroll
    for (uint32_t j = 0; j < kSCSmall; ++j) {
      const uint64_t g = lo + 64ull * j + lane;
      pre.X[j] = g < n ? __builtin_nontemporal_load(ev + e0 + g) : ~0ull;
    }
    pre.xprev = lo > 0 ? (uint32_t)ev[e0 + lo - 1] : 0u;
    pre.xnext = lo + kSpan < n ? (uint32_t)ev[e0 + lo + kSpan] : 0u;
    return true;
  };
  bool have_pre = n_rounds > 0 && prefetch(0);
  for (uint32_t r = 0; r < n_rounds; ++r) {
    GDSM_RSTAMP(1, r, 0);
    if (!have_pre) {
      ne0 = (uint64_t)eoff[r];
      nn = (uint64_t)eoff[r + 1] - ne0;
    }
    const uint64_t e0 = ne0, n = nn;
    const uint64_t nb = (n + kSpan - 1) / kSpan, nfull = n / kSpan;
    // (the launcher zeroed every round's totals: no flag to wait for before adding to them)
    const CohChain ch{epoch0 + r, nullptr, r};
    unsigned long long* const tot = totals + 10ull * r;
    uint32_t acc = 0;  // lane q < 10: this wave's spans' total q
    for (uint64_t b = wv; b < nb; b += nw) {
      const bool up = b == wv && have_pre;
      if (b < nfull)
        coh_stream_wave<kSCSmall, true, true, true, kXcd>(pt, n_pages, ev + e0, n, b, status,
                                                          nullptr, err, n_nodes, tot, ch, up, pre,
                                                          &acc);
      else
        coh_stream_wave<kSCSmall, false, true, true, kXcd>(pt, n_pages, ev + e0, n, b, status,
                                                           nullptr, err, n_nodes, tot, ch, up, pre,
                                                           &acc);
    }
    GDSM_RSTAMP(1, r, 1);
    grid_arrive_wt<kXcd>(bar);
    have_pre = r + 1 < n_rounds && prefetch(r + 1);
    if (lane < 10 && acc) atomicAdd(tot + lane, (unsigned long long)acc);
    grid_wait_wt(bar, (r + 1) * team.n, err, kErrRoundsBarrier);
  }
}

// ---- DSM rounds, page-table side on ONE workgroup (gdsm_rounds with a small page table and
// small rounds, config 5): the page table sits in LDS for the whole launch, so a round needs no
// page-table gathers, no look-back and no grid barrier — two workgroup barriers. Per round: the
// round's events (loaded a round ahead, event 1024k + t in thread t) are checked (high dword,
// node) and their low dwords staged in LDS; every thread then folds the segments (page runs)
// whose head lies in its contiguous chunk of the round, each from its page's LDS word to the
// segment's end (SPEC §5's rules one event at a time, as oracle/gdsm_oracle.c or_coherence), and
// the round's totals are summed per wave, added in LDS and stored as row r. Pages are folded by
// exactly one thread per round (a page's events are one run of the sorted round), so the rounds
// need no other ordering. The page table is written back once, after the last round.
// Several workgroups (gridDim.x = W): workgroup w keeps pages [w S, w S + S) (S = `slice`) and
// folds the events of those pages only — every workgroup stages the whole round and counts the
// events below its slice and below its slice's end (their index range, the round being sorted),
// so a round's work is split W ways with no hand-off between workgroups; the totals are added to
// row r by each workgroup (the launcher zeroes the rows). A page outside the folding workgroup's
// slice (only an unsorted round puts one there) fails the call.
constexpr uint32_t kRLThreads = 1024;
constexpr uint32_t kRLEvents = kRoundsLdsEvents;    // a round's events staged (64 KiB)
constexpr uint32_t kRLPer = kRLEvents / kRLThreads;  // of them loaded per thread

__global__ __launch_bounds__(kRLThreads) void rounds_fold_lds_kernel(
    uint64_t* __restrict__ pt, uint64_t n_pages, const uint64_t* __restrict__ ev,
    const int64_t* __restrict__ eoff, uint32_t n_rounds, uint32_t* __restrict__ err,
    uint32_t n_nodes, unsigned long long* __restrict__ totals, uint32_t slice) {
  __shared__ uint64_t spt[kRoundsLdsPages];
  __shared__ uint32_t sev[kRLEvents];
  __shared__ int64_t soff[kRoundsLdsRounds + 1];
  __shared__ uint32_t red[10];
  __shared__ uint32_t rng[2][2];  // per round parity: events below the slice, below its end
  const uint32_t t = threadIdx.x, lane = t & 63;
  // this workgroup's slice of pages [base, base + np) (slice <= kRoundsLdsPages, by the caller)
  const uint32_t base = blockIdx.x * slice;
  const uint32_t np = base < n_pages ? (uint32_t)min((uint64_t)slice, n_pages - base) : 0u;
  const uint32_t lim = base + slice;
  for (uint32_t i = t; i < np; i += kRLThreads) spt[i] = pt[base + i];
  // every round's event offsets in LDS (n_rounds <= kRoundsLdsRounds, checked by the caller):
  // read from memory inside the loop, their scalar loads shared lgkmcnt with the walk's LDS
  // reads, and the first LDS wait of every round waited for them too (a memory round trip)
  for (uint32_t i = t; i <= n_rounds; i += kRLThreads) soff[i] = eoff[i];
  if (t < 10) red[t] = 0;
  if (t < 4) rng[t >> 1][t & 1] = 0;
  __syncthreads();
  uint32_t bad = 0;
  uint64_t X[kRLPer];
  uint32_t nn = 0;
  auto load = [&](uint32_t r) {
    const uint64_t e0 = (uint64_t)soff[r];
    nn = (uint32_t)((uint64_t)soff[r + 1] - e0);  // (<= kRLEvents, checked by the caller)
#pragma unroll
    for (uint32_t k = 0; k < kRLPer; ++k) {
      const uint32_t g = k * kRLThreads + t;
      X[k] = g < nn ? __builtin_nontemporal_load(ev + e0 + g) : 0ull;
    }
  };
  if (n_rounds) load(0);
  GDSM_RSTAMP_WG(true);
  for (uint32_t r = 0; r < n_rounds; ++r) {
    GDSM_RSTAMP(1, r, 0);
    // (a round past the staging area fails the call instead of walking past it; gdsm_rounds
    // never picks this kernel for one)
    const uint32_t n = nn <= kRLEvents ? nn : 0u;
    if (nn > kRLEvents) bad = 1;
    uint32_t below = 0, below_end = 0;  // this thread's events of pages < base / < lim
#pragma unroll
    for (uint32_t k = 0; k < kRLPer; ++k) {
      const uint32_t g = k * kRLThreads + t;
      if (g < n) {
        const uint64_t x = X[k];
        if ((x >> 32) || ((((uint32_t)x >> 1) & 7u) >= n_nodes)) bad = 1;
        sev[g] = (uint32_t)x;
        below += ((uint32_t)x >> 4) < base ? 1u : 0u;
        below_end += ((uint32_t)x >> 4) < lim ? 1u : 0u;
      }
    }
    if (gridDim.x > 1) {
      const uint32_t b0 = wave_sum(below), b1 = wave_sum(below_end);
      if (lane == 0) {
        if (b0) atomicAdd(&rng[r & 1][0], b0);
        if (b1) atomicAdd(&rng[r & 1][1], b1);
      }
    }
    __syncthreads();  // the round staged; the previous round's words and totals settled
    uint32_t lo = 0, hi = n;  // this slice's events (the whole round for one workgroup)
    if (gridDim.x > 1) {
      lo = min(rng[r & 1][0], n);
      hi = min(max(rng[r & 1][1], lo), n);
      if (t < 2) rng[(r + 1) & 1][t] = 0;  // (round r - 1's pair: read before this barrier)
    }
    GDSM_RSTAMP(1, r, 2);
    if (r + 1 < n_rounds) load(r + 1);  // in flight while this round is folded
    // (an odd C, which puts the lanes' chunk starts on distinct LDS banks, measured 20-40 % slower
    // on config 5 at 4 and 8 nodes: its rounds' page runs are P events long, which an even C
    // splits evenly between threads and an odd one does not)
    const uint32_t C = (hi - lo + kRLThreads - 1) / kRLThreads;
    const uint32_t c0 = min(lo + t * C, hi), c1 = min(c0 + C, hi);
    uint32_t inv = 0, xfer = 0;
    uint64_t nf_lo = 0, nf_hi = 0;  // fault counts of nodes 0-3 / 4-7, 16 bits each
    // One flat walk per thread (a nested per-head loop diverged: every head position of the
    // wave's lanes ran a whole segment walk): from the chunk's start, skipping the events of a
    // segment headed before it, through every segment headed inside it to that segment's end.
    uint32_t pp = c0 > 0 ? sev[c0 - 1] >> 4 : 0u;  // the page of the event before j
    uint32_t cur = 0, f = 0, cs = 0, owner = 0, st = 0, dirty = 0;
    bool have = false;  // folding the segment of page `cur`
    uint32_t y = c0 < n ? sev[c0] : 0u;
    for (uint32_t j = c0; j < n; ++j) {
      const uint32_t x = y, yn = j + 1 < n ? sev[j + 1] : 0u;  // (read one event ahead)
      const uint32_t pg = x >> 4;
      const bool head = j == 0 || pg != pp;
      if (j >= c1 && (head || !have)) break;  // the next segment is the next thread's
      if (head) {
        if (have)
          spt[cur] = (uint64_t)(cs | (owner << 8) | (st << 16) | (dirty << 18)) | ((uint64_t)f << 32);
        if (j > 0 && pg < pp) bad = 1;  // pages must not decrease
        have = pg >= base && pg - base < np;  // (outside the slice: an unsorted round)
        if (!have) bad = 1;
        const uint64_t w = spt[have ? pg - base : 0u];
        const uint32_t s = (uint32_t)w;
        cur = pg - base;
        f = (uint32_t)(w >> 32);
        cs = s & 0xFFu;
        owner = (s >> 8) & 0xFFu;
        st = (s >> 16) & 3u;
        dirty = (s >> 18) & 1u;
      }
      pp = pg;
      y = yn;
      if (!have) continue;
      // (a select-only form of this step measured slower: 4.4 vs 3.7 us per 4-node round)
      const uint32_t node = (x >> 1) & 7u, bit = 1u << node;
      bool fault;
      if (!(x & 1u)) {
        fault = !(cs & bit);
        if (fault) {
          cs |= bit;
          if (st == 2u) st = 1u;
        }
      } else {
        dirty = 1u;
        fault = !(st == 2u && owner == node);
        if (fault) {
          inv += (uint32_t)__popc(cs & ~bit);
          xfer += owner != node ? 1u : 0u;
        }
        owner = node;
        cs = bit;
        st = 2u;
      }
      if (fault) {
        ++f;
        const uint64_t one = 1ull << (16u * (node & 3u));
        if (node < 4u)
          nf_lo += one;
        else
          nf_hi += one;
      }
    }
    if (have) spt[cur] = (uint64_t)(cs | (owner << 8) | (st << 16) | (dirty << 18)) | ((uint64_t)f << 32);
    GDSM_RSTAMP(1, r, 3);
    // the round's totals: per wave, then in LDS (a thread's 16-bit node counts cannot overflow:
    // a round holds at most kRLEvents events)
    uint32_t v[10] = {inv, xfer};
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      v[2 + q] = (uint32_t)(nf_lo >> (16 * q)) & 0xFFFFu;
      v[6 + q] = (uint32_t)(nf_hi >> (16 * q)) & 0xFFFFu;
    }
#pragma unroll
    for (uint32_t q = 0; q < 10; ++q) {
      const uint32_t sq = wave_sum(v[q]);
      if (lane == 0 && sq) atomicAdd(&red[q], sq);
    }
    __syncthreads();  // the round's words and totals are in LDS
    GDSM_RSTAMP(1, r, 1);
    if (t < 10) {
      if (red[t]) atomicAdd(totals + 10ull * r + t, (unsigned long long)red[t]);
      red[t] = 0;  // (the next round adds after its first barrier)
    }
  }
  __syncthreads();
  for (uint32_t i = t; i < np; i += kRLThreads) pt[base + i] = spt[i];
  if (__syncthreads_or(bad) && t == 0) atomicOr(err, 2u);  // (kErrEvents)
}

const void* rounds_fold_kernel_ptr(bool xcd) {
  return xcd ? reinterpret_cast<const void*>(rounds_fold_kernel<true>)
             : reinterpret_cast<const void*>(rounds_fold_kernel<false>);
}

hipError_t launch_rounds_fold(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                              const uint64_t* events, const int64_t* eoff, uint32_t n_rounds,
                              uint32_t grid, uint64_t* totals, uint32_t* err, CohChainState* chain,
                              uint32_t* bar, bool xcd, bool lds, hipStream_t s, Prof* prof) {
  if (n_rounds == 0) return hipSuccess;
  if (lds) {  // `grid` workgroups, the page table in LDS slices (no chain workspace or barrier)
    const uint64_t slice = (n_pages + grid - 1) / max(grid, 1u);
    if (grid == 0 || grid > kRoundsLdsMaxWGs || slice > kRoundsLdsPages ||
        n_rounds > kRoundsLdsRounds)
      return hipErrorInvalidValue;
    const hipError_t e = hipMemsetAsync(totals, 0, 80ull * n_rounds, s);  // rows: added to
    if (e != hipSuccess) return e;
    ProfScope ps(prof, GDSM_PROF_COH_FOLD, s);
    hipLaunchKernelGGL(rounds_fold_lds_kernel, dim3(grid), dim3(kRLThreads), 0, s, pt, n_pages,
                       events, eoff, n_rounds, err, n_nodes,
                       reinterpret_cast<unsigned long long*>(totals), (uint32_t)max(slice, (uint64_t)1));
    return hipGetLastError();
  }
  if (!chain || !chain->ws) return hipErrorInvalidValue;
  // the rounds take epochs [epoch0, epoch0 + n_rounds); the chain is zeroed again afterwards by
  // its next launch (its ticket sets are not kept in step here)
  if (chain->epoch == 0 || chain->epoch + n_rounds >= (1u << 29)) {
    const hipError_t e = hipMemsetAsync(chain->ws, 0, coh_chain_bytes(), s);
    if (e != hipSuccess) return e;
    chain->epoch = 1;
  }
  const uint32_t epoch0 = chain->epoch;
  chain->epoch = 0;
  hipError_t e = hipMemsetAsync(bar, 0, kRoundsBarBytes, s);  // arrivals + team words
  if (e == hipSuccess) e = hipMemsetAsync(totals, 0, 80ull * n_rounds, s);  // every round's row
  if (e != hipSuccess) return e;
  ProfScope ps(prof, GDSM_PROF_COH_FOLD, s);
  hipLaunchKernelGGL(xcd ? rounds_fold_kernel<true> : rounds_fold_kernel<false>, dim3(grid),
                     dim3(256), 0, s, pt, n_pages, events, eoff,
                     n_rounds, chain->ws, err, n_nodes,
                     reinterpret_cast<unsigned long long*>(totals), epoch0, bar);
  return hipGetLastError();
}

// The small-batch path's zeroing (batch totals and the tickets + status granules) in one launch.
__global__ __launch_bounds__(256) void coh_zero_kernel(uint64_t* __restrict__ a, uint64_t na,
                                                       uint64_t* __restrict__ b, uint64_t nb) {
  const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = t0; i < na; i += st) a[i] = 0;
  for (uint64_t i = t0; i < nb; i += st) b[i] = 0;
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
// Coherence variant (gdsm_tune "coh_variant" or GDSM_COH_VARIANT): 0 (default) = automatic: the
// streaming fold with 256-event spans up to kCohSmall events, the single-pass fold
// (coh_fold_kernel) beyond; 1 = the streaming fold with 4096-event spans at every size; 2 = the
// single-pass fold at every size. All write the same page table and totals
// (tests/test_gpu_coherence.py runs each). Measurement builds (-DGDSM_MEASURE,
// scripts/dev/build_measure.sh; output invalid) add 4 / 5 / 6 = the fold without its walk /
// without its look-back / without the ordered look-back, and 7 = with its events read from a hot
// 64 MB window (coh_fold_wave kM 4). (1-3, the round-2 four-pass path, were
// removed in round 4; its last version is in git history, commit 585a356.)
#ifdef GDSM_MEASURE
constexpr int kCohVariants = 8;
static bool coh_variant_ok(int v) { return v <= 2 || (v >= 4 && v < kCohVariants); }
#else
static bool coh_variant_ok(int v) { return v >= 0 && v <= 2; }
#endif
static int coh_variant_from_env() {
  const char* e = getenv("GDSM_COH_VARIANT");
  const int v = e ? atoi(e) : 0;
  return coh_variant_ok(v) ? v : 0;
}
static std::atomic<int> g_coh_variant{coh_variant_from_env()};
// Small batches of a context outside graph capture: the chained one-launch form (CohChain) unless
// gdsm_tune("coh_chain", 0) or GDSM_COH_CHAIN=0 at load (then the zeroing launch before the fold).
static std::atomic<int> g_coh_chain{getenv("GDSM_COH_CHAIN") && atoi(getenv("GDSM_COH_CHAIN")) == 0 ? 0 : 1};
// the chained fold's span (gdsm_tune("coh_span", 1 | 2 | 4) 64-event chunks, GDSM_COH_SPAN).
// Config 5, same box, rounds/s, span 4 / 2 / 1 (and 8, not kept): 4 nodes 93.6k / 95.4k / 85.0k
// (71.6k); 8 nodes 83.1k / 73.8k / 60.8k (66.3k); 1 node 94.3k / 96.2k (71.2k).
static int coh_span_from_env() {
  const char* e = getenv("GDSM_COH_SPAN");
  const int v = e ? atoi(e) : 4;
  return (v == 1 || v == 2 || v == 4) ? v : 4;
}
static std::atomic<int> g_coh_span{coh_span_from_env()};
int coh_tune(const char* key, int64_t value) {
  if (!strcmp(key, "coh_span") && (value == 1 || value == 2 || value == 4)) {
    g_coh_span.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  if (!strcmp(key, "coh_chain") && (value == 0 || value == 1)) {
    g_coh_chain.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  if (!strcmp(key, "coh_variant") && value >= 0 && value < 8 && coh_variant_ok((int)value)) {
    g_coh_variant.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  return -1;
}

static inline uint64_t fold_blocks(uint64_t n) { return (n + kFBlock - 1) / kFBlock; }

// Batches up to kCohSmall events take the streaming fold with 256-event spans (S above): the
// fold's 2048-event blocks would leave most of the GPU idle, and a block's serial load -> walk
// -> look-back chain is the whole batch's time (config 5: ~8000 events per round).
constexpr uint64_t kCohSmall = 1u << 20;

uint64_t coh_workspace_bytes(uint64_t n_events) {
  // ticket counters + one status granule per block (or span), one partial row of totals each;
  // non-decreasing in n (a workspace reserved for n serves every smaller batch)
  const uint64_t ns = (min(n_events, kCohSmall) + 64 * kSCSmall - 1) / (64 * kSCSmall);
  const uint64_t nf = max(ns, fold_blocks(n_events));
  return 8 * (kFoldStatus + nf) + 40 * nf + 512;
}

hipError_t launch_coh_init(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes, hipStream_t s) {
  if (n_pages == 0) return hipSuccess;
  const uint64_t per = (n_pages + n_nodes - 1) / n_nodes;
  uint64_t g = (n_pages + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(coh_init_kernel, dim3((unsigned)g), dim3(256), 0, s, pt, n_pages, per);
  return hipGetLastError();
}

uint64_t coh_chain_bytes() {
  return 8 * (kCohChainStatus + kCohSmall / 64);  // spans of at least one 64-event chunk
}

hipError_t launch_coherence(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                            const uint64_t* events, uint64_t n_events, uint64_t* totals,
                            uint8_t* ws, uint64_t ws_bytes, uint32_t* err, hipStream_t s,
                            Prof* prof, CohChainState* chain) {
  const int cv = g_coh_variant.load(std::memory_order_relaxed);
  const bool small = cv == 0 && n_events <= kCohSmall;
  if (n_events == 0) return hipMemsetAsync(totals, 0, 10 * sizeof(uint64_t), s);
  if (small && chain && chain->ws && g_coh_chain.load(std::memory_order_relaxed)) {
    // one launch: epoch-tagged granules, counters and totals row the previous launch zeroed
    if (chain->epoch == 0) {
      const hipError_t e = hipMemsetAsync(chain->ws, 0, coh_chain_bytes(), s);
      if (e != hipSuccess) return e;
      chain->epoch = 1;
    }
    const uint32_t sc = (uint32_t)g_coh_span.load(std::memory_order_relaxed);  // chunks per span
    const uint64_t span = 64ull * sc;
    const uint64_t ns = (n_events + span - 1) / span, full = n_events / span;
    ProfScope ps(prof, GDSM_PROF_COH_FOLD, s);
    auto kern = sc == 1   ? coh_stream_kernel<1, true>
                : sc == 2 ? coh_stream_kernel<2, true>
                          : coh_stream_kernel<kSCSmall, true>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, s, pt, n_pages, events,
                       n_events, ns, full, chain->ws, nullptr, err, n_nodes,
                       reinterpret_cast<unsigned long long*>(totals), chain->epoch);
    const hipError_t e = hipGetLastError();
    // a launch that did not run leaves its successor's set unzeroed: start the chain over
    chain->epoch = e != hipSuccess || chain->epoch + 1 >= (1u << 29) ? 0 : chain->epoch + 1;
    return e;
  }
  if (coh_workspace_bytes(n_events) > ws_bytes) return hipErrorInvalidValue;
  hipError_t r;
  if (cv == 1 || small) {
    const uint64_t span = 64ull * (small ? kSCSmall : kSCBig);
    const uint64_t ns = (n_events + span - 1) / span;
    uint64_t* fws = reinterpret_cast<uint64_t*>(ws);
    uint32_t* fpart = reinterpret_cast<uint32_t*>(fws + kFoldStatus + ns);
    // the totals and the tickets + status granules zeroed by one launch
    const uint64_t nz = kFoldStatus + ns;
    hipLaunchKernelGGL(coh_zero_kernel, dim3((unsigned)min((nz + 255) / 256, (uint64_t)1024)),
                       dim3(256), 0, s, totals, (uint64_t)10, fws, nz);
    {
      ProfScope ps(prof, GDSM_PROF_COH_FOLD, s);
      const uint64_t full = n_events / span;
      auto kern = small ? coh_stream_kernel<kSCSmall> : coh_stream_kernel<kSCBig>;
      unsigned long long* direct = small ? reinterpret_cast<unsigned long long*>(totals) : nullptr;
      hipLaunchKernelGGL(kern, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, s, pt, n_pages,
                         events, n_events, ns, full, fws, fpart, err, n_nodes, direct, 0u);
    }
    if (small) return hipGetLastError();
    uint64_t g = (ns + 255) / 256;
    if (g > 1024) g = 1024;
    ProfScope ps(prof, GDSM_PROF_COH_REDUCE, s);
    hipLaunchKernelGGL(coh_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, fpart, ns,
                       reinterpret_cast<unsigned long long*>(totals));
    return hipGetLastError();
  }
  r = hipMemsetAsync(totals, 0, 10 * sizeof(uint64_t), s);
  if (r != hipSuccess) return r;
  if (cv == 0 || cv == 2 || cv >= 4) {
    const uint64_t nf = fold_blocks(n_events);
    uint64_t* fws = reinterpret_cast<uint64_t*>(ws);
    uint32_t* fpart = reinterpret_cast<uint32_t*>(fws + kFoldStatus + nf);
    r = hipMemsetAsync(fws, 0, 8 * (kFoldStatus + nf), s);  // tickets + status granules
    if (r != hipSuccess) return r;
    {
      ProfScope ps(prof, GDSM_PROF_COH_FOLD, s);
      const bool vec = (reinterpret_cast<uintptr_t>(events) & 15) == 0;
      const bool nodes = n_nodes < 8;
      const uint64_t full = n_events / kFBlock;
      if (full) {
        auto kern = vec ? (nodes ? coh_fold_kernel<true, true, true> : coh_fold_kernel<true, true, false>)
                        : (nodes ? coh_fold_kernel<false, true, true> : coh_fold_kernel<false, true, false>);
#ifdef GDSM_MEASURE
        if (vec && !nodes && cv == 4) kern = coh_fold_kernel<true, true, false, 1>;
        if (vec && !nodes && cv == 5) kern = coh_fold_kernel<true, true, false, 2>;
        if (vec && !nodes && cv == 6) kern = coh_fold_kernel<true, true, false, 3>;
        if (vec && !nodes && cv == 7) kern = coh_fold_kernel<true, true, false, 4>;
#endif
        hipLaunchKernelGGL(kern, dim3((unsigned)((full + kFoldWaves - 1) / kFoldWaves)),
                           dim3(64 * kFoldWaves), 0, s, pt, n_pages, events, n_events, full, fws,
                           fpart, err, n_nodes);
      }
      if (nf > full) {
        auto kern = nodes ? coh_fold_kernel<false, false, true> : coh_fold_kernel<false, false, false>;
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, s, pt, n_pages, events, n_events, nf, fws,
                           fpart, err, n_nodes);
      }
    }
    uint64_t g = (nf + 255) / 256;
    if (g > 1024) g = 1024;
    ProfScope ps(prof, GDSM_PROF_COH_REDUCE, s);
    hipLaunchKernelGGL(coh_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, fpart, nf,
                       reinterpret_cast<unsigned long long*>(totals));
    return hipGetLastError();
  }
  return hipErrorInvalidValue;  // coh_variant 1-3 (the four-pass path) no longer exist
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

#ifdef GDSM_ROUNDS_STAMPS
extern "C" int gdsm_debug_fold_spans(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gdsm::g_fold_spans), bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -EIO;
}
extern "C" int gdsm_debug_round_stamps_pt(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gdsm::g_round_stamps), bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -5;
}
#endif
#ifdef GDSM_COH_STAMPS
extern "C" int gdsm_debug_coh_stamps(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gdsm::g_coh_stamps), bytes, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -1;
}
#endif
