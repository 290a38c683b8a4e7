// GPU Needleman-Wunsch for the legacy diff() symbol: the alignment of
// gallocy/utils/diff.cpp:73-167 for a batch of byte-string pairs, bit-exact with the CPU
// restatement (legacy_diff.cpp, oracle or_nw_diff) and therefore with the reference wherever the
// reference survives (n, m <= 1180), and without its size limit.
//
// Recurrence (diff.cpp:104-123): H[y][x] = max(dg, lf, up) with dg = H[y-1][x-1] + (a==b)
// (the MATCH ternary quirk, diff.cpp:107-108), lf = H[y][x-1] - 1, up = H[y-1][x] - 1, borders
// H[0][x] = -x, H[y][0] = -y (diff.cpp:94-102); the traceback prefers diag > left > up
// (diff.cpp:115-120) and runs from (n, m) to (0, 0) (diff.cpp:126-158).
//
// Fill (nw_fill_kernel): one 8-wave workgroup per pair. Rows are cut into strips of 512; a strip
// belongs to one wave, 8 consecutive rows per lane (8 rows spread the per-step DPP and feed work
// over twice the cells of 4: the fill of 512 x 4 KiB pairs 1.27 -> 1.01 ms). Lane l computes
// column x = t - l + 1 at step t, so the value from the row above (lane l-1's bottom row one step
// earlier) arrives by one DPP wave_shr:1, and the byte of b by one LDS byte read (b is staged in
// LDS). Strip s+1 follows strip s two 64-step phases behind (one workgroup barrier per phase);
// the bottom row of a strip reaches the next wave through a 256-column LDS ring (or, from the
// last wave to wave 0 of the next group of strips, through the strip's bottom row in global
// memory). No MFMA: the recurrence is max/add on int32, not a contraction.
//
// Scores are kept as U = H + y + x, which makes every border 0 and a cell one compare, one
// add-with-carry and one max3: U = max3(U[y-1][x-1] + 2 + (a==b), U[y][x-1], U[y-1][x]). The three
// candidates are H's candidates shifted by the same y + x, so every comparison (and the traceback)
// is the reference's.
//
// No traceback leaves the fill. It stores, per strip, the lanes' state every 64 steps (a
// checkpoint: 8 left values, diag, pass; 40 B per lane) and the strip's bottom row (the next
// strip's input, one word per column). The trace recomputes one 64-step region of a strip from
// its checkpoint when the path enters it, with the traceback bits this time: two bits per cell,
// nd = "not diag" (dg < max(lf, up)) and u = "up beats left" (up > left, only read when nd), a
// 16-byte record per lane per 8 steps, into LDS. The path crosses ~10 regions of a strip, so the
// trace recomputes a few % of the matrix where the fill used to write 2 bits for every cell.
//
// Trace (nw_trace_kernel, 8 waves per pair): the strips are walked in parallel from guessed
// entries, then checked in order (a strip whose real entry differs is walked again until it meets
// its first walk), and every DP row's share of the output is written at once (see below).
#include "gdsm_common.h"
#include "gdsm_launch.h"

// v_writelane_b32 as the compiler's own intrinsic (this clang has no __builtin for it): the
// compiler then picks M0 for the lane select and knows it is written.
extern "C" __device__ int nw_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace gdsm {
namespace {

// Geometry (compile-time; the defaults are the measured best for 4 KiB pairs): rows
// per lane, waves per fill workgroup, steps per phase and phases between strips, steps per
// checkpoint, waves per trace workgroup.
#ifndef GDSM_NW_ROWS
#define GDSM_NW_ROWS 8
#endif
constexpr uint32_t kRows = GDSM_NW_ROWS;  // DP rows per lane
#ifndef GDSM_NW_WAVES
#define GDSM_NW_WAVES 8
#endif
constexpr uint32_t kWaves = GDSM_NW_WAVES;  // waves per fill workgroup
constexpr uint32_t kStrip = 64 * kRows;   // rows per strip
#ifndef GDSM_NW_PHASE
#define GDSM_NW_PHASE 64
#endif
#ifndef GDSM_NW_LAG
#define GDSM_NW_LAG 2
#endif
constexpr uint32_t kPhase = GDSM_NW_PHASE;  // steps per phase (between barriers)
constexpr uint32_t kLag = GDSM_NW_LAG;      // phases between consecutive strips
constexpr uint32_t kRing = 256;           // ring slots per wave (>= 193 live columns)
constexpr uint32_t kBlk = 16;             // steps per block (one feed word per lane, ...)
constexpr uint32_t kRecK = 64 / kRows;    // steps per traceback record (a lane's rows x kRecK
constexpr uint32_t kRecPerBlk = kBlk / kRecK;  // cells = one 64-bit mask per bit)
static_assert(kRows == 4 || kRows == 8, "rows per lane");
#ifndef GDSM_NW_CK
#define GDSM_NW_CK 64
#endif
constexpr uint32_t kCk = GDSM_NW_CK;      // steps per checkpoint = per recomputed region
constexpr uint32_t kCkBlk = kCk / kBlk;   // records per lane per region
constexpr uint32_t kCkBytes = 64 * (4 * kRows + 8);  // one checkpoint: 64 x (left[] | diag, pass)

__device__ __forceinline__ uint32_t wave_shr1_or(uint32_t old, uint32_t v) {
  // Lane l gets lane l-1's v; lane 0 keeps `old` (bound_ctrl off).
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t wave_rol1(uint32_t v) {
  // Lane l gets lane l+1's v, lane 63 gets lane 0's.
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x134, 0xF, 0xF, false);
}

struct Strip {
  uint32_t a[kRows];
  int32_t left[kRows];  // U[y][x-1]
  int32_t diag;         // U[ytop-1][x-1]
  int32_t pass;         // U[ybottom][x]: the row above for lane l+1 one step later
};

__device__ __forceinline__ uint32_t shift_in_sign(uint32_t acc, int32_t v) {
  return __builtin_amdgcn_alignbit(acc, (uint32_t)v, 31);  // (acc << 1) | (v < 0)
}

// Pair geometry shared by the fill and the trace (max_len fixes the workspace strides).
__host__ __device__ inline uint32_t step_blocks(uint32_t n2) { return (n2 + 63 + kBlk - 1) / kBlk; }
struct Geo {
  uint32_t CK;   // checkpoints per strip slot
  uint64_t RS;   // words per stored bottom row
  uint64_t ck_bytes, row_bytes, rec_bytes;
  __host__ __device__ explicit Geo(uint32_t max_len) {
    const uint64_t S = max_len ? (max_len + kStrip - 1) / kStrip : 1;
    CK = (step_blocks(max_len) * kBlk + kCk - 1) / kCk;
    RS = (uint64_t)max_len + 64;
    ck_bytes = S * CK * kCkBytes;
    row_bytes = (S * RS * 4 + 255) & ~255ull;
    rec_bytes = (((uint64_t)max_len + 2) * 4 + 255) & ~255ull;  // the trace's row records
  }
  __host__ __device__ uint64_t per_pair() const { return ck_bytes + row_bytes + rec_bytes; }
};

// One block of 16 steps [t0, t0 + 16) of a strip. R: lane i holds the word lane 0 consumes at
// step t0 + i (the row above the strip, up to 64 steps ahead); bx[x] is b's byte at column x
// (1..n2). One register carries both ways: each step R rotates down a lane (lane 0 meets the next
// feed word, the consumed one wraps to lane 63) and lane 63 takes the new bottom word, so after
// the block lanes 48..63 hold the bottom words of steps t0..t0+15 (columns t0-62 .. t0-47) and
// lanes 0..47 the feed words of the next 48 steps. With kRec the traceback bits of the lane's
// kRows x 16 cells go to rec[0 .. kRecPerBlk), one 64-bit mask pair per kRecK steps.
// GDSM_NW_ASM: a step's diagonal candidates dg[r] + 2 + (a[r] == b) four rows per asm statement,
// the four compares into four SGPR pairs before the four add-with-carries, so no carry is read
// right after the compare that wrote it (the compiler reuses VCC and waits a cycle per cell).
// 2 (default): in the trace's region recomputation only, 3.6 % off the trace (0.388 -> 0.374 ms
// per batch, 1.3 % off the step); 1: in the fill too, which then runs 5 % slower (its compares
// lose their SDWA byte selects on the packed feed word); 0: the compiler's code everywhere.
#ifndef GDSM_NW_ASM
#define GDSM_NW_ASM 2
#endif
__device__ __forceinline__ void diag4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                      uint32_t b, int32_t g0, int32_t g1, int32_t g2, int32_t g3,
                                      int32_t& d0, int32_t& d1, int32_t& d2, int32_t& d3) {
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_cmp_eq_u32_e64 %4, %8, %12\n\t"
      "v_cmp_eq_u32_e64 %5, %9, %12\n\t"
      "v_cmp_eq_u32_e64 %6, %10, %12\n\t"
      "v_cmp_eq_u32_e64 %7, %11, %12\n\t"
      "v_addc_co_u32_e64 %0, %4, 2, %13, %4\n\t"
      "v_addc_co_u32_e64 %1, %5, 2, %14, %5\n\t"
      "v_addc_co_u32_e64 %2, %6, 2, %15, %6\n\t"
      "v_addc_co_u32_e64 %3, %7, 2, %16, %7"
      : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b), "v"(g0), "v"(g1), "v"(g2), "v"(g3));
}

template <bool kMasked, bool kRec>
__device__ __forceinline__ uint32_t fill_block(Strip& st, uint32_t R, const uint8_t* bx,
                                               uint32_t t0, uint32_t n2, uint32_t lane,
                                               uint4* rec) {
  constexpr uint32_t kW = kBlk * kRows / 32;  // 32-bit words per mask per block
  uint32_t ndw[kW], uw[kW];
#pragma unroll
  for (uint32_t i = 0; i < kW; ++i) ndw[i] = uw[i] = 0;
  const int32_t x0 = (int32_t)(t0 + 1) - (int32_t)lane;  // this lane's column at step t0
  const bool top = lane == 63;
#pragma unroll
  for (uint32_t k = 0; k < kBlk; ++k) {
    const int32_t x = x0 + (int32_t)k;
    bool act = true;
    uint32_t bb;
    if (kMasked) {
      act = x >= 1 && x <= (int32_t)n2;
      bb = bx[min(max(x, 1), (int32_t)n2)];
    } else {
      bb = bx[x];
    }
    const int32_t up_in = (int32_t)wave_shr1_or(R, (uint32_t)st.pass);
    R = wave_rol1(R);  // lane 0: the next feed word; lane 63: free (this step's feed, consumed)
    int32_t up = up_in, dgv = st.diag;
    uint32_t* acc_nd = &ndw[k / (32 / kRows)];
    uint32_t* acc_u = &uw[k / (32 / kRows)];
    int32_t dd[kRows];
    if (GDSM_NW_ASM && (GDSM_NW_ASM == 1 || kRec) && kRows == 8) {
      diag4(st.a[0], st.a[1], st.a[2], st.a[3], bb, st.diag, st.left[0], st.left[1], st.left[2],
            dd[0], dd[1], dd[2], dd[3]);
      diag4(st.a[4], st.a[5], st.a[6], st.a[7], bb, st.left[3], st.left[4], st.left[5],
            st.left[6], dd[4], dd[5], dd[6], dd[7]);
    }
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
      const int32_t lf = st.left[r];
      const int32_t d = (GDSM_NW_ASM && (GDSM_NW_ASM == 1 || kRec) && kRows == 8)
                            ? dd[r]
                            : dgv + 2 + (st.a[r] == bb ? 1 : 0);
      const int32_t mx = max(max(d, lf), up);
      if (kRec) {
        *acc_nd = shift_in_sign(*acc_nd, d - mx);
        *acc_u = shift_in_sign(*acc_u, lf - up);
      }
      dgv = lf;
      up = mx;
      if (kMasked) st.left[r] = act ? mx : lf;
      else st.left[r] = mx;
    }
    if (kMasked) st.diag = act ? up_in : st.diag;
    else st.diag = up_in;
    st.pass = up;
    R = top ? (uint32_t)up : R;
  }
  if (kRec) {
#pragma unroll
    for (uint32_t h = 0; h < kRecPerBlk; ++h)
      rec[h] = make_uint4(ndw[2 * h], ndw[2 * h + 1], uw[2 * h], uw[2 * h + 1]);
  }
  return R;
}

__device__ __forceinline__ void strip_start(Strip& st, const uint8_t* a, uint64_t ao, uint32_t n1,
                                            uint32_t s, uint32_t lane) {
  const uint32_t y0 = s * kStrip + lane * kRows + 1;
#pragma unroll
  for (uint32_t r = 0; r < kRows; ++r) {
    st.a[r] = (y0 + r <= n1) ? a[ao + y0 + r - 1] : 0u;
    st.left[r] = 0;
  }
  st.diag = 0;
  st.pass = 0;
}

constexpr uint32_t kBLds = 48 * 1024 - 16;  // b staged in LDS up to this length (64 KiB in all)
extern __shared__ uint8_t nw_dyn_lds[];

template <bool kLdsB>
__global__ __launch_bounds__(64 * kWaves) void nw_fill_kernel(
    const uint8_t* __restrict__ a, const uint64_t* __restrict__ a_off,
    const uint8_t* __restrict__ b, const uint64_t* __restrict__ b_off, uint64_t first_pair,
    uint32_t max_len, uint8_t* __restrict__ ws, uint32_t* __restrict__ err) {
  __shared__ uint32_t ring[kWaves][kRing];
  const uint64_t pair = first_pair + blockIdx.x;
  const uint64_t ao = a_off[pair], bo = b_off[pair];
  const uint64_t l1 = a_off[pair + 1] - ao, l2 = b_off[pair + 1] - bo;
  if (l1 > max_len || l2 > max_len) {
    if (threadIdx.x == 0) atomicOr(err, 4u);
    return;
  }
  const uint32_t n1 = (uint32_t)l1, n2 = (uint32_t)l2;
  if (!n1 || !n2) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint8_t* bx = b + bo - 1;
  if (kLdsB) {
    for (uint32_t i = threadIdx.x; i < n2; i += 64 * kWaves) nw_dyn_lds[i + 1] = bx[i + 1];
    bx = nw_dyn_lds;
    __syncthreads();
  }
  const uint32_t S = (n1 + kStrip - 1) / kStrip;
  const uint32_t nblk = step_blocks(n2);                        // step blocks per strip
  const uint32_t T = (nblk * kBlk + kPhase - 1) / kPhase;      // phases per strip
  // Group g of 16 strips starts at phase g * TT; strip 16g + w at g * TT + kLag * w. TT lets wave
  // 15 finish a strip before wave 0 of the next group reads its bottom row, and a wave's ring
  // outlive its previous reader.
  const uint32_t TT = T + kLag * (kWaves - 1);
  const uint32_t Q = ((S - 1) / kWaves) * TT + kLag * ((S - 1) % kWaves) + T;
  const Geo geo(max_len);
  uint8_t* ck = ws + blockIdx.x * geo.per_pair();
  uint32_t* rows = reinterpret_cast<uint32_t*>(ck + geo.ck_bytes);
  const uint32_t* ring_in = ring[(w + kWaves - 1) % kWaves];
  uint32_t* ring_out = ring[w];

  Strip st;
  for (uint32_t q = 0; q < Q; ++q) {
    const int32_t rel = (int32_t)q - (int32_t)(kLag * w);
    if (rel >= 0) {
      const uint32_t g = (uint32_t)rel / TT, lp = (uint32_t)rel - g * TT;
      const uint32_t s = g * kWaves + w;
      if (s < S && lp < T) {
        if (lp == 0) strip_start(st, a, ao, n1, s, lane);
        // The phase's 64 feed words, one per lane: column x = 64 lp + 1 + lane of the row above.
        const uint32_t x = lp * kPhase + 1 + lane;
        uint32_t R = 0;
        if (s == 0) {
          R = 0;
        } else if (w == 0) {
          const uint32_t* src = rows + (uint64_t)(s - 1) * geo.RS;
          R = (x <= n2) ? __hip_atomic_load(src + x - 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : 0u;
        } else {
          R = ring_in[(x - 1) & (kRing - 1)];
        }
        for (uint32_t bi = 0; bi < kPhase / kBlk; ++bi) {
          const uint32_t t0 = lp * kPhase + bi * kBlk;
          if (t0 >= nblk * kBlk) break;
          if ((t0 & (kCk - 1)) == 0) {  // checkpoint: the state before step t0
            uint8_t* c = ck + ((uint64_t)s * geo.CK + t0 / kCk) * kCkBytes;
#pragma unroll
            for (uint32_t q = 0; q < kRows / 4; ++q)
              reinterpret_cast<int4*>(c + 64 * 16 * q)[lane] =
                  make_int4(st.left[4 * q], st.left[4 * q + 1], st.left[4 * q + 2], st.left[4 * q + 3]);
            reinterpret_cast<int2*>(c + 64 * 4 * kRows)[lane] = make_int2(st.diag, st.pass);
          }
          const bool masked = t0 < 64 || t0 + kBlk > n2;
          R = masked ? fill_block<true, false>(st, R, bx, t0, n2, lane, nullptr)
                     : fill_block<false, false>(st, R, bx, t0, n2, lane, nullptr);
          // Lanes 48..63 of R: lane 63's bottom words at steps t0..t0+15, columns t0-62 ..
          if (lane >= 48) {
            const int32_t xo = (int32_t)(t0 + lane) - 110;
            ring_out[(uint32_t)(xo - 1) & (kRing - 1)] = R;
            if (s + 1 < S && xo >= 1 && xo <= (int32_t)n2) rows[(uint64_t)s * geo.RS + xo - 1] = R;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---- trace: strips in parallel from guessed entries, then checked in order -------------------
// The path is recorded per DP row y as (lo, how it leaves the row): it enters row y at column hi,
// moves left to lo, then up (3) or diagonally (1) into row y - 1, so hi of row y is where row
// y + 1 left it (lo - 1 after a diagonal, lo after an up; n2 for row n1) and row 0 holds the
// final run of left moves. Phase A: the pair's waves walk all strips at once, each from a guessed
// entry on its strip's bottom row (the last strip's, (n1, n2), is exact; the others y * n2 / n1).
// Phase B: wave 0 takes the strips in order from the end: a strip whose real entry (the exit of
// the strip below) is not its guess is walked again from the real one until it meets its
// recorded path (a cell inside that row's [lo, hi]: from a common cell on the two paths agree).
// Phase C: every row's share of the output by a scan, and its characters.
#ifndef GDSM_NW_TW
#define GDSM_NW_TW 8
#endif
constexpr uint32_t kTW = GDSM_NW_TW;     // trace waves per pair
constexpr uint32_t kX21 = (1u << 21) - 1;  // columns <= 2^20 (gdsm_nw_diff_batch's limit)

__device__ __forceinline__ uint32_t ld_row(const uint32_t* p) {  // other waves' rows (L2)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_row_u(const uint32_t* p) {  // the same, wave-uniform
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_row(p));
}
// the column a row record hands to the row above it (its entry column there)
__device__ __forceinline__ uint32_t row_exit(uint32_t v) {
  return (v & kX21) - ((v >> 21) == 1u ? 1u : 0u);
}

__global__ __launch_bounds__(64 * kTW) void nw_trace_kernel(
    const uint8_t* __restrict__ a, const uint64_t* __restrict__ a_off,
    const uint8_t* __restrict__ b, const uint64_t* __restrict__ b_off, uint64_t first_pair,
    uint32_t max_len, uint8_t* __restrict__ ws, uint8_t* __restrict__ out1,
    uint8_t* __restrict__ out2, uint64_t* __restrict__ out_len) {
  __shared__ uint4 lrec_all[kTW][kCkBlk * kRecPerBlk][64];  // each wave's region (64 KiB)
  __shared__ uint8_t bwin_all[kTW][256];         // each wave's region of b (kCk + 63 columns)
  const uint64_t pair = first_pair + blockIdx.x;
  // the wave index as a scalar: everything a wave walks with is wave-uniform
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t ao = a_off[pair], bo = b_off[pair];
  const uint64_t l1 = a_off[pair + 1] - ao, l2 = b_off[pair + 1] - bo;
  if (l1 > max_len || l2 > max_len) return;  // flagged by the fill kernel
  const uint32_t n1 = (uint32_t)l1, n2 = (uint32_t)l2;
  const uint32_t nblk = step_blocks(n2);
  const uint8_t* bx = b + bo - 1;
  const Geo geo(max_len);
  const uint8_t* ck = ws + blockIdx.x * geo.per_pair();
  const uint32_t* rows = reinterpret_cast<const uint32_t*>(ck + geo.ck_bytes);
  uint32_t* rr = reinterpret_cast<uint32_t*>(ws + blockIdx.x * geo.per_pair() + geo.ck_bytes +
                                             geo.row_bytes);  // rr[y]: lo | exit << 21
  uint4(*lrec)[64] = lrec_all[w];
  constexpr int32_t kRecs = (int32_t)(kCkBlk * kRecPerBlk);  // records per lane per region
  const uint32_t S = (n1 + kStrip - 1) / kStrip;
  auto guess = [&](uint32_t s) -> uint32_t {
    if (s + 1 == S) return n2;
    return (uint32_t)(((uint64_t)kStrip * (s + 1) * n2 + n1 / 2) / n1);
  };

  // A record holds a lane's kRows rows x kRecK steps as two 64-bit masks (nd, u), cell (k, r) at
  // bit 63 - (kRows k + r): inside a record a left move is bit + kRows, up + 1, diag + kRows + 1,
  // all scalar; the record changes when the path leaves the lane's rows or the record's steps.
  int32_t rs = -1, rq = 0;             // the region in LDS: strip rs, steps [rq*kCk, +kCk)
  int32_t ws_ = -1, wl0 = 0, wb0 = 0;  // the record window in VGPRs
  uint4 rec = make_uint4(0, 0, 0, 0);
  // Row records leave 64 at a time: lane j of rbuf holds row ystart - (nbase + j). Every cell
  // writes its row's candidate record into slot nrow % 64; the slot only advances when the row
  // ends (no branch per cell).
  uint32_t rbuf = 0, nrow = 0, ystart = 0;
  auto put = [&](uint32_t v, uint32_t dr) {
    uint32_t j = nrow & 63;
    asm volatile("" : "+s"(v), "+s"(j));  // both in SGPRs (a literal is no writelane operand)
    // One scalar operand per VALU on gfx950: the compiler routes the lane select through M0
    // itself (it owns M0, so nothing it keeps there is clobbered behind its back).
    rbuf = (uint32_t)nw_writelane((int)v, (int)j, (int)rbuf);
    nrow += dr;
    if ((j + dr) & 64) rr[ystart - (nrow - 64) - lane] = rbuf;  // slot 63 filled: 64 rows out
  };
  auto flush_rows = [&]() {
    const uint32_t j = nrow & 63;
    if (j && lane < j) rr[ystart - (nrow - j) - lane] = rbuf;
    nrow = 0;
  };

  // Walk strip s from (y, x) on until the path leaves the strip's top row. With `merge`, stop
  // at the first cell inside the recorded row's [lo, hi] (the row keeps its lo and exit).
  auto walk = [&](uint32_t s, uint32_t y, uint32_t x, bool merge) {
    const uint32_t top = s * kStrip + 1;
    ystart = y;
    uint32_t spec = merge ? ld_row_u(rr + y) : 0;  // the recorded row y
    uint32_t spec_hi = x == n2 && y == n1 ? n2 : guess(s);  // its entry column
    while (y >= top) {
      if (merge && (spec & kX21) <= x && x <= spec_hi) {
        put(spec, 1);  // merged: this row and the ones above are the recorded path
        break;
      }
      if (x == 0) {  // column 0: straight up
        put(3u << 21, 1);
        --y;
        if (merge && y >= top) {
          spec_hi = row_exit(spec);
          spec = ld_row_u(rr + y);
        }
        continue;
      }
      const uint32_t yy = y - 1;
      const int32_t l = (int32_t)((yy / kRows) & 63);
      const uint32_t r = yy & (kRows - 1);
      const uint32_t t = x - 1 + (uint32_t)l;
      const int32_t blk = (int32_t)(t / kRecK);  // the record (kRecK steps) holding the cell
      const uint32_t k = t & (kRecK - 1);
      if ((int32_t)s != rs || blk < rq * kRecs ||
          blk >= (rq + 1) * kRecs) {  // recompute the region from its checkpoint
        rs = (int32_t)s;
        rq = blk / kRecs;
        const uint8_t* c = ck + ((uint64_t)s * geo.CK + (uint32_t)rq) * kCkBytes;
        const int2 dp = reinterpret_cast<const int2*>(c + 64 * 4 * kRows)[lane];
        Strip st;
        strip_start(st, a, ao, n1, s, lane);
#pragma unroll
        for (uint32_t q = 0; q < kRows / 4; ++q) {
          const int4 lv = reinterpret_cast<const int4*>(c + 64 * 16 * q)[lane];
          st.left[4 * q] = lv.x;
          st.left[4 * q + 1] = lv.y;
          st.left[4 * q + 2] = lv.z;
          st.left[4 * q + 3] = lv.w;
        }
        st.diag = dp.x;
        st.pass = dp.y;
        // the row above the strip: 64 columns per register, both halves loaded at once
        const uint32_t* above = rows + (uint64_t)(s > 0 ? s - 1 : 0) * geo.RS;
        auto feed = [&](uint32_t t0) -> uint32_t {
          const uint32_t xf = t0 + 1 + lane;
          return (s > 0 && xf <= n2) ? above[xf - 1] : 0u;
        };
        uint32_t R = feed((uint32_t)rq * kCk);
        const uint32_t R2 = kCkBlk > kPhase / kBlk ? feed((uint32_t)rq * kCk + kPhase) : 0u;
        // the region's columns of b, loaded with the checkpoint: bw[x] for x in
        // [rq kCk - 62, rq kCk + kCk] (masked blocks clamp x inside it)
        uint8_t* bwin = bwin_all[w];
        const int32_t xb = (int32_t)((uint32_t)rq * kCk) - 63;
        static_assert(kCk + 64 <= 256, "b window");
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const int32_t xc = xb + (int32_t)(4 * lane + j);
          bwin[4 * lane + j] = (xc >= 1 && xc <= (int32_t)n2) ? bx[xc] : (uint8_t)0;
        }
        const uint8_t* bw = bwin - xb;
        for (uint32_t bi = 0; bi < kCkBlk; ++bi) {
          const uint32_t t0 = (uint32_t)rq * kCk + bi * kBlk;
          if (t0 >= nblk * kBlk) break;
          if (bi == kPhase / kBlk) R = R2;
          uint4 rr4[kRecPerBlk];
          R = (t0 < 64 || t0 + kBlk > n2) ? fill_block<true, true>(st, R, bw, t0, n2, lane, rr4)
                                          : fill_block<false, true>(st, R, bw, t0, n2, lane, rr4);
#pragma unroll
          for (uint32_t h = 0; h < kRecPerBlk; ++h) lrec[bi * kRecPerBlk + h][lane] = rr4[h];
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes are done
        __builtin_amdgcn_wave_barrier();
        ws_ = -1;
      }
      // (a walk moves to smaller l and blk; a new walk may start anywhere)
      if ((int32_t)s != ws_ || l < wl0 || blk < wb0 || l > wl0 + 15 || blk > wb0 + 3) {
        ws_ = (int32_t)s;
        wl0 = l - 15;
        wb0 = max(blk - 3, rq * kRecs);
        const int32_t il = wl0 + (int32_t)(lane >> 2), ib = wb0 + (int32_t)(lane & 3);
        rec = il >= 0 ? lrec[ib - rq * kRecs][il] : make_uint4(0, 0, 0, 0);
      }
      const int idx = (l - wl0) * 4 + (blk - wb0);
      const uint64_t nd = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rec.x, idx) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)rec.y, idx);
      const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rec.z, idx) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)rec.w, idx);
      // Leaving the record: the row above lane l's rows (r < 0), the step before the record
      // (k < 0) or column 0 (k < l - kRecK blk): bit > bmax.
      const int32_t kmin = max(0, l - (int32_t)kRecK * blk);
      const uint32_t bmax = 63 - kRows * (uint32_t)kmin;
      uint32_t bit = 63 - (kRows * k + r);
      const uint32_t y0 = y;
      for (;;) {  // inside record (l, blk); integer flags keep it all scalar
        const uint32_t ndb = (uint32_t)(nd >> bit) & 1u, ub = (uint32_t)(u >> bit) & 1u;
        const uint32_t upm = ndb & ub;         // 1: up
        const uint32_t code = 1u + ndb + upm;  // 1 diag, 2 left, 3 up
        const uint32_t dk = 1u - upm;          // x moves
        const uint32_t dr = 1u - ndb + upm;    // y moves
        put(x | (code << 21), dr);             // this row's record, if the row ends here
        x -= dk;
        y -= dr;
        const uint32_t wrap = ((bit & (kRows - 1)) + dr) & kRows;  // r was 0 and y moved
        bit += kRows * dk + dr;
        if (merge || (int32_t)((bmax - bit) | (0u - wrap)) < 0) break;
      }
      if (merge && y != y0 && y >= top) {
        spec_hi = row_exit(spec);
        spec = ld_row_u(rr + y);
      }
    }
    flush_rows();
  };

  // ---- phase A: every strip from its guessed entry
  for (int32_t s = (int32_t)S - 1 - (int32_t)w; s >= 0; s -= (int32_t)kTW)
    walk((uint32_t)s, min(kStrip * ((uint32_t)s + 1), n1), guess((uint32_t)s), false);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's row stores have landed
  __syncthreads();

  // ---- phase B: in order from the last strip, each strip's real entry. The strips' top rows
  // are loaded 64 at a time up front; only a strip walked again reloads its own.
  if (w == 0) {
    uint32_t topv = 0;  // lane j: the top row of strip sb + j
    int32_t sb = -1;
    bool again = false;  // strip s + 1 was walked again
    for (int32_t s = (int32_t)S - 2; s >= 0; --s) {
      if (s + 1 < sb || sb < 0) {
        sb = max(s + 1 - 63, 1);
        const uint32_t sj = (uint32_t)sb + lane;
        topv = sj < S ? ld_row(rr + kStrip * sj + 1) : 0;
      }
      uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)topv, s + 1 - sb);
      if (again) v = ld_row_u(rr + kStrip * ((uint32_t)s + 1) + 1);
      const uint32_t xe = row_exit(v);
      again = xe != guess((uint32_t)s);
      if (again) {
        walk((uint32_t)s, kStrip * ((uint32_t)s + 1), xe, true);
        __builtin_amdgcn_s_waitcnt(0x0F70);
      }
    }
  }
  __syncthreads();

  // ---- phase C: thread i owns rows [i m, i m + m); row y's characters (1 + hi - lo, row 0: hi)
  // start at the number of characters of rows 0 .. y-1 (one block scan)
  uint32_t* wsum = reinterpret_cast<uint32_t*>(&lrec_all[0][0][0]);
  const uint64_t oo = ao + bo + pair;
  const uint32_t m = (n1 + 64 * kTW) / (64 * kTW);  // ceil((n1 + 1) / threads)
  const uint32_t y0 = threadIdx.x * m, y1 = min(y0 + m, n1 + 1);
  // row y: lo (0 for row 0) and hi (the exit of row y + 1; n2 for row n1)
  auto row_at = [&](uint32_t y, uint32_t& lo, uint32_t& hi, uint32_t& code) {
    const uint32_t v = y ? ld_row(rr + y) : 0u;
    lo = v & kX21;
    code = v >> 21;
    hi = y < n1 ? row_exit(ld_row(rr + y + 1)) : n2;
  };
  uint32_t cnt = 0;
#pragma unroll 4
  for (uint32_t y = y0; y < y1; ++y) {
    uint32_t lo, hi, code;
    row_at(y, lo, hi, code);
    cnt += y ? 1u + hi - lo : hi;
  }
  const uint32_t incl = wave_incl_sum(cnt);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t off = 0, carry = 0;
#pragma unroll
  for (uint32_t i = 0; i < kTW; ++i) {
    const uint32_t q = wsum[i];
    off += i < w ? q : 0u;
    carry += q;
  }
  uint64_t p = oo + off + incl - cnt;
  for (uint32_t y = y0; y < y1; ++y) {
    uint32_t lo, hi, code;
    row_at(y, lo, hi, code);
    if (y) {
      out1[p] = a[ao + y - 1];
      out2[p] = code == 1u ? b[bo + lo - 1] : (uint8_t)'-';
      ++p;
    }
    for (uint32_t xx = y ? lo + 1 : 1u; xx <= hi; ++xx, ++p) {
      out1[p] = (uint8_t)'-';
      out2[p] = b[bo + xx - 1];
    }
  }
  if (threadIdx.x == 0) {
    out1[oo + carry] = 0;
    out2[oo + carry] = 0;
    out_len[pair] = carry;
  }
}

}  // namespace

uint64_t nw_pair_ws_bytes(uint32_t max_len) { return Geo(max_len).per_pair(); }

hipError_t launch_nw(const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                     const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                     uint8_t* out2, uint64_t* out_len, uint8_t* ws, uint64_t ws_bytes,
                     uint32_t* err, hipStream_t s, Prof* prof) {
  if (!n) return hipSuccess;
  const uint64_t per = nw_pair_ws_bytes(max_len);
  const uint64_t chunk = ws_bytes / per;
  if (!chunk) return hipErrorInvalidValue;
  for (uint64_t first = 0; first < n; first += chunk) {
    const uint64_t cnt = n - first < chunk ? n - first : chunk;
    {
      ProfScope ps(prof, GDSM_PROF_NW_FILL, s);
      const bool lds_b = max_len <= kBLds;
      auto kern = lds_b ? nw_fill_kernel<true> : nw_fill_kernel<false>;
      hipLaunchKernelGGL(kern, dim3((uint32_t)cnt), dim3(64 * kWaves), lds_b ? max_len + 4 : 0,
                         s, a, a_off, b, b_off, first, max_len, ws, err);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    {
      ProfScope ps(prof, GDSM_PROF_NW_TRACE, s);
      hipLaunchKernelGGL(nw_trace_kernel, dim3((uint32_t)cnt), dim3(64 * kTW), 0, s, a, a_off, b,
                         b_off, first, max_len, ws, out1, out2, out_len);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace gdsm
