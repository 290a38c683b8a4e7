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
// Fill (nw_fill_kernel): one 16-wave workgroup per pair. Rows are cut into strips of 256; a strip
// belongs to one wave, 4 consecutive rows per lane. Lane l computes column x = t - l + 1 at step
// t, so the value from the row above (lane l-1's bottom row one step earlier) arrives by one DPP
// wave_shr:1 of a packed (score << 8 | b byte) word: no LDS traffic inside a strip. Strip s+1
// follows strip s two 64-step phases behind (one workgroup barrier per phase); the bottom row
// of a strip reaches the next wave through a 256-column LDS ring (or, from wave 15 to wave 0 of
// the next group of 16 strips, through a double-buffered row in global memory). No MFMA: the
// recurrence is max/add on int32, not a contraction.
//
// Traceback bits: per cell two bits, nd = "not diag" (dg < max(lf, up)) and u = "up beats left"
// (up > left, only read when nd). A lane accumulates them for its 4 rows over 16 steps into
// one 16-byte record; record (strip, block, lane) lives at ((strip * NB + block) * 64 + lane),
// so the 64 lanes of a wave store 1 KiB contiguously.
//
// Trace (nw_trace_kernel): one wave per pair walks the path with wave-uniform (scalar) state,
// reading directions out of a 64-record window held in VGPRs (v_readlane with a uniform lane),
// writes the moves, then turns them into the two alignment strings with wave prefix counts.
#include "gdsm_common.h"
#include "gdsm_launch.h"

namespace gdsm {
namespace {

constexpr uint32_t kRows = 4;             // DP rows per lane
constexpr uint32_t kWaves = 16;           // waves per fill workgroup
constexpr uint32_t kStrip = 64 * kRows;   // rows per strip
constexpr uint32_t kPhase = 64;           // steps per phase (between barriers)
constexpr uint32_t kLag = 2;              // phases between consecutive strips
constexpr uint32_t kRing = 256;           // ring slots per wave (>= 193 live columns)
constexpr uint32_t kBlk = 16;             // steps per traceback record

__device__ __forceinline__ uint32_t wave_shr1_or(uint32_t old, uint32_t v) {
  // Lane l gets lane l-1's v; lane 0 keeps `old` (bound_ctrl off).
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t pack(int32_t score, uint32_t byte) {
  return ((uint32_t)score << 8) | byte;
}

// Scores are kept minus one (H - 1): then lf and up of the recurrence are the stored values,
// dg = stored diag + 1 + (a == b) is one add-with-carry, mx = max3(dg, lf, up), and both
// traceback bits are sign bits shifted in by v_alignbit (nd = dg < mx, u = lf < up).
struct Strip {
  uint32_t a[kRows];
  int32_t left[kRows];  // H[y][x-1] - 1
  int32_t diag;         // H[ytop-1][x-1] - 1
  uint32_t pass;        // (H[ybottom][x] - 1) << 8 | b byte
};

__device__ __forceinline__ uint32_t shift_in_sign(uint32_t acc, int32_t v) {
  return __builtin_amdgcn_alignbit(acc, (uint32_t)v, 31);  // (acc << 1) | (v < 0)
}

// One block of 16 steps [t0, t0 + 16) of a strip. fv: lanes 0..15 hold the packed words lane 0
// consumes at steps t0..t0+15. Returns (in lanes 0..15) the packed bottom words of lane 63.
template <bool kMasked>
__device__ __forceinline__ uint32_t fill_block(Strip& st, uint32_t fv, uint32_t t0, uint32_t n2,
                                               uint32_t lane, uint4* rec) {
  uint32_t ndA = 0, ndB = 0, uA = 0, uB = 0, wv = 0;
#pragma unroll
  for (uint32_t k = 0; k < kBlk; ++k) {
    const uint32_t feed = (uint32_t)__builtin_amdgcn_readlane((int)fv, (int)k);
    const uint32_t in = wave_shr1_or(feed, st.pass);
    const int32_t up_in = (int32_t)in >> 8;
    const uint32_t bb = in & 0xFFu;
    bool act = true;
    if (kMasked) {
      const int32_t x = (int32_t)(t0 + k) - (int32_t)lane + 1;
      act = x >= 1 && x <= (int32_t)n2;
    }
    int32_t up = up_in, dgv = st.diag;
    uint32_t* acc_nd[2] = {&ndA, &ndB};
    uint32_t* acc_u[2] = {&uA, &uB};
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
      const int32_t lf = st.left[r];
      const int32_t d = dgv + 1 + (st.a[r] == bb ? 1 : 0);
      const int32_t mx = max(max(d, lf), up);
      *acc_nd[r >> 1] = shift_in_sign(*acc_nd[r >> 1], d - mx);
      *acc_u[r >> 1] = shift_in_sign(*acc_u[r >> 1], lf - up);
      dgv = lf;
      up = mx - 1;
      if (kMasked) st.left[r] = act ? up : lf;
      else st.left[r] = up;
    }
    if (kMasked) st.diag = act ? up_in : st.diag;
    else st.diag = up_in;
    st.pass = pack(up, bb);
    const uint32_t bot = (uint32_t)__builtin_amdgcn_readlane((int)st.pass, 63);
    wv = (lane == k) ? bot : wv;
  }
  *rec = make_uint4(ndA, ndB, uA, uB);
  return wv;
}

__global__ __launch_bounds__(1024) void nw_fill_kernel(
    const uint8_t* __restrict__ a, const uint64_t* __restrict__ a_off,
    const uint8_t* __restrict__ b, const uint64_t* __restrict__ b_off, uint64_t first_pair,
    uint32_t max_len, uint32_t NB, uint64_t slot_recs, uint4* __restrict__ tb,
    uint32_t* __restrict__ rowbuf, uint32_t* __restrict__ err) {
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
  const uint32_t S = (n1 + kStrip - 1) / kStrip;
  const uint32_t nblk = (n2 + 63 + kBlk - 1) / kBlk;           // step blocks per strip
  const uint32_t T = (nblk * kBlk + kPhase - 1) / kPhase;      // phases per strip
  // Group g of 16 strips starts at phase g * TT; strip 16g + w at g * TT + kLag * w. TT lets wave
  // 15 finish a strip before wave 0 of the next group reads its bottom row, and a wave's ring
  // outlive its previous reader.
  const uint32_t TT = T + kLag * (kWaves - 1);
  const uint32_t Q = ((S - 1) / kWaves) * TT + kLag * ((S - 1) % kWaves) + T;
  uint4* tbp = tb + blockIdx.x * slot_recs;
  uint32_t* rb = rowbuf + (uint64_t)blockIdx.x * 2 * (max_len + 64);
  const uint32_t* ring_in = ring[(w + kWaves - 1) % kWaves];
  uint32_t* ring_out = ring[w];

  Strip st;
  for (uint32_t q = 0; q < Q; ++q) {
    const int32_t rel = (int32_t)q - (int32_t)(kLag * w);
    if (rel >= 0) {
      const uint32_t g = (uint32_t)rel / TT, lp = (uint32_t)rel - g * TT;
      const uint32_t s = g * kWaves + w;
      if (s < S && lp < T) {
        if (lp == 0) {  // strip start: rows y0 .. y0+3 of this lane
          const uint32_t y0 = s * kStrip + lane * kRows + 1;
#pragma unroll
          for (uint32_t r = 0; r < kRows; ++r) {
            st.a[r] = (y0 + r <= n1) ? a[ao + y0 + r - 1] : 0u;
            st.left[r] = -(int32_t)(y0 + r) - 1;
          }
          st.diag = -(int32_t)(y0 - 1) - 1;
          st.pass = 0;
        }
        for (uint32_t bi = 0; bi < kPhase / kBlk; ++bi) {
          const uint32_t t0 = lp * kPhase + bi * kBlk;
          if (t0 >= nblk * kBlk) break;
          // Lane 0's feed for steps t0 + i: column x = t0 + 1 + i of the row above the strip.
          const uint32_t x = t0 + 1 + (lane & 15);
          uint32_t fv = 0;
          if (s == 0) {
            fv = (x <= n2) ? pack(-(int32_t)x - 1, b[bo + x - 1]) : 0u;
          } else if (w == 0) {
            const uint32_t* src = rb + ((g - 1) & 1) * (max_len + 64);
            fv = (x <= n2) ? __hip_atomic_load(src + x - 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0u;
          } else {
            fv = ring_in[(t0 + (lane & 15)) & (kRing - 1)];
          }
          uint4 rec;
          const bool masked = t0 < 64 || t0 + kBlk > n2;
          const uint32_t wv = masked ? fill_block<true>(st, fv, t0, n2, lane, &rec)
                                     : fill_block<false>(st, fv, t0, n2, lane, &rec);
          tbp[((uint64_t)s * NB + t0 / kBlk) * 64 + lane] = rec;
          // Lane 63's bottom words at steps t0..t0+15 are columns t0-62 .. t0-47.
          if (lane < 16) {
            ring_out[(t0 + lane - 63) & (kRing - 1)] = wv;
            const int32_t xo = (int32_t)(t0 + lane) - 62;
            if (w == kWaves - 1 && s + 1 < S && xo >= 1 && xo <= (int32_t)n2)
              rb[(g & 1) * (max_len + 64) + xo - 1] = wv;
          }
        }
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) void nw_trace_kernel(
    const uint8_t* __restrict__ a, const uint64_t* __restrict__ a_off,
    const uint8_t* __restrict__ b, const uint64_t* __restrict__ b_off, uint64_t first_pair,
    uint32_t max_len, uint32_t NB, uint64_t slot_recs, const uint4* __restrict__ tb,
    uint8_t* __restrict__ mv, uint8_t* __restrict__ out1, uint8_t* __restrict__ out2,
    uint64_t* __restrict__ out_len) {
  const uint64_t pair = first_pair + blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const uint64_t ao = a_off[pair], bo = b_off[pair];
  const uint64_t l1 = a_off[pair + 1] - ao, l2 = b_off[pair + 1] - bo;
  if (l1 > max_len || l2 > max_len) return;  // flagged by the fill kernel
  const uint32_t n1 = (uint32_t)l1, n2 = (uint32_t)l2;
  const uint4* tbp = tb + blockIdx.x * slot_recs;
  uint8_t* mvp = mv + (uint64_t)blockIdx.x * (2 * (uint64_t)max_len + 64);

  // ---- walk (n1, n2) -> (0, 0); codes 1 diag, 2 left, 3 up, in path order from the end
  uint32_t y = n1, x = n2, L = 0;
  int32_t ws = -1, wl0 = 0, wb0 = 0;
  uint4 rec = make_uint4(0, 0, 0, 0);
  uint32_t mvreg = 0;
  while (y | x) {
    uint32_t code;
    if (x == 0) {
      code = 3;
    } else if (y == 0) {
      code = 2;
    } else {
      const uint32_t yy = y - 1;
      const int32_t s = (int32_t)(yy / kStrip), l = (int32_t)((yy / kRows) & 63);
      const uint32_t r = yy & (kRows - 1);
      const uint32_t t = x - 1 + (uint32_t)l;
      const int32_t blk = (int32_t)(t / kBlk);
      const uint32_t k = t & (kBlk - 1);
      if (s != ws || l < wl0 || blk < wb0) {  // the path only moves to smaller l and blk
        ws = s;
        wl0 = l - 15;
        wb0 = blk - 3;
        const int32_t il = wl0 + (int32_t)(lane >> 2), ib = wb0 + (int32_t)(lane & 3);
        rec = (il >= 0 && ib >= 0) ? tbp[((uint64_t)s * NB + (uint32_t)ib) * 64 + (uint32_t)il]
                                   : make_uint4(0, 0, 0, 0);
      }
      const int idx = (l - wl0) * 4 + (blk - wb0);
      const uint32_t ndw = (uint32_t)__builtin_amdgcn_readlane((int)(r < 2 ? rec.x : rec.y), idx);
      const uint32_t uw = (uint32_t)__builtin_amdgcn_readlane((int)(r < 2 ? rec.z : rec.w), idx);
      const uint32_t bit = 31 - (2 * k + (r & 1));
      code = !((ndw >> bit) & 1u) ? 1u : !((uw >> bit) & 1u) ? 2u : 3u;
    }
    mvreg = (lane == (L & 63)) ? code : mvreg;
    if ((L & 63) == 63) mvp[L - 63 + lane] = (uint8_t)mvreg;
    ++L;
    y -= (code != 2);
    x -= (code != 3);
  }
  if ((L & 63) && lane < (L & 63)) mvp[(L & ~63u) + lane] = (uint8_t)mvreg;
  __syncthreads();

  // ---- alignment strings: move i (from the end) fills position L-1-i
  const uint64_t oo = ao + bo + pair;
  uint32_t cy = 0, cx = 0;
  for (uint32_t base = 0; base < L; base += 64) {
    const uint32_t i = base + lane;
    const uint32_t c = i < L ? mvp[i] : 0u;
    const uint32_t isy = (c == 1 || c == 3), isx = (c == 1 || c == 2);
    const uint32_t ey = wave_incl_sum(isy) - isy, ex = wave_incl_sum(isx) - isx;
    if (i < L) {
      const uint32_t yk = n1 - cy - ey, xk = n2 - cx - ex;
      out1[oo + L - 1 - i] = isy ? a[ao + yk - 1] : (uint8_t)'-';
      out2[oo + L - 1 - i] = isx ? b[bo + xk - 1] : (uint8_t)'-';
    }
    cy += wave_sum(isy);
    cx += wave_sum(isx);
  }
  if (lane == 0) {
    out1[oo + L] = 0;
    out2[oo + L] = 0;
    out_len[pair] = L;
  }
}

}  // namespace

uint64_t nw_slot_recs(uint32_t max_len) {
  const uint64_t S = (max_len + kStrip - 1) / kStrip;
  const uint64_t NB = (max_len + 63 + kBlk - 1) / kBlk;
  return (S ? S : 1) * NB * 64;
}

uint64_t nw_pair_ws_bytes(uint32_t max_len) {
  return nw_slot_recs(max_len) * 16 + 2 * ((uint64_t)max_len + 64) * 4 +
         (2 * (uint64_t)max_len + 64);
}

hipError_t launch_nw(const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                     const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                     uint8_t* out2, uint64_t* out_len, uint8_t* ws, uint64_t ws_bytes,
                     uint32_t* err, hipStream_t s, Prof* prof) {
  if (!n) return hipSuccess;
  const uint64_t per = nw_pair_ws_bytes(max_len);
  const uint64_t chunk = ws_bytes / per;
  if (!chunk) return hipErrorInvalidValue;
  const uint64_t recs = nw_slot_recs(max_len);
  const uint32_t NB = (uint32_t)((max_len + 63 + kBlk - 1) / kBlk);
  for (uint64_t first = 0; first < n; first += chunk) {
    const uint64_t cnt = n - first < chunk ? n - first : chunk;
    uint4* tb = reinterpret_cast<uint4*>(ws);
    uint32_t* rowbuf = reinterpret_cast<uint32_t*>(ws + cnt * recs * 16);
    uint8_t* mv = reinterpret_cast<uint8_t*>(rowbuf + cnt * 2 * ((uint64_t)max_len + 64));
    {
      ProfScope ps(prof, GDSM_PROF_NW_FILL, s);
      hipLaunchKernelGGL(nw_fill_kernel, dim3((uint32_t)cnt), dim3(64 * kWaves), 0, s, a, a_off,
                         b, b_off, first, max_len, NB, recs, tb, rowbuf, err);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    {
      ProfScope ps(prof, GDSM_PROF_NW_TRACE, s);
      hipLaunchKernelGGL(nw_trace_kernel, dim3((uint32_t)cnt), dim3(64), 0, s, a, a_off, b,
                         b_off, first, max_len, NB, recs, tb, mv, out1, out2, out_len);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace gdsm
