// gdsm page kernels for gfx950: synthetic pages, twin, run diff (SPEC §3), apply (SPEC §4).
//
// Replaces the twin/diff/apply step of gallocy's described-but-unimplemented DSM flow
// (resources/NUTSHELL.md:59-69); the only diff in the reference is the NW alignment
// gallocy/utils/diff.cpp:73-167, see legacy_diff.cpp.
//
// Diff (HBM-bound, no MFMA): diff_single_kernel, one pass. A wave diffs a unit of 16 or 32
// consecutive list entries (the next page's loads in flight): 4 x 16 B coalesced loads of twin and
// current per lane, 16-bit byte-diff mask per 16-B chunk, dirty chunks compacted by ballot into
// LDS, run starts/ends from the neighbour entry's edge bit, ranks by wave prefix sums; the record
// image is built in the wave's LDS buffer. Its offset in the stream comes from a decoupled
// look-back over the other waves' published totals, then the records are stored once, in place.
// No wave waits for a ticket that a wave not yet running holds.
#include "gdsm_common.h"
#include "gdsm_launch.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>

namespace gdsm {

// ------------------------------------------------------------------------- synthetic pages
__global__ __launch_bounds__(256) void gen_pages_kernel(uint8_t* __restrict__ twin,
                                                        uint8_t* __restrict__ cur,
                                                        uint8_t* __restrict__ replica,
                                                        uint64_t n_chunks16, uint64_t first_global,
                                                        uint64_t stride, uint64_t seed, int mode,
                                                        uint32_t ppm) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_chunks16;
       g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = g >> 8;           // arena page
    const uint64_t w0 = (g & 255) * 2;   // first word of this 16-B chunk
    const uint64_t p = first_global + i * stride;  // global page id
    uint64_t tv[2], cv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t w = w0 + h;
      const uint64_t v = hash3(seed ^ 0xDA7Aull, p, w);
      bool changed;
      if (mode == 0)
        changed = (hash3(seed ^ 0x5E1EC7EDull, p, w) % 1000000ull) < ppm;
      else
        changed = (hash3(seed ^ 0xC1057E12ull, p, w >> 3) % 1000000ull) < ppm;
      uint64_t x = 0;
      if (changed) {
        x = hash3(seed ^ 0x0F11E5ull, p, w);
        if (x == 0) x = 1;
      }
      tv[h] = v;
      cv[h] = v ^ x;
    }
    const uint4 T = make_uint4((uint32_t)tv[0], (uint32_t)(tv[0] >> 32), (uint32_t)tv[1],
                               (uint32_t)(tv[1] >> 32));
    const uint4 C = make_uint4((uint32_t)cv[0], (uint32_t)(cv[0] >> 32), (uint32_t)cv[1],
                               (uint32_t)(cv[1] >> 32));
    if (twin) reinterpret_cast<uint4*>(twin)[g] = T;
    if (cur) reinterpret_cast<uint4*>(cur)[g] = C;
    if (replica) reinterpret_cast<uint4*>(replica)[g] = T;
  }
}

// ------------------------------------------------------------------------- twin (SPEC §2)
// TWIN := CURRENT for listed pages: a wave per kP pages per step, every 16-B load of them in
// flight before the stores (kNT: bit 0 nontemporal loads, bit 1 nontemporal stores). A caller
// list is guarded in place (as check_ids_kernel below, without a launch of its own): an id >=
// n_pages twins the guard page n_pages instead and sets err bit 8.
template <uint32_t kP, int kNT>
__global__ __launch_bounds__(256) void twin_kernel(uint8_t* __restrict__ twin,
                                                   const uint8_t* __restrict__ cur,
                                                   const uint32_t* __restrict__ ids, uint64_t n,
                                                   uint64_t n_pages, uint32_t* __restrict__ err) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t steps = (n + kP - 1) / kP;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < steps;
       i += (uint64_t)gridDim.x * 4) {
    u32x4 v[kP][4];
    uint64_t pg[kP];
#pragma unroll
    for (uint32_t k = 0; k < kP; ++k) {
      const uint64_t e = i * kP + k;
      pg[k] = e < n ? (ids ? ids[e] : e) : ~0ull;
      if (pg[k] == ~0ull) continue;
      if (pg[k] >= n_pages) {  // (wave-uniform: one page per wave step)
        pg[k] = n_pages;
        if (err && lane == 0) atomicOr(err, 8u);
      }
      const u32x4* src = reinterpret_cast<const u32x4*>(cur + pg[k] * kPage);
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q)
        v[k][q] = (kNT & 1) ? __builtin_nontemporal_load(src + lane + 64 * q) : src[lane + 64 * q];
    }
#pragma unroll
    for (uint32_t k = 0; k < kP; ++k) {
      if (pg[k] == ~0ull) continue;
      u32x4* dst = reinterpret_cast<u32x4*>(twin + pg[k] * kPage);
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        if (kNT & 2)
          __builtin_nontemporal_store(v[k][q], dst + lane + 64 * q);
        else
          dst[lane + 64 * q] = v[k][q];
      }
    }
  }
}

// Re-twin after a release (gdsm_release, GDSM_RELEASE_RETWIN) on the multi-workgroup diff path:
// TWIN := CURRENT for list entry i's page when its record was stored (rec_off[i + 1] <= cap), so
// a release that overflowed its stream leaves the pages it could not ship dirty. A wave per page;
// ids are the launch's checked list (out-of-range entries already name the guard page).
__global__ __launch_bounds__(256) void retwin_kernel(uint8_t* __restrict__ twin,
                                                     const uint8_t* __restrict__ cur,
                                                     const uint32_t* __restrict__ ids, uint64_t n,
                                                     const uint64_t* __restrict__ rec_off,
                                                     uint64_t cap, uint64_t n_pages) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n;
       i += (uint64_t)gridDim.x * 4) {
    if (rec_off[i + 1] > cap) continue;  // wave-uniform
    const uint64_t pg = ids ? ids[i] : i;
    if (n_pages && pg >= n_pages) continue;  // the guard page (a bad entry): left alone
    const u32x4* src = reinterpret_cast<const u32x4*>(cur + pg * kPage);
    u32x4 v[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) v[q] = src[lane + 64 * q];
    u32x4* dst = reinterpret_cast<u32x4*>(twin + pg * kPage);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) dst[lane + 64 * q] = v[q];
  }
}

// ------------------------------------------------------------------------- page-id guard
// A context-level id list is copied with every out-of-range id replaced by n_pages, the guard
// page every arena carries past its last page, so a bad list can never address outside the
// arenas; the call then fails at the next gdsm_sync (err bit 8).
__global__ __launch_bounds__(256) void check_ids_kernel(const uint32_t* __restrict__ ids,
                                                        uint64_t n, uint64_t n_pages,
                                                        uint32_t* __restrict__ safe,
                                                        uint32_t* __restrict__ err) {
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t p = ids[i];
    const bool ok = p < n_pages;
    safe[i] = ok ? p : (uint32_t)n_pages;
    bad |= !ok;
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(err, 8u);
}

// Everything a diff launch needs zeroed or checked, as ONE launch before it (instead of a memset
// per workspace range and a check launch per caller list: a small release is a handful of
// microsecond operations, config 5's rounds): z64[0, n64) and z32[0, n32) := 0, and the caller
// lists guarded as check_ids_kernel does (g.ids -> g.safe_ids, g.tids -> g.safe_tids).
__global__ __launch_bounds__(256) void diff_prep_kernel(uint64_t* __restrict__ z64, uint64_t n64,
                                                        uint32_t* __restrict__ z32, uint64_t n32,
                                                        IdGuard g, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = t0; i < n64; i += st) z64[i] = 0;
  for (uint64_t i = t0; i < n32; i += st) z32[i] = 0;
  bool bad = false;
  for (uint64_t i = t0; i < n; i += st) {
    if (g.ids) {
      const uint32_t p = g.ids[i];
      bad |= p >= g.n_pages;
      g.safe_ids[i] = p < g.n_pages ? p : (uint32_t)g.n_pages;
    }
    if (g.tids) {
      const uint32_t p = g.tids[i];
      bad |= p >= g.n_pages;
      g.safe_tids[i] = p < g.n_pages ? p : (uint32_t)g.n_pages;
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(g.err, 8u);
}

// ------------------------------------------------------------------------- exchanged streams
// Every stream gdsm_exchange applies (received ones and the rank's own) is checked whole before
// the apply: rec_off[0] == 0, offsets non-decreasing and 4-aligned, rec_off[n] <= budget, and
// every page index < n_pages (copied to `safe`). Two launches, so no block ever judges a stream
// another block has already zeroed: the check ORs its verdict into one word (bit 0 malformed
// offsets, bit 1 over budget, bit 2 bad page index) and the err word (16 / 32 / 8); the zeroing
// pass then empties every record of a rejected stream, so the apply writes nothing of it.
__global__ __launch_bounds__(256) void xchg_check_kernel(const uint64_t* __restrict__ rec_off,
                                                         const uint32_t* __restrict__ ids,
                                                         uint64_t n, uint64_t budget,
                                                         uint64_t n_pages,
                                                         uint32_t* __restrict__ safe,
                                                         uint32_t* __restrict__ verdict,
                                                         uint32_t* __restrict__ err) {
  uint32_t v = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = rec_off[i];
    if (o & 3u) v |= 1u;
    if (i == 0 && o != 0) v |= 1u;
    if (i < n) {
      if (rec_off[i + 1] < o) v |= 1u;
      const uint32_t p = ids[i];
      const bool ok = p < n_pages;
      safe[i] = ok ? p : (uint32_t)n_pages;
      if (!ok) v |= 4u;
    } else if (o > budget) {
      v |= 2u;
    }
  }
  // one atomic per wave that found something
  const uint64_t any = __ballot(v != 0);
  if (any) {
    uint32_t w = v;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) w |= __shfl_xor(w, d, 64);
    if ((threadIdx.x & 63) == (uint32_t)__builtin_ctzll(any)) {
      atomicOr(verdict, w);
      atomicOr(err, ((w & 1u) ? 16u : 0u) | ((w & 2u) ? 32u : 0u) | ((w & 4u) ? 8u : 0u));
    }
  }
}

// The sender's view of a stream it shipped with a fixed budget: err |= 32 if it did not fit.
__global__ void budget_check_kernel(const uint64_t* __restrict__ rec_off, uint64_t n,
                                    uint64_t budget, uint32_t* __restrict__ err) {
  if (threadIdx.x == 0 && rec_off[n] > budget) atomicOr(err, 32u);
}

__global__ __launch_bounds__(256) void xchg_zero_kernel(uint64_t* __restrict__ rec_off, uint64_t n,
                                                        const uint32_t* __restrict__ verdict) {
  if (*verdict == 0) return;  // written by the previous launch: every block reads the same word
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n;
       i += (uint64_t)gridDim.x * blockDim.x)
    rec_off[i] = 0;
}

// ------------------------------------------------------------------------- diff (SPEC §3)
// Bit j of the result is set iff byte j of x is non-zero (j = 0..3).
__device__ __forceinline__ uint32_t nz4(uint32_t x) {
  const uint32_t y = ((((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u) >> 7;
  return ((y * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ uint32_t diffmask16(const uint4& a, const uint4& b) {
  return nz4(a.x ^ b.x) | (nz4(a.y ^ b.y) << 4) | (nz4(a.z ^ b.z) << 8) | (nz4(a.w ^ b.w) << 12);
}
// Byte b (0..15) of a 16-byte chunk, by 64-bit shifts (a select chain over the four words gets
// turned into an indexed private array, which the compiler then parks in LDS).
__device__ __forceinline__ uint32_t byte_of(const uint4& v, uint32_t b) {
  const uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  const uint64_t h = (b & 8u) ? hi : lo;
  return (uint32_t)(h >> ((b & 7u) * 8)) & 0xFFu;
}

// Writes the headers of the runs ENDING in chunk `ch` and the chunk's changed bytes. A run's
// start is the last run start at or before its end: inside this chunk, or `ps` - 1 where `ps` is
// the exclusive prefix maximum of (last start + 1) over the earlier chunks. (Called once per k
// with scalars, so no per-thread array is ever indexed at run time.)
template <bool kWT = false>
__device__ __forceinline__ void emit_chunk(uint32_t ch, uint32_t s, uint32_t e, uint32_t m,
                                           uint32_t ps, uint32_t excl, const uint4 c,
                                           uint32_t* __restrict__ hdr, uint8_t* __restrict__ pay) {
  const uint32_t pos = ch * 16u;
  uint32_t r = excl & 0xFFFFu;
  while (e) {
    const uint32_t b = (uint32_t)__builtin_ctz(e);
    e &= e - 1;
    const uint32_t upto = s & ((2u << b) - 1u);
    const uint32_t start = upto ? pos + 31u - (uint32_t)__builtin_clz(upto) : ps - 1u;
    st_<kWT>(hdr + r++, start | ((pos + b - start + 1u) << 16));
  }
  uint32_t q = excl >> 16;
  while (m) {
    const uint32_t b = (uint32_t)__builtin_ctz(m);
    m &= m - 1;
    st_<kWT>(pay + q++, (uint8_t)byte_of(c, b));
  }
}

__device__ __forceinline__ void load_page(const uint8_t* __restrict__ twin,
                                          const uint8_t* __restrict__ cur, uint64_t p,
                                          uint32_t lane, uint4 (&t)[4], uint4 (&c)[4]) {
  const uint4* T = reinterpret_cast<const uint4*>(twin + p * kPage);
  const uint4* C = reinterpret_cast<const uint4*>(cur + p * kPage);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t[k] = ld_nt16(T + k * 64 + lane);
    c[k] = ld_nt16(C + k * 64 + lane);
  }
}

// v_perm_b32 selectors compacting the bytes of a dword whose bit is set in a 4-bit mask to its
// low bytes, in order; selector 0x0C yields a zero byte.
__device__ __forceinline__ uint32_t compact_sel(uint32_t nib) {
  uint32_t sel = 0x0C0C0C0Cu, sh = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j)
    if ((nib >> j) & 1u) {
      sel = (sel & ~(0xFFu << sh)) | (j << sh);
      sh += 8;
    }
  return sel;
}

// ORs the bytes of v (little-endian) into the 3-word window w at byte offset o (o + 8 <= 24).
__device__ __forceinline__ void or_at(uint64_t v, uint32_t o, uint64_t& w0, uint64_t& w1,
                                      uint64_t& w2) {
  const uint32_t ob = (o & 7u) * 8u;
  const uint64_t lo = v << ob;
  const uint64_t hi = ob ? v >> (64u - ob) : 0ull;
  const bool up = o >= 8u;
  w0 |= up ? 0ull : lo;
  w1 |= up ? lo : hi;
  w2 |= up ? hi : 0ull;
}

// Emits the headers of the runs ending in one 16-B chunk and the chunk's changed bytes into the
// wave's LDS record image (payload region pre-zeroed): the changed bytes are compacted in
// registers (v_perm_b32 per dword), shifted to their byte position and OR-ed into <= 5 dwords,
// so the cost does not grow with the number of changed bytes.
__device__ __forceinline__ void emit_compact(uint32_t ch, uint32_t s, uint32_t e, uint32_t m,
                                             uint32_t ps, uint32_t excl, const uint4 c,
                                             uint32_t* __restrict__ img, uint32_t pay_base,
                                             const uint32_t* __restrict__ sel_tab) {
  const uint32_t pos = ch * 16u;
  uint32_t r = excl & 0xFFFFu;
  while (e) {
    const uint32_t b = (uint32_t)__builtin_ctz(e);
    e &= e - 1;
    const uint32_t upto = s & ((2u << b) - 1u);
    const uint32_t start = upto ? pos + 31u - (uint32_t)__builtin_clz(upto) : ps - 1u;
    img[1 + r++] = start | ((pos + b - start + 1u) << 16);
  }
  const uint32_t n0 = m & 0xFu, n1 = (m >> 4) & 0xFu, n2 = (m >> 8) & 0xFu, n3 = m >> 12;
  const uint32_t p0 = __builtin_amdgcn_perm(0u, c.x, sel_tab[n0]);
  const uint32_t p1 = __builtin_amdgcn_perm(0u, c.y, sel_tab[n1]);
  const uint32_t p2 = __builtin_amdgcn_perm(0u, c.z, sel_tab[n2]);
  const uint32_t p3 = __builtin_amdgcn_perm(0u, c.w, sel_tab[n3]);
  const uint32_t l0 = (uint32_t)__popc(n0), l1 = (uint32_t)__popc(n1);
  const uint32_t l2 = (uint32_t)__popc(n2), l3 = (uint32_t)__popc(n3);
  const uint64_t A = (uint64_t)p0 | ((uint64_t)p1 << (8u * l0));
  const uint64_t B = (uint64_t)p2 | ((uint64_t)p3 << (8u * l2));
  const uint32_t P = pay_base + (excl >> 16);  // byte address of the first payload byte
  const uint32_t sh = P & 3u, len = l0 + l1 + l2 + l3;
  uint64_t w0 = 0, w1 = 0, w2 = 0;
  or_at(A, sh, w0, w1, w2);
  or_at(B, sh + l0 + l1, w0, w1, w2);
  const uint32_t nw = (sh + len + 3u) >> 2;  // dwords touched (<= 5)
  uint32_t* d = img + (P >> 2);
  if (nw > 0) atomicOr(d + 0, (uint32_t)w0);
  if (nw > 1) atomicOr(d + 1, (uint32_t)(w0 >> 32));
  if (nw > 2) atomicOr(d + 2, (uint32_t)w1);
  if (nw > 3) atomicOr(d + 3, (uint32_t)(w1 >> 32));
  if (nw > 4) atomicOr(d + 4, (uint32_t)w2);
}

// Run structure of one page held in registers (chunk (k, lane) = bytes [(64k + lane) * 16, +16),
// page order = (k, lane)): per chunk the byte-diff mask m, run-start bits s, run-end bits e, the
// exclusive ranks excl (runs ending before the chunk in the low 16 bits, changed bytes before it
// in the high 16) and ps (1 + the last run start before the chunk); NR / NP = the page's runs /
// payload bytes (wave-uniform).
struct PageRuns {
  uint32_t m[4], s[4], e[4], excl[4], ps[4];
  uint32_t NR, NP;
};

__device__ __forceinline__ void scan_page(const uint4 (&t)[4], const uint4 (&c)[4], uint32_t lane,
                                          PageRuns& P) {
#pragma unroll
  for (int k = 0; k < 4; ++k) P.m[k] = diffmask16(t[k], c[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // neighbour chunks' edge bytes: lane-1 / lane+1 of the same k, wrapping across k
    uint32_t up = from_prev_lane(P.m[k]);
    uint32_t dn = from_next_lane(P.m[k]);
    if (k > 0 && lane == 0) up = lane_bcast(P.m[k > 0 ? k - 1 : 0], 63);
    if (k < 3 && lane == 63) dn = lane_bcast(P.m[k < 3 ? k + 1 : 3], 0);
    P.s[k] = P.m[k] & ~((P.m[k] << 1) | ((up >> 15) & 1u)) & 0xFFFFu;   // first byte of a run
    P.e[k] = P.m[k] & ~((P.m[k] >> 1) | ((dn & 1u) << 15)) & 0xFFFFu;   // last byte of a run
  }
  // Ranks: runs (counted at their ends) in the low 16 bits, payload bytes in the high 16.
  uint32_t carry = 0, cmax = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t v = (uint32_t)__popc(P.e[k]) | ((uint32_t)__popc(P.m[k]) << 16);
    const uint32_t inc = wave_incl_sum(v);
    P.excl[k] = carry + inc - v;
    carry += lane_bcast(inc, 63);
    const uint32_t pos = (uint32_t)(k * 64 + lane) * 16u;
    const uint32_t ls = P.s[k] ? pos + 32u - (uint32_t)__builtin_clz(P.s[k]) : 0u;  // last start + 1
    const uint32_t mx = wave_incl_max(ls);
    P.ps[k] = max(cmax, from_prev_lane(mx));
    cmax = max(cmax, lane_bcast(mx, 63));
  }
  P.NR = carry & 0xFFFFu;
  P.NP = carry >> 16;
}

__device__ __forceinline__ uint32_t record_size(const PageRuns& P) {
  return P.NR ? 4u + 4u * P.NR + ((P.NP + 3u) & ~3u) : 0u;
}

// Byte-loop emission of a whole record (headers and payload bytes one store each) to `rec`
// (LDS or global); lane 0 writes the run count and the zero padding.
__device__ __forceinline__ void emit_bytes(const PageRuns& P, const uint4 (&c)[4], uint32_t lane,
                                           uint8_t* __restrict__ rec) {
  uint32_t* hdr = reinterpret_cast<uint32_t*>(rec + 4);
  uint8_t* pay = rec + 4 + 4 * P.NR;
  if (lane == 0) {
    *reinterpret_cast<uint32_t*>(rec) = P.NR;
    for (uint32_t q = P.NP; q & 3u; ++q) pay[q] = 0;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    emit_chunk(k * 64 + lane, P.s[k], P.e[k], P.m[k], P.ps[k], P.excl[k], c[k], hdr, pay);
}

// Size of the record of a page whose byte-diff masks m[k] (chunk (k, lane)) are in registers
// (the run ends need the next chunk's first bit: DPP from lane + 1, wrapping across k).
__device__ __forceinline__ uint32_t record_size_masks(const uint32_t (&m)[4], uint32_t lane) {
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t dn = from_next_lane(m[k]);
    if (k < 3 && lane == 63) dn = lane_bcast(m[k < 3 ? k + 1 : 3], 0);
    const uint32_t e = m[k] & ~((m[k] >> 1) | ((dn & 1u) << 15)) & 0xFFFFu;
    v += (uint32_t)__popc(e) | ((uint32_t)__popc(m[k]) << 16);
  }
  const uint32_t tot = wave_sum(v);
  const uint32_t NR = tot & 0xFFFFu, NP = tot >> 16;
  return NR ? 4u + 4u * NR + ((NP + 3u) & ~3u) : 0u;
}

// The bytes of a 16-B chunk selected by `m` (bit j = byte j), stored from registers: one 16-B
// store for a whole chunk, 8-B stores for whole halves, dword stores for whole dwords, else bytes.
template <bool kWT = false>
__device__ __forceinline__ void store_masked16(uint8_t* __restrict__ dst, uint32_t m,
                                               const uint4& c) {
  if (m == 0xFFFFu) {
    if (kWT)
      st_wt16(dst, c);
    else
      *reinterpret_cast<uint4*>(dst) = c;
    return;
  }
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t lo = h ? c.z : c.x, hi = h ? c.w : c.y;
    if (((m >> (8 * h)) & 0xFFu) == 0xFFu) {
      if (kWT)
        st_wt(reinterpret_cast<uint64_t*>(dst + 8 * h), (uint64_t)lo | ((uint64_t)hi << 32));
      else
        *reinterpret_cast<u32x2*>(dst + 8 * h) = (u32x2){lo, hi};
      continue;
    }
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const uint32_t wv = d ? hi : lo, nib = (m >> (8 * h + 4 * d)) & 0xFu;
      uint8_t* q = dst + 8 * h + 4 * d;
      if (nib == 0xFu) {
        st_<kWT>(reinterpret_cast<uint32_t*>(q), wv);
      } else if (nib) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((nib >> k) & 1u) st_<kWT>(q + k, (uint8_t)(wv >> (8 * k)));
      }
    }
  }
}

// ---- single-pass diff (default): every record is written straight to its final place in the
// packed stream, so the stream crosses HBM once (no workspace slots, no scan, no pack).
// A WAVE is the unit of work: it draws a ticket (atomic counter; tickets are drawn in dispatch
// order, so every lower ticket belongs to a wave that is already running) and diffs the kSpU
// consecutive list entries of unit `ticket` exactly like the compacted kernel above (next page's
// loads in flight, ballot/mbcnt compaction, DPP scans, record image built in LDS). Records that
// fit the wave's LDS buffer stay there; a page with > 64 dirty 16-B chunks, or one that no longer
// fits, is only sized ("late"). The wave then publishes its byte total as an 8-B {flag, value}
// granule (agent-scope relaxed atomic store, i.e. one sc1 store: MI355X_MICROARCH.md
// "granule") and finds its exclusive offset by decoupled look-back over the 64 nearest
// predecessors' granules (agent-scope relaxed loads, s_sleep while one is unpublished). It
// publishes its inclusive prefix, writes rec_off for its pages, copies its buffered records
// from LDS to the stream with coalesced dword stores (nontemporal), and re-reads its late pages
// from the arenas to emit them byte-wise in place. No wave ever waits for a ticket that a
// non-running wave holds, so the look-back cannot deadlock whatever the dispatch order.
constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62, kStVal = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// kApply: the same runs are also applied to `target` (a home copy on this GPU, pages indexed by
// the same ids): each dirty chunk's changed bytes, exactly the bytes its runs cover (SPEC §4),
// are stored from the registers that found them, so the stream is not read back.
// kSpill (bytes, 0 = none): when a record no longer fits the wave's LDS buffer, the buffer's
// records are flushed to the wave's slot of a global spill pool and the buffer starts over, so a
// unit holds kBuf + kSpill bytes of records before any page has to be re-read ("late"). The pool
// has kSpillWGs workgroup slots (4 wave slots each); workgroup ticket t uses slot t % kSpillWGs
// once the workgroup with ticket t - kSpillWGs has released it (a generation word per slot;
// that workgroup drew its ticket earlier, so it is running or done and never waits for t).
constexpr uint32_t kSpillWGs = 1280;  // > the workgroups of this kernel one MI355X holds at once

// kSolo (a release of at most kSoloUnits one-page units, one stream): ONE workgroup, a wave per
// unit, no ticket and no workspace. The exclusive offsets come from the waves' totals through LDS
// and one barrier instead of the look-back, and the caller's id lists are guarded in the kernel
// (g, as diff_prep_kernel does), so the release is this one launch (config 5's rounds).
constexpr uint32_t kSoloUnits = 16;

// A re-twin store may go to page pj: not the guard page, where every out-of-range entry of a
// checked list points (those workgroups would write the guard page's TWIN while others read it,
// and the records emitted for the bad entries would depend on the race). g.n_pages == 0: the
// launch has no checked list, so no entry names the guard page.
__device__ __forceinline__ bool twin_ok(const IdGuard& g, uint64_t pj) {
  return g.n_pages == 0 || pj < g.n_pages;
}

__device__ __forceinline__ uint64_t guarded_value(uint32_t p, uint64_t n_pages, uint32_t& bad) {
  bad |= p >= n_pages ? 1u : 0u;
  return p < n_pages ? p : n_pages;
}

__device__ __forceinline__ uint64_t guarded_id(const uint32_t* __restrict__ ids, uint64_t i,
                                               uint64_t n_pages, uint32_t& bad) {
  const uint32_t p = ids[i];
  bad |= p >= n_pages ? 1u : 0u;
  return p < n_pages ? p : n_pages;
}

// kChain (a context's lists of at most kDiffTiny pages outside graph capture; DiffChain): the
// grid form without a zeroing launch. ws = two ticket counters, then one granule per unit tagged
// with the launch's epoch sp.epoch: launch E draws its tickets from counter E & 1 and zeroes
// counter (E + 1) & 1 for the next launch, and the look-back counts a granule only when it carries
// E (granule = flag << 62 | E << 32 | value). The caller's lists are guarded in the kernel (g).
template <uint32_t kU, uint32_t kBuf, int kWaves, bool kApply, uint32_t kSpill = 0,
          bool kSolo = false, bool kRetwin = false, uint32_t kChainW = 0, uint32_t kSkip = 0>
__global__ __launch_bounds__(kSolo ? 64 * kSoloUnits : kChainW ? 64 * kChainW : 256) __attribute__((amdgpu_waves_per_eu(kWaves))) void diff_single_kernel(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, const DiffSplit sp, uint64_t* __restrict__ ws,
    uint8_t* __restrict__ target, uint32_t* __restrict__ gen, uint8_t* __restrict__ pool,
    const uint32_t* __restrict__ tids, const IdGuard g) {
  static_assert(kU <= 64 && (kU & (kU - 1)) == 0, "unit size");
  static_assert(!kRetwin || kU == 1, "re-twin: one-page units");
  // kRetwin (gdsm_release): TWIN is also written, through a pointer derived from `twin` itself,
  // so the compiler never treats this kernel's twin loads as invariant
  uint8_t* const twin_w = const_cast<uint8_t*>(twin);
  static_assert(!kSolo || (kU == 1 && kSpill == 0), "solo: one-page units, no spill slot");
  constexpr bool kChain = kChainW != 0;  // kChainW: waves per workgroup of the chained form
  // kSkip (MEASUREMENT ONLY, -DGDSM_MEASURE builds, output invalid): 1 = no home-apply stores,
  // 2 = no late-record stores (still scanned), 4 = no re-twin stores, 8 = no late path at all,
  // 16 = no look-back (every unit at offset 0), 32 = no copy of buffered records
  static_assert(!kChain || (kU == 1 && kSpill == 0 && !kSolo), "chain: one-page grid units");
  constexpr bool kGuard = kSolo || kChain;  // the caller's id lists are guarded in this kernel
  const uint64_t tag = kChain ? (uint64_t)sp.epoch << 32 : 0ull;  // granule epoch (kChain)
  constexpr uint64_t kVal = kChain ? 0xFFFFFFFFull : kStVal;
  constexpr uint32_t kNW = kSolo ? kSoloUnits : kChain ? kChainW : 4;  // waves per workgroup
  __shared__ uint32_t sel_tab[16];
  __shared__ uint32_t ent_all[kNW][64];
  __shared__ uint4 dat_all[kNW][64];
  __shared__ __attribute__((aligned(16))) uint32_t buf_all[kNW][kBuf / 4];
  __shared__ uint32_t tab_all[kNW][2 * kU + 1];  // [0, kU]: record offsets; [kU+1, 2kU]: LDS source
  if (threadIdx.x < 16) sel_tab[threadIdx.x] = compact_sel(threadIdx.x);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* ent = ent_all[wave];
  uint4* dat = dat_all[wave];
  uint32_t* buf = buf_all[wave];
  uint32_t* tab = tab_all[wave];
  const uint64_t nunits = sp.ustart[sp.G];
  // one ticket per workgroup (a single counter takes ~88 returning atomics per us, so per-wave
  // tickets would queue on it); unit = 4 * ticket + wave
  __shared__ uint32_t ticket, done_waves;
  if (!kSolo && threadIdx.x == 0) {
    uint32_t* const ctr = reinterpret_cast<uint32_t*>(ws);
    const uint32_t t = atomicAdd(ctr + (kChain ? sp.epoch & 1u : 0u), 1u);
    if (kChain && blockIdx.x == 0)  // the next launch's counter (this launch never draws from it)
      __hip_atomic_store(ctr + ((sp.epoch + 1u) & 1u), 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    ticket = t;
    done_waves = 0;
    if (kSpill && (uint64_t)t * 4 < nunits) {  // wait for the spill slot's previous user
      const uint32_t want = t / kSpillWGs;
      while (__hip_atomic_load(gen + t % kSpillWGs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
             want)
        __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  const uint64_t u = kSolo ? (uint64_t)wave : (uint64_t)ticket * kNW + wave;
  if (u >= nunits) return;  // wave-uniform: the grid's spare waves (none in a solo launch)
  uint32_t bad_id = 0;      // kGuard: a caller id out of range
  // the output stream this unit belongs to (units never straddle two of them) and its place in it
  uint32_t d = 0;
#pragma unroll
  for (uint32_t t = 1; t < kMaxSplit; ++t)
    if (t < sp.G && sp.ustart[t] <= u) d = t;
  const uint64_t u0 = sp.ustart[d];            // the stream's first unit
  uint64_t* __restrict__ rec_off = sp.rec_off[d];
  uint8_t* __restrict__ data = sp.data[d];
  const uint64_t cap = sp.cap[d];
  uint32_t* slot = kSpill ? reinterpret_cast<uint32_t*>(
                                pool + ((uint64_t)(ticket % kSpillWGs) * 4 + wave) * kSpill)
                          : nullptr;
  uint32_t spilled = 0;  // bytes of this wave's records flushed to its slot
  uint64_t* status = ws + 1;
  const uint64_t l0 = (u - u0) * kU;              // first record of the unit in its stream
  const uint64_t i0 = sp.first[d] + l0;           // ... and its list entry
  const uint32_t cnt = (uint32_t)min((uint64_t)kU, sp.first[d + 1] - i0);

  uint32_t acc = 0;       // LDS bytes used by buffered records
  uint64_t late = 0;      // bit j: page j is emitted from the arenas after the look-back
  uint32_t my_size = 0;   // lane j: record size of page j
  uint32_t my_src = 0;    // lane j: LDS byte offset of page j's record
  uint4 t[4], c[4];
  // Re-twin (gdsm_release), one-page units only (a late page is emitted from the registers, so
  // the twin page is never read again by this wave): with room in the stream for every record of
  // the launch, the twin's dirty chunks are stored with the first pass's other stores; otherwise
  // (kSolo) at the end, for a page whose record was stored. (The grid takes kRetwin only when the
  // stream has that room.)
  const bool retwin_now = kRetwin && cap >= (sp.first[1] - sp.first[0]) * GDSM_MAX_RECORD;
  uint64_t pj = ids ? (kGuard && g.ids ? guarded_id(ids, i0, g.n_pages, bad_id) : ids[i0]) : i0;
  load_page(twin, cur, pj, lane, t, c);
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint64_t pt_ =
        kApply ? (tids ? (kGuard && g.tids ? guarded_id(tids, i0 + j, g.n_pages, bad_id)
                                          : (uint64_t)tids[i0 + j])
                       : pj)
               : 0;  // page at target
    uint32_t m[4], D = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m[k] = diffmask16(t[k], c[k]);
      const uint64_t B = __ballot(m[k] != 0u);
      const uint32_t rank = D + __builtin_amdgcn_mbcnt_hi(
                                    (uint32_t)(B >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
      if (m[k] && rank < 64u) {
        ent[rank] = ((uint32_t)(k * 64 + lane) << 16) | m[k];
        dat[rank] = c[k];
      }
      D += (uint32_t)__popcll(B);
      if (kApply && !(kSkip & 1) && m[k]) store_masked16(target + pt_ * kPage + (k * 64 + lane) * 16u, m[k], c[k]);
      // (whole chunks: a chunk's clean bytes are equal in TWIN and CURRENT, and TWIN is this
      // writer's own, so no byte stores)
      if (!(kSkip & 4) && retwin_now && m[k] && twin_ok(g, pj))
        *reinterpret_cast<uint4*>(twin_w + pj * kPage + (k * 64 + lane) * 16u) = c[k];
    }
    if (j + 1 < cnt) {
      pj = ids ? ids[i0 + j + 1] : i0 + j + 1;
      load_page(twin, cur, pj, lane, t, c);
    }
    uint32_t size = 0;
    uint32_t src = spilled + acc;  // logical offset: [0, spilled) in the slot, then LDS
    if (D > 64u) {
      size = record_size_masks(m, lane);
      late |= 1ull << j;
    } else if (D) {
      wave_lds_sync();
      const bool valid = lane < D;
      const uint32_t E = valid ? ent[lane] : 0u;
      const uint32_t Ep = from_prev_lane(E), En = from_next_lane(E);
      const uint32_t g = E >> 16, mm = E & 0xFFFFu;
      const uint32_t up = (Ep != 0u && (Ep >> 16) + 1u == g) ? (Ep >> 15) & 1u : 0u;
      const uint32_t dn = (En != 0u && (En >> 16) == g + 1u) ? En & 1u : 0u;
      const uint32_t s = mm & ~((mm << 1) | up) & 0xFFFFu;
      const uint32_t e = mm & ~((mm >> 1) | (dn << 15)) & 0xFFFFu;
      const uint32_t v = (uint32_t)__popc(e) | ((uint32_t)__popc(mm) << 16);
      const uint32_t inc = wave_incl_sum(v);
      const uint32_t tot = lane_bcast(inc, 63);
      const uint32_t ls = s ? g * 16u + 32u - (uint32_t)__builtin_clz(s) : 0u;
      const uint32_t ps = from_prev_lane(wave_incl_max(ls));
      const uint32_t NR = tot & 0xFFFFu, NP = tot >> 16;
      size = 4u + 4u * NR + ((NP + 3u) & ~3u);
      if (kSpill && acc + size > kBuf && spilled + acc <= kSpill) {
        // the buffer is full: its records go to the slot (coalesced dword stores), then it starts
        // over (every record with <= 64 dirty chunks fits an empty 8 KiB buffer)
        for (uint32_t q = lane; q < acc / 4u; q += 64) slot[spilled / 4u + q] = buf[q];
        wave_lds_sync();
        spilled += acc;
        acc = 0;
        src = spilled;
      }
      if (acc + size > kBuf) {
        late |= 1ull << j;
      } else {
        uint32_t* img = buf + acc / 4u;
        for (uint32_t q = lane; q < size / 4u; q += 64) img[q] = 0u;
        const uint4 cc = valid ? dat[lane] : make_uint4(0, 0, 0, 0);
        wave_lds_sync();
        if (lane == 0) img[0] = NR;
        if (valid) emit_compact(g, s, e, mm, ps, inc - v, cc, img, 4u + 4u * NR, sel_tab);
        wave_lds_sync();
        acc += size;
      }
    }
    if (lane == j) {
      my_size = size;
      my_src = src;
    }
  }

  // ---- publish the aggregate, look back for the exclusive offset, publish the inclusive prefix
  const uint32_t incl = wave_incl_sum(my_size);  // lanes >= cnt hold 0
  const uint32_t agg = lane_bcast(incl, 63);
  uint64_t excl = 0;
  if (kSolo) {  // the waves' totals through LDS (every wave of the launch gets here)
    __shared__ uint32_t solo_agg[kSoloUnits];
    if (lane == 0) solo_agg[wave] = agg;
    __syncthreads();
    for (uint32_t w = 0; w < wave; ++w) excl += solo_agg[w];
    if (g.err && __ballot(bad_id != 0) && lane == 0) atomicOr(g.err, 8u);
  }
  if (kChain && g.err && __ballot(bad_id != 0) && lane == 0) atomicOr(g.err, 8u);
  if (!kSolo && lane == 0)
    __hip_atomic_store(status + u, (u == u0 ? kStIncl : kStAgg) | tag | agg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (!kSolo && !(kSkip & 16) && u > u0) {
    int64_t pos = (int64_t)u - 1;
    for (;;) {
      const int64_t q = pos - (int64_t)lane;
      uint64_t st = q >= (int64_t)u0
                        ? __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : kStIncl | tag;  // before the stream's first unit: a prefix of 0
      // unpublished: no flag yet (kChain: or a granule of an earlier launch)
      auto unpub = [&](uint64_t w) {
        return (w >> 62) == 0 || (kChain && ((w >> 32) & 0x3FFFFFFFull) != sp.epoch);
      };
      while (__ballot(unpub(st))) {  // a predecessor has not published yet
        __builtin_amdgcn_s_sleep(1);
        if (unpub(st))
          st = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint64_t im = __ballot((st >> 62) == 2);
      if (im) {
        const uint32_t k = (uint32_t)__builtin_ctzll(im);
        excl += wave_sum_u64(lane <= k ? (st & kVal) : 0ull);
        break;
      }
      excl += wave_sum_u64(st & kVal);
      pos -= 64;
    }
    if (lane == 0)
      __hip_atomic_store(status + u, kStIncl | tag | (excl + agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- rec_off, then the records: buffered ones from LDS, late ones from the arenas
  if (lane < cnt) rec_off[l0 + lane + 1] = excl + incl;
  if (u == u0 && lane == 0) rec_off[0] = 0;
  if (lane < kU) {
    tab[lane] = lane < cnt ? incl - my_size : agg;
    tab[kU + 1 + lane] = ((late >> lane) & 1ull) ? 0xFFFFFFFFu : my_src;
  }
  if (lane == 0) tab[kU] = agg;
  // only records that end inside the capacity are stored (SPEC §3)
  uint32_t limit = agg;
  if (excl + agg > cap) {
    const bool fits = lane < cnt && excl + incl <= cap;
    limit = lane_bcast(wave_incl_max(fits ? incl : 0u), 63);
  }
  wave_lds_sync();
  // The buffered records between two late pages are contiguous both in the wave's logical stream
  // (slot, then LDS) and in the output: each such run of records is one dword copy, no per-dword
  // record search.
  uint32_t* dst = reinterpret_cast<uint32_t*>(data + excl);
  // (the slot is read at agent scope: past this CU's L1, which may hold lines of the slot's
  // previous user)
  if (kSpill && spilled) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the flushes landed
  const uint64_t all = cnt >= 64 ? ~0ull : ((1ull << cnt) - 1ull);
  for (uint64_t rest = (kSkip & 32) ? 0ull : all & ~late; rest;) {  // wave-uniform
    const uint32_t j0 = (uint32_t)__builtin_ctzll(rest);
    const uint64_t above = j0 < 63 ? late & ~((2ull << j0) - 1ull) : 0ull;
    const uint32_t j1 = above ? (uint32_t)__builtin_ctzll(above) : cnt;  // first late page after
    rest = j1 >= 64 ? 0ull : rest & ~((1ull << j1) - 1ull);
    const uint32_t o0 = tab[j0], o1 = min(tab[j1], limit);
    if (o1 <= o0) continue;
    const uint32_t s0 = tab[kU + 1 + j0] / 4u, d0 = o0 / 4u, nd = (o1 - o0) / 4u;
    if (!kSpill || spilled == 0) {
      for (uint32_t g = lane; g < nd; g += 64) __builtin_nontemporal_store(buf[s0 + g], dst + d0 + g);
    } else {
      const uint32_t sp = spilled / 4u;
      for (uint32_t g0 = 0; g0 < nd; g0 += 256) {  // four dwords per lane in flight
        uint32_t v[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          const uint32_t g = g0 + 64 * q + lane, lg = s0 + g;
          v[q] = 0;
          if (g < nd)
            v[q] = lg < sp ? __hip_atomic_load(slot + lg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : buf[lg - sp];
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
          if (g0 + 64 * q + lane < nd) __builtin_nontemporal_store(v[q], dst + d0 + g0 + 64 * q + lane);
      }
    }
  }
  // (short units, kU <= 2: the registers still hold the unit's last page, so a late last page
  // that no earlier late page displaced is emitted without reading it again — two dependent
  // round trips less for a dense page of a small release)
  constexpr bool kKeep = kU <= 2;
  for (uint64_t rem = (kSkip & 8) ? 0ull : late; rem;) {  // wave-uniform
    const uint32_t j = (uint32_t)__builtin_ctzll(rem);
    const bool first_late = rem == late;
    rem &= rem - 1;
    if (excl + tab[j + 1] > cap) continue;
    const uint64_t i = i0 + j;
    if (!(kKeep && first_late && j + 1 == cnt)) {
      uint32_t unused = 0;
      load_page(twin, cur,
                ids ? (kGuard && g.ids ? guarded_id(ids, i, g.n_pages, unused) : ids[i]) : i, lane,
                t, c);
    }
    PageRuns P;
    scan_page(t, c, lane, P);
    if (kSkip & 2) {
      if (P.NR == 12345u) data[lane] = 0;  // keep the scan
    } else {
      emit_bytes(P, c, lane, data + excl + tab[j]);
    }
  }
  if (kGuard && kRetwin && !(kSkip & 4) && !retwin_now && excl + tab[1] <= cap && twin_ok(g, pj)) {
    // gdsm_release's re-twin (TWIN := CURRENT, the dirty bytes only), once the record is out: the
    // registers still hold the unit's one page (kKeep: a late page was emitted from them)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (diffmask16(t[k], c[k])) *reinterpret_cast<uint4*>(twin_w + pj * kPage + (k * 64 + lane) * 16u) = c[k];
    }
  }
  if (kSpill) {
    // the last active wave of the workgroup hands the slot to ticket + kSpillWGs once every wave's
    // slot reads have returned
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    uint32_t prev = 0;
    if (lane == 0) prev = atomicAdd(&done_waves, 1u);
    prev = lane_bcast(prev, 0);
    const uint32_t active = (uint32_t)min((uint64_t)4, nunits - (uint64_t)ticket * 4);
    if (prev + 1 == active && lane == 0)
      __hip_atomic_store(gen + ticket % kSpillWGs, ticket / kSpillWGs + 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- chained release, a page per workgroup (DiffChain lists of up to kChainPerPage pages).
// A few dense pages are latency: one wave per page issues its page's ~80 home-apply and ~36
// record store instructions one after another, four cycles per wave64 VALU step. Here the four
// waves of a workgroup take a quarter of the page each (wave w: chunks 64w .. 64w + 63, one
// 16-B chunk per lane), so the stores and the run scan of a page are spread over the CU's four
// SIMDs. The quarters meet through LDS: the edge chunks' masks (a run may cross a quarter),
// each quarter's run / payload counts and last run start (the record's prefix), and the
// record's offset in the stream, which wave 0 finds by the decoupled look-back over the chained
// epoch-tagged granules (as diff_single_kernel<..., kChainW> does; ticket per workgroup, the
// next launch's counter zeroed). Records are written straight from the registers (run headers
// and payload bytes, emit_chunk), the home copy's changed bytes with store_masked16, the twin's
// dirty chunks whole (kRetwin). Same stream, apply and re-twin as every other diff form.
// One page (list entry u of n) by the calling four-wave workgroup; the kernel below draws u as a
// ticket, rounds_data_kernel assigns it (every workgroup resident, pages in ascending order per
// workgroup, so the look-back only ever waits for running workgroups).
// A round's writes for release_page_wg<..., kFuse>: copy descriptors [d0, d1) of desc, each
// (dst, src, bytes) 8-B aligned; `covered` counts the 8-B words laid onto released pages.
// (Holding a round's first 8 descriptors in registers, loaded a round ahead, measured ~0.6 us
// per round SLOWER in the release than these scalar-cached loads: profiles/r06_rounds_ab.txt.)
struct RoundWrites {
  const uint64_t* desc;
  uint64_t d0, d1;
  unsigned long long* covered;
};

// Lays descriptor (dst, src, bytes) onto the 16-B CURRENT chunk at address a: the 8-B halves
// it covers (bit h of wm) take their bytes from src.
__device__ __forceinline__ void lay_desc(uint64_t a, uint64_t dst, uint64_t src, uint64_t bytes,
                                         uint64_t (&hv)[2], uint32_t& wm) {
  if (a + 16 <= dst || a >= dst + bytes) return;
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    const uint64_t ha = a + 8 * h;
    if (ha >= dst && ha + 8 <= dst + bytes) {
      hv[h] = *reinterpret_cast<const uint64_t*>(src + (ha - dst));
      wm |= 1u << h;
    }
  }
}

// kWT: every store write-through and the page loads past L1 (st_wt / ld_wt16): the persistent
// rounds grid hands CURRENT, TWIN, REPLICA and the stream from one workgroup to another with no
// fences. kFuse: the round's writes (rw) that fall on this page are laid onto its CURRENT chunk
// in registers and stored to CURRENT here, so the release needs no copy step and no barrier
// before it (a word outside every released page is never written: `covered` falls short and the
// launch flags it). kL2 (with kWT: a one-XCD team, xcd_team): the stores stay plain (kept in the
// team's L2, where the sc1 loads of the other members find them).
template <bool kApply, bool kRetwin, bool kWT = false, bool kFuse = false, bool kL2 = false>
__device__ __forceinline__ void release_page_wg(
    const uint64_t u, const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, const DiffSplit& sp, uint64_t* __restrict__ ws,
    uint8_t* __restrict__ target, const uint32_t* __restrict__ tids, const IdGuard& g,
    const RoundWrites& rw = RoundWrites{}, const int64_t pre_id = -1) {
  uint8_t* const twin_w = const_cast<uint8_t*>(twin);  // (kRetwin: see diff_single_kernel)
  constexpr bool kWTs = kWT && !kL2;                  // write-through stores
  __shared__ uint32_t edge_first[4], edge_last[4], tot[4], lastst[4];
  __shared__ uint64_t rec_at;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t E = sp.epoch;
  const uint64_t tag = (uint64_t)E << 32;
  const uint64_t n = sp.first[1] - sp.first[0];
  uint32_t bad = 0;
  const uint64_t i = sp.first[0] + u;
  // (pre_id >= 0: the list entry, loaded ahead by the caller)
  const uint64_t pj =
      pre_id >= 0 ? (g.ids ? guarded_value((uint32_t)pre_id, g.n_pages, bad) : (uint64_t)pre_id)
      : ids       ? (g.ids ? guarded_id(ids, i, g.n_pages, bad) : ids[i])
                  : i;
  const uint64_t cap = sp.cap[0];
  const bool ample = kRetwin && cap >= n * GDSM_MAX_RECORD;
  const uint32_t ch = w * 64 + lane;  // this lane's chunk of the page
  const uint4 t = kWT ? ld_wt16(twin + pj * kPage + ch * 16u) : ld_nt16(twin + pj * kPage + ch * 16u);
  uint4 c = kWT ? ld_wt16(cur + pj * kPage + ch * 16u) : ld_nt16(cur + pj * kPage + ch * 16u);
  if (kFuse) {
    const uint64_t a = reinterpret_cast<uint64_t>(cur + pj * kPage + ch * 16u);
    uint32_t wm = 0;  // bit h: 8-B half h of the chunk written this round
    uint64_t hv[2] = {(uint64_t)c.x | ((uint64_t)c.y << 32), (uint64_t)c.z | ((uint64_t)c.w << 32)};
    for (uint64_t d = rw.d0; d < rw.d1; ++d)
      lay_desc(a, rw.desc[3 * d], rw.desc[3 * d + 1], rw.desc[3 * d + 2], hv, wm);
    if (wm) {
      c = make_uint4((uint32_t)hv[0], (uint32_t)(hv[0] >> 32), (uint32_t)hv[1],
                     (uint32_t)(hv[1] >> 32));
      uint8_t* const cw = const_cast<uint8_t*>(cur) + pj * kPage + ch * 16u;
#pragma unroll
      for (uint32_t h = 0; h < 2; ++h)
        if ((wm >> h) & 1u) st_<kWTs>(reinterpret_cast<uint64_t*>(cw + 8 * h), hv[h]);
    }
    const uint32_t words = wave_sum((uint32_t)__popc(wm));
    if (words && lane == 0) atomicAdd(rw.covered, (unsigned long long)words);
  }
  const uint32_t m = diffmask16(t, c);
  const uint64_t pt = kApply ? (tids ? (g.tids ? guarded_id(tids, i, g.n_pages, bad) : tids[i]) : pj)
                             : 0;  // page at target
  if (kApply && m) store_masked16<kWTs>(target + pt * kPage + ch * 16u, m, c);
  if (ample && m && twin_ok(g, pj)) {
    if (kWTs)
      st_wt16(twin_w + pj * kPage + ch * 16u, c);
    else
      *reinterpret_cast<uint4*>(twin_w + pj * kPage + ch * 16u) = c;
  }
  if (lane == 0) edge_first[w] = m;
  if (lane == 63) edge_last[w] = m;
  __syncthreads();
  // run starts / ends with the neighbour chunks' edge bytes (across quarters through LDS)
  uint32_t up = from_prev_lane(m), dn = from_next_lane(m);
  if (lane == 0) up = w > 0 ? edge_last[w - 1] : 0u;
  if (lane == 63) dn = w < 3 ? edge_first[w + 1] : 0u;
  const uint32_t st = m & ~((m << 1) | ((up >> 15) & 1u)) & 0xFFFFu;
  const uint32_t en = m & ~((m >> 1) | ((dn & 1u) << 15)) & 0xFFFFu;
  const uint32_t v = (uint32_t)__popc(en) | ((uint32_t)__popc(m) << 16);  // runs | bytes << 16
  const uint32_t inc = wave_incl_sum(v);
  const uint32_t ls = st ? ch * 16u + 32u - (uint32_t)__builtin_clz(st) : 0u;  // last start + 1
  const uint32_t mx = wave_incl_max(ls);
  if (lane == 63) {
    tot[w] = inc;
    lastst[w] = mx;
  }
  __syncthreads();
  uint32_t carry = 0, cmax = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    if (q < w) {
      carry += tot[q];
      cmax = max(cmax, lastst[q]);
    }
    all += tot[q];
  }
  const uint32_t NR = all & 0xFFFFu, NP = all >> 16;
  const uint32_t size = NR ? 4u + 4u * NR + ((NP + 3u) & ~3u) : 0u;
  if (w == 0) {
    if (g.err && __ballot(bad != 0) && lane == 0) atomicOr(g.err, 8u);
    uint64_t* status = ws + 1;
    if (lane == 0)
      __hip_atomic_store(status + u, (u == 0 ? kStIncl : kStAgg) | tag | size, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    if (u > 0) {
      int64_t pos = (int64_t)u - 1;
      auto unpub = [&](uint64_t x) { return (x >> 62) == 0 || ((x >> 32) & 0x3FFFFFFFull) != E; };
      for (;;) {
        const int64_t q = pos - (int64_t)lane;
        uint64_t sw = q >= 0 ? __hip_atomic_load(status + q, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : kStIncl | tag;  // before the first page: a prefix of 0
        while (__ballot(unpub(sw))) {
          __builtin_amdgcn_s_sleep(1);
          if (unpub(sw))
            sw = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t im = __ballot((sw >> 62) == 2);
        if (im) {
          const uint32_t kk = (uint32_t)__builtin_ctzll(im);
          excl += wave_sum_u64(lane <= kk ? (sw & 0xFFFFFFFFull) : 0ull);
          break;
        }
        excl += wave_sum_u64(sw & 0xFFFFFFFFull);
        pos -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(status + u, kStIncl | tag | (excl + size), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      st_<kWTs>(sp.rec_off[0] + u + 1, (uint64_t)(excl + size));
      if (u == 0) st_<kWTs>(sp.rec_off[0], (uint64_t)0);
      rec_at = excl;
    }
  }
  __syncthreads();
  const uint64_t at = rec_at;
  if (at + size > cap) return;  // only records that end inside the capacity are stored (SPEC §3)
  if (size) {
    uint8_t* rec = sp.data[0] + at;
    if (threadIdx.x == 0) {
      st_<kWTs>(reinterpret_cast<uint32_t*>(rec), NR);
      for (uint32_t q = NP; q & 3u; ++q) st_<kWTs>(rec + 4 + 4 * NR + q, (uint8_t)0);
    }
    emit_chunk<kWTs>(ch, st, en, m, max(cmax, from_prev_lane(mx)), carry + inc - v, c,
               reinterpret_cast<uint32_t*>(rec + 4), rec + 4 + 4 * NR);
  }
  if (kRetwin && !ample && m && twin_ok(g, pj)) {
    if (kWTs)
      st_wt16(twin_w + pj * kPage + ch * 16u, c);
    else
      *reinterpret_cast<uint4*>(twin_w + pj * kPage + ch * 16u) = c;
  }
}

template <bool kApply, bool kRetwin>
__global__ __launch_bounds__(256) void release_page_kernel(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, const DiffSplit sp, uint64_t* __restrict__ ws,
    uint8_t* __restrict__ target, const uint32_t* __restrict__ tids, const IdGuard g) {
  __shared__ uint32_t ticket;
  const uint32_t E = sp.epoch;
  uint32_t* const ctr = reinterpret_cast<uint32_t*>(ws);
  if (threadIdx.x == 0) {
    ticket = atomicAdd(ctr + (E & 1u), 1u);
    if (blockIdx.x == 0)
      __hip_atomic_store(ctr + ((E + 1u) & 1u), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint64_t u = ticket;  // one page per workgroup (one stream: first[0] = 0)
  if (u >= sp.first[1] - sp.first[0]) return;  // workgroup-uniform
  release_page_wg<kApply, kRetwin>(u, twin, cur, ids, sp, ws, target, tids, g);
}

// ------------------------------------------------------------------------- apply (SPEC §4)
// A wave takes 64 (short lists: 4) consecutive records. It stages as many of them as fit in an LDS
// window (kApplyWin*) with coalesced loads, one global round trip per window, then
// applies them four at a time, one record per 16-lane DPP row (apply_rows: validate every header,
// then spread the (run, 16-B chunk) pairs over the row). The replica is only STORED to (16-B
// stores for whole chunks, 8-B / dword stores for whole words, byte stores otherwise), never
// read. A record larger than the window is read from global by row 0.
// Bytes of records staged per wave: 8 KiB for long lists (LDS for occupancy), 12 KiB for short
// ones (every well-formed record fits, so dense records never take the global path).
constexpr uint32_t kApplyWinLong = 8192, kApplyWinShort = 12288;
static_assert(kApplyWinShort >= 10244, "every well-formed record (GDSM_MAX_RECORD) fits");

// Stores the payload bytes selected by `mask` (16 bits, chunk of 16 B at dst) from pay[pp..].
// Replica store; kNT = nontemporal (streaming) cache policy.
template <bool kNT, typename T>
__device__ __forceinline__ void st(T* p, T v) {
  if (kNT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Payload bytes [q, q + 4) of a record (4-B aligned base `pay`), all inside the record: two
// aligned dword loads and a funnel shift (the second load only when q is unaligned).
template <typename P8>
__device__ __forceinline__ uint32_t pay_dw(P8 pay, uint32_t q) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&pay[0]);
  const uint32_t i = q >> 2, sh = (q & 3u) * 8u;
  const uint32_t lo = w[i];
  return sh ? __builtin_amdgcn_alignbit(w[i + 1], lo, sh) : lo;
}

// Stores the payload bytes selected by `mask` (16 bits, chunk of 16 B at dst) from pay[pp..]:
// one 16-B store for a whole chunk, one 8-B store per whole 8-B half, else dword stores for
// whole dwords and byte stores for the rest. kNT = nontemporal (streaming) cache policy.
template <bool kNT, typename P8>
__device__ __forceinline__ void store_chunk(uint8_t* __restrict__ dst, uint32_t mask, P8 pay,
                                            uint32_t pp) {
  if (mask == 0xFFFFu) {
    st<kNT>(reinterpret_cast<u32x4*>(dst), (u32x4){pay_dw(pay, pp), pay_dw(pay, pp + 4),
                                                    pay_dw(pay, pp + 8), pay_dw(pay, pp + 12)});
    return;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t hm = (mask >> (8 * h)) & 0xFFu;
    if (hm == 0xFFu) {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      st<kNT>(reinterpret_cast<u32x2*>(dst + 8 * h), (u32x2){pay_dw(pay, pp), pay_dw(pay, pp + 4)});
      pp += 8;
      continue;
    }
#pragma unroll
    for (int d = 2 * h; d < 2 * h + 2; ++d) {
      const uint32_t nib = (mask >> (4 * d)) & 0xFu;
      if (nib == 0xFu) {
        st<kNT>(reinterpret_cast<uint32_t*>(dst + 4 * d), pay_dw(pay, pp));
        pp += 4;
      } else if (nib) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((nib >> k) & 1u) st<kNT>(dst + 4 * d + k, (uint8_t)pay[pp++]);
      }
    }
  }
}

// Stores the run bytes that fall into one 16-B destination chunk: chunk [cs, cs+16) of `page`,
// run [off, end), payload of the run starting at pay[pp].
template <bool kNT, typename P8>
__device__ __forceinline__ void store_run_chunk(uint8_t* __restrict__ page, uint32_t cs,
                                                uint32_t off, uint32_t end, P8 pay, uint32_t pp) {
  const uint32_t lo = max(off, cs), hi = min(end, cs + 16u);
  const uint32_t mask = ((hi - cs >= 16u) ? 0xFFFFu : ((1u << (hi - cs)) - 1u)) &
                        ~((1u << (lo - cs)) - 1u);
  store_chunk<kNT>(page + cs, mask, pay, pp + (lo - off));
}

// Applies up to four records at once, one per 16-lane DPP row (a lane per run), or, with kW = 64,
// one record over the whole wave. Pass 1 validates every header of the row's record (length,
// bounds, sorted and non-overlapping, total size), so a malformed record writes nothing. Pass 2
// spreads the record's (run, 16-B chunk) pairs over the row's lanes — a run is found by a binary
// search over the row's pair offsets — so short and long runs cost the same per byte. `has` is
// false for rows without a record. Returns false in the lanes of a row whose record is malformed.
// kMode: 0 = plain stores, 1 = MEASUREMENT ONLY (no replica stores), 2 = nontemporal stores.
template <uint32_t kW>
__device__ __forceinline__ uint32_t grp_incl_sum(uint32_t x) {
  return kW == 16 ? row_incl_sum(x) : wave_incl_sum(x);
}
template <uint32_t kW>
__device__ __forceinline__ uint32_t grp_incl_max(uint32_t x) {
  return kW == 16 ? row_incl_max(x) : wave_incl_max(x);
}
template <uint32_t kW>
__device__ __forceinline__ uint32_t grp_last(uint32_t x) {
  return kW == 16 ? row_last(x) : lane_bcast(x, 63);
}
template <uint32_t kW>
__device__ __forceinline__ uint32_t grp_prev(uint32_t x) {
  return kW == 16 ? row_prev(x) : from_prev_lane(x);
}

template <int kMode, typename P32, typename P8, uint32_t kW = 16>
__device__ __forceinline__ bool apply_rows(uint8_t* __restrict__ page, P32 rec32, P8 rec8,
                                           uint32_t size, bool has, uint32_t& sink) {
  static_assert(kW == 16 || kW == 64, "a DPP row or the wave");
  const uint32_t lane = lane_id(), lr = lane & (kW - 1), rb = lane & ~(kW - 1);
  uint32_t nr = has ? rec32[0] : 0u;
  bool bad = has && (nr == 0 || nr > kMaxRuns || size < 4u + 4u * nr);
  if (bad) nr = 0;
  const uint32_t nit = lane_bcast(wave_incl_max((nr + kW - 1) / kW), 63);
  uint32_t pay = 0, prev_end = 0, lbad = 0;
  for (uint32_t it = 0; it < nit; ++it) {
    const uint32_t r = it * kW + lr;
    const bool v = r < nr;
    const uint32_t h = v ? rec32[1 + r] : 0u;
    const uint32_t off = h & 0xFFFFu, len = h >> 16, end = v ? off + len : 0u;
    uint32_t pe = grp_prev<kW>(end);
    if (lr == 0) pe = prev_end;
    if (v && (len == 0 || end > kPage || off < pe)) lbad = 1;
    pay += grp_last<kW>(grp_incl_sum<kW>(v ? len : 0u));
    prev_end = grp_last<kW>(end);
  }
  if (grp_last<kW>(grp_incl_max<kW>(lbad))) bad = true;
  if (has && !bad && size != 4u + 4u * nr + ((pay + 3u) & ~3u)) bad = true;
  const uint32_t nrw = bad ? 0u : nr;  // runs this row writes
  const uint32_t nit2 = lane_bcast(wave_incl_max((nrw + kW - 1) / kW), 63);
  uint32_t pcarry = 0;
  for (uint32_t it = 0; it < nit2; ++it) {
    const uint32_t r = it * kW + lr;
    const bool v = r < nrw;
    const uint32_t h = v ? rec32[1 + r] : 0u;
    const uint32_t off = h & 0xFFFFu, len = v ? h >> 16 : 0u, end = off + len;
    const uint32_t pinc = grp_incl_sum<kW>(len);
    const uint32_t pp = 4u + 4u * nr + pcarry + pinc - len;  // payload of this run
    pcarry += grp_last<kW>(pinc);
    const uint32_t nch = len ? ((end - 1u) >> 4) - (off >> 4) + 1u : 0u;
    const uint32_t cinc = grp_incl_sum<kW>(nch);
    const uint32_t cex = cinc - nch;
    const uint32_t T = grp_last<kW>(cinc);
    if (__ballot(nch > 2u) == 0) {
      // short runs (<= 2 chunks each, e.g. word-sized edits): every lane stores its own run, no
      // cross-lane lookup (a 4-step bpermute search per 16 pairs dominated many-run records);
      // longer runs keep the spread below, whose lanes store consecutive chunks
      for (uint32_t c = 0; c < nch; ++c) {
        if (kMode != 1)
          store_run_chunk<kMode == 2>(page, ((off >> 4) + c) << 4, off, end, rec8, pp);
        else
          sink += off ^ end ^ (uint32_t)rec8[pp];
      }
      continue;
    }
    const uint32_t tmax = lane_bcast(wave_incl_max(T), 63);
    for (uint32_t g = lr; g < ((tmax + kW - 1) & ~(kW - 1)); g += kW) {
      uint32_t i = 0;
#pragma unroll
      for (uint32_t step = kW / 2; step; step >>= 1) {
        const uint32_t c = (uint32_t)__shfl(cex, (int)(rb + i + step), 64);
        if (c <= g) i += step;
      }
      const uint32_t oi = (uint32_t)__shfl(off, (int)(rb + i), 64);
      const uint32_t ei = (uint32_t)__shfl(end, (int)(rb + i), 64);
      const uint32_t pi = (uint32_t)__shfl(pp, (int)(rb + i), 64);
      const uint32_t ci = (uint32_t)__shfl(cex, (int)(rb + i), 64);
      if (g < T) {
        if (kMode != 1)
          store_run_chunk<kMode == 2>(page, ((oi >> 4) + (g - ci)) << 4, oi, ei, rec8, pi);
        else  // measurement variant: everything but the replica stores
          sink += oi ^ ei ^ (uint32_t)rec8[pi];
      }
    }
  }
  return !bad;
}

// Tiny lists (<= kApplyTiny records): one wave per record, its runs 64 at a time over the whole
// wave. Such a list costs latency, not bandwidth: a page of rewritten doubles is ~500 runs of ~7
// bytes (config 5), which one 16-lane row of apply_kernel walked in 33 steps with 4 records per
// wave. The record is staged in LDS first (16 B per lane by LDS-DMA, every load in flight at
// once): read from global memory, each of the run loops' steps waited one round trip.
constexpr uint64_t kApplyTiny = 4096;
template <int kMode>
__global__ __launch_bounds__(256) void apply_tiny_kernel(uint8_t* __restrict__ target,
                                                         const uint32_t* __restrict__ ids,
                                                         uint64_t n,
                                                         const uint64_t* __restrict__ rec_off,
                                                         const uint8_t* __restrict__ data,
                                                         uint32_t* __restrict__ err) {
  // +4 dwords: pay_dw's second dword at the record's end stays inside the buffer
  __shared__ __attribute__((aligned(16))) uint32_t win_all[4][kApplyWinShort / 4 + 4];
  const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const uint32_t lane = lane_id();
  uint32_t* win = win_all[threadIdx.x >> 6];
  const uint64_t o0 = rec_off[r], o1 = rec_off[r + 1];
  const uint64_t p = ids ? ids[r] : r;
  const uint8_t* rec = data + o0;
  const uint32_t size = o1 > o0 ? (uint32_t)min(o1 - o0, (uint64_t)0xFFFFFFFFu) : 0u;
  uint32_t sink = 0;
  bool ok;
  if (size <= kApplyWinShort) {
    typedef __attribute__((address_space(1))) void* gptr;
    typedef __attribute__((address_space(3))) void* lptr;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rec);
    const uint32_t words = size >> 2, n16 = words >> 2;
    for (uint32_t q0 = 0; q0 < 4 * n16; q0 += 256) {
      const uint32_t q = q0 / 4 + lane;
      if (q < n16) __builtin_amdgcn_global_load_lds((gptr)(src + 4 * q), (lptr)(win + q0), 16, 0, 0);
    }
    const uint32_t qt = 4 * n16 + lane;
    if (qt < words) __builtin_amdgcn_global_load_lds((gptr)(src + qt), (lptr)(win + 4 * n16), 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the record has landed
    wave_lds_sync();
    ok = apply_rows<kMode, const uint32_t*, const uint8_t*, 64>(
        target + p * kPage, win, reinterpret_cast<const uint8_t*>(win), size, size > 0, sink);
  } else {  // larger than any well-formed record: validated (and refused) from global memory
    ok = apply_rows<kMode, const uint32_t*, const uint8_t*, 64>(
        target + p * kPage, reinterpret_cast<const uint32_t*>(rec), rec, size, true, sink);
  }
  if (__ballot(!ok) && lane == 0) atomicOr(err, 1u);
  if (kMode == 1 && sink == 0x9E3779B9u) atomicOr(err, 2u);
}

template <int kMode, uint32_t kApplyWin>
__global__ __launch_bounds__(256) void apply_kernel(uint8_t* __restrict__ target,
                                                    const uint32_t* __restrict__ ids, uint64_t n,
                                                    const uint64_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ data,
                                                    uint32_t* __restrict__ err, uint32_t per_task) {
  __shared__ __attribute__((aligned(16))) uint32_t win_all[4][kApplyWin / 4];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = lane >> 4;
  uint32_t* win = win_all[wave];
  const uint64_t ntask = (n + per_task - 1) / per_task;
  uint32_t bad = 0, sink = 0;
  for (uint64_t task = (uint64_t)blockIdx.x * 4 + wave; task < ntask;
       task += (uint64_t)gridDim.x * 4) {
    const uint64_t a = task * per_task;
    const uint32_t cnt = (uint32_t)min((uint64_t)per_task, n - a);
    const uint64_t my_off = rec_off[a + min(lane, cnt)];  // lane l: start of record a+l
    const uint64_t end_off = rec_off[a + cnt];
    uint32_t j = 0;
    while (j < cnt) {
      const uint64_t start = lane_bcast64(my_off, j);
      // records j..k-1 fit the window: rec_off[a+k] - start <= kApplyWin
      const bool fits = lane > j && lane <= cnt && (my_off - start) <= kApplyWin;
      const uint64_t fm = __ballot(fits);
      uint32_t k = fm ? 63u - (uint32_t)__clzll(fm) : j;  // highest lane whose offset fits
      if (cnt == 64 && (end_off - start) <= kApplyWin) k = 64;
      if (k == j) {  // record j alone exceeds the window: straight from global, row 0 only
        const uint64_t r1 = (j + 1 < 64) ? lane_bcast64(my_off, j + 1) : end_off;
        const uint64_t p = ids ? ids[a + j] : a + j;
        const uint8_t* rec = data + start;
        const bool has = row == 0 && r1 > start;
        if (!apply_rows<kMode>(target + p * kPage, reinterpret_cast<const uint32_t*>(rec), rec,
                                (uint32_t)(r1 - start), has, sink))
          bad = 1;
        ++j;
        continue;
      }
      const uint64_t stop = (k == 64) ? end_off : lane_bcast64(my_off, k);
      const uint32_t words = (uint32_t)((stop - start) >> 2);
      // the window is filled by LDS-DMA (global_load_lds_dword: 256 B per wave instruction, all
      // of them in flight at once), so a wave waits one round trip per window, not one per 256 B
      const uint32_t* src = reinterpret_cast<const uint32_t*>(data + start);
      for (uint32_t q0 = 0; q0 < words; q0 += 64) {
        const uint32_t q = q0 + lane;
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void*)(src + (q < words ? q : 0)),
            (__attribute__((address_space(3))) void*)(win + q0), 4, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window has landed
      wave_lds_sync();
      const uint8_t* win8 = reinterpret_cast<const uint8_t*>(win);
      for (uint32_t jj = j; jj < k; jj += 4) {
        const uint32_t mine = jj + row;  // this row's record
        const bool in = mine < k;
        const uint32_t ms = in ? mine : jj;
        // both shuffles run in every lane: a bpermute from a lane that is switched off by a
        // branch returns garbage, and `?:` would evaluate the second one in some rows only
        const uint64_t r0 = __shfl(my_off, (int)ms, 64);
        const uint64_t nx = __shfl(my_off, (int)min(ms + 1, 63u), 64);
        const uint64_t r1 = (ms + 1 == k) ? stop : nx;
        const bool has = in && r1 > r0;
        const uint32_t base = (uint32_t)(r0 - start);
        const uint64_t p = ids ? ids[a + ms] : a + ms;
        if (!apply_rows<kMode>(target + p * kPage, win + base / 4, win8 + base,
                                (uint32_t)(r1 - r0), has, sink))
          bad = 1;
      }
      wave_lds_sync();
      j = k;
    }
  }
  if (__ballot(bad != 0) && lane == 0) atomicOr(err, 1u);
  if (kMode == 1 && sink == 0x9E3779B9u) atomicOr(err, 2u);
}

// 16 payload bytes starting at LDS byte offset q (4-B aligned base `pay32`): five aligned dword
// reads and four funnel shifts.
__device__ __forceinline__ u32x4 lds_load16(const uint32_t* __restrict__ pay32, uint32_t q) {
  const uint32_t i = q >> 2, sh = (q & 3u) * 8u;
  const uint32_t w0 = pay32[i], w1 = pay32[i + 1], w2 = pay32[i + 2], w3 = pay32[i + 3],
                 w4 = pay32[i + 4];
  if (!sh) return (u32x4){w0, w1, w2, w3};
  return (u32x4){__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                 __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh)};
}

// One 16-B destination chunk per lane (where `valid`): bytes [lo, hi) of the chunk at `dst`
// (16-B aligned), their payload at LDS byte offset q (the byte for lo). The wave stores
//   whole chunks with one 16-B store, chunks whose bytes are one aligned 8-B half with one 8-B
//   store, and every other chunk's bytes 16 lanes per chunk, four chunks per step,
// so no lane walks a byte mask on its own while the others wait (a partial chunk among 64 made
// every lane of the old per-lane mask walk pay for it).
// kNT: 1 = half chunks (whole aligned 8-B words) stored nontemporally, 2 = whole chunks too.
// (Alone, scattered whole 64-B segments are written 1.3x faster nontemporally,
// scripts/dev/cluster_probe.hip; inside the apply, beside the partial chunks' cached byte stores to
// the same segments, nontemporal whole chunks measured slower.)
template <int kNT>
__device__ __forceinline__ void store_chunks_wave(bool valid, uint8_t* dst, uint32_t lo,
                                                  uint32_t hi, const uint32_t* __restrict__ pay32,
                                                  uint32_t q) {
  const bool full = valid && lo == 0 && hi == 16;
  const bool half = valid && (hi - lo) == 8 && (lo & 7u) == 0;
  if (full) {
    st<(kNT >= 2)>(reinterpret_cast<u32x4*>(dst), lds_load16(pay32, q));
  } else if (half) {
    const u32x4 v = lds_load16(pay32, q);
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    st<(kNT >= 1)>(reinterpret_cast<u32x2*>(dst + lo), (u32x2){v.x, v.y});
  }
  uint64_t G = __ballot(valid && !full && !half);
  const uint32_t lane = lane_id(), r = lane >> 4, b = lane & 15u;
  const uint8_t* pay8 = reinterpret_cast<const uint8_t*>(pay32);
  while (G) {  // wave-uniform
    // the four lowest remaining chunks, one per 16-lane row
    uint32_t own[4];
    uint64_t g = G;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      own[k] = g ? (uint32_t)__builtin_ctzll(g) : 64u;
      g &= g ? g - 1 : 0ull;
    }
    G = g;
    const uint32_t o = r == 0 ? own[0] : r == 1 ? own[1] : r == 2 ? own[2] : own[3];
    const uint32_t os = o < 64u ? o : 0u;
    const uint64_t d = shfl64((uint64_t)(uintptr_t)dst, (int)os);
    const uint32_t l2 = (uint32_t)__shfl((int)lo, (int)os, 64);
    const uint32_t h2 = (uint32_t)__shfl((int)hi, (int)os, 64);
    const uint32_t q2 = (uint32_t)__shfl((int)q, (int)os, 64);
    if (o < 64u && b >= l2 && b < h2)
      *reinterpret_cast<__attribute__((address_space(1))) uint8_t*>((uintptr_t)d + b) =
          pay8[q2 + b - l2];
  }
}

// ---- apply, flat form (long lists): a wave stages a window of records in LDS as above, then
// works on the window's RUNS, one lane per run, instead of on records row by row:
//   records  lane per record: header checks and a lane-serial walk over its run headers (sorted,
//            in the page, sizes adding up: SPEC §4), exclusive scan of the run counts;
//   runs     64 at a time, lane q = the window's run q: its record by a 6-step search over the
//            records' run offsets, its header, its payload offset (segmented scan of the lengths
//            within the record), then its 16-B chunks spread over the wave by a search over the
//            batch's chunk offsets (consecutive lanes, consecutive chunks of a run), or lane by
//            lane when every run of the batch spans at most two chunks.
// A malformed record writes nothing (its runs are dropped after the record walk); a record
// larger than the window goes through apply_rows from global memory, as in apply_kernel.
constexpr uint32_t kChunkMap = 512;  // chunks of one run batch mapped through LDS (else: search)

// One staged window of the flat form: records j..k-1 of the wave's task (lane l's my_off / my_page:
// record a + l's stream offset and page), their bytes [start, stop) in `win`. Returns 1 when a
// record of the window is malformed (its runs are not written).
template <int kNT>
__device__ __forceinline__ uint32_t flat_window(uint8_t* __restrict__ target,
                                                const uint32_t* __restrict__ win, uint4* ri,
                                                uint4* rp, uint8_t* cm, uint64_t my_off,
                                                uint32_t my_page, uint32_t j, uint32_t k,
                                                uint64_t start, uint64_t stop) {
  const uint32_t lane = lane_id();
  uint32_t bad = 0;
  // ---- records: lane l = record j + l of the window
  const uint32_t nrec = k - j;
  const bool inrec = lane < nrec;
  const uint32_t r = min(j + lane, 63u);
  const uint64_t o0 = __shfl(my_off, (int)r, 64);
  const uint64_t o1n = __shfl(my_off, (int)min(r + 1, 63u), 64);
  const uint64_t o1 = (j + lane + 1 == k) ? stop : o1n;
  // offsets out of order (an unchecked caller stream) can put a record of the window outside
  // [start, stop): it is malformed and writes nothing (its bytes are not in the window)
  const bool outside = inrec && (o0 < start || o1 < o0 || o1 > stop);
  const uint32_t rs = inrec && !outside ? (uint32_t)(o0 - start) : 0u;
  const uint32_t size = inrec && !outside ? (uint32_t)(o1 - o0) : 0u;
  uint32_t nr = size ? win[rs / 4] : 0u;
  bool rbad = outside || (size && (nr == 0 || nr > kMaxRuns || size < 4u + 4u * nr));
  if (rbad) nr = 0;
  if (nr) {  // the record's run headers, lane-serially: sorted, inside the page, sizes add up
    // (four independent LDS reads per step, not one dependent read per header)
    uint32_t prev_end = 0, tot = 0;
    for (uint32_t i = 0; i < nr; i += 4) {
      uint32_t hv[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) hv[u] = win[rs / 4 + 1 + min(i + u, nr - 1u)];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        if (i + u < nr) {
          const uint32_t off = hv[u] & 0xFFFFu, len = hv[u] >> 16;
          if (len == 0 || off + len > kPage || off < prev_end) rbad = true;
          prev_end = off + len;
          tot += len;
        }
      }
    }
    if (size != 4u + 4u * nr + ((tot + 3u) & ~3u)) rbad = true;
    if (rbad) nr = 0;
  }
  bad |= rbad ? 1u : 0u;
  const uint32_t rinc = wave_incl_sum(nr);
  const uint32_t RB = rinc - nr;                 // the record's first run in the window
  const uint32_t NRW = lane_bcast(rinc, 63);     // runs in the window
  const uint32_t RBs = inrec ? RB : 0xFFFFFFFFu;  // search key (records past the window: never)
  ri[lane] = make_uint4(rs, nr, RB, __shfl(my_page, (int)r, 64));
  wave_lds_sync();

  // ---- runs: 64 at a time
  uint32_t carry_sum = 0;  // payload bytes of the previous batch's last record so far
  for (uint32_t q0 = 0; q0 < NRW; q0 += 64) {
    const uint32_t q = q0 + lane;
    const bool vq = q < NRW;
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = 32; st; st >>= 1) {
      const uint32_t c = (uint32_t)__shfl((int)RBs, (int)(pos + st), 64);
      if (c <= q) pos += st;
    }
    const uint4 R = ri[pos];  // .x LDS offset, .y runs, .z first run, .w page
    const uint32_t i = q - R.z;
    const uint32_t h = vq ? win[R.x / 4 + 1 + i] : 0u;
    const uint32_t off = h & 0xFFFFu, len = h >> 16, end = off + len;
    // payload offset: lengths summed within the record (segments start at a record's run 0)
    const uint32_t sg = wave_incl_segsum_dpp(len | ((vq && i == 0) ? kSegStart : 0u));
    const uint32_t incl = (sg & ~kSegStart) + ((sg & kSegStart) ? 0u : carry_sum);
    const uint32_t pp = R.x + 4u + 4u * R.y + incl - len;
    carry_sum = lane_bcast(incl, 63);
    const uint32_t nch = len ? ((end - 1u) >> 4) - (off >> 4) + 1u : 0u;
    const uint32_t M = lane_bcast(wave_incl_max(nch), 63);
    uint8_t* page = target + (uint64_t)R.w * kPage;
    if (M <= 2) {
      // short runs (word-sized edits): each lane stores its own run's one or two chunks
      for (uint32_t c = 0; c < M; ++c) {
        const uint32_t cs = ((off >> 4) + c) << 4;
        const uint32_t lo = max(off, cs), hi = min(end, cs + 16u);
        store_chunks_wave<kNT>(c < nch, page + cs, lo - cs, hi - cs, win, pp + (lo - off));
      }
    } else {
      // the batch's (run, chunk) pairs spread over the wave, 64 per step: consecutive lanes
      // store consecutive chunks of a run, so one store instruction writes whole segments
      // (lane-per-run stores, 16 B into 64 different runs per instruction, measured 1.3x
      // slower on clustered records)
      const uint32_t cinc = wave_incl_sum(nch), cex = cinc - nch;
      const uint32_t T = lane_bcast(cinc, 63);
      if (T <= kChunkMap) {
        // chunk -> run through LDS: each run writes its index over its chunks' slots and its
        // parameters once; a chunk lane then needs two LDS reads (a 6-step search over the
        // runs' chunk offsets was 6 dependent ds_bpermute round trips per 64 chunks)
        if (vq) rp[lane] = make_uint4(R.w, off | (end << 16), pp, cex);
        for (uint32_t c = 0; c < M; ++c)
          if (c < nch) cm[cex + c] = (uint8_t)lane;
        wave_lds_sync();
        for (uint32_t g0 = 0; g0 < T; g0 += 64) {
          const uint32_t g = g0 + lane;
          const uint4 P = rp[cm[g < T ? g : 0]];
          const uint32_t oi = P.y & 0xFFFFu, ei = P.y >> 16;
          const uint32_t cs = ((oi >> 4) + (g - P.w)) << 4;
          const uint32_t lo = max(oi, cs), hi = min(ei, cs + 16u);
          store_chunks_wave<kNT>(g < T, target + (uint64_t)P.x * kPage + cs, lo - cs, hi - cs, win,
                            P.z + (lo - oi));
        }
        wave_lds_sync();  // the next batch rewrites rp / cm
        continue;
      }
      for (uint32_t g0 = 0; g0 < T; g0 += 64) {
        const uint32_t g = g0 + lane;
        uint32_t p2 = 0;
#pragma unroll
        for (uint32_t st = 32; st; st >>= 1) {
          const uint32_t c = (uint32_t)__shfl((int)cex, (int)(p2 + st), 64);
          if (c <= g) p2 += st;
        }
        const uint32_t oi = (uint32_t)__shfl((int)off, (int)p2, 64);
        const uint32_t ei = (uint32_t)__shfl((int)end, (int)p2, 64);
        const uint32_t pi = (uint32_t)__shfl((int)pp, (int)p2, 64);
        const uint32_t ci = (uint32_t)__shfl((int)cex, (int)p2, 64);
        const uint32_t wi = (uint32_t)__shfl((int)R.w, (int)p2, 64);
        const uint32_t cs = ((oi >> 4) + (g - ci)) << 4;
        const uint32_t lo = max(oi, cs), hi = min(ei, cs + 16u);
        store_chunks_wave<kNT>(g < T, target + (uint64_t)wi * kPage + cs, lo - cs, hi - cs, win,
                          pi + (lo - oi));
      }
    }
  }
  wave_lds_sync();
  return bad;
}

template <uint32_t kWin, bool kX4 = true, int kNT = 0>
__global__ __launch_bounds__(256) void apply_flat_kernel(uint8_t* __restrict__ target,
                                                         const uint32_t* __restrict__ ids,
                                                         uint64_t n,
                                                         const uint64_t* __restrict__ rec_off,
                                                         const uint8_t* __restrict__ data,
                                                         uint32_t* __restrict__ err) {
  // +4 dwords: an unaligned payload read of the window's last bytes stays inside the buffer
  // (every fill instruction writes whole 1 KiB / 256-B blocks inside roundup(window, 64 dwords))
  __shared__ __attribute__((aligned(16))) uint32_t win_all[4][kWin / 4 + 4];
  __shared__ uint4 ri_all[4][64];  // per record of the window: LDS offset, runs, first run, page
  __shared__ uint4 rp_all[4][64];  // per run of a batch: page, off | end << 16, payload offset
  __shared__ uint8_t cm_all[4][kChunkMap];  // chunk -> run of the batch
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = lane >> 4;
  uint32_t* win = win_all[wave];
  uint4* ri = ri_all[wave];
  uint4* rp = rp_all[wave];
  uint8_t* cm = cm_all[wave];
  const uint64_t ntask = (n + 63) / 64;
  uint32_t bad = 0, sink = 0;
  for (uint64_t task = (uint64_t)blockIdx.x * 4 + wave; task < ntask;
       task += (uint64_t)gridDim.x * 4) {
    const uint64_t a = task * 64;
    const uint32_t cnt = (uint32_t)min((uint64_t)64, n - a);
    const uint64_t my_off = rec_off[a + min(lane, cnt)];  // lane l: start of record a+l
    const uint64_t end_off = rec_off[a + cnt];
    const uint32_t my_page = lane < cnt ? (ids ? ids[a + lane] : (uint32_t)(a + lane)) : 0u;
    uint32_t j = 0;
    while (j < cnt) {
      const uint64_t start = lane_bcast64(my_off, j);
      const bool fits = lane > j && lane <= cnt && (my_off - start) <= kWin;
      const uint64_t fm = __ballot(fits);
      uint32_t k = fm ? 63u - (uint32_t)__clzll(fm) : j;
      if (cnt == 64 && (end_off - start) <= kWin) k = 64;
      if (k == j) {  // record j alone exceeds the window: straight from global, row 0 only
        const uint64_t r1 = (j + 1 < 64) ? lane_bcast64(my_off, j + 1) : end_off;
        const uint32_t p = lane_bcast(my_page, j);
        const uint8_t* rec = data + start;
        const bool has = row == 0 && r1 > start;
        if (!apply_rows<0>(target + (uint64_t)p * kPage, reinterpret_cast<const uint32_t*>(rec),
                           rec, (uint32_t)(r1 - start), has, sink))
          bad = 1;
        ++j;
        continue;
      }
      const uint64_t stop = (k == 64) ? end_off : lane_bcast64(my_off, k);
      const uint32_t words = (uint32_t)((stop - start) >> 2);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(data + start);
      typedef __attribute__((address_space(1))) void* gptr;
      typedef __attribute__((address_space(3))) void* lptr;
      uint32_t q0 = 0;
      if (kX4) {
        // 16 B per lane (global_load_lds_dwordx4, gfx950), then the last < 4 dwords. Lanes past
        // the pieces are switched off, not clamped: an LDS-DMA lane writes only when active, and
        // a clamped x4 lane would write into the tail's dwords, which the second fill also
        // writes (two DMA writes of one LDS dword land in no fixed order)
        const uint32_t n16 = words >> 2;
        for (; q0 < 4 * n16; q0 += 256) {
          const uint32_t q = q0 / 4 + lane;
          if (q < n16)
            __builtin_amdgcn_global_load_lds((gptr)(src + 4 * q), (lptr)(win + q0), 16, 0, 0);
        }
        q0 = 4 * n16;
        const uint32_t q = q0 + lane;
        if (q < words) __builtin_amdgcn_global_load_lds((gptr)(src + q), (lptr)(win + q0), 4, 0, 0);
        q0 = words;
      }
      for (; q0 < words; q0 += 64) {
        const uint32_t q = q0 + lane;
        __builtin_amdgcn_global_load_lds((gptr)(src + (q < words ? q : 0)), (lptr)(win + q0), 4, 0,
                                         0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window has landed
      wave_lds_sync();

      bad |= flat_window<kNT>(target, win, ri, rp, cm, my_off, my_page, j, k, start, stop);
      j = k;
    }
  }
  if (__ballot(bad != 0) && lane == 0) atomicOr(err, 1u);
  (void)sink;  // apply_rows<0> leaves it alone (measurement builds only)
}

// ------------------------------------------------------------------------- launchers
// Diff geometry, gdsm_tune("diff_variant", v) or GDSM_DIFF_VARIANT=v; every variant writes the
// same canonical stream (tests/test_gpu_pages.py checks each):
//   0  automatic (default): 2 pages per wave for short lists (n <= 32768: a wave walks its
//      pages one after the other, so a few dozen pages must not share one wave); longer lists by
//      the density the context last saw (gdsm_runs_total, a sized exchange): <= kDense64 B/page
//      64 pages with the spill slot (5), <= kDense16 16 pages (1), beyond 16 pages with the spill
//      slot (7); density unknown: 64 pages with the spill slot (5), correct and fast at any
//      density but 14 % behind 16 pages on dense clustered pages. Never the caller's capacity,
//      except for a raw caller whose workspace predates the spill pool (round 2's rule:
//      64 / 32 / 16 pages at <= 128 / 384 / more bytes of capacity per page)
//   1  16 pages per wave, 8 KiB LDS record buffer per wave, 4 waves/SIMD
//   2  32 pages per wave, 8 KiB LDS record buffer per wave, 4 waves/SIMD
//   3  2 pages per wave
//   4  64 pages per wave, 8 KiB LDS record buffer per wave, 4 waves/SIMD (no spill)
//   5  64 pages per wave, 8 KiB LDS buffer + 24 KiB global spill slot per wave
//   6  32 pages per wave, 8 KiB LDS buffer + 24 KiB global spill slot per wave
//   7  16 pages per wave, 8 KiB LDS buffer + 24 KiB global spill slot per wave
//   8  1 page per wave (automatic for lists of <= kDiffTiny pages: a wave per page, and a dense
//      page's record, ~4.6 KiB for a page of rewritten doubles, fits the LDS buffer instead of
//      being re-read as the second page of a 2-page unit); one stream of a context outside graph
//      capture: the one-workgroup kSolo launch up to diff_solo_max pages, the chained grid launch
//      (kChain, no zeroing launch) beyond; otherwise kSolo up to kSoloUnits pages
// Measurement-only kernels (invalid output) are not part of the library.
static int diff_variant_from_env() {
  const char* e = getenv("GDSM_DIFF_VARIANT");
  const int v = e ? atoi(e) : 0;
  return (v >= 0 && v <= 8) ? v : 0;
}
static std::atomic<int> g_diff_variant{diff_variant_from_env()};
static int diff_variant() { return g_diff_variant.load(std::memory_order_relaxed); }
// Apply geometry, gdsm_tune("apply_variant", v) or GDSM_APPLY_VARIANT=v (same output):
//   0  default: long lists (> 16384 records) the flat form (apply_flat_kernel: the window's runs
//      64 at a time, chunks spread over the wave) with a 4 KiB window filled 16 B per lane, whole
//      aligned 8-B words stored nontemporally; short lists apply_kernel with 4 records per task
//      and a 12 KiB window
//   1  long lists: apply_kernel (records row by row), 8 KiB window (round 2's default)
//   2  long lists: apply_kernel, 4 KiB window
//   3  long lists: flat form, 8 KiB window
//   4  long lists: flat form, 2 KiB window
//   5  long lists: flat form, 4 KiB window filled by dword LDS-DMA (round 3's first default)
//   6  long lists: flat form, whole chunks stored nontemporally too
//   7  long lists: flat form, every store cached (round 3's first flat default)
// Same box, 4M pages: uniform 1 % 0.966 ms (7) -> 0.932 (0); clustered 1.058 (7), 1.065 (0),
// 1.234 (6).
// Same-box, 2M clustered pages (config-3 shard): 0.79 ms (1) -> 0.64 (2) -> 0.55 (0); config 2:
// 0.250 -> 0.241 ms.
constexpr int kApplyVariants = 8;
static int apply_variant_from_env() {
  const char* e = getenv("GDSM_APPLY_VARIANT");
  const int v = e ? atoi(e) : 0;
  return (v >= 0 && v < kApplyVariants) ? v : 0;
}
static std::atomic<int> g_apply_variant{apply_variant_from_env()};
// Short lists of one-page units (variant 8), gdsm_tune("diff_solo_max", k) and ("diff_chain", c):
// up to k units the one-workgroup kSolo launch, beyond it a chained launch when the context
// offers its DiffChain: c = 1 / 4: diff_single_kernel<..., kChainW> with 1 / 4 waves (pages) per
// workgroup, c = 3: release_page_kernel (a page per four-wave workgroup), c = 2 (default):
// release_page_kernel up to kChainPerPage pages, four pages per workgroup beyond (per-page
// tickets would queue on the counter); c = 0: the grid with its zeroing launch. Release of m
// dense pages (profiles/r05_release_chain_probe.txt), us per launch, one-workgroup / one page per
// wave / page per workgroup: m = 1 8.2 / 9.1 / 3.6; m = 10 11.9 / 12.0 / 6.1; m = 200 (four
// pages per workgroup 12.5) / 13.2 / 8.5; m = 2048 four per workgroup 30.7, page per workgroup
// 45.1. Default k = 0: the one-workgroup form (up to kSoloUnits pages) serves graph capture,
// which has no chain, and callers without a context.
constexpr int kSoloDefault = 0;
// (also GDSM_DIFF_SOLO_MAX / GDSM_DIFF_CHAIN at load)
static int env_int(const char* name, int lo, int hi, int dflt) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : dflt;
  return (e && v >= lo && v <= hi) ? v : dflt;
}
static std::atomic<int> g_solo_max{env_int("GDSM_DIFF_SOLO_MAX", 0, (int)kSoloUnits, kSoloDefault)};
constexpr uint64_t kChainPerPage = 512;
static std::atomic<int> g_chain{env_int("GDSM_DIFF_CHAIN", 0, 4, 2)};
#ifdef GDSM_MEASURE
static std::atomic<int> g_diff_skip{0};  // the chained release's kSkip (measurement builds)
#endif


int tune(const char* key, int64_t value) {
  if (!strcmp(key, "diff_variant") && value >= 0 && value <= 8) {
    g_diff_variant.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  if (!strcmp(key, "diff_solo_max") && value >= 0 && value <= (int64_t)kSoloUnits) {
    g_solo_max.store((int)value, std::memory_order_relaxed);
    return 0;
  }
#ifdef GDSM_MEASURE
  if (!strcmp(key, "diff_skip") && value >= 0 && value < 64) {
    g_diff_skip.store((int)value, std::memory_order_relaxed);
    return 0;
  }
#endif
  if (!strcmp(key, "diff_chain") && value >= 0 && value <= 4) {
    g_chain.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  if (!strcmp(key, "apply_variant") && value >= 0 && value < kApplyVariants) {
    g_apply_variant.store((int)value, std::memory_order_relaxed);
    return 0;
  }
  return coh_tune(key, value);
}

// Single-pass diff workspace: the ticket counter and one status granule per unit of the
// smallest geometry that n may take (2 pages up to kDiffShort, else 16), then the spill pool of
// the 64-page geometry (a generation word per workgroup slot, then kSpillWGs or
// fewer workgroup slots of 4 x kDiffSpill bytes). Non-decreasing in n, so a workspace reserved
// for n fits every shorter list.
constexpr uint64_t kDiffShort = 32768, kDiffTiny = 2048;
static_assert(kDiffChainUnits == kDiffTiny, "every automatic one-page list fits the chain");
constexpr uint32_t kDiffSpill = 24576;
// Densities (stream bytes per page) the automatic geometry switches at: up to kDense64, 64 pages
// per wave (their records fill the 8 KiB buffer at 128 B); up to kDense16, 16 pages (8 KiB / 16
// = 512 B fit without spilling); beyond, 16 pages with the spill slot. Measured, 1M pages:
// 1 % words (66 B/page) 64 pages 1.40 ms vs 16 pages 1.50; clustered 10 % (442 B/page) 16 pages
// 1.56-1.66 ms vs 64 pages with the spill slot 1.79-1.93 (the spill's write and read-back).
constexpr uint32_t kDense64 = 112, kDense16 = 480;
static inline uint64_t up256(uint64_t v) { return (v + 255) & ~255ull; }
// Sized for the smallest spill unit (16 pages), plus the partial units of up to kMaxSplit output
// streams (launch_diff_split: each stream's last unit may be partial): two more workgroups. None
// for short lists, which take the 2-page geometry, unless a spill geometry is forced (gdsm_tune).
static uint64_t spill_pool_bytes(uint64_t n) {
  if (n <= kDiffShort && (diff_variant() < 5 || diff_variant() > 7)) return 0;
  const uint64_t wgs = ((n + 15) / 16 + 3) / 4 + 2;
  return (uint64_t)(wgs < kSpillWGs ? wgs : kSpillWGs) * 4 * kDiffSpill;
}
uint64_t diff_workspace_bytes(uint64_t n) {
  const uint64_t u16 = (n + 15) / 16, u2 = (min(n, kDiffShort) + 1) / 2;
  const uint64_t u1 = diff_variant() == 8 ? n : min(n, kDiffTiny);  // 1-page units
  const uint64_t base = 8 * (1 + max(max(u16, u2), u1)) + 64;
  return up256(base) + up256(4 * (uint64_t)kSpillWGs) + spill_pool_bytes(n);
}

static inline unsigned grid_for(uint64_t work, unsigned per_block, unsigned cap) {
  uint64_t g = (work + per_block - 1) / per_block;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  return (unsigned)g;
}

hipError_t launch_gen_pages(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t n,
                            uint64_t first_global, uint64_t stride, uint64_t seed, int mode,
                            uint32_t ppm, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t chunks = n * 256;
  hipLaunchKernelGGL(gen_pages_kernel, dim3(grid_for(chunks, 256, 65536)), dim3(256), 0, s, twin,
                     cur, replica, chunks, first_global, stride ? stride : 1, seed, mode, ppm);
  return hipGetLastError();
}

hipError_t launch_check_ids(const uint32_t* ids, uint64_t n, uint64_t n_pages, uint32_t* safe,
                            uint32_t* err, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(check_ids_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, ids, n,
                     n_pages, safe, err);
  return hipGetLastError();
}

hipError_t launch_xchg_guard(uint64_t* rec_off, const uint32_t* ids, uint64_t n, uint64_t budget,
                             uint64_t n_pages, uint32_t* safe, uint32_t* verdict, uint32_t* err,
                             hipStream_t s) {
  hipError_t e = hipMemsetAsync(verdict, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  const unsigned g = grid_for(n + 1, 256, 2048);
  hipLaunchKernelGGL(xchg_check_kernel, dim3(g), dim3(256), 0, s, rec_off, ids, n, budget, n_pages,
                     safe, verdict, err);
  hipLaunchKernelGGL(xchg_zero_kernel, dim3(g), dim3(256), 0, s, rec_off, n, verdict);
  return hipGetLastError();
}

hipError_t launch_budget_check(const uint64_t* rec_off, uint64_t n, uint64_t budget,
                               uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(budget_check_kernel, dim3(1), dim3(64), 0, s, rec_off, n, budget, err);
  return hipGetLastError();
}

hipError_t launch_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       hipStream_t s, Prof* prof, uint64_t n_pages, uint32_t* err) {
  if (n == 0) return hipSuccess;
  ProfScope ps(prof, GDSM_PROF_TWIN, s);
  // one page per wave step, cached loads and stores: two or four pages per step and
  // nontemporal loads and/or stores measured 0.3-4.5 % slower in one process (round 4)
  auto kern = twin_kernel<1, 0>;
  hipLaunchKernelGGL(kern, dim3(grid_for(n, 4, 16384)), dim3(256), 0, s, twin, cur, ids, n,
                     n_pages, err);
  return hipGetLastError();
}

// A workgroup copies n words of T, four per lane in flight before their stores (a load-store
// pair per step would wait out one memory latency per step).
template <bool kWT, typename T>
__device__ __forceinline__ void st_word(T* p, const T& v) {
  if constexpr (sizeof(T) == 16) {
    if (kWT)
      st_wt16(p, v);
    else
      *p = v;
  } else {
    st_<kWT>(p, v);
  }
}
template <typename T, bool kWT = false>
__device__ __forceinline__ void copy_words(T* __restrict__ d, const T* __restrict__ s,
                                           uint64_t n) {
  const uint64_t st = blockDim.x;
  uint64_t i = threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    const T a = s[i], b = s[i + st], c = s[i + 2 * st], e = s[i + 3 * st];
    st_word<kWT>(d + i, a);
    st_word<kWT>(d + i + st, b);
    st_word<kWT>(d + i + 2 * st, c);
    st_word<kWT>(d + i + 3 * st, e);
  }
  for (; i < n; i += st) st_word<kWT>(d + i, s[i]);
}

// One (dst, src, bytes) copy by the calling workgroup, in the widest words (16, 8, 4 or 1 B)
// that dst and src are both aligned to, the remainder bytes after them. (Config 5's rows are 8-B
// aligned: copied byte by byte they took 13-16 us of a ~45 us round.)
// kWT: write-through stores (the persistent rounds grid: the release of another workgroup reads
// the bytes after a fence-free barrier). The sources are never written in the launch.
template <bool kWT = false>
__device__ __forceinline__ void copy_desc_wg(const uint64_t* __restrict__ d) {
  {
    uint8_t* dst = reinterpret_cast<uint8_t*>(d[0]);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(d[1]);
    const uint64_t bytes = d[2];
    const uintptr_t al = (uintptr_t)dst | (uintptr_t)src;
    uint64_t done;
    if (!(al & 15u)) {
      copy_words<uint4, kWT>(reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src),
                             bytes / 16);
      done = bytes & ~15ull;
    } else if (!(al & 7u)) {
      copy_words<uint64_t, kWT>(reinterpret_cast<uint64_t*>(dst),
                                reinterpret_cast<const uint64_t*>(src), bytes / 8);
      done = bytes & ~7ull;
    } else if (!(al & 3u)) {
      copy_words<uint32_t, kWT>(reinterpret_cast<uint32_t*>(dst),
                                reinterpret_cast<const uint32_t*>(src), bytes / 4);
      done = bytes & ~3ull;
    } else {
      copy_words<uint8_t, kWT>(dst, src, bytes);
      done = bytes;
    }
    for (uint64_t b = done + threadIdx.x; b < bytes; b += blockDim.x) st_<kWT>(dst + b, src[b]);
  }
}

// n device-to-device copies in one launch (gdsm_memcpy_batch): copy i = desc[3i .. 3i+2] =
// (dst, src, bytes), one workgroup per copy.
__global__ __launch_bounds__(256) void copy_batch_kernel(const uint64_t* __restrict__ desc,
                                                         uint64_t n) {
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) copy_desc_wg(desc + 3 * i);
}

// ---- DSM rounds on the device (gdsm_rounds, page-data side): one persistent launch runs every
// round's row writes (the application's stores, as copy descriptors) and its release (diff of the
// written pages + home apply + re-twin, release_page_wg), a grid barrier between rounds. The
// writes are laid onto the released pages inside the release (kFuse: the workgroup releasing a
// page first applies the round's descriptors that fall on it, in order), so a round is one step:
// separate launches needed a copy, a boundary and the release. Round r's pages are list entries
// [off[r], off[r+1]) of ids / tids (r's records land in the one stream sp describes, as a release
// of those pages would write them), its writes descriptors [doff[r], doff[r+1]).
// Look-back granules carry epoch epoch0 + r (DiffChain's ws and layout; the launcher leaves the
// chain to be zeroed again by its next chained launch). Every byte one workgroup hands another
// (CURRENT rows, TWIN, REPLICA, the stream) is stored write-through and the pages are loaded past
// L1 (kWT), so the barriers need no L2 write-back or L1 invalidate.
// kXcd: the rounds run on a one-XCD team (xcd_team, team control words at bar + 32): every hand-off
// meets in that XCD's L2, so the stores stay plain and the arrivals are L2 atomics.
template <bool kXcd>
__global__ __launch_bounds__(256) void rounds_data_kernel(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, const uint32_t* __restrict__ tids,
    const int64_t* __restrict__ off, const uint64_t* __restrict__ desc,
    const int64_t* __restrict__ doff, uint32_t n_rounds, DiffSplit sp, uint64_t* __restrict__ ws,
    uint8_t* __restrict__ target, IdGuard g, uint32_t epoch0, uint32_t* __restrict__ bar) {
  // bar[0]: barrier arrivals; bar[2..3]: the words laid onto released pages minus the words
  // the descriptors hold (0 at the end, else a write fell outside the released pages)
  unsigned long long* const covered = reinterpret_cast<unsigned long long*>(bar + 2);
  const XcdTeam team = kXcd ? xcd_team(bar + 32, g.err, kErrRoundsBarrier)
                            : XcdTeam{blockIdx.x, gridDim.x};
  if (team.idx == ~0u) return;  // (workgroup-uniform: not on the team's XCD)
  const uint32_t wg = team.idx, nwg = team.n;
  GDSM_RSTAMP_WG(team.idx == 0);
  // member 0's first wave accounts for each round's descriptors (their 8-B words, their
  // alignment), lane-parallel, loaded one round ahead so the loads wait out a barrier
  const bool acct = wg == 0 && threadIdx.x < 64;
  uint32_t acct_words = 0, acct_mis = 0;
  auto acct_load = [&](uint32_t r) {
    acct_words = acct_mis = 0;
    for (uint64_t d = (uint64_t)doff[r] + threadIdx.x; d < (uint64_t)doff[r + 1]; d += 64) {
      const uint64_t dst = desc[3 * d], src = desc[3 * d + 1], bytes = desc[3 * d + 2];
      acct_words += (uint32_t)(bytes / 8);
      acct_mis |= (uint32_t)((dst | src | bytes) & 7u);
    }
  };
  if (acct && n_rounds) acct_load(0);
  // round r's list and descriptor bounds and this workgroup's first list entry, loaded a round
  // ahead (uniform scalar loads: the lists are never written in the launch), so the release's
  // first loads go out as soon as the barrier ends
  RoundWrites rw{desc, 0, 0, covered};
  int64_t next_id = -1;
  uint64_t na = 0, nn = 0, nd0 = 0, nd1 = 0;
  auto load_ahead = [&](uint32_t r) {
    na = (uint64_t)off[r];
    nn = (uint64_t)off[r + 1] - na;
    nd0 = (uint64_t)doff[r];
    nd1 = (uint64_t)doff[r + 1];
    next_id = wg < nn ? (int64_t)ids[na + wg] : -1;
  };
  if (n_rounds) load_ahead(0);
  uint32_t phase = 0;
  for (uint32_t r = 0; r < n_rounds; ++r) {
    GDSM_RSTAMP(0, r, 0);
    const uint64_t a = na, n = nn;
    rw.d0 = nd0;
    rw.d1 = nd1;
    if (acct) {
      const uint32_t words = wave_sum(acct_words);
      if (threadIdx.x == 0 && words) atomicAdd(covered, 0ull - (unsigned long long)words);
      if (__ballot(acct_mis != 0) && threadIdx.x == 0 && g.err) atomicOr(g.err, kErrRoundsWrites);
    }
    DiffSplit rs = sp;
    rs.first[0] = 0;
    rs.first[1] = n;
    rs.epoch = epoch0 + r;
    GDSM_RSTAMP(0, r, 1);
    GDSM_RSTAMP(0, r, 2);
    for (uint64_t u = wg; u < n; u += nwg) {
      release_page_wg<true, true, true, true, kXcd>(u, twin, cur, ids + a, rs, ws, target,
                                                    tids + a, g, rw, u == wg ? next_id : -1);
      __syncthreads();  // (the page's LDS exchange is reused by the workgroup's next page)
    }
    if (n == 0 && wg == 0 && threadIdx.x == 0) st_<!kXcd>(rs.rec_off[0], (uint64_t)0);
    GDSM_RSTAMP(0, r, 3);
    grid_arrive_wt<kXcd>(bar);
    if (acct && r + 1 < n_rounds) acct_load(r + 1);
    if (r + 1 < n_rounds) load_ahead(r + 1);  // (landed by the barrier's end)
    grid_wait_wt(bar, ++phase * nwg, g.err, kErrRoundsBarrier);
  }
  if (wg == 0 && threadIdx.x == 0 && g.err &&
      __hip_atomic_load(covered, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
    atomicOr(g.err, kErrRoundsWrites);
}

const void* rounds_data_kernel_ptr(bool xcd) {
  return xcd ? reinterpret_cast<const void*>(rounds_data_kernel<true>)
             : reinterpret_cast<const void*>(rounds_data_kernel<false>);
}

hipError_t launch_rounds_data(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                              const uint32_t* tids, const int64_t* off, const uint64_t* desc,
                              const int64_t* doff, uint32_t n_rounds, uint32_t grid,
                              uint64_t* rec_off, uint8_t* data, uint64_t cap, uint64_t* chain_ws,
                              uint8_t* target, uint64_t n_pages, uint32_t* err, uint32_t epoch0,
                              uint32_t* bar, bool xcd, hipStream_t s, Prof* prof) {
  if (n_rounds == 0) return hipSuccess;
  DiffSplit sp{};
  sp.G = 1;
  sp.rec_off[0] = rec_off;
  sp.data[0] = data;
  sp.cap[0] = cap;
  const IdGuard g{ids, tids, nullptr, nullptr, n_pages, err};
  // arrivals, the coverage count and the team's control words (bar + 32)
  hipError_t e = hipMemsetAsync(bar, 0, kRoundsBarBytes, s);
  if (e != hipSuccess) return e;
  ProfScope ps(prof, GDSM_PROF_DIFF, s);
  hipLaunchKernelGGL(xcd ? rounds_data_kernel<true> : rounds_data_kernel<false>, dim3(grid),
                     dim3(256), 0, s, twin, cur, ids, tids, off, desc, doff, n_rounds, sp, chain_ws,
                     target, g, epoch0, bar);
  return hipGetLastError();
}

hipError_t launch_copy_batch(const uint64_t* desc, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(copy_batch_kernel, dim3(grid_for(n, 1, 65536)), dim3(256), 0, s, desc, n);
  return hipGetLastError();
}

static hipError_t launch_diff_impl(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                                   DiffSplit sp, uint8_t* ws, uint64_t ws_bytes, hipStream_t s,
                                   Prof* prof, uint8_t* target, uint32_t bpp_hint, uint64_t cap,
                                   const uint32_t* tids, const IdGuard* guard, uint8_t* retwin,
                                   DiffChain* chain = nullptr);

uint64_t diff_chain_bytes() { return 8 * (1 + kDiffChainUnits); }

hipError_t launch_diff(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       uint64_t* rec_off, uint8_t* data, uint64_t cap, uint8_t* ws,
                       uint64_t ws_bytes, hipStream_t s, Prof* prof, uint8_t* target,
                       uint32_t bpp_hint, const uint32_t* tids, const IdGuard* guard,
                       uint8_t* retwin, DiffChain* chain) {
  if (n == 0) return hipMemsetAsync(rec_off, 0, sizeof(uint64_t), s);
  DiffSplit sp{};
  sp.G = 1;
  sp.rec_off[0] = rec_off;
  sp.data[0] = data;
  sp.cap[0] = cap;
  sp.first[0] = 0;
  sp.first[1] = n;
  return launch_diff_impl(twin, cur, ids, sp, ws, ws_bytes, s, prof, target, bpp_hint, cap, tids,
                          guard, retwin, chain);
}

hipError_t launch_diff_split(const uint8_t* twin, const uint8_t* cur, DiffSplit sp, uint8_t* ws,
                             uint64_t ws_bytes, hipStream_t s, Prof* prof, uint32_t bpp_hint) {
  if (sp.G < 1 || sp.G > kMaxSplit) return hipErrorInvalidValue;
  uint64_t mincap = ~0ull;
  for (uint32_t d = 0; d < sp.G; ++d) {
    if (sp.first[d + 1] < sp.first[d]) return hipErrorInvalidValue;
    mincap = sp.cap[d] < mincap ? sp.cap[d] : mincap;
    if (sp.first[d + 1] == sp.first[d]) {  // an empty stream: rec_off[0] = 0, no work unit
      const hipError_t e = hipMemsetAsync(sp.rec_off[d], 0, sizeof(uint64_t), s);
      if (e != hipSuccess) return e;
    }
  }
  if (sp.first[sp.G] == sp.first[0]) return hipSuccess;
  return launch_diff_impl(twin, cur, nullptr, sp, ws, ws_bytes, s, prof, nullptr, bpp_hint,
                          mincap, nullptr, nullptr, nullptr);
}

// `cap` (the smallest stream capacity) only matters to workspaces that predate the spill pool.
static hipError_t launch_diff_impl(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                                   DiffSplit sp, uint8_t* ws, uint64_t ws_bytes, hipStream_t s,
                                   Prof* prof, uint8_t* target, uint32_t bpp_hint, uint64_t cap,
                                   const uint32_t* tids, const IdGuard* guard, uint8_t* retwin,
                                   DiffChain* chain) {
  const uint64_t n = sp.first[sp.G] - sp.first[0];
  if (retwin && sp.G != 1) return hipErrorInvalidValue;
  int v = diff_variant();
  // the spill pool's place in the workspace (after the largest status area n may need)
  const uint64_t u1 = v == 8 ? n : min(n, kDiffTiny);
  const uint64_t status_end =
      up256(8 * (1 + max(max((n + 15) / 16, (min(n, kDiffShort) + 1) / 2), u1)) + 64);
  const uint64_t pool_at = status_end + up256(4 * (uint64_t)kSpillWGs);
  const bool pool_ok = ws_bytes >= pool_at + spill_pool_bytes(n);
  if (v == 0) {
    if (n <= kDiffTiny)
      v = 8;
    else if (n <= kDiffShort)
      v = 3;
    else if (bpp_hint)  // the density this context saw last: sparse -> 64 pages, denser -> 16
      v = bpp_hint <= kDense64 ? (pool_ok ? 5 : 4) : bpp_hint <= kDense16 || !pool_ok ? 1 : 7;
    else  // unknown density: 64 pages with the spill slot, valid at any density
      v = pool_ok ? 5 : (cap <= 128 * n) ? 4 : (cap <= 384 * n) ? 2 : 1;
  }
  const bool spill = v >= 5 && v <= 7;  // 8: one page per wave, no spill slot
  if (spill && !pool_ok) return hipErrorInvalidValue;
  const uint32_t U = (v == 4 || v == 5) ? 64 : v == 3 ? 2 : v == 8 ? 1 : (v == 2 || v == 6) ? 32 : 16;
  sp.ustart[0] = 0;
  for (uint32_t d = 0; d < sp.G; ++d)
    sp.ustart[d + 1] = sp.ustart[d] + (sp.first[d + 1] - sp.first[d] + U - 1) / U;
  const uint64_t nunits = sp.ustart[sp.G];
  if ((1 + nunits) * 8 > ws_bytes) return hipErrorInvalidValue;
  // every workgroup's spill slot (ticket % kSpillWGs) lies inside the pool
  const uint64_t wgs = (nunits + 3) / 4;
  if (spill && (wgs < kSpillWGs ? wgs : kSpillWGs) * 4 * kDiffSpill > spill_pool_bytes(n))
    return hipErrorInvalidValue;
  uint32_t* gen = spill ? reinterpret_cast<uint32_t*>(ws + status_end) : nullptr;
  // short lists: the chained launch (when the context offers it) from solo_max + 1 units, the
  // one-workgroup launch below (up to kSoloUnits without the chain)
  const bool chain_ok = v == 8 && sp.G == 1 && chain && chain->ws && nunits <= kDiffChainUnits &&
                        g_chain.load(std::memory_order_relaxed);
  const uint64_t solo_max =
      chain_ok ? (uint64_t)g_solo_max.load(std::memory_order_relaxed) : (uint64_t)kSoloUnits;
  if (v == 8 && sp.G == 1 && nunits <= solo_max) {
    // one workgroup, no workspace: the caller's lists are guarded by the kernel itself
    const IdGuard g = guard ? *guard : IdGuard{};
    ProfScope ps(prof, GDSM_PROF_DIFF, s);
    auto kern = retwin ? (target ? diff_single_kernel<1, 4096, 4, true, 0, true, true>
                                 : diff_single_kernel<1, 4096, 4, false, 0, true, true>)
                       : (target ? diff_single_kernel<1, 4096, 4, true, 0, true>
                                 : diff_single_kernel<1, 4096, 4, false, 0, true>);
    hipLaunchKernelGGL(kern, dim3(1), dim3((unsigned)(64 * nunits)), 0, s, twin, cur, ids, sp,
                       reinterpret_cast<uint64_t*>(ws), target, nullptr, nullptr, tids, g);
    return hipGetLastError();
  }
  if (chain_ok) {
    // one launch: epoch-tagged granules, the caller's lists guarded by the kernel (DiffChain)
    if (chain->epoch == 0) {
      const hipError_t e = hipMemsetAsync(chain->ws, 0, diff_chain_bytes(), s);
      if (e != hipSuccess) return e;
      chain->epoch = 1;
    }
    sp.epoch = chain->epoch;
    const IdGuard g = guard ? *guard : IdGuard{};
    ProfScope ps(prof, GDSM_PROF_DIFF, s);
    const int cw = g_chain.load(std::memory_order_relaxed);
    if (cw == 3 || (cw == 2 && nunits <= kChainPerPage)) {  // a page per four-wave workgroup
      auto kp = retwin ? (target ? release_page_kernel<true, true> : release_page_kernel<false, true>)
                       : (target ? release_page_kernel<true, false> : release_page_kernel<false, false>);
      hipLaunchKernelGGL(kp, dim3((unsigned)nunits), dim3(256), 0, s, twin, cur, ids, sp, chain->ws,
                         target, tids, g);
      const hipError_t e = hipGetLastError();
      chain->epoch = e != hipSuccess || chain->epoch + 1 >= (1u << 30) ? 0 : chain->epoch + 1;
      return e;
    }
    const uint32_t W = cw == 1 ? 1 : 4;  // waves per workgroup
#ifdef GDSM_MEASURE
    if (g_diff_skip.load(std::memory_order_relaxed) && retwin && target && W == 1) {
      const int k = g_diff_skip.load(std::memory_order_relaxed);
      auto km = k == 1   ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 1>
                : k == 2  ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 2>
                : k == 4  ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 4>
                : k == 5  ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 5>
                : k == 8  ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 8>
                : k == 13 ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 13>
                : k == 16 ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 16>
                : k == 32 ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 32>
                          : diff_single_kernel<1, 8192, 4, true, 0, false, true, 1, 61>;
      hipLaunchKernelGGL(km, dim3((unsigned)nunits), dim3(64), 0, s, twin, cur, ids, sp, chain->ws,
                         target, nullptr, nullptr, tids, g);
      const hipError_t e = hipGetLastError();
      chain->epoch = e != hipSuccess || chain->epoch + 1 >= (1u << 30) ? 0 : chain->epoch + 1;
      return e;
    }
#endif
    auto kern = W == 1 ? (retwin ? (target ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 1>
                                           : diff_single_kernel<1, 8192, 4, false, 0, false, true, 1>)
                                 : (target ? diff_single_kernel<1, 8192, 4, true, 0, false, false, 1>
                                           : diff_single_kernel<1, 8192, 4, false, 0, false, false, 1>))
                       : (retwin ? (target ? diff_single_kernel<1, 8192, 4, true, 0, false, true, 4>
                                           : diff_single_kernel<1, 8192, 4, false, 0, false, true, 4>)
                                 : (target ? diff_single_kernel<1, 8192, 4, true, 0, false, false, 4>
                                           : diff_single_kernel<1, 8192, 4, false, 0, false, false, 4>));
    hipLaunchKernelGGL(kern, dim3((unsigned)((nunits + W - 1) / W)), dim3(64 * W), 0, s, twin, cur,
                       ids, sp, chain->ws, target, nullptr, nullptr, tids, g);
    const hipError_t e = hipGetLastError();
    // a launch that did not run leaves its successor's counter unzeroed: start the chain over
    chain->epoch = e != hipSuccess || chain->epoch + 1 >= (1u << 30) ? 0 : chain->epoch + 1;
    return e;
  }
  // ticket counter + status granules (+ the spill slots' generation words), zeroed per launch
  // (outside the timed kernel), and the caller's lists checked, in one prep launch
  IdGuard g{};
  {
    if (guard) {
      g = *guard;
      if (g.ids) ids = g.safe_ids;
      if (g.tids) tids = g.safe_tids;
    }
    const uint64_t nz = 1 + nunits, nchk = (g.ids || g.tids) ? n : 0;
    const uint64_t work = nz > nchk ? nz : nchk;
    hipLaunchKernelGGL(diff_prep_kernel, dim3(grid_for(work, 256, 1024)), dim3(256), 0, s,
                       reinterpret_cast<uint64_t*>(ws), nz, gen, spill ? (uint64_t)kSpillWGs : 0,
                       g, nchk);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  uint8_t* pool = spill ? ws + pool_at : nullptr;
  ProfScope ps(prof, GDSM_PROF_DIFF, s);
  auto kern = target ? (v == 5   ? diff_single_kernel<64, 8192, 4, true, kDiffSpill>
                       : v == 6 ? diff_single_kernel<32, 8192, 4, true, kDiffSpill>
                       : v == 7 ? diff_single_kernel<16, 8192, 4, true, kDiffSpill>
                       : v == 4 ? diff_single_kernel<64, 8192, 4, true>
                       : v == 3 ? diff_single_kernel<2, 8192, 4, true>
                       : v == 8 ? diff_single_kernel<1, 8192, 4, true>
                       : v == 2 ? diff_single_kernel<32, 8192, 4, true>
                                : diff_single_kernel<16, 8192, 4, true>)
                     : (v == 5   ? diff_single_kernel<64, 8192, 4, false, kDiffSpill>
                       : v == 6 ? diff_single_kernel<32, 8192, 4, false, kDiffSpill>
                       : v == 7 ? diff_single_kernel<16, 8192, 4, false, kDiffSpill>
                       : v == 4 ? diff_single_kernel<64, 8192, 4, false>
                       : v == 3 ? diff_single_kernel<2, 8192, 4, false>
                       : v == 8 ? diff_single_kernel<1, 8192, 4, false>
                       : v == 2 ? diff_single_kernel<32, 8192, 4, false>
                                : diff_single_kernel<16, 8192, 4, false>);
  // one-page units with room for every record re-twin inside the kernel; otherwise a second
  // launch once the diff has read every twin page (late pages of longer units are re-read)
  const bool retwin_in = retwin && U == 1 && sp.cap[0] >= n * (uint64_t)GDSM_MAX_RECORD;
  if (retwin_in)
    kern = target ? diff_single_kernel<1, 8192, 4, true, 0, false, true>
                  : diff_single_kernel<1, 8192, 4, false, 0, false, true>;
  // (the lists are checked already: the kernel only learns n_pages, for twin_ok)
  const IdGuard gn{nullptr, nullptr, nullptr, nullptr, g.n_pages, nullptr};
  hipLaunchKernelGGL(kern, dim3((unsigned)((nunits + 3) / 4)), dim3(256), 0, s, twin, cur, ids, sp,
                     reinterpret_cast<uint64_t*>(ws), target, gen, pool, tids, gn);
  if (retwin && !retwin_in) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(retwin_kernel, dim3(grid_for(n, 4, 16384)), dim3(256), 0, s, retwin, cur,
                       ids, n, sp.rec_off[0], sp.cap[0], g.n_pages);
  }
  return hipGetLastError();
}

hipError_t launch_apply(uint8_t* target, const uint32_t* ids, uint64_t n,
                        const uint64_t* rec_off, const uint8_t* data, uint32_t* err,
                        hipStream_t s, Prof* prof) {
  if (n == 0) return hipSuccess;
  ProfScope ps(prof, GDSM_PROF_APPLY, s);
  // one task per wave, 4 waves per workgroup: no workgroup launched without work. A task is 64
  // records (one staging window serves many small records); short lists take 4 per task, so a
  // few dense records are spread over waves instead of queueing in one
  const bool short_list = n <= 16384;
  const uint32_t per_task = short_list ? 4u : 64u;
  const int av = g_apply_variant.load(std::memory_order_relaxed);
  if (n <= kApplyTiny && av == 0) {
    hipLaunchKernelGGL(apply_tiny_kernel<0>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s,
                       target, ids, n, rec_off, data, err);
    return hipGetLastError();
  }
  if (!short_list && (av == 0 || av >= 3)) {
    auto kf = av == 0 ? apply_flat_kernel<4096, true, 1>
              : av == 3 ? apply_flat_kernel<8192, true, 1>
              : av == 5 ? apply_flat_kernel<4096, false, 1>
              : av == 6 ? apply_flat_kernel<4096, true, 2>
              : av == 7 ? apply_flat_kernel<4096, true, 0>
                        : apply_flat_kernel<2048, true, 1>;
    hipLaunchKernelGGL(kf, dim3(grid_for(n, 4 * 64, 65536)), dim3(256), 0, s, target, ids, n,
                       rec_off, data, err);
    return hipGetLastError();
  }
  auto kern = short_list ? apply_kernel<0, kApplyWinShort>
              : av == 2  ? apply_kernel<0, 4096>
                         : apply_kernel<0, kApplyWinLong>;
  hipLaunchKernelGGL(kern, dim3(grid_for(n, 4 * per_task, 65536)), dim3(256), 0, s, target, ids,
                     n, rec_off, data, err, per_task);
  return hipGetLastError();
}

}  // namespace gdsm

#ifdef GDSM_ROUNDS_STAMPS
extern "C" int gdsm_debug_round_stamps(void* out, size_t bytes) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gdsm::g_round_stamps), bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -5;
}
#endif
