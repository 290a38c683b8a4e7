// gdsm page kernels for gfx950: synthetic pages, twin, run diff (SPEC §3), apply (SPEC §4).
//
// Replaces the twin/diff/apply step of gallocy's described-but-unimplemented DSM flow
// (resources/NUTSHELL.md:59-69); the only diff in the reference is the NW alignment
// gallocy/utils/diff.cpp:73-167, see legacy_diff.cpp.
//
// Diff pipeline (all HBM-bound, no MFMA):
//   1. diff_pages_kernel   one wave per page: 4 x 16 B coalesced loads of twin and current per
//                          lane, 16-bit byte-diff mask per 16-B chunk, run starts/ends from the
//                          neighbour chunk's edge bit (shuffles), ranks by wave prefix sums;
//                          the record goes to the page's fixed slot of the workspace, its size
//                          to sizes[], the workgroup's sum to block_sum[].
//   2. scan_blocks_kernel  one workgroup: exclusive scan of block_sum -> block_off.
//   3. pack_kernel         per workgroup: page offsets inside the block -> rec_off, then
//                          copies each record from its slot to its packed place.
// No workgroup waits on another, so nothing can hang on dispatch order.
#include "gdsm_common.h"
#include "gdsm_launch.h"

#include <stdlib.h>
#include <string.h>

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
__global__ __launch_bounds__(256) void twin_kernel(uint8_t* __restrict__ twin,
                                                   const uint8_t* __restrict__ cur,
                                                   const uint32_t* __restrict__ ids, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n;
       i += (uint64_t)gridDim.x * 4) {
    const uint64_t p = ids ? ids[i] : i;
    const uint4* src = reinterpret_cast<const uint4*>(cur + p * kPage);
    uint4* dst = reinterpret_cast<uint4*>(twin + p * kPage);
    const uint4 a = src[lane], b = src[lane + 64], c = src[lane + 128], d = src[lane + 192];
    dst[lane] = a;
    dst[lane + 64] = b;
    dst[lane + 128] = c;
    dst[lane + 192] = d;
  }
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
    hdr[r++] = start | ((pos + b - start + 1u) << 16);
  }
  uint32_t q = excl >> 16;
  while (m) {
    const uint32_t b = (uint32_t)__builtin_ctz(m);
    m &= m - 1;
    pay[q++] = (uint8_t)byte_of(c, b);
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

// Diffs one page held in registers (chunk (k, lane) = bytes [(64k + lane) * 16, +16), page
// order = (k, lane)); writes its record to `out` and returns the record size (wave-uniform).
constexpr uint32_t kDiffStage = 2048;  // per-wave LDS record stage (bytes)

template <bool kWrite>
__device__ __forceinline__ uint32_t diff_one(const uint4 (&t)[4], const uint4 (&c)[4],
                                             uint32_t lane, uint8_t* __restrict__ out,
                                             uint32_t* __restrict__ stage) {
  uint32_t m[4], s[4], e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = diffmask16(t[k], c[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // neighbour chunks' edge bytes: lane-1 / lane+1 of the same k, wrapping across k
    uint32_t up = from_prev_lane(m[k]);
    uint32_t dn = from_next_lane(m[k]);
    if (k > 0 && lane == 0) up = lane_bcast(m[k > 0 ? k - 1 : 0], 63);
    if (k < 3 && lane == 63) dn = lane_bcast(m[k < 3 ? k + 1 : 3], 0);
    s[k] = m[k] & ~((m[k] << 1) | ((up >> 15) & 1u)) & 0xFFFFu;   // first byte of a run
    e[k] = m[k] & ~((m[k] >> 1) | ((dn & 1u) << 15)) & 0xFFFFu;   // last byte of a run
  }
  // Ranks: runs (counted at their ends) in the low 16 bits, payload bytes in the high 16.
  uint32_t excl[4], ps[4], carry = 0, cmax = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t v = (uint32_t)__popc(e[k]) | ((uint32_t)__popc(m[k]) << 16);
    const uint32_t inc = wave_incl_sum(v);
    excl[k] = carry + inc - v;
    carry += lane_bcast(inc, 63);
    const uint32_t pos = (uint32_t)(k * 64 + lane) * 16u;
    const uint32_t ls = s[k] ? pos + 32u - (uint32_t)__builtin_clz(s[k]) : 0u;  // last start + 1
    const uint32_t mx = wave_incl_max(ls);
    ps[k] = max(cmax, from_prev_lane(mx));
    cmax = max(cmax, lane_bcast(mx, 63));
  }
  const uint32_t NR = carry & 0xFFFFu, NP = carry >> 16;
  if (NR == 0) return 0;
  const uint32_t size = 4u + 4u * NR + ((NP + 3u) & ~3u);
  if (!kWrite) {  // measurement variant: keep the emit work's inputs alive, store nothing
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) h ^= s[k] ^ e[k] ^ ps[k] ^ excl[k] ^ c[k].x;
    return size + ((wave_sum(h) == 0x9E3779B9u) ? 4u : 0u);
  }
  // Assemble the record in the wave's LDS stage when it fits, then write it with 16-B stores
  // (a handful of VMEM instructions instead of one per header and per payload byte).
  const bool staged = stage != nullptr && size <= kDiffStage;
  uint8_t* rec = staged ? reinterpret_cast<uint8_t*>(stage) : out;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(rec + 4);
  uint8_t* pay = rec + 4 + 4 * NR;
  if (lane == 0) {
    *reinterpret_cast<uint32_t*>(rec) = NR;
    for (uint32_t q = NP; q & 3u; ++q) pay[q] = 0;  // zero padding
  }
  emit_chunk(0 * 64 + lane, s[0], e[0], m[0], ps[0], excl[0], c[0], hdr, pay);
  emit_chunk(1 * 64 + lane, s[1], e[1], m[1], ps[1], excl[1], c[1], hdr, pay);
  emit_chunk(2 * 64 + lane, s[2], e[2], m[2], ps[2], excl[2], c[2], hdr, pay);
  emit_chunk(3 * 64 + lane, s[3], e[3], m[3], ps[3], excl[3], c[3], hdr, pay);
  if (staged) {
    wave_lds_sync();
    const uint4* src = reinterpret_cast<const uint4*>(stage);
    uint4* dst = reinterpret_cast<uint4*>(out);
    for (uint32_t q = lane; q < (size + 15u) / 16u; q += 64) dst[q] = src[q];
    wave_lds_sync();
  }
  return size;
}

// One workgroup = 4 waves = kDiffPagesPerBlock consecutive pages; wave w takes the 16 pages
// [16w, 16w + 16) of the block in order and appends their records, each rounded up to 16 B, to
// its own region of the workspace (16 slots = the worst case): every wave writes one contiguous,
// 16-B aligned stream, so partially written cache lines merge in L2 instead of going to HBM as
// one partial line per record, and the pack kernel reads near-contiguous memory.
// kVar (gdsm_tune "diff_variant"; in-process A/B, scripts/ab_diff.py):
//   0  records assembled in the wave's LDS stage, written with 16-B stores (default)
//   1  records written straight from the lanes (per-header / per-byte stores)
//   2  as 0, and the next page's 8 loads issued before the current page is processed
//   3  MEASUREMENT ONLY: full diff, records not written (sizes only) -- output is invalid
//   4  MEASUREMENT ONLY: loads + a change count per page -- the read roofline of this kernel
//   5  as 0, register budget capped at 64 VGPRs (8 waves/SIMD)
template <int kVar>
__device__ __forceinline__ void diff_pages_body(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, uint64_t first, uint64_t n, uint8_t* __restrict__ ws,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ block_sum) {
  constexpr bool kPrefetch = kVar == 2;
  constexpr bool kStage = kVar == 0 || kVar == 2 || kVar == 5;
  __shared__ uint32_t wsum[4];
  __shared__ __attribute__((aligned(16))) uint32_t stage_all[kStage ? 4 : 1][kStage ? kDiffStage / 4 : 1];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* stage = kStage ? stage_all[kStage ? wave : 0] : nullptr;
  const uint64_t w0 = (uint64_t)blockIdx.x * kDiffPagesPerBlock + wave * kDiffPagesPerWave;
  uint8_t* region = ws + w0 * kRecSlot;
  uint32_t acc = 0, acc16 = 0;
  uint4 t[4], c[4];
  if (kPrefetch && w0 < n) load_page(twin, cur, ids ? ids[first + w0] : first + w0, lane, t, c);
  for (uint32_t j = 0; j < kDiffPagesPerWave; ++j) {
    const uint64_t i = w0 + j;  // index within chunk
    if (i >= n) break;
    if (!kPrefetch) load_page(twin, cur, ids ? ids[first + i] : first + i, lane, t, c);
    uint4 tn[4], cn[4];
    const bool nx = kPrefetch && j + 1 < kDiffPagesPerWave && i + 1 < n;
    if (nx) load_page(twin, cur, ids ? ids[first + i + 1] : first + i + 1, lane, tn, cn);
    uint32_t size;
    if constexpr (kVar == 4) {
      uint32_t d = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        d |= (t[k].x ^ c[k].x) | (t[k].y ^ c[k].y) | (t[k].z ^ c[k].z) | (t[k].w ^ c[k].w);
      size = wave_sum(d ? 1u : 0u);
    } else if constexpr (kVar == 3) {
      size = diff_one<false>(t, c, lane, nullptr, nullptr);
    } else {
      size = diff_one<true>(t, c, lane, region + acc16, stage);
    }
    if (lane == 0) sizes[i] = size;
    acc += size;
    acc16 += (size + 15u) & ~15u;
    if (kPrefetch) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t[k] = tn[k];
        c[k] = cn[k];
      }
    }
  }
  if (lane == 0) wsum[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) block_sum[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

template <int kVar>
__global__ __launch_bounds__(256) void diff_pages_kernel(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, uint64_t first, uint64_t n, uint8_t* __restrict__ ws,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ block_sum) {
  diff_pages_body<kVar>(twin, cur, ids, first, n, ws, sizes, block_sum);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void
diff_pages_kernel_o8(const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
                     const uint32_t* __restrict__ ids, uint64_t first, uint64_t n,
                     uint8_t* __restrict__ ws, uint32_t* __restrict__ sizes,
                     uint32_t* __restrict__ block_sum) {
  diff_pages_body<5>(twin, cur, ids, first, n, ws, sizes, block_sum);
}

// One workgroup: block_off[b] = base + sum(block_sum[0..b)), base = rec_off[first].
__global__ __launch_bounds__(1024) void scan_blocks_kernel(const uint32_t* __restrict__ block_sum,
                                                           uint64_t nb,
                                                           const uint64_t* __restrict__ base_ptr,
                                                           uint64_t* __restrict__ block_off) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t lo = min(nb, (uint64_t)t * per), hi = min(nb, lo + per);
  uint64_t s = 0;
  for (uint64_t b = lo; b < hi; ++b) s += block_sum[b];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint64_t v = (t >= d) ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = (base_ptr ? *base_ptr : 0) + part[t] - s;
  for (uint64_t b = lo; b < hi; ++b) {
    block_off[b] = run;
    run += block_sum[b];
  }
}

// Per workgroup (64 pages): page offsets inside the block -> rec_off; then every thread copies
// output dwords of the block's packed range, finding each dword's record by binary search over
// the 65 block-relative offsets in LDS (all loads independent, stores contiguous). A record's
// source is its wave region (diff_pages_body) at the 16-B rounded prefix `src` of its row.
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ ws,
                                                   const uint32_t* __restrict__ sizes,
                                                   const uint64_t* __restrict__ block_off,
                                                   uint64_t first, uint64_t n,
                                                   uint64_t* __restrict__ rec_off,
                                                   uint8_t* __restrict__ data, uint64_t cap) {
  __shared__ uint32_t off[kDiffPagesPerBlock + 1];
  __shared__ uint32_t src[kDiffPagesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kDiffPagesPerBlock;
  const uint64_t base = block_off[blockIdx.x];
  if (wave == 0) {
    static_assert(kDiffPagesPerWave == 16, "one DPP row per wave region");
    const uint64_t i = b0 + lane;
    const uint32_t sz = (i < n) ? sizes[i] : 0u;
    const uint32_t inc = wave_incl_sum(sz);
    const uint32_t s16 = (sz + 15u) & ~15u;
    src[lane] = row_incl_sum(s16) - s16;
    off[lane] = inc - sz;
    if (lane == 63) off[64] = inc;
    if (i < n) rec_off[first + i + 1] = base + inc;
    if (first == 0 && blockIdx.x == 0 && lane == 0) rec_off[0] = 0;
  }
  __syncthreads();
  // Only records that end inside the capacity are copied.
  uint32_t limit = off[64];
  if (base + limit > cap) {
    limit = 0;
    for (uint32_t r = 0; r < kDiffPagesPerBlock; ++r)
      if (base + off[r + 1] <= cap) limit = off[r + 1];
  }
  uint32_t* dst = reinterpret_cast<uint32_t*>(data + base);
  for (uint32_t g = threadIdx.x; g < limit / 4; g += 256) {
    const uint32_t byte = g * 4;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
      if (off[r + step] <= byte) r += step;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(
        ws + (b0 + (r & ~(kDiffPagesPerWave - 1))) * kRecSlot + src[r] + (byte - off[r]));
    dst[g] = *p;
  }
}

// ------------------------------------------------------------------------- apply (SPEC §4)
// A wave takes 64 consecutive records. It stages as many of them as fit in an 8 KiB LDS window
// with coalesced loads (one global round trip for the whole window), then handles them one by
// one out of LDS: the run list becomes the page's 4096-bit dirty mask by toggling a bit at each
// run start and end and taking a prefix-XOR (lane l owns bytes [64l, 64l+64)); the payload index
// of a byte is the popcount of the dirty bits before it. The replica is only STORED to (16-B
// stores for whole chunks, dword stores for whole dwords, byte stores otherwise), never read, so
// no wave ever waits on a replica load. A record larger than the window is read from global.
constexpr uint32_t kApplyWin = 8192;  // bytes of records staged per wave

// Stores the payload bytes selected by `mask` (16 bits, chunk of 16 B at dst) from pay[pp..].
template <typename P8>
__device__ __forceinline__ void store_chunk(uint8_t* __restrict__ dst, uint32_t mask, P8 pay,
                                            uint32_t pp) {
  if (mask == 0xFFFFu) {
    uint32_t w[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
      w[d] = (uint32_t)pay[pp + 4 * d] | ((uint32_t)pay[pp + 4 * d + 1] << 8) |
             ((uint32_t)pay[pp + 4 * d + 2] << 16) | ((uint32_t)pay[pp + 4 * d + 3] << 24);
    *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
    return;
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t nib = (mask >> (4 * d)) & 0xFu;
    if (nib == 0xFu) {
      const uint32_t v = (uint32_t)pay[pp] | ((uint32_t)pay[pp + 1] << 8) |
                         ((uint32_t)pay[pp + 2] << 16) | ((uint32_t)pay[pp + 3] << 24);
      *reinterpret_cast<uint32_t*>(dst + 4 * d) = v;
      pp += 4;
    } else if (nib) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((nib >> k) & 1u) dst[4 * d + k] = pay[pp++];
    }
  }
}

// Stores the run bytes that fall into one 16-B destination chunk: chunk [cs, cs+16) of `page`,
// run [off, end), payload of the run starting at pay[pp].
template <typename P8>
__device__ __forceinline__ void store_run_chunk(uint8_t* __restrict__ page, uint32_t cs,
                                                uint32_t off, uint32_t end, P8 pay, uint32_t pp) {
  const uint32_t lo = max(off, cs), hi = min(end, cs + 16u);
  const uint32_t mask = ((hi - cs >= 16u) ? 0xFFFFu : ((1u << (hi - cs)) - 1u)) &
                        ~((1u << (lo - cs)) - 1u);
  store_chunk(page + cs, mask, pay, pp + (lo - off));
}

// Applies up to four records at once, one per 16-lane DPP row (a lane per run). Pass 1 validates
// every header of the row's record (length, bounds, sorted and non-overlapping, total size), so
// a malformed record writes nothing. Pass 2 spreads the record's (run, 16-B chunk) pairs over
// the row's lanes — a run is found by a 4-step binary search over the row's pair offsets — so
// short and long runs cost the same per byte. `has` is false for rows without a record.
// Returns false in the lanes of a row whose record is malformed.
template <typename P32, typename P8>
__device__ __forceinline__ bool apply_rows(uint8_t* __restrict__ page, P32 rec32, P8 rec8,
                                           uint32_t size, bool has) {
  const uint32_t lane = lane_id(), lr = lane & 15, rb = lane & ~15u;
  uint32_t nr = has ? rec32[0] : 0u;
  bool bad = has && (nr == 0 || nr > kMaxRuns || size < 4u + 4u * nr);
  if (bad) nr = 0;
  const uint32_t nit = lane_bcast(wave_incl_max((nr + 15u) >> 4), 63);
  uint32_t pay = 0, prev_end = 0, lbad = 0;
  for (uint32_t it = 0; it < nit; ++it) {
    const uint32_t r = it * 16u + lr;
    const bool v = r < nr;
    const uint32_t h = v ? rec32[1 + r] : 0u;
    const uint32_t off = h & 0xFFFFu, len = h >> 16, end = v ? off + len : 0u;
    uint32_t pe = row_prev(end);
    if (lr == 0) pe = prev_end;
    if (v && (len == 0 || end > kPage || off < pe)) lbad = 1;
    pay += row_last(row_incl_sum(v ? len : 0u));
    prev_end = row_last(end);
  }
  if (row_last(row_incl_max(lbad))) bad = true;
  if (has && !bad && size != 4u + 4u * nr + ((pay + 3u) & ~3u)) bad = true;
  const uint32_t nrw = bad ? 0u : nr;  // runs this row writes
  const uint32_t nit2 = lane_bcast(wave_incl_max((nrw + 15u) >> 4), 63);
  uint32_t pcarry = 0;
  for (uint32_t it = 0; it < nit2; ++it) {
    const uint32_t r = it * 16u + lr;
    const bool v = r < nrw;
    const uint32_t h = v ? rec32[1 + r] : 0u;
    const uint32_t off = h & 0xFFFFu, len = v ? h >> 16 : 0u, end = off + len;
    const uint32_t pinc = row_incl_sum(len);
    const uint32_t pp = 4u + 4u * nr + pcarry + pinc - len;  // payload of this run
    pcarry += row_last(pinc);
    const uint32_t nch = len ? ((end - 1u) >> 4) - (off >> 4) + 1u : 0u;
    const uint32_t cinc = row_incl_sum(nch);
    const uint32_t cex = cinc - nch;
    const uint32_t T = row_last(cinc);
    const uint32_t tmax = lane_bcast(wave_incl_max(T), 63);
    for (uint32_t g = lr; g < ((tmax + 15u) & ~15u); g += 16) {
      uint32_t i = 0;
#pragma unroll
      for (uint32_t step = 8; step; step >>= 1) {
        const uint32_t c = (uint32_t)__shfl(cex, (int)(rb + i + step), 64);
        if (c <= g) i += step;
      }
      const uint32_t oi = (uint32_t)__shfl(off, (int)(rb + i), 64);
      const uint32_t ei = (uint32_t)__shfl(end, (int)(rb + i), 64);
      const uint32_t pi = (uint32_t)__shfl(pp, (int)(rb + i), 64);
      const uint32_t ci = (uint32_t)__shfl(cex, (int)(rb + i), 64);
      if (g < T) store_run_chunk(page, ((oi >> 4) + (g - ci)) << 4, oi, ei, rec8, pi);
    }
  }
  return !bad;
}

__global__ __launch_bounds__(256) void apply_kernel(uint8_t* __restrict__ target,
                                                    const uint32_t* __restrict__ ids, uint64_t n,
                                                    const uint64_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ data,
                                                    uint32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint32_t win_all[4][kApplyWin / 4];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = lane >> 4;
  uint32_t* win = win_all[wave];
  const uint64_t ntask = (n + 63) / 64;
  uint32_t bad = 0;
  for (uint64_t task = (uint64_t)blockIdx.x * 4 + wave; task < ntask;
       task += (uint64_t)gridDim.x * 4) {
    const uint64_t a = task * 64;
    const uint32_t cnt = (uint32_t)min((uint64_t)64, n - a);
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
        if (!apply_rows(target + p * kPage, reinterpret_cast<const uint32_t*>(rec), rec,
                        (uint32_t)(r1 - start), has))
          bad = 1;
        ++j;
        continue;
      }
      const uint64_t stop = (k == 64) ? end_off : lane_bcast64(my_off, k);
      const uint32_t words = (uint32_t)((stop - start) >> 2);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(data + start);
      for (uint32_t q = lane; q < words; q += 64) win[q] = src[q];
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
        if (!apply_rows(target + p * kPage, win + base / 4, win8 + base, (uint32_t)(r1 - r0),
                        has))
          bad = 1;
      }
      wave_lds_sync();
      j = k;
    }
  }
  if (__ballot(bad != 0) && lane == 0) atomicOr(err, 1u);
}

// ------------------------------------------------------------------------- launchers
// Diff kernel variant (see diff_pages_kernel); gdsm_tune("diff_variant", v) or
// GDSM_DIFF_VARIANT=v; used for in-process A/B measurements.
static int g_diff_variant = -1;
static int diff_variant() {
  if (g_diff_variant < 0) {
    const char* e = getenv("GDSM_DIFF_VARIANT");
    g_diff_variant = e ? atoi(e) : 0;
    if (g_diff_variant < 0 || g_diff_variant > 5) g_diff_variant = 0;
  }
  return g_diff_variant;
}
int tune(const char* key, int64_t value) {
  if (!strcmp(key, "diff_variant") && value >= 0 && value <= 5) {
    g_diff_variant = (int)value;
    return 0;
  }
  return -1;
}

uint64_t diff_workspace_bytes(uint64_t n_chunk) {
  const uint64_t nb = (n_chunk + kDiffPagesPerBlock - 1) / kDiffPagesPerBlock;
  return n_chunk * kRecSlot + n_chunk * 4 + nb * 4 + nb * 8 + 64;
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

hipError_t launch_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       hipStream_t s, Prof* prof) {
  if (n == 0) return hipSuccess;
  ProfScope ps(prof, 4, s);
  hipLaunchKernelGGL(twin_kernel, dim3(grid_for(n, 4, 16384)), dim3(256), 0, s, twin, cur, ids,
                     n);
  return hipGetLastError();
}

hipError_t launch_diff(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       uint64_t* rec_off, uint8_t* data, uint64_t cap, uint8_t* ws,
                       uint64_t ws_bytes, hipStream_t s, Prof* prof) {
  if (n == 0) return hipMemsetAsync(rec_off, 0, sizeof(uint64_t), s);
  // Largest chunk whose workspace fits.
  uint64_t chunk = n < kDiffChunk ? n : kDiffChunk;
  while (chunk > kDiffPagesPerBlock && diff_workspace_bytes(chunk) > ws_bytes) chunk >>= 1;
  if (diff_workspace_bytes(chunk) > ws_bytes) return hipErrorInvalidValue;
  const uint64_t nbmax = (chunk + kDiffPagesPerBlock - 1) / kDiffPagesPerBlock;
  uint8_t* slots = ws;
  uint32_t* sizes = reinterpret_cast<uint32_t*>(ws + chunk * kRecSlot);
  uint32_t* block_sum = sizes + chunk;
  uint64_t* block_off =
      reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(block_sum + nbmax) + 15) & ~15ull);
  for (uint64_t first = 0; first < n; first += chunk) {
    const uint64_t m = (n - first < chunk) ? n - first : chunk;
    const uint64_t nb = (m + kDiffPagesPerBlock - 1) / kDiffPagesPerBlock;
    {
      ProfScope ps(prof, 0, s);
      static void (*const kVariants[])(const uint8_t*, const uint8_t*, const uint32_t*, uint64_t,
                                       uint64_t, uint8_t*, uint32_t*, uint32_t*) = {
          diff_pages_kernel<0>, diff_pages_kernel<1>, diff_pages_kernel<2>,
          diff_pages_kernel<3>, diff_pages_kernel<4>, diff_pages_kernel_o8};
      auto kern = kVariants[diff_variant()];
      hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(256), 0, s, twin, cur, ids, first, m,
                         slots, sizes, block_sum);
    }
    {
      ProfScope ps(prof, 1, s);
      hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, s, block_sum, nb,
                         first ? rec_off + first : nullptr, block_off);
    }
    {
      ProfScope ps(prof, 2, s);
      hipLaunchKernelGGL(pack_kernel, dim3((unsigned)nb), dim3(256), 0, s, slots, sizes,
                         block_off, first, m, rec_off, data, cap);
    }
  }
  return hipGetLastError();
}

hipError_t launch_apply(uint8_t* target, const uint32_t* ids, uint64_t n,
                        const uint64_t* rec_off, const uint8_t* data, uint32_t* err,
                        hipStream_t s, Prof* prof) {
  if (n == 0) return hipSuccess;
  ProfScope ps(prof, 3, s);
  hipLaunchKernelGGL(apply_kernel, dim3(grid_for(n, 4, 65536)), dim3(256), 0, s, target, ids, n,
                     rec_off, data, err);
  return hipGetLastError();
}

}  // namespace gdsm
