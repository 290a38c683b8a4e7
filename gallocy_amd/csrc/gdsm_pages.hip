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

// Writes the headers of the runs starting in chunk `ch` and the chunk's changed bytes.
// (Called once per k with scalars, so no per-thread array is ever indexed at run time.)
__device__ __forceinline__ void emit_chunk(uint32_t ch, uint32_t s, uint32_t e, uint32_t m,
                                           uint32_t ne, uint32_t excl, const uint4 c,
                                           uint32_t* __restrict__ hdr, uint8_t* __restrict__ pay) {
  const uint32_t pos = ch * 16u;
  uint32_t r = excl & 0xFFFFu;
  while (s) {
    const uint32_t b = (uint32_t)__builtin_ctz(s);
    s &= s - 1;
    const uint32_t later = (e >> b) << b;
    const uint32_t end = later ? pos + (uint32_t)__builtin_ctz(later) : ne;
    hdr[r++] = (pos + b) | ((end - pos - b + 1u) << 16);
  }
  uint32_t q = excl >> 16;
  while (m) {
    const uint32_t b = (uint32_t)__builtin_ctz(m);
    m &= m - 1;
    pay[q++] = (uint8_t)byte_of(c, b);
  }
}

__global__ __launch_bounds__(256) void diff_pages_kernel(
    const uint8_t* __restrict__ twin, const uint8_t* __restrict__ cur,
    const uint32_t* __restrict__ ids, uint64_t first, uint64_t n, uint8_t* __restrict__ ws,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ block_sum) {
  __shared__ uint32_t wsum[4];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (uint32_t j = wave; j < kDiffPagesPerBlock; j += 4) {
    const uint64_t i = (uint64_t)blockIdx.x * kDiffPagesPerBlock + j;  // index within chunk
    if (i >= n) break;
    const uint64_t p = ids ? ids[first + i] : first + i;
    const uint4* T = reinterpret_cast<const uint4*>(twin + p * kPage);
    const uint4* C = reinterpret_cast<const uint4*>(cur + p * kPage);
    uint4 t[4], c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k] = ld_nt16(T + k * 64 + lane);
      c[k] = ld_nt16(C + k * 64 + lane);
    }
    // Chunk (k, lane) covers bytes [(64k + lane) * 16, +16): page order = (k, lane).
    uint32_t m[4], s[4], e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = diffmask16(t[k], c[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t up = __shfl_up(m[k], 1, 64);
      const uint32_t dn = __shfl_down(m[k], 1, 64);
      const uint32_t wrap_prev = (k > 0) ? __shfl(m[k > 0 ? k - 1 : 0], 63, 64) : 0u;
      const uint32_t wrap_next = (k < 3) ? __shfl(m[k < 3 ? k + 1 : 3], 0, 64) : 0u;
      const uint32_t prev_top = ((lane == 0 ? wrap_prev : up) >> 15) & 1u;
      const uint32_t next_low = (lane == 63 ? wrap_next : dn) & 1u;
      s[k] = m[k] & ~((m[k] << 1) | prev_top) & 0xFFFFu;           // first byte of a run
      e[k] = m[k] & ~((m[k] >> 1) | (next_low << 15)) & 0xFFFFu;   // last byte of a run
    }
    // Packed counts: runs in the low 16 bits, payload bytes in the high 16 (totals <= 4096).
    uint32_t excl[4], carry = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t v = (uint32_t)__popc(s[k]) | ((uint32_t)__popc(m[k]) << 16);
      const uint32_t inc = wave_incl_sum(v);
      excl[k] = carry + inc - v;
      carry += __shfl(inc, 63, 64);
    }
    const uint32_t NR = carry & 0xFFFFu, NP = carry >> 16;
    const uint32_t size = NR ? 4u + 4u * NR + ((NP + 3u) & ~3u) : 0u;
    if (lane == 0) sizes[i] = size;
    acc += size;
    if (NR == 0) continue;  // wave-uniform

    // Next run end after each chunk: suffix minimum of the chunks' first end positions.
    uint32_t ne[4];
    uint32_t emin = 0xFFFFu;
#pragma unroll
    for (int k = 3; k >= 0; --k) {
      const uint32_t pos = (uint32_t)(k * 64 + lane) * 16u;
      const uint32_t fe = e[k] ? pos + (uint32_t)__builtin_ctz(e[k]) : 0xFFFFu;
      const uint32_t sm = wave_incl_suffix_min(fe);
      uint32_t after = __shfl_down(sm, 1, 64);
      if (lane == 63) after = 0xFFFFu;
      ne[k] = min(after, emin);
      emin = min(emin, __shfl(sm, 0, 64));
    }
    uint8_t* out = ws + i * kRecSlot;
    uint32_t* hdr = reinterpret_cast<uint32_t*>(out + 4);
    uint8_t* pay = out + 4 + 4 * NR;
    if (lane == 0) {
      *reinterpret_cast<uint32_t*>(out) = NR;
      for (uint32_t q = NP; q & 3u; ++q) pay[q] = 0;  // zero padding
    }
    emit_chunk(0 * 64 + lane, s[0], e[0], m[0], ne[0], excl[0], c[0], hdr, pay);
    emit_chunk(1 * 64 + lane, s[1], e[1], m[1], ne[1], excl[1], c[1], hdr, pay);
    emit_chunk(2 * 64 + lane, s[2], e[2], m[2], ne[2], excl[2], c[2], hdr, pay);
    emit_chunk(3 * 64 + lane, s[3], e[3], m[3], ne[3], excl[3], c[3], hdr, pay);
  }
  if (lane == 0) wsum[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) block_sum[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
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

__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ ws,
                                                   const uint32_t* __restrict__ sizes,
                                                   const uint64_t* __restrict__ block_off,
                                                   uint64_t first, uint64_t n,
                                                   uint64_t* __restrict__ rec_off,
                                                   uint8_t* __restrict__ data, uint64_t cap) {
  __shared__ uint64_t off[kDiffPagesPerBlock];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kDiffPagesPerBlock;
  if (wave == 0) {
    const uint64_t i = b0 + lane;
    const uint32_t sz = (i < n) ? sizes[i] : 0u;
    const uint32_t inc = wave_incl_sum(sz);
    const uint64_t base = block_off[blockIdx.x];
    off[lane] = base + inc - sz;
    if (i < n) rec_off[first + i + 1] = base + inc;
    if (first == 0 && blockIdx.x == 0 && lane == 0) rec_off[0] = 0;
  }
  __syncthreads();
  for (uint32_t j = wave; j < kDiffPagesPerBlock; j += 4) {
    const uint64_t i = b0 + j;
    if (i >= n) break;
    const uint32_t sz = sizes[i];
    const uint64_t o = off[j];
    if (sz == 0 || o + sz > cap) continue;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(ws + i * kRecSlot);
    uint32_t* dst = reinterpret_cast<uint32_t*>(data + o);
    for (uint32_t q = lane; q < sz / 4; q += 64) dst[q] = src[q];
  }
}

// ------------------------------------------------------------------------- apply (SPEC §4)
// One wave per record. The run list is turned back into the page's 4096-bit dirty mask by
// toggling a bit at every run start and end in LDS and taking a prefix-XOR (lane l owns bits
// [64l, 64l+64)); payload index of a byte = popcount of the dirty bits before it. Each lane
// then rewrites its four 16-byte chunks (read-modify-write only for partly dirty chunks).
__global__ __launch_bounds__(256) void apply_kernel(uint8_t* __restrict__ target,
                                                    const uint32_t* __restrict__ ids, uint64_t n,
                                                    const uint64_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ data,
                                                    uint32_t* __restrict__ err) {
  __shared__ uint32_t bm_all[4][128];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* bm = bm_all[wave];
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + wave; i < n; i += (uint64_t)gridDim.x * 4) {
    const uint64_t r0 = rec_off[i], r1 = rec_off[i + 1];
    if (r0 == r1) continue;
    const uint32_t* rec = reinterpret_cast<const uint32_t*>(data + r0);
    const uint32_t nr = rec[0];
    bool bad = (nr == 0) || (nr > kMaxRuns) || (r1 < r0) || (r1 - r0 < 4u + 4u * (uint64_t)nr);
    if (bad) {
      if (lane == 0) atomicOr(err, 1u);
      continue;
    }
    bm[lane] = 0;
    bm[lane + 64] = 0;
    wave_lds_sync();
    uint32_t paysum = 0, badrun = 0;
    for (uint32_t r = lane; r < nr; r += 64) {
      const uint32_t h = rec[1 + r];
      const uint32_t off = h & 0xFFFFu, len = h >> 16, end = off + len;
      if (len == 0 || end > kPage) { badrun = 1; continue; }
      paysum += len;
      atomicXor(&bm[off >> 5], 1u << (off & 31));
      if (end < kPage) atomicXor(&bm[end >> 5], 1u << (end & 31));
    }
    paysum = wave_sum(paysum);
    badrun = wave_sum(badrun);
    if (badrun || (r1 - r0) != 4u + 4u * (uint64_t)nr + ((paysum + 3u) & ~3u)) {
      if (lane == 0) atomicOr(err, 1u);
      continue;
    }
    wave_lds_sync();
    uint64_t w = (uint64_t)bm[2 * lane] | ((uint64_t)bm[2 * lane + 1] << 32);
    const uint32_t par = (uint32_t)__popcll(w) & 1u;
    w ^= w << 1;
    w ^= w << 2;
    w ^= w << 4;
    w ^= w << 8;
    w ^= w << 16;
    w ^= w << 32;
    const uint32_t pinc = wave_incl_sum(par);
    const uint64_t D = ((pinc - par) & 1u) ? ~w : w;
    const uint32_t cnt = (uint32_t)__popcll(D);
    const uint32_t pbase = wave_incl_sum(cnt) - cnt;
    const uint8_t* pay = reinterpret_cast<const uint8_t*>(rec + 1 + nr);
    const uint64_t p = ids ? ids[i] : i;
    uint8_t* dst = target + p * kPage + (uint64_t)lane * 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t mq = (uint32_t)(D >> (16 * q)) & 0xFFFFu;
      if (!mq) continue;
      const uint32_t pp = pbase + (q ? (uint32_t)__popcll(D & ((1ull << (16 * q)) - 1)) : 0u);
      uint4* d4 = reinterpret_cast<uint4*>(dst + 16 * q);
      uint4 v = (mq == 0xFFFFu) ? make_uint4(0, 0, 0, 0) : *d4;
      uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if ((mq >> j) & 1u) {
          const uint32_t src = pp + (uint32_t)__popc(mq & ((1u << j) - 1u));
          const uint32_t byte = pay[src];
          wv[j >> 2] = (wv[j >> 2] & ~(0xFFu << ((j & 3) * 8))) | (byte << ((j & 3) * 8));
        }
      }
      *d4 = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
  }
}

// ------------------------------------------------------------------------- launchers
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
      hipLaunchKernelGGL(diff_pages_kernel, dim3((unsigned)nb), dim3(256), 0, s, twin, cur, ids,
                         first, m, slots, sizes, block_sum);
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
