// Read-roofline probe for the diff kernel's access pattern on gfx950: two 4 GiB arenas (TWIN and
// CURRENT, 1M x 4 KiB pages) streamed once, one wave per page, XOR-OR reduced to one word per
// page. Variants: pages per wave, pages in flight per wave, nt vs default loads, grid shape.
// Not product code: it measures the ceiling the diff kernel is held against.
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/read_probe.hip -o scripts/dev/read_probe
//   read_probe <pages> [w]   (w: the record-stream variants only)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// PPW pages per wave, processed INF at a time (INF pages' loads issued before any is reduced).
template <int PPW, int INF, bool NT>
__global__ __launch_bounds__(256) void rd_pages(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                uint32_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wave) * PPW;
  for (int j = 0; j < PPW; j += INF) {
    u32x4 t[INF][4], c[INF][4];
#pragma unroll
    for (int q = 0; q < INF; ++q) {
      const uint64_t p = w0 + j + q;
      if (p < n) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          t[q][k] = ld<NT>(a + p * 256 + k * 64 + lane);
          c[q][k] = ld<NT>(b + p * 256 + k * 64 + lane);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < INF; ++q) {
      const uint64_t p = w0 + j + q;
      if (p >= n) break;
      uint32_t d = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32x4 x = t[q][k] ^ c[q][k];
        d |= x.x | x.y | x.z | x.w;
      }
      const uint64_t m = __ballot(d != 0);
      if (lane == 0) out[p] = (uint32_t)__popcll(m);
    }
  }
}

// The diff kernel's own shape: PPW pages per wave, the next page's 8 loads issued before the
// current page is reduced (one page in flight ahead).
template <int PPW>
__global__ __launch_bounds__(256) void rd_pipe(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                               uint32_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wave) * PPW;
  if (w0 >= n) return;
  u32x4 t[4], c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t[k] = ld<true>(a + w0 * 256 + k * 64 + lane);
    c[k] = ld<true>(b + w0 * 256 + k * 64 + lane);
  }
  for (int j = 0; j < PPW && w0 + j < n; ++j) {
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 x = t[k] ^ c[k];
      d |= x.x | x.y | x.z | x.w;
    }
    const uint64_t p = w0 + j + 1;
    if (j + 1 < PPW && p < n) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t[k] = ld<true>(a + p * 256 + k * 64 + lane);
        c[k] = ld<true>(b + p * 256 + k * 64 + lane);
      }
    }
    const uint64_t m = __ballot(d != 0);
    if (lane == 0) out[w0 + j] = (uint32_t)__popcll(m);
  }
}

// rd_pipe plus a record stream: WB bytes per page stored to out_w (dword stores, the diff's
// coalesced copy shape), either right after each page (kEnd false) or for the whole unit after its
// last page (kEnd true, the diff's order: records leave after the unit's look-back). The ceiling
// for a diff whose records are not small (config 3: ~850 B per page).
template <int PPW, uint32_t WB, bool kNT, bool kEnd, bool kX4 = false>
__global__ __launch_bounds__(256) void rd_pipe_w(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                 uint32_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wave) * PPW;
  if (w0 >= n) return;
  uint32_t* ow = out + n;  // the record stream, after the per-page words
  u32x4 t[4], c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t[k] = ld<true>(a + w0 * 256 + k * 64 + lane);
    c[k] = ld<true>(b + w0 * 256 + k * 64 + lane);
  }
  uint32_t acc = 0;
  for (int j = 0; j < PPW && w0 + j < n; ++j) {
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 x = t[k] ^ c[k];
      d |= x.x | x.y | x.z | x.w;
    }
    const uint64_t p = w0 + j + 1;
    if (j + 1 < PPW && p < n) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t[k] = ld<true>(a + p * 256 + k * 64 + lane);
        c[k] = ld<true>(b + p * 256 + k * 64 + lane);
      }
    }
    acc ^= d;
    if (!kEnd) {
      uint32_t* dst = ow + (w0 + j) * (WB / 4);
      for (uint32_t g = lane; g < WB / 4; g += 64) {
        if (kNT) __builtin_nontemporal_store(d ^ g, dst + g); else dst[g] = d ^ g;
      }
    }
    const uint64_t m = __ballot(d != 0);
    if (lane == 0) out[w0 + j] = (uint32_t)__popcll(m);
  }
  if (kEnd) {
    const uint64_t np = min((uint64_t)PPW, n - w0);
    uint32_t* dst = ow + w0 * (WB / 4);
    if (kX4) {  // 16-B stores (the unit's stream starts 16-B aligned here: 832 = 52 * 16)
      u32x4* d4 = reinterpret_cast<u32x4*>(dst);
      for (uint32_t g = lane; g < np * (WB / 16); g += 64) {
        const u32x4 v = (u32x4){acc ^ g, acc, g, 1u};
        if (kNT) __builtin_nontemporal_store(v, d4 + g); else d4[g] = v;
      }
    } else {
      for (uint32_t g = lane; g < np * (WB / 4); g += 64) {
        if (kNT) __builtin_nontemporal_store(acc ^ g, dst + g); else dst[g] = acc ^ g;
      }
    }
  }
}

// LDS-DMA: PPW pages per wave, each page's 8 KiB (twin + current) by 8 global_load_lds_dwordx4
// into one of two per-wave LDS buffers, the next page's DMA issued before the current page is
// read back from LDS and reduced. 64 KiB of LDS per workgroup: 2 workgroups per CU.
template <int PPW>
__global__ __launch_bounds__(256) void rd_dma(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                              uint32_t* __restrict__ out, uint64_t n) {
  __shared__ __attribute__((aligned(16))) u32x4 buf[4][2][512];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wave) * PPW;
  if (w0 >= n) return;
  typedef __attribute__((address_space(1))) void* gptr;
  typedef __attribute__((address_space(3))) void* lptr;
#define RD_DMA(p_, s_)                                                                      \
  do {                                                                                      \
    for (int k = 0; k < 4; ++k) {                                                           \
      __builtin_amdgcn_global_load_lds((gptr)(a + (p_) * 256 + k * 64 + lane),              \
                                       (lptr)(&buf[wave][s_][k * 64]), 16, 0, 0);           \
      __builtin_amdgcn_global_load_lds((gptr)(b + (p_) * 256 + k * 64 + lane),              \
                                       (lptr)(&buf[wave][s_][256 + k * 64]), 16, 0, 0);     \
    }                                                                                       \
  } while (0)
  RD_DMA(w0, 0);
  for (int j = 0; j < PPW && w0 + j < n; ++j) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t p = w0 + j + 1;
    if (j + 1 < PPW && p < n) RD_DMA(p, (j + 1) & 1);
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 x = buf[wave][j & 1][k * 64 + lane] ^ buf[wave][j & 1][256 + k * 64 + lane];
      d |= x.x | x.y | x.z | x.w;
    }
    const uint64_t m = __ballot(d != 0);
    if (lane == 0) out[w0 + j] = (uint32_t)__popcll(m);
  }
#undef RD_DMA
}

// Persistent grid-stride over pages, one page per wave iteration.
template <bool NT>
__global__ __launch_bounds__(256) void rd_persist(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                  uint32_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t p = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < n; p += nw) {
    u32x4 t[4], c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k] = ld<NT>(a + p * 256 + k * 64 + lane);
      c[k] = ld<NT>(b + p * 256 + k * 64 + lane);
    }
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 x = t[k] ^ c[k];
      d |= x.x | x.y | x.z | x.w;
    }
    const uint64_t m = __ballot(d != 0);
    if (lane == 0) out[p] = (uint32_t)__popcll(m);
  }
}

// Flat streaming: every thread reads consecutive 16-B chunks of both arenas (no page structure).
template <bool NT>
__global__ __launch_bounds__(256) void rd_flat(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                               uint32_t* __restrict__ out, uint64_t nchunks) {
  uint32_t d = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < nchunks; g += stride * 4) {
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t i = g + u * stride;
      if (i < nchunks) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); } else { x[u] = y[u] = (u32x4){0,0,0,0}; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { const u32x4 z = x[u] ^ y[u]; d |= z.x | z.y | z.z | z.w; }
  }
  if (d == 0x12345678u) out[0] = d;
}

__global__ void fill(u32x4* p, uint64_t n, uint32_t s) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (u32x4){(uint32_t)i ^ s, (uint32_t)(i >> 7), s, (uint32_t)i * 2654435761u};
}

typedef void (*Kern)(const u32x4*, const u32x4*, uint32_t*, uint64_t);

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1 << 20), chunks = n * 256;
  u32x4 *a, *b;
  uint32_t* out;
  CK(hipMalloc(&a, chunks * 16));
  CK(hipMalloc(&b, chunks * 16));
  const bool wmode = argc > 2 && argv[2][0] == 'w';  // record-stream variants only
  CK(hipMalloc(&out, n * 4 + (wmode ? n * 832 : 0)));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, a, chunks, 1u);
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, b, chunks, 1u);
  CK(hipDeviceSynchronize());
  struct V { const char* name; Kern k; unsigned grid; uint64_t arg; };
  std::vector<V> vs = {
      {"pages ppw16 inf1 nt", rd_pages<16, 1, true>, (unsigned)(n / 64), n},
      {"pages ppw16 inf1   ", rd_pages<16, 1, false>, (unsigned)(n / 64), n},
      {"pages ppw16 inf2 nt", rd_pages<16, 2, true>, (unsigned)(n / 64), n},
      {"pages ppw16 inf4 nt", rd_pages<16, 4, true>, (unsigned)(n / 64), n},
      {"pages ppw4  inf1 nt", rd_pages<4, 1, true>, (unsigned)(n / 16), n},
      {"pages ppw1  inf1 nt", rd_pages<1, 1, true>, (unsigned)(n / 4), n},
      {"pages ppw64 inf2 nt", rd_pages<64, 2, true>, (unsigned)(n / 256), n},
      {"pipe ppw64 nt      ", rd_pipe<64>, (unsigned)(n / 256), n},
      {"pipe ppw16 nt      ", rd_pipe<16>, (unsigned)(n / 64), n},
      {"dma ppw64          ", rd_dma<64>, (unsigned)(n / 256), n},
      {"dma ppw16          ", rd_dma<16>, (unsigned)(n / 64), n},
      {"persist 2048 nt    ", rd_persist<true>, 2048, n},
      {"persist 4096 nt    ", rd_persist<true>, 4096, n},
      {"persist 8192 nt    ", rd_persist<true>, 8192, n},
      {"persist 2048       ", rd_persist<false>, 2048, n},
      {"flat 4096 nt       ", rd_flat<true>, 4096, chunks},
      {"flat 8192 nt       ", rd_flat<true>, 8192, chunks},
      {"flat 8192          ", rd_flat<false>, 8192, chunks},
  };
  if (wmode)
    vs = {
        {"pipe ppw16 nt      ", rd_pipe<16>, (unsigned)(n / 64), n},
        {"pipe16 +832 end nt ", rd_pipe_w<16, 832, true, true>, (unsigned)(n / 64), n},
        {"pipe16 +832 end    ", rd_pipe_w<16, 832, false, true>, (unsigned)(n / 64), n},
        {"pipe16 +832 page nt", rd_pipe_w<16, 832, true, false>, (unsigned)(n / 64), n},
        {"pipe64 +832 end nt ", rd_pipe_w<64, 832, true, true>, (unsigned)(n / 256), n},
        {"pipe16 +832 end nt x4", rd_pipe_w<16, 832, true, true, true>, (unsigned)(n / 64), n},
        {"pipe16 +832 end x4 ", rd_pipe_w<16, 832, false, true, true>, (unsigned)(n / 64), n},
    };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 5, K = 10;
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      hipLaunchKernelGGL(vs[v].k, dim3(vs[v].grid), dim3(256), 0, 0, a, b, out, vs[v].arg);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < K; ++i)
        hipLaunchKernelGGL(vs[v].k, dim3(vs[v].grid), dim3(256), 0, 0, a, b, out, vs[v].arg);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / K);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(ms[v].begin(), ms[v].end());
    const double med = ms[v][R / 2];
    const double wb = (wmode && v > 0) ? 832.0 * n : 0.0;
    printf("%s  median %.4f ms  min %.4f ms  %.0f GB/s (read + written)\n", vs[v].name, med,
           ms[v][0], (2.0 * chunks * 16 + wb) / (med * 1e-3) / 1e9);
  }
  return 0;
}
