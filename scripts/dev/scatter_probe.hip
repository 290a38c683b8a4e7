// Scattered-write probe for the apply kernel's access pattern on gfx950 (not product code):
// 1M pages x 5 dirty 8-B words per page (BASELINE config 2's 1 % word writes) written into a
// 4 GiB REPLICA arena, followed by the diff-shaped read stream over two other 4 GiB arenas.
// Reports the write kernel's time and how much longer the following read stream takes than
// after an empty kernel (the deferred write-back of the dirty lines), per write shape:
//   w8      one lane per word, 8-B store (what apply does), pages in order
//   w8rand  the same words, pages in random order
//   l64     the 64-B line holding the word stored whole (16 lanes x 4 B)
//   l128    the 128-B line holding the word stored whole (32 lanes x 4 B)
//   rmw64   the 64-B line read, the word merged in, the line stored whole
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/scatter_probe.hip -o scripts/dev/scatter_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27; z *= 0x94D049BB133111EBull; z ^= z >> 31;
  return z;
}
constexpr uint32_t kWordsPerPage = 5;

// word w (0..n*5): page, byte offset (8-B aligned) of the w-th dirty word
__device__ __forceinline__ void word_at(uint64_t w, uint64_t n, bool rnd, uint64_t& page, uint32_t& off) {
  page = w / kWordsPerPage;
  if (rnd) page = mix(page * 7 + 1) % n;
  off = (uint32_t)(mix(w * 131 + 5) % 512) * 8;
}

template <bool RND>
__global__ void w8(uint8_t* __restrict__ rep, uint64_t n) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n * kWordsPerPage) return;
  uint64_t p; uint32_t o;
  word_at(w, n, RND, p, o);
  *reinterpret_cast<uint64_t*>(rep + p * 4096 + o) = w * 0x9E3779B97F4A7C15ull;
}

template <int LINE>
__global__ void wline(uint8_t* __restrict__ rep, uint64_t n) {
  constexpr int L = LINE / 4;  // lanes per line
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t w = t / L;
  const uint32_t l = (uint32_t)(t % L);
  if (w >= n * kWordsPerPage) return;
  uint64_t p; uint32_t o;
  word_at(w, n, false, p, o);
  uint32_t* line = reinterpret_cast<uint32_t*>(rep + p * 4096 + (o & ~(uint32_t)(LINE - 1)));
  line[l] = (uint32_t)w ^ l;
}

__global__ void rmw64(uint8_t* __restrict__ rep, uint64_t n) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t w = t / 16;
  const uint32_t l = (uint32_t)(t % 16);
  if (w >= n * kWordsPerPage) return;
  uint64_t p; uint32_t o;
  word_at(w, n, false, p, o);
  uint32_t* line = reinterpret_cast<uint32_t*>(rep + p * 4096 + (o & ~63u));
  uint32_t v = line[l];
  if (l == ((o & 63u) >> 2) || l == ((o & 63u) >> 2) + 1) v ^= (uint32_t)w;
  line[l] = v;
}

__global__ void nop(uint8_t*, uint64_t) {}

__global__ __launch_bounds__(256) void rd_flat(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                               uint32_t* __restrict__ out, uint64_t nchunks) {
  uint32_t d = 0;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < nchunks; g += stride * 4) {
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t i = g + u * stride;
      if (i < nchunks) { x[u] = __builtin_nontemporal_load(a + i); y[u] = __builtin_nontemporal_load(b + i); }
      else { x[u] = y[u] = (u32x4){0, 0, 0, 0}; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { const u32x4 z = x[u] ^ y[u]; d |= z.x | z.y | z.z | z.w; }
  }
  if (d == 0x12345678u) out[0] = d;
}

typedef void (*WK)(uint8_t*, uint64_t);

int main() {
  const uint64_t n = 1 << 20, chunks = n * 256, words = n * kWordsPerPage;
  u32x4 *a, *b;
  uint8_t* rep;
  uint32_t* out;
  CK(hipMalloc(&a, chunks * 16));
  CK(hipMalloc(&b, chunks * 16));
  CK(hipMalloc(&rep, n * 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, chunks * 16));
  CK(hipMemset(b, 2, chunks * 16));
  CK(hipMemset(rep, 3, n * 4096));
  CK(hipDeviceSynchronize());
  struct V { const char* name; WK k; uint64_t threads; };
  std::vector<V> vs = {{"nop   ", nop, 64},
                       {"w8    ", w8<false>, words},
                       {"w8rand", w8<true>, words},
                       {"l64   ", wline<64>, words * 16},
                       {"l128  ", wline<128>, words * 32},
                       {"rmw64 ", rmw64, words * 16}};
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  const int R = 7;
  std::vector<std::vector<float>> tw(vs.size()), tr(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      hipLaunchKernelGGL(rd_flat, dim3(8192), dim3(256), 0, 0, a, b, out, chunks);  // settle
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(vs[v].k, dim3((unsigned)((vs[v].threads + 255) / 256)), dim3(256), 0, 0, rep, n);
      CK(hipEventRecord(e1, 0));
      hipLaunchKernelGGL(rd_flat, dim3(8192), dim3(256), 0, 0, a, b, out, chunks);
      CK(hipEventRecord(e2, 0));
      CK(hipEventSynchronize(e2));
      float x, y;
      CK(hipEventElapsedTime(&x, e0, e1));
      CK(hipEventElapsedTime(&y, e1, e2));
      tw[v].push_back(x);
      tr[v].push_back(y);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(tw[v].begin(), tw[v].end());
    std::sort(tr[v].begin(), tr[v].end());
    printf("%s write %.4f ms  following read %.4f ms  (sum %.4f)\n", vs[v].name, tw[v][R / 2],
           tr[v][R / 2], tw[v][R / 2] + tr[v][R / 2]);
  }
  return 0;
}
