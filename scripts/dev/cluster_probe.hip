// Write-side probe for the clustered apply (BASELINE config 3 shape) on gfx950 (not product
// code): 4M pages, each 64-B cluster dirty with probability 10 % (the bench's clustered pages),
// i.e. ~1.7 GB of aligned 64-B segments scattered over a 16 GiB REPLICA arena. Kernels, each one
// thread per 16-B chunk of the dirty clusters in page order (a precomputed cluster list, 4 B per
// cluster), so they are the apply without any record parsing:
//   copy    16 B read from a contiguous payload stream, stored to its place in the arena
//           (the ideal apply: the stream is read once, every segment written whole)
//   write   the same stores, no payload read
//   read    the payload read alone (stores skipped)
//   rand    copy with the clusters taken in a random page order (no locality between waves)
//   copynt / writent   copy / write with nontemporal stores
//   hipcc --offload-arch=gfx950 -O3 scripts/dev/cluster_probe.hip -o /tmp/cluster_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __host__ inline uint64_t mix(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

// dirty-cluster mask of page p (10 %)
__device__ __host__ inline uint64_t page_mask(uint64_t p) {
  uint64_t m = 0;
  for (int c = 0; c < 64; ++c)
    if (mix(p * 64 + c + 12345) % 10 == 0) m |= 1ull << c;
  return m;
}

__global__ void count_kernel(uint32_t* __restrict__ cnt, uint64_t n) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) cnt[p] = (uint32_t)__popcll(page_mask(p));
}

__global__ void list_kernel(const uint32_t* __restrict__ off, uint32_t* __restrict__ list,
                            uint64_t n) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint64_t m = page_mask(p);
  uint32_t o = off[p];
  while (m) {
    const int c = __builtin_ctzll(m);
    m &= m - 1;
    list[o++] = (uint32_t)(p * 64 + c);
  }
}

template <int kMode, bool kNT = false>  // 0 copy, 1 write only, 2 read only
__global__ __launch_bounds__(256) void chunk_kernel(uint8_t* __restrict__ arena,
                                                    const u32x4* __restrict__ pay,
                                                    const uint32_t* __restrict__ list,
                                                    uint64_t nchunks, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < nchunks;
       g += (uint64_t)gridDim.x * 256) {
    const uint32_t cl = list[g >> 2];
    u32x4 v = (u32x4){(uint32_t)g, 1, 2, 3};
    if (kMode != 1) v = __builtin_nontemporal_load(pay + g);
    if (kMode != 2) {
      u32x4* d = reinterpret_cast<u32x4*>(arena + (uint64_t)cl * 64 + (g & 3) * 16);
      if (kNT)
        __builtin_nontemporal_store(v, d);
      else
        *d = v;
    }
    else
      acc ^= v.x ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t n = 4ull << 20;
  std::vector<uint32_t> hc(n);
  uint32_t *cnt, *off, *list, *sink;
  uint8_t* arena;
  u32x4* pay;
  CK(hipMalloc(&cnt, n * 4));
  CK(hipMalloc(&off, n * 4));
  CK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(count_kernel, dim3((unsigned)(n / 256)), dim3(256), 0, 0, cnt, n);
  CK(hipMemcpy(hc.data(), cnt, n * 4, hipMemcpyDeviceToHost));
  uint64_t tot = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t c = hc[i];
    hc[i] = (uint32_t)tot;
    tot += c;
  }
  CK(hipMemcpy(off, hc.data(), n * 4, hipMemcpyHostToDevice));
  const uint64_t nchunks = tot * 4;
  printf("pages %llu, dirty clusters %llu, payload %.3f GB\n", (unsigned long long)n,
         (unsigned long long)tot, tot * 64 / 1e9);
  CK(hipMalloc(&list, tot * 4));
  CK(hipMalloc(&arena, n * 4096));
  CK(hipMalloc(&pay, nchunks * 16));
  CK(hipMemset(arena, 3, n * 4096));
  CK(hipMemset(pay, 5, nchunks * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    int mode;
    int rnd;
    bool nt;
  };
  const V vs[] = {{"copy ", 0, 0, false},  {"write", 1, 0, false},   {"read ", 2, 0, false},
                  {"copynt", 0, 0, true},  {"writent", 1, 0, true},  {"rand ", 0, 1, false}};
  for (const V& v : vs) {
    hipLaunchKernelGGL(list_kernel, dim3((unsigned)(n / 256)), dim3(256), 0, 0, off, list, n);
    CK(hipDeviceSynchronize());
    if (v.rnd) {  // shuffle whole pages' cluster runs on the host
      std::vector<uint32_t> hl(tot);
      CK(hipMemcpy(hl.data(), list, tot * 4, hipMemcpyDeviceToHost));
      std::vector<uint32_t> order(n);
      for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
      for (uint64_t i = n - 1; i > 0; --i) std::swap(order[i], order[mix(i) % (i + 1)]);
      std::vector<uint32_t> out;
      out.reserve(tot);
      for (uint64_t k = 0; k < n; ++k) {
        const uint32_t p = order[k];
        const uint32_t a = hc[p], b = p + 1 < n ? hc[p + 1] : (uint32_t)tot;
        out.insert(out.end(), hl.begin() + a, hl.begin() + b);
      }
      CK(hipMemcpy(list, out.data(), tot * 4, hipMemcpyHostToDevice));
    }
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(e0, 0));
      auto k = v.mode == 0 ? (v.nt ? chunk_kernel<0, true> : chunk_kernel<0>)
               : v.mode == 1 ? (v.nt ? chunk_kernel<1, true> : chunk_kernel<1>)
                             : chunk_kernel<2>;
      hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, arena, pay, list, nchunks, sink);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float x;
      CK(hipEventElapsedTime(&x, e0, e1));
      ts.push_back(x);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[3];
    const double bytes = (v.mode != 1 ? nchunks * 16.0 : 0) + (v.mode != 2 ? nchunks * 16.0 : 0) +
                         tot * 4.0;
    printf("%s %.4f ms  %.2f TB/s of payload read + written + list\n", v.name, ms,
           bytes / ms / 1e9);
  }
  return 0;
}
