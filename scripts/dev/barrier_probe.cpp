// Dev probe (not product code): the pure cost of gdsm_common.h's grid_barrier_wt, 1000 barriers
// back to back in one persistent launch, against the grid size and the poll's sleep.
//   hipcc -x hip --offload-arch=gfx950 -O3 -I include -I gallocy_amd/csrc \
//     scripts/dev/barrier_probe.cpp -o scripts/dev/barrier_probe && scripts/dev/barrier_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gdsm_common.h"

template <int kSleep>
__device__ __forceinline__ void barrier_v(uint32_t* bar, uint32_t target, uint32_t* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (kSleep) __builtin_amdgcn_s_sleep(kSleep);
      if (++spins > (1u << 24)) {
        atomicOr(err, 1u);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}

// One XCD's workgroups only (blockIdx % 8 == 0 under round-robin dispatch, checked through
// XCC_ID): arrivals as workgroup-scope atomics (performed in that XCD's L2), polls as sc0 loads.
__device__ __forceinline__ void barrier_xcd(uint32_t* bar, uint32_t target, uint32_t* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
      if (++spins > (1u << 24)) {
        atomicOr(err, 1u);
        break;
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void xcd_kernel(uint32_t* bar, uint32_t* err, uint32_t n,
                                                  unsigned long long* t) {
  if (blockIdx.x % 8 != 0) return;
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0 && (xcc & 0xF) != 0) atomicOr(err, 2u);  // not on XCD 0: the probe is void
  const uint32_t parts = (gridDim.x + 7) / 8;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t r = 0; r < n; ++r) barrier_xcd(bar, (r + 1) * parts, err);
  if (blockIdx.x == 0 && threadIdx.x == 0) t[0] = __builtin_amdgcn_s_memtime() - t0;
}

template <int kMode>
__global__ __launch_bounds__(256) void bar_kernel(uint32_t* bar, uint32_t* err, uint32_t n,
                                                  unsigned long long* t) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t r = 0; r < n; ++r) {
    if (kMode == 0) gdsm::grid_barrier_wt(bar, (r + 1) * gridDim.x, err, 1u);
    if (kMode == 1) barrier_v<0>(bar, (r + 1) * gridDim.x, err);
    if (kMode == 2) barrier_v<2>(bar, (r + 1) * gridDim.x, err);
    if (kMode == 3) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) t[0] = __builtin_amdgcn_s_memtime() - t0;
}

int main() {
  uint32_t *bar, *err;
  unsigned long long* t;
  (void)hipMalloc(&bar, 256);
  (void)hipMalloc(&err, 256);
  (void)hipMalloc(&t, 256);
  const uint32_t n = 1000;
  const char* names[4] = {"grid_barrier_wt (s_sleep 1)", "no sleep", "s_sleep 2", "syncthreads only"};
  for (int mode = 0; mode < 4; ++mode) {
    for (unsigned grid : {1u, 2u, 8u, 32u, 256u}) {
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipMemset(bar, 0, 256);
        (void)hipMemset(err, 0, 256);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        if (mode == 0) hipLaunchKernelGGL(bar_kernel<0>, dim3(grid), dim3(256), 0, 0, bar, err, n, t);
        if (mode == 1) hipLaunchKernelGGL(bar_kernel<1>, dim3(grid), dim3(256), 0, 0, bar, err, n, t);
        if (mode == 2) hipLaunchKernelGGL(bar_kernel<2>, dim3(grid), dim3(256), 0, 0, bar, err, n, t);
        if (mode == 3) hipLaunchKernelGGL(bar_kernel<3>, dim3(grid), dim3(256), 0, 0, bar, err, n, t);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long ht = 0;
        uint32_t he = 0;
        (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
        if (rep == 1)
          printf("%-28s grid %3u: %.3f us per barrier (event), %.3f us (memtime @2.4GHz) err %u\n",
                 names[mode], grid, ms * 1000.0 / n, ht / 2400.0 / n, he);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
      }
    }
  }
  for (unsigned grid : {8u, 16u, 64u, 256u}) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemset(bar, 0, 256);
      (void)hipMemset(err, 0, 256);
      hipLaunchKernelGGL(xcd_kernel, dim3(grid), dim3(256), 0, 0, bar, err, n, t);
      (void)hipDeviceSynchronize();
      unsigned long long ht = 0;
      uint32_t he = 0;
      (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
      if (rep == 1)
        printf("one XCD, L2 atomics, %3u of %3u workgroups: %.3f us per barrier (memtime) err %u\n",
               (grid + 7) / 8, grid, ht / 2400.0 / n, he);
    }
  }
  return 0;
}
