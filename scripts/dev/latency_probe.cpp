// Dev probe (not product code): dependent-load latency on one wave for the load forms the rounds
// kernels use: plain (L1/L2-cached), write-through hand-off loads (agent-scope relaxed atomic =
// global_load ... sc1) and nontemporal loads, over a small chain that stays in cache after the
// first pass, plus the store->load round trip of a write-through store.
//   hipcc -x hip --offload-arch=gfx950 -O3 scripts/dev/latency_probe.cpp -o scripts/dev/latency_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int kMode>
__global__ void chase(const uint32_t* __restrict__ next, uint32_t steps, uint32_t* out,
                      unsigned long long* t) {
  uint32_t p = threadIdx.x >> 6;  // 0 in the one-wave launch, but a vector value (vector loads)
  // one warm pass
  for (uint32_t i = 0; i < steps; ++i) p = next[p];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < steps; ++i) {
    if (kMode == 0) p = next[p];
    if (kMode == 1)
      p = __hip_atomic_load(const_cast<uint32_t*>(next) + p, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    if (kMode == 2) p = __builtin_nontemporal_load(next + p);
    if (kMode == 3)
      p = __hip_atomic_load(const_cast<uint32_t*>(next) + p, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = p;
    t[0] = t1 - t0;
  }
}

int main() {
  const uint32_t n = 4096, steps = 2000;  // 16 KiB chain, 64-B stride between hops
  uint32_t h[n];
  for (uint32_t i = 0; i < n; ++i) h[i] = (i * 16 + 16 * 37) % n;
  uint32_t *d, *o;
  unsigned long long* t;
  (void)hipMalloc(&d, n * 4);
  (void)hipMalloc(&o, 64);
  (void)hipMalloc(&t, 64);
  (void)hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  const char* names[4] = {"plain (cached)", "agent relaxed atomic (sc1)", "nontemporal",
                          "workgroup relaxed atomic"};
  for (int m = 0; m < 4; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      if (m == 0) hipLaunchKernelGGL(chase<0>, dim3(1), dim3(64), 0, 0, d, steps, o, t);
      if (m == 1) hipLaunchKernelGGL(chase<1>, dim3(1), dim3(64), 0, 0, d, steps, o, t);
      if (m == 2) hipLaunchKernelGGL(chase<2>, dim3(1), dim3(64), 0, 0, d, steps, o, t);
      if (m == 3) hipLaunchKernelGGL(chase<3>, dim3(1), dim3(64), 0, 0, d, steps, o, t);
      (void)hipDeviceSynchronize();
      unsigned long long ht = 0;
      (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-28s %.1f ns per dependent load (s_memtime at 2.4 GHz)\n", names[m],
                      ht / 2.4 / steps);
    }
  }
  return 0;
}
