// Checks the wave/row cross-lane primitives of gallocy_amd/csrc/gdsm_common.h on the GPU
// against their definitions (test infrastructure; prints PASS/FAIL per primitive).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "gdsm_common.h"
using namespace gdsm;

__global__ void prims(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  const uint32_t x = (l * 7 + 3) % 11;
  uint32_t* o = out + l;
  o[0 * 64] = wave_incl_sum(x);
  o[1 * 64] = wave_incl_max(x);
  o[2 * 64] = row_incl_sum(x);
  o[3 * 64] = row_incl_max(x);
  o[4 * 64] = row_last(x);
  o[5 * 64] = row_prev(x);
  o[6 * 64] = from_prev_lane(x);
  o[7 * 64] = from_next_lane(x);
  o[8 * 64] = lane_bcast(x, 63);
  o[9 * 64] = wave_sum(x);
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 10 * 64 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(prims, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[640];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  uint32_t x[64];
  for (int l = 0; l < 64; ++l) x[l] = (l * 7 + 3) % 11;
  const char* names[10] = {"wave_incl_sum", "wave_incl_max", "row_incl_sum", "row_incl_max",
                           "row_last", "row_prev", "from_prev_lane", "from_next_lane",
                           "lane_bcast63", "wave_sum"};
  int fails = 0;
  for (int f = 0; f < 10; ++f) {
    int bad = -1;
    for (int l = 0; l < 64; ++l) {
      uint32_t e = 0, rb = l & ~15;
      switch (f) {
        case 0: for (int k = 0; k <= l; ++k) e += x[k]; break;
        case 1: for (int k = 0; k <= l; ++k) e = x[k] > e ? x[k] : e; break;
        case 2: for (int k = rb; k <= l; ++k) e += x[k]; break;
        case 3: for (int k = rb; k <= l; ++k) e = x[k] > e ? x[k] : e; break;
        case 4: e = x[rb + 15]; break;
        case 5: e = (l & 15) ? x[l - 1] : 0; break;
        case 6: e = l ? x[l - 1] : 0; break;
        case 7: e = l < 63 ? x[l + 1] : 0; break;
        case 8: e = x[63]; break;
        case 9: for (int k = 0; k < 64; ++k) e += x[k]; break;
      }
      if (h[f * 64 + l] != e && bad < 0) bad = l;
    }
    if (bad >= 0) {
      ++fails;
      printf("FAIL %s lane %d got %u\n", names[f], bad, h[f * 64 + bad]);
      for (int l = 0; l < 64; ++l) printf("%u ", h[f * 64 + l]);
      printf("\n");
    } else {
      printf("PASS %s\n", names[f]);
    }
  }
  return fails ? 1 : 0;
}
