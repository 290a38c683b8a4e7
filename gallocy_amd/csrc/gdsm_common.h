// Shared device helpers for the gdsm kernels (gfx950, wave64). Internal header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdsm {

constexpr uint32_t kPage = 4096;
// Per-page record slot in the diff workspace: the largest record (SPEC §3: 10244 B) rounded to
// 16 B, so every slot starts 16-byte aligned.
constexpr uint32_t kRecSlot = 10256;
constexpr uint32_t kMaxRuns = 2048;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load (read-once data: nontemporal hint).
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Inclusive prefix sum across the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  return __shfl(wave_incl_sum(v), 63, 64);
}

// Inclusive suffix minimum across lanes (lane l gets min over lanes >= l).
__device__ __forceinline__ uint32_t wave_incl_suffix_min(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_down(v, d, 64);
    if (lane + d < 64u) v = min(v, t);
  }
  return v;
}

// Orders LDS traffic of ONE wave: LDS executes a wave's instructions in issue order, so only the
// compiler has to be kept from moving accesses across this point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// SPEC §6 mixers (must match oracle/gdsm_oracle.c bit for bit).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}
__device__ __forceinline__ uint64_t hash3(uint64_t s, uint64_t a, uint64_t b) {
  return mix64(mix64(s ^ (a * 0x9E3779B97F4A7C15ull)) + b * 0xC2B2AE3D27D4EB4Full +
               0x165667B19E3779F9ull);
}

}  // namespace gdsm
