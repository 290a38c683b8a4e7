// Shared device helpers for the gdsm kernels (gfx950, wave64). Internal header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdsm {

constexpr uint32_t kPage = 4096;
constexpr uint32_t kMaxRuns = 2048;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load (read-once data: nontemporal hint).
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// ---- write-through access for hand-offs inside one launch (gdsm_rounds' persistent grids):
// stores `sc1` (written through to memory, so another XCD's reader needs no release fence from
// the writer) and loads `sc1` (past this CU's L1, so the reader needs no acquire), both as
// agent-scope relaxed atomics, which gfx950 lowers to plain global_store / global_load with sc1
// (MI355X_MICROARCH.md, inter-workgroup visibility: valid forms). 16 B = two 8-B accesses.
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt16(void* p, const uint4& v) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
  st_wt(q, (uint64_t)v.x | ((uint64_t)v.y << 32));
  st_wt(q + 1, (uint64_t)v.z | ((uint64_t)v.w << 32));
}
__device__ __forceinline__ uint4 ld_wt16(const void* p) {
  uint64_t* q = const_cast<uint64_t*>(reinterpret_cast<const uint64_t*>(p));
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}
template <typename T>
__device__ __forceinline__ T ld_wt(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a store, write-through when kWT
template <bool kWT, typename T>
__device__ __forceinline__ void st_(T* p, T v) {
  if (kWT)
    st_wt(p, v);
  else
    *p = v;
}
// an add to a word other workgroups read: kL2 (every reader on this XCD) performed in the XCD's
// L2 (workgroup scope: no sc1), else an agent-scope atomic
template <bool kL2>
__device__ __forceinline__ void add_u32(uint32_t* p, uint32_t v) {
  if (kL2)
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    atomicAdd(p, v);
}

// ---- wave64 cross-lane primitives on DPP (VALU, no LDS traffic) -------------------------
// gfx9-family DPP controls: row_shr:n = 0x110+n, row_bcast:15 = 0x142, row_bcast:31 = 0x143,
// wave_shl:1 = 0x130, wave_shr:1 = 0x138. Lanes whose source is out of range (or whose row is
// masked off) read 0, which is the identity of every scan below.
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, false);
}

// Inclusive prefix sum across the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  x += dpp0<0x142, 0xA>(x);
  x += dpp0<0x143, 0xC>(x);
  return x;
}

// Inclusive prefix maximum across lanes (values >= 0; 0 is the identity).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, dpp0<0x111>(x));
  x = max(x, dpp0<0x112>(x));
  x = max(x, dpp0<0x114>(x));
  x = max(x, dpp0<0x118>(x));
  x = max(x, dpp0<0x142, 0xA>(x));
  x = max(x, dpp0<0x143, 0xC>(x));
  return x;
}

__device__ __forceinline__ uint32_t lane_bcast(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t lane_bcast64(uint64_t v, int lane) {
  return (uint64_t)lane_bcast((uint32_t)v, lane) | ((uint64_t)lane_bcast((uint32_t)(v >> 32), lane) << 32);
}

// A 64-bit value from lane `src` (both halves as unsigned dwords: __shfl returns int, and a
// negative int widened to 64 bits would sign-extend into the high half).
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return lane_bcast(wave_incl_sum(v), 63); }

// Value of lane l-1 (lane 0 gets 0) / of lane l+1 (lane 63 gets 0).
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) { return dpp0<0x138>(v); }
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) { return dpp0<0x130>(v); }

// ---- 16-lane DPP rows
__device__ __forceinline__ uint32_t row_incl_sum(uint32_t x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  return x;
}
__device__ __forceinline__ uint32_t row_incl_max(uint32_t x) {
  x = max(x, dpp0<0x111>(x));
  x = max(x, dpp0<0x112>(x));
  x = max(x, dpp0<0x114>(x));
  x = max(x, dpp0<0x118>(x));
  return x;
}
// Lane 15 of the row, broadcast to the whole row (row_newbcast:15).
__device__ __forceinline__ uint32_t row_last(uint32_t x) { return dpp0<0x15F>(x); }
// Lane r-1 of the row (lane 0 of the row gets 0).
__device__ __forceinline__ uint32_t row_prev(uint32_t x) { return dpp0<0x111>(x); }

// Segmented sum: bit 31 = "a segment starts in here", low bits = the sum since the last start
// (the sums stay below 2^31). 0 is the identity.
constexpr uint32_t kSegStart = 1u << 31;
__device__ __forceinline__ uint32_t segsum(uint32_t a, uint32_t b) {
  return ((b & kSegStart) ? (b & ~kSegStart) : ((a & ~kSegStart) + (b & ~kSegStart))) |
         ((a | b) & kSegStart);
}
__device__ __forceinline__ uint32_t wave_incl_segsum_dpp(uint32_t v) {
  v = segsum(dpp0<0x111>(v), v);
  v = segsum(dpp0<0x112>(v), v);
  v = segsum(dpp0<0x114>(v), v);
  v = segsum(dpp0<0x118>(v), v);
  v = segsum(dpp0<0x142, 0xA>(v), v);
  v = segsum(dpp0<0x143, 0xC>(v), v);
  return v;
}

// Inclusive suffix minimum across lanes (lane l gets min over lanes >= l); bpermute based.
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

// A barrier of a persistent grid (every workgroup resident) whose hand-offs are all write-through
// (st_wt / ld_wt above): no release or acquire fence (their L2 write-back and L1 invalidate cost
// ~1.7 us each); every wave drains its stores (vmcnt(0)) before the workgroup's arrival, and the
// arrival counter `bar` (zeroed before the launch; the k-th barrier waits for k x gridDim.x
// arrivals) is an agent atomic polled by sc1 loads. A wait that never ends (a workgroup not
// resident: never expected, the launcher sizes the grid below the occupancy) sets `err_bit` in
// *err and lets the workgroup go on, so the grid always drains.
// Split form: grid_arrive_wt drains the workgroup's stores and counts it in; loads issued between
// it and grid_wait_wt (the next round's inputs) overlap the wait instead of delaying the arrival
// (gfx9's vmcnt counts loads and stores alike, so a load issued before the drain is waited for).
// kL2 (a one-XCD team, below): the arrival is added in the XCD's L2, where every member's sc1
// polls read it.
template <bool kL2 = false>
__device__ __forceinline__ void grid_arrive_wt(uint32_t* __restrict__ bar) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (kL2)
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void grid_wait_wt(uint32_t* __restrict__ bar, uint32_t target,
                                             uint32_t* __restrict__ err, uint32_t err_bit) {
  if (threadIdx.x == 0) {
    uint32_t spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023u) == 0 &&
          (spins > (1u << 22) ||
           (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & err_bit))) {
        atomicOr(err, err_bit);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps loads below)
  __syncthreads();
}
__device__ __forceinline__ void grid_barrier_wt(uint32_t* __restrict__ bar, uint32_t target,
                                                uint32_t* __restrict__ err, uint32_t err_bit) {
  grid_arrive_wt(bar);
  grid_wait_wt(bar, target, err, err_bit);
}

// A one-XCD team of a persistent grid: of the launch's workgroups, those running on the XCD of
// the workgroup that checked in first take part (member idx of n), the others leave at once. The
// XCD is read from HW_REG_XCC_ID, so no dispatch order or placement is assumed; the members' hand-
// offs then meet in that XCD's L2 (plain stores kept there, sc1 loads served from it, arrivals and
// count adds performed there) instead of crossing to memory. ctl: 4 words zeroed before the launch
// ([0] check-ins, [1] home XCC + 1, [2] members, [3] settled). A member waits for every
// workgroup's check-in, so the launch must be resident at once (as every grid barrier needs).
struct XcdTeam {
  uint32_t idx, n;  // idx == ~0u: not a member
};
__device__ __forceinline__ XcdTeam xcd_team(uint32_t* __restrict__ ctl, uint32_t* __restrict__ err,
                                            uint32_t err_bit) {
  __shared__ uint32_t s_idx, s_n;
  if (threadIdx.x == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 0xFu;
    const uint32_t t = __hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) __hip_atomic_store(ctl + 1, xcc + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t home, spins = 0;
    while ((home = __hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        atomicOr(err, err_bit);
        break;
      }
    }
    uint32_t idx = ~0u, n = 0;
    if (home == xcc + 1u)
      idx = __hip_atomic_fetch_add(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the member count is final before settling)
    __hip_atomic_fetch_add(ctl + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (idx != ~0u) {
      spins = 0;
      while (__hip_atomic_load(ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {
          atomicOr(err, err_bit);
          idx = ~0u;
          break;
        }
      }
      n = __hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_idx = idx;
    s_n = n;
  }
  __syncthreads();
  return XcdTeam{s_idx, s_n};
}

// Measurement builds only (-DGDSM_ROUNDS_STAMPS): s_memtime stamps of gdsm_rounds' grids,
// workgroup 0, [kernel: 0 data, 1 page table][round][point], read by gdsm_debug_round_stamps
// (gdsm_pages.hip's copy: the data side) and gdsm_debug_round_stamps_pt (the page-table side).
// The stamping workgroup is the kernel's member 0 (GDSM_RSTAMP_WG, set and read by thread 0).
#ifdef GDSM_ROUNDS_STAMPS
static __device__ unsigned long long g_round_stamps[2][4096][4];  // (one copy per file)
__device__ __forceinline__ uint32_t& gdsm_stamp_wg() {
  __shared__ uint32_t f;
  return f;
}
#define GDSM_RSTAMP_WG(is0_)                    \
  do {                                          \
    if (threadIdx.x == 0) gdsm_stamp_wg() = (is0_); \
  } while (0)
#define GDSM_RSTAMP(k_, r_, i_)                                                          \
  do {                                                                                  \
    if (threadIdx.x == 0 && gdsm_stamp_wg() && (r_) < 4096)                             \
      g_round_stamps[k_][r_][i_] = __builtin_amdgcn_s_memtime();                        \
  } while (0)
#else
#define GDSM_RSTAMP_WG(is0_) \
  do {                       \
  } while (0)
#define GDSM_RSTAMP(k_, r_, i_) \
  do {                          \
  } while (0)
#endif

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
