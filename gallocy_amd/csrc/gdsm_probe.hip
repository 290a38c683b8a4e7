// Box ceilings for bench.py's roofline lines (gdsm_probe_ceiling, include/gdsm.h): how fast THIS
// GPU streams the workload's own arenas, measured in the bench's process before its timed region,
// so every line can state its kernel's fraction of the box it ran on beside the fraction of the
// 8 TB/s spec. Not part of the DSM path; no caller outside the bench needs it.
//
// read: two page arenas read once (the diff's input), one wave per 4 pages, each page's 8 x 16-B
//   nontemporal loads per lane in flight before the XOR-reduce; the best of the read shapes
//   measured in round 3 (scripts/dev/read_probe.hip "pages ppw4 inf1 nt", 6.63 TB/s at 16M pages).
// copy: dst := src over whole pages (the twin step's traffic), the fastest of three shapes: a
//   flat grid-stride 16-B copy (four loads per lane in flight before the four stores, 8
//   workgroups per CU) and two page-shaped grid-stride copies (a wave per page per step, its 4 x
//   16 B per lane loaded before the stores; cached or nontemporal loads).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "gdsm_common.h"
#include "gdsm_ctx.h"

namespace gdsm {
namespace {

typedef uint32_t u32x4p __attribute__((ext_vector_type(4)));
constexpr uint32_t kProbePPW = 4;           // pages per wave (read)
constexpr uint32_t kProbeSentinel = 0x9E3779B9u;

__global__ __launch_bounds__(256) void probe_read_kernel(const u32x4p* __restrict__ a,
                                                         const u32x4p* __restrict__ b, uint64_t n,
                                                         uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wave) * kProbePPW;
  uint32_t acc = 0;
  for (uint32_t j = 0; j < kProbePPW; ++j) {
    const uint64_t p = w0 + j;
    if (p >= n) break;
    u32x4p t[4], c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k] = __builtin_nontemporal_load(a + p * 256 + k * 64 + lane);
      c[k] = __builtin_nontemporal_load(b + p * 256 + k * 64 + lane);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4p x = t[k] ^ c[k];
      acc |= x.x | x.y | x.z | x.w;
    }
  }
  if (acc == kProbeSentinel) sink[0] = acc;  // (never in practice: it keeps the loads)
}

__global__ __launch_bounds__(256) void probe_copy_kernel(u32x4p* __restrict__ dst,
                                                         const u32x4p* __restrict__ src,
                                                         uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4p v0 = __builtin_nontemporal_load(src + i);
    const u32x4p v1 = __builtin_nontemporal_load(src + i + stride);
    const u32x4p v2 = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4p v3 = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = v0;
    dst[i + stride] = v1;
    dst[i + 2 * stride] = v2;
    dst[i + 3 * stride] = v3;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// Page-shaped copies: a wave per page per step over a grid-stride loop (grid capped at 16384
// workgroups), each lane's 4 x 16 B of the page loaded before any store; kNT: nontemporal loads.
template <bool kNT>
__global__ __launch_bounds__(256) void probe_copy_pages_kernel(u32x4p* __restrict__ dst,
                                                               const u32x4p* __restrict__ src,
                                                               uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t p = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < n;
       p += (uint64_t)gridDim.x * 4) {
    u32x4p v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = kNT ? __builtin_nontemporal_load(src + p * 256 + k * 64 + lane)
                 : src[p * 256 + k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[p * 256 + k * 64 + lane] = v[k];
  }
}

}  // namespace
}  // namespace gdsm

using namespace gdsm::detail;

extern "C" int gdsm_probe_ceiling(gdsm_ctx* ctx, int kind, const void* a, const void* b, void* dst,
                                  uint64_t n_pages, int reps, float* best_ms, float* median_ms) {
  if (!ctx || !a || n_pages == 0 || reps < 1 || reps > 64 || !best_ms || !median_ms) return -EINVAL;
  if (kind == GDSM_PROBE_READ ? !b : kind == GDSM_PROBE_COPY ? !dst : true) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  GDSM_TRY(hipEventCreate(&e0));
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -EIO;
  }
  // the read takes one shape; the copy takes three (flat; page-shaped with cached or nontemporal
  // loads) and reports the fastest: the ceiling is the best copy this box does
  const int shapes = kind == GDSM_PROBE_READ ? 1 : 3;
  const uint64_t waves = (n_pages + gdsm::kProbePPW - 1) / gdsm::kProbePPW;
  const dim3 page_grid((unsigned)((waves + 3) / 4));
  int rc = 0;
  float best = 0, med = 0;
  for (int sh = 0; sh < shapes && !rc; ++sh) {
    std::vector<float> ms;
    for (int r = 0; r < reps && !rc; ++r) {
      hipError_t e = hipEventRecord(e0, ctx->stream);
      if (e == hipSuccess) {
        if (kind == GDSM_PROBE_READ) {
          hipLaunchKernelGGL(gdsm::probe_read_kernel, page_grid, dim3(256), 0, ctx->stream,
                             static_cast<const gdsm::u32x4p*>(a),
                             static_cast<const gdsm::u32x4p*>(b), n_pages,
                             ctx->err + 8);  // (a spare word of the error block)
        } else if (sh == 0) {
          hipLaunchKernelGGL(gdsm::probe_copy_kernel, dim3((unsigned)(8 * cus)), dim3(256), 0,
                             ctx->stream, static_cast<gdsm::u32x4p*>(dst),
                             static_cast<const gdsm::u32x4p*>(a), n_pages * 256);
        } else {
          const uint64_t g = std::min<uint64_t>((n_pages + 3) / 4, 16384);
          hipLaunchKernelGGL(sh == 1 ? gdsm::probe_copy_pages_kernel<false>
                                     : gdsm::probe_copy_pages_kernel<true>,
                             dim3((unsigned)g), dim3(256), 0, ctx->stream,
                             static_cast<gdsm::u32x4p*>(dst), static_cast<const gdsm::u32x4p*>(a),
                             n_pages);
        }
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipEventRecord(e1, ctx->stream);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      float t = 0;
      if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
      if (e != hipSuccess) rc = map_err(e);
      ms.push_back(t);
    }
    if (rc) break;
    std::sort(ms.begin(), ms.end());
    if (sh == 0 || ms.front() < best) {
      best = ms.front();
      med = ms[ms.size() / 2];
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc) return rc;
  *best_ms = best;
  *median_ms = med;
  return 0;
}
