// Diff wire format (docs/SPEC.md §7): a diff stream framed, checksummed and
// base64-encoded into the text of a Raft log command (gallocy Command{string},
// gallocy/include/gallocy/consensus/log.h:18-27, shipped in append-entries JSON by
// consensus/client.cpp:133-142), and back. All byte work, HBM-bound, one pass each:
//   wire_sum_kernel    — Σ mix64(w_i + i·φ) over the frame's 8-byte words (checksum field = 0)
//   b64_encode_kernel  — 12 frame bytes -> 16 characters per thread (3 dword loads, 1 uint4 store)
//   b64_decode_kernel  — 16 characters -> 12 bytes per thread; bad characters flag the error word
//   wire_check_kernel  — rec_off monotone / 4-aligned / ending at D, ids inside the arena
#include "gdsm_common.h"
#include "gdsm_launch.h"

namespace gdsm {
namespace {

constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint32_t b64_char(uint32_t v) {
  return v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '+' : '/';
}

// 6-bit value of a base64 character, or 64 for anything outside the alphabet.
__device__ __forceinline__ uint32_t b64_val(uint32_t c) {
  if (c - 'A' < 26u) return c - 'A';
  if (c - 'a' < 26u) return c - 'a' + 26;
  if (c - '0' < 10u) return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return 64;
}

__global__ __launch_bounds__(256) void wire_sum_kernel(const uint64_t* __restrict__ w,
                                                       uint64_t nw, uint64_t* __restrict__ sum) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = i == 3 ? 0 : w[i];  // word 3 = the checksum field
    acc += mix64(v + i * kPhi);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) acc += __shfl_down(acc, d, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(reinterpret_cast<unsigned long long*>(sum), acc);
}

__global__ __launch_bounds__(256) void b64_encode_kernel(const uint8_t* __restrict__ frame,
                                                         uint64_t F, uint8_t* __restrict__ text,
                                                         uint64_t T) {
  const uint64_t g = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t ib = g * 12, ob = g * 16;
  if (ob >= T) return;
  const uint32_t* fw = reinterpret_cast<const uint32_t*>(frame + ib);
  // F is a multiple of 8, so each of the three dwords is wholly inside or outside the frame.
  const uint32_t d0 = ib + 4 <= F ? fw[0] : 0u;
  const uint32_t d1 = ib + 8 <= F ? fw[1] : 0u;
  const uint32_t d2 = ib + 12 <= F ? fw[2] : 0u;
  uint32_t out[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // triplet q = bytes 3q .. 3q+2 of the 12
    auto byte = [&](int k) -> uint32_t {
      const uint32_t d = k < 4 ? d0 : k < 8 ? d1 : d2;
      return (d >> (8 * (k & 3))) & 0xFFu;
    };
    const uint32_t v = (byte(3 * q) << 16) | (byte(3 * q + 1) << 8) | byte(3 * q + 2);
    const uint64_t tb = ib + 3 * q;  // first frame byte of the triplet
    const uint32_t have = tb >= F ? 0u : (uint32_t)(F - tb < 3 ? F - tb : 3);
    uint32_t c0 = b64_char(v >> 18), c1 = b64_char((v >> 12) & 63);
    uint32_t c2 = have >= 2 ? b64_char((v >> 6) & 63) : '=';
    uint32_t c3 = have >= 3 ? b64_char(v & 63) : '=';
    out[q] = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
  }
  if (ob + 16 <= T) {
    *reinterpret_cast<uint4*>(text + ob) = make_uint4(out[0], out[1], out[2], out[3]);
  } else {
    for (uint64_t k = 0; k < T - ob; ++k) text[ob + k] = (uint8_t)(out[k >> 2] >> (8 * (k & 3)));
  }
}

__global__ __launch_bounds__(256) void b64_decode_kernel(const uint8_t* __restrict__ text,
                                                         uint64_t T, uint32_t pad,
                                                         uint8_t* __restrict__ frame, uint64_t F,
                                                         uint32_t* __restrict__ err) {
  const uint64_t g = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t ib = g * 16, ob = g * 12;
  if (ib >= T) return;
  uint32_t c[16];
  if (ib + 16 <= T) {
    const uint4 v = *reinterpret_cast<const uint4*>(text + ib);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = ib + k < T ? text[ib + k] : 'A';
  }
  uint32_t bad = 0, bytes[12];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t pos = ib + 4 * q + k;
      uint32_t x = b64_val(c[4 * q + k]);
      if (x == 64 && c[4 * q + k] == '=' && pos >= T - pad) x = 0;  // trailing padding only
      bad |= x >> 6;
      v = (v << 6) | (x & 63);
    }
    bytes[3 * q] = v >> 16;
    bytes[3 * q + 1] = (v >> 8) & 0xFFu;
    bytes[3 * q + 2] = v & 0xFFu;
  }
  if (bad) atomicOr(err, 8u);
  if (ob + 12 <= F) {
    uint32_t* fw = reinterpret_cast<uint32_t*>(frame + ob);
#pragma unroll
    for (int d = 0; d < 3; ++d)
      fw[d] = bytes[4 * d] | (bytes[4 * d + 1] << 8) | (bytes[4 * d + 2] << 16) |
              (bytes[4 * d + 3] << 24);
  } else {
    for (uint64_t k = 0; ob + k < F && k < 12; ++k) frame[ob + k] = (uint8_t)bytes[k];
  }
}

__global__ __launch_bounds__(256) void wire_check_kernel(const uint32_t* __restrict__ ids,
                                                         const uint64_t* __restrict__ rec_off,
                                                         uint64_t n, uint64_t D, uint64_t n_pages,
                                                         uint32_t* __restrict__ err) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i > n) return;
  const uint64_t o = rec_off[i];
  bool bad = (o & 3) != 0;
  if (i == 0) bad |= o != 0;
  if (i == n) bad |= o != D;
  else bad |= rec_off[i + 1] < o || ids[i] >= n_pages;
  if (bad) atomicOr(err, 16u);
}

__global__ __launch_bounds__(256) void iota_kernel(uint32_t* __restrict__ dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    dst[i] = (uint32_t)i;
}

uint32_t grid(uint64_t threads) {
  const uint64_t b = (threads + 255) / 256;
  return (uint32_t)(b ? (b < (1u << 30) ? b : (1u << 30)) : 1);
}

}  // namespace

uint64_t wire_frame_bytes(uint64_t n, uint64_t D) {
  return 32 + 4 * ((n + 1) & ~1ull) + 8 * (n + 1) + ((D + 7) & ~7ull);
}

hipError_t launch_wire_sum(const uint8_t* frame, uint64_t F, uint64_t* sum, hipStream_t s) {
  hipError_t e = hipMemsetAsync(sum, 0, 8, s);
  if (e != hipSuccess) return e;
  const uint64_t nw = F / 8;
  const uint32_t blocks = grid(nw) < 4096 ? grid(nw) : 4096;
  hipLaunchKernelGGL(wire_sum_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<const uint64_t*>(frame), nw, sum);
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* dst, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = grid(n) < 4096 ? grid(n) : 4096;
  hipLaunchKernelGGL(iota_kernel, dim3(blocks), dim3(256), 0, s, dst, n);
  return hipGetLastError();
}

hipError_t launch_b64_encode(const uint8_t* frame, uint64_t F, uint8_t* text, hipStream_t s) {
  const uint64_t T = 4 * ((F + 2) / 3);
  hipLaunchKernelGGL(b64_encode_kernel, dim3(grid((T + 15) / 16)), dim3(256), 0, s, frame, F,
                     text, T);
  return hipGetLastError();
}

hipError_t launch_b64_decode(const uint8_t* text, uint64_t T, uint32_t pad, uint8_t* frame,
                             uint64_t F, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(b64_decode_kernel, dim3(grid((T + 15) / 16)), dim3(256), 0, s, text, T, pad,
                     frame, F, err);
  return hipGetLastError();
}

hipError_t launch_wire_check(const uint32_t* ids, const uint64_t* rec_off, uint64_t n,
                             uint64_t D, uint64_t n_pages, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(wire_check_kernel, dim3(grid(n + 1)), dim3(256), 0, s, ids, rec_off, n, D,
                     n_pages, err);
  return hipGetLastError();
}

}  // namespace gdsm
