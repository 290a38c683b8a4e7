// Coherence across GPUs (SPEC §5b): the kernels behind gdsm_route_events (a node's
// fault events to the pages' home shards) and gdsm_coherence_notify (the homes' access-change
// notices back to the nodes). The transfers themselves are in gdsm_exchange.cpp.
//
// The reference describes the step these replace as "negotiate access, copy over the latest
// contents, update page tables and protections" (resources/NUTSHELL.md:61-69), carried by its
// HTTP fan-out (gallocy/http/client.cpp:39-91) from the Raft leader (consensus/client.cpp:15-42);
// none of it is implemented there.
//
// Integer / index work, HBM-bound and tiny next to the fold itself: binary searches over sorted
// event lists (split, merge by rank), one gather of the touched pages' words before the fold and
// one after, and a per-destination compaction of the notices (ballot + mbcnt ranks inside a
// block, one scan of the block counts).
#include "gdsm_common.h"
#include "gdsm_launch.h"

namespace gdsm {

constexpr int kStampShift = 36;  // stamped event: page << 36 | seq << 4 | node << 1 | rw

// ------------------------------------------------------------------------- node side: split
// Validates a node's stamped events (sorted, page < total_pages, node < G) and finds each home's
// slice: bounds[d] = first event of a page >= d * per. counts[d] = its length (u64, the all-to-all
// input). bad |= 1 on any invalid event (then the bounds mean nothing and the call is refused).
__global__ __launch_bounds__(256) void route_split_kernel(const uint64_t* __restrict__ ev,
                                                          uint64_t n, uint64_t total_pages,
                                                          uint64_t per, uint32_t G,
                                                          uint64_t* __restrict__ counts,
                                                          uint64_t* __restrict__ bounds,
                                                          uint32_t* __restrict__ bad) {
  uint32_t v = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = ev[i];
    if ((x >> kStampShift) >= total_pages || ((x >> 1) & 7u) >= G) v = 1;
    if (i + 1 < n && ev[i + 1] < x) v = 1;
  }
  if (__ballot(v) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
  if (blockIdx.x != 0) return;  // block-uniform
  __shared__ uint64_t b[GDSM_MAX_NODES + 1];
  const uint32_t t = threadIdx.x;
  if (t <= G) {
    const uint64_t first = (uint64_t)t * per;
    uint64_t lo = 0, hi = n;
    if (t == G || first >= total_pages) {
      lo = n;
    } else {
      const uint64_t key = first << kStampShift;
      while (lo < hi) {  // first index with ev >= key
        const uint64_t mid = (lo + hi) >> 1;
        if (ev[mid] < key) lo = mid + 1; else hi = mid;
      }
    }
    b[t] = lo;
  }
  __syncthreads();
  if (t <= G) bounds[t] = b[t];
  if (t < G) counts[t] = b[t + 1] - b[t];
}

// ------------------------------------------------------------------------- home side: merge
// The received slices (one sorted run per source node, back to back at off[s]) merged into one
// page-sorted batch by rank: an element's place is its index in its own run plus, for every other
// run, the number of elements before it (equal keys: lower-numbered sources first). Output in
// SPEC §5 packing with the local page: (page - base) << 4 | node << 1 | rw.
struct RunOffsets {
  uint64_t o[GDSM_MAX_NODES + 1];
};

__global__ __launch_bounds__(256) void route_merge_kernel(const uint64_t* __restrict__ runs,
                                                          RunOffsets off, uint32_t G,
                                                          uint64_t base,
                                                          uint64_t* __restrict__ out) {
  const uint64_t total = off.o[G];
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s = 0;
    for (uint32_t t = 1; t < G; ++t)
      if (off.o[t] <= idx) s = t;
    const uint64_t x = runs[idx];
    uint64_t pos = idx - off.o[s];
    for (uint32_t t = 0; t < G; ++t) {
      if (t == s) continue;
      uint64_t lo = off.o[t], hi = off.o[t + 1];
      const bool le = t < s;  // an earlier source's equal key goes first
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint64_t y = runs[mid];
        if (le ? y <= x : y < x) lo = mid + 1; else hi = mid;
      }
      pos += lo - off.o[t];
    }
    out[pos] = (((x >> kStampShift) - base) << 4) | (x & 15u);
  }
}

// ------------------------------------------------------------------------- notices (SPEC §5b)
// A node's access to a page, from the page's state word: 0 none, 1 read, 2 write.
__device__ __forceinline__ uint32_t access_of(uint32_t w, uint32_t node) {
  const uint32_t st = (w >> 16) & 3u;
  if (st == 0 || !((w >> node) & 1u)) return 0;
  return (st == 2 && ((w >> 8) & 0xFFu) == node) ? 2u : 1u;
}

// Nodes (< G) that get a notice: their access changed, or they are the old or the new owner of a
// page whose owner changed.
__device__ __forceinline__ uint32_t notice_mask(uint32_t pre, uint32_t post, uint32_t G) {
  const uint32_t ob = (pre >> 8) & 0xFFu, oa = (post >> 8) & 0xFFu;
  uint32_t m = 0;
  for (uint32_t d = 0; d < G; ++d) {
    const bool chg = access_of(pre, d) != access_of(post, d) || (ob != oa && (d == ob || d == oa));
    m |= (uint32_t)chg << d;
  }
  return m;
}

__device__ __forceinline__ uint64_t notice_word(uint64_t gpage, uint32_t pre, uint32_t post,
                                                uint32_t d) {
  return gpage | ((uint64_t)access_of(pre, d) << 32) | ((uint64_t)access_of(post, d) << 34) |
         ((uint64_t)((pre >> 8) & 0xFFu) << 40) | ((uint64_t)((post >> 8) & 0xFFu) << 48);
}

__device__ __forceinline__ bool batch_head(const uint64_t* __restrict__ batch, uint64_t i,
                                           uint32_t& page) {
  page = (uint32_t)batch[i] >> 4;
  return i == 0 || ((uint32_t)batch[i - 1] >> 4) != page;
}

// Before the fold: the state word of every page the batch touches, at its first event, and the
// number of such pages (heads += one atomic per wave; the bound on any node's notices).
__global__ __launch_bounds__(256) void notice_pre_kernel(const uint64_t* __restrict__ pt,
                                                         uint64_t n_pages,
                                                         const uint64_t* __restrict__ batch,
                                                         uint64_t n, uint32_t* __restrict__ pre,
                                                         unsigned long long* __restrict__ heads) {
  uint32_t cnt = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t page;
    if (batch_head(batch, i, page)) {
      ++cnt;
      if (page < n_pages) pre[i] = (uint32_t)pt[page];
    }
  }
  const uint32_t w = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(heads, (unsigned long long)w);
}

// After the fold, one event per thread, 256 per block. kEmit = false: per-block notice counts per
// destination node (blk[b * 8 + d]). kEmit = true: the notices, written destination-major at
// dest_base[d] + blk_off[b * 8 + d] + their rank inside the block (event order).
template <bool kEmit>
__global__ __launch_bounds__(256) void notice_kernel(const uint64_t* __restrict__ pt,
                                                     uint64_t n_pages,
                                                     const uint64_t* __restrict__ batch,
                                                     uint64_t n, const uint32_t* __restrict__ pre,
                                                     uint32_t G, uint64_t base,
                                                     uint32_t* __restrict__ blk,
                                                     const uint64_t* __restrict__ blk_off,
                                                     const uint64_t* __restrict__ dest_base,
                                                     uint64_t* __restrict__ out) {
  __shared__ uint32_t wcnt[4][GDSM_MAX_NODES];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t mask = 0, pw = 0, qw = 0, page = 0;
  if (i < n && batch_head(batch, i, page) && page < n_pages) {
    pw = pre[i];
    qw = (uint32_t)pt[page];
    mask = notice_mask(pw, qw, G);
  }
  uint32_t rank[GDSM_MAX_NODES];
#pragma unroll
  for (uint32_t d = 0; d < GDSM_MAX_NODES; ++d) {
    const uint64_t B = __ballot((mask >> d) & 1u);
    rank[d] = __builtin_amdgcn_mbcnt_hi((uint32_t)(B >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
    if (lane == 0) wcnt[wave][d] = (uint32_t)__popcll(B);
  }
  __syncthreads();
  if (!kEmit) {
    if (threadIdx.x < GDSM_MAX_NODES)
      blk[blockIdx.x * GDSM_MAX_NODES + threadIdx.x] =
          wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] +
          wcnt[3][threadIdx.x];
    return;
  }
#pragma unroll
  for (uint32_t d = 0; d < GDSM_MAX_NODES; ++d) {
    if (!((mask >> d) & 1u)) continue;
    uint64_t at = dest_base[d] + blk_off[blockIdx.x * GDSM_MAX_NODES + d] + rank[d];
    for (uint32_t w = 0; w < wave; ++w) at += wcnt[w][d];
    out[at] = notice_word(base + page, pw, qw, d);
  }
}

// One workgroup: exclusive scan of the block counts per destination (blk -> blk_off), the
// destinations' totals (u64, the all-to-all input) and their exclusive bases.
__global__ __launch_bounds__(256) void notice_scan_kernel(const uint32_t* __restrict__ blk,
                                                          uint64_t nblk, uint32_t G,
                                                          uint64_t* __restrict__ blk_off,
                                                          uint64_t* __restrict__ dest_total,
                                                          uint64_t* __restrict__ dest_base) {
  __shared__ uint32_t wtot[4];
  __shared__ uint64_t tot[GDSM_MAX_NODES];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t d = 0; d < GDSM_MAX_NODES; ++d) {
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nblk; c0 += 256) {
      const uint64_t b = c0 + threadIdx.x;
      const uint32_t v = b < nblk ? blk[b * GDSM_MAX_NODES + d] : 0u;
      const uint32_t inc = wave_incl_sum(v);
      if (lane == 63) wtot[wave] = inc;
      __syncthreads();
      uint64_t pre = carry;
      for (uint32_t w = 0; w < wave; ++w) pre += wtot[w];
      if (b < nblk) blk_off[b * GDSM_MAX_NODES + d] = pre + inc - v;
      carry += (uint64_t)wtot[0] + wtot[1] + wtot[2] + wtot[3];
      __syncthreads();
    }
    if (threadIdx.x == 0) tot[d] = d < G ? carry : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (uint32_t d = 0; d < GDSM_MAX_NODES; ++d) {
      if (d < G) {
        dest_total[d] = tot[d];
        dest_base[d] = acc;
      }
      acc += tot[d];
    }
  }
}

// ------------------------------------------------------------------------- launchers
static inline unsigned grid_of(uint64_t work, unsigned cap) {
  uint64_t g = (work + 255) / 256;
  if (g > cap) g = cap;
  return g ? (unsigned)g : 1u;
}

hipError_t launch_route_split(const uint64_t* ev, uint64_t n, uint64_t total_pages, uint64_t per,
                              uint32_t G, uint64_t* counts, uint64_t* bounds, uint32_t* bad,
                              hipStream_t s) {
  hipLaunchKernelGGL(route_split_kernel, dim3(grid_of(n, 2048)), dim3(256), 0, s, ev, n,
                     total_pages, per, G, counts, bounds, bad);
  return hipGetLastError();
}

hipError_t launch_route_merge(const uint64_t* runs, const uint64_t* off, uint32_t G, uint64_t base,
                              uint64_t* out, hipStream_t s) {
  RunOffsets o{};
  for (uint32_t t = 0; t <= G; ++t) o.o[t] = off[t];
  if (o.o[G] == 0) return hipSuccess;
  hipLaunchKernelGGL(route_merge_kernel, dim3(grid_of(o.o[G], 8192)), dim3(256), 0, s, runs, o, G,
                     base, out);
  return hipGetLastError();
}

uint64_t notice_blocks(uint64_t n) { return (n + 255) / 256; }

hipError_t launch_notice_pre(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                             uint64_t n, uint32_t* pre, uint64_t* heads, hipStream_t s) {
  hipError_t e = hipMemsetAsync(heads, 0, 8, s);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(notice_pre_kernel, dim3(grid_of(n, 8192)), dim3(256), 0, s, pt, n_pages, batch,
                     n, pre, reinterpret_cast<unsigned long long*>(heads));
  return hipGetLastError();
}

hipError_t launch_notice_count(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                               uint64_t n, const uint32_t* pre, uint32_t G, uint32_t* blk,
                               uint64_t* blk_off, uint64_t* dest_total, uint64_t* dest_base,
                               hipStream_t s) {
  const uint64_t nb = notice_blocks(n);
  if (nb)
    hipLaunchKernelGGL(notice_kernel<false>, dim3((unsigned)nb), dim3(256), 0, s, pt, n_pages,
                       batch, n, pre, G, 0ull, blk, nullptr, nullptr, nullptr);
  hipLaunchKernelGGL(notice_scan_kernel, dim3(1), dim3(256), 0, s, blk, nb, G, blk_off,
                     dest_total, dest_base);
  return hipGetLastError();
}

hipError_t launch_notice_emit(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                              uint64_t n, const uint32_t* pre, uint32_t G, uint64_t base,
                              const uint64_t* blk_off, const uint64_t* dest_base, uint64_t* out,
                              hipStream_t s) {
  const uint64_t nb = notice_blocks(n);
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(notice_kernel<true>, dim3((unsigned)nb), dim3(256), 0, s, pt, n_pages, batch,
                     n, pre, G, base, nullptr, blk_off, dest_base, out);
  return hipGetLastError();
}

}  // namespace gdsm
