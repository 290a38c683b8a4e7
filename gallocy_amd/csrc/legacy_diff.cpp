// Legacy drop-in for the reference diff() (gallocy/include/gallocy/utils/diff.h:9-11,
// gallocy/utils/diff.cpp:73-167): Needleman-Wunsch global alignment of two byte strings, CPU.
//
// Same observable behaviour as the reference for every input it survives (n, m <= 1180):
//   * scores: match +1, mismatch 0 (the ternary `Cost::MATCH ? a == b : Cost::MISMATCH` at
//     diff.cpp:107-108 always takes the (a == b) arm), gap -1 (diff.cpp:21-26, 94-102, 109-110);
//   * tie-break diag > left > up (diff.cpp:115-120);
//   * traceback from (n, m) to (0, 0), gaps written as '-' into the other string (142-158);
//   * outputs are NUL-terminated and allocated by the installed allocator, which gallocy sets to
//     internal_malloc so its callers keep calling internal_free (diff.cpp:135-136);
//   * returns 0.
// Different by design: the DP keeps an int32 score row pair and a 1-byte direction per cell
// (the reference keeps a 24-byte Element per cell in its 32 MiB internal zone and crashes from
// n = m = 1181 on), the output buffers are L + 1 bytes (the reference writes one byte past an
// L-byte buffer, diff.cpp:139-140), and row 0 / column 0 never read out of bounds
// (diff.cpp:146-152 index _matrix[-1]).
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "gdsm.h"

namespace gdsm {
int nw_host(gdsm_ctx* ctx, const char* m1, size_t n1, const char* m2, size_t n2,
            void* (*alloc)(size_t), void (*release)(void*), char** o1, char** o2, size_t* len);
}

namespace {
void* (*g_alloc)(size_t) = malloc;
void (*g_free)(void*) = free;
gdsm_ctx* g_dev_ctx = nullptr;    // gdsm_set_diff_device
uint64_t g_dev_min_cells = 0;
// The offload path stages through one context (its stream, staging buffers and error word):
// concurrent diff() calls are serialised there. The CPU path is reentrant like the reference's
// (every call allocates its own DP rows).
std::mutex g_dev_mu;

int nw_align(const char* m1, size_t n1, const char* m2, size_t n2, char** o1, char** o2,
             size_t* len) {
  if (g_dev_ctx && (uint64_t)n1 * n2 >= g_dev_min_cells) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    return gdsm::nw_host(g_dev_ctx, m1, n1, m2, n2, g_alloc, g_free, o1, o2, len);
  }
  const size_t C = n2 + 1;
  std::vector<int32_t> prev(C), row(C);
  std::vector<uint8_t> dir((n1 + 1) * C);  // 1 diag, 2 left, 3 up
  for (size_t x = 0; x < C; ++x) {
    prev[x] = -(int32_t)x;
    dir[x] = x ? 2 : 0;
  }
  for (size_t y = 1; y <= n1; ++y) {
    row[0] = -(int32_t)y;
    uint8_t* d = &dir[y * C];
    d[0] = 3;
    const char a = m1[y - 1];
    for (size_t x = 1; x < C; ++x) {
      const int32_t dg = prev[x - 1] + (a == m2[x - 1]);
      const int32_t lf = row[x - 1] - 1;
      const int32_t up = prev[x] - 1;
      const int32_t mx = dg >= lf ? (dg >= up ? dg : up) : (lf >= up ? lf : up);
      d[x] = (dg == mx) ? 1 : (lf == mx) ? 2 : 3;
      row[x] = mx;
    }
    prev.swap(row);
  }
  size_t L = 0;
  for (size_t y = n1, x = n2; y || x; ++L) {
    const uint8_t d = dir[y * C + x];
    if (d == 1) { --y; --x; } else if (d == 2) { --x; } else { --y; }
  }
  char* a1 = static_cast<char*>(g_alloc(L + 1));
  char* a2 = static_cast<char*>(g_alloc(L + 1));
  if (!a1 || !a2) {
    if (a1) g_free(a1);
    if (a2) g_free(a2);
    return -ENOMEM;
  }
  a1[L] = 0;
  a2[L] = 0;
  size_t k = L;
  for (size_t y = n1, x = n2; y || x;) {
    const uint8_t d = dir[y * C + x];
    --k;
    if (d == 1) { a1[k] = m1[y - 1]; a2[k] = m2[x - 1]; --y; --x; }
    else if (d == 2) { a1[k] = '-'; a2[k] = m2[x - 1]; --x; }
    else { a1[k] = m1[y - 1]; a2[k] = '-'; --y; }
  }
  *o1 = a1;
  *o2 = a2;
  if (len) *len = L;
  return 0;
}
}  // namespace

extern "C" int gdsm_set_allocator(void* (*alloc_fn)(size_t), void (*free_fn)(void*)) {
  if (!alloc_fn || !free_fn) return -EINVAL;
  g_alloc = alloc_fn;
  g_free = free_fn;
  return 0;
}

extern "C" int gdsm_set_diff_device(gdsm_ctx* ctx, uint64_t min_cells) {
  g_dev_ctx = ctx;
  g_dev_min_cells = min_cells;
  return 0;
}

extern "C" int gdsm_nw_diff(const char* mem1, size_t mem1_len, char** out1, const char* mem2,
                            size_t mem2_len, char** out2, size_t* len) {
  if (!out1 || !out2 || (!mem1 && mem1_len) || (!mem2 && mem2_len)) return -EINVAL;
  return nw_align(mem1, mem1_len, mem2, mem2_len, out1, out2, len);
}

int diff(const char* mem1, size_t mem1_len, char*& mem1_alignment, const char* mem2,
         size_t mem2_len, char*& mem2_alignment) {
  char* a = nullptr;
  char* b = nullptr;
  // 0 like the reference; a GPU failure (gdsm_set_diff_device) leaves both outputs NULL and
  // returns its negative errno instead of falling back.
  const int rc = nw_align(mem1, mem1_len, mem2, mem2_len, &a, &b, nullptr);
  mem1_alignment = a;
  mem2_alignment = b;
  return rc;
}
