// TEST INFRASTRUCTURE ONLY. A compiled C++ caller of libgdsm.so that uses gallocy's own internal
// heap, built by oracle/Makefile into oracle/_ref/legacy_caller from the reference's
// gallocy/allocators/internal.cpp and gallocy/utils/constants.cpp (compiled in place; nothing is
// copied). It proves the ownership contract of the legacy diff() symbol end to end:
//
//   1. gdsm_set_allocator(internal_malloc, internal_free) — the allocator pair whose outputs
//      callers free with internal_free (gallocy/utils/diff.cpp:135-136, 160-164;
//      gallocy/allocators/internal.cpp:31-57);
//   2. the three test/test_diff.cpp bodies (DiffTinyTest :10-20, DiffGeneral_1 :23-35,
//      DiffGeneral_2 :38-57), linked against libgdsm's diff() (mangled _Z4diffPKcmRPcS0_mS2_);
//   3. every output checked to lie inside the internal heap's 32 MiB zone, to have an
//      internal_malloc_usable_size covering the string, and released with internal_free; the
//      freed space is handed out again by the next internal_malloc (first-fit reuse,
//      test/test_internal_allocator.cpp:105-138).
// The zone is taken from what the heap actually mapped: SourceMmapHeap passes
// get_heap_location(PURPOSE_INTERNAL_HEAP) (utils/constants.cpp:36-54) to mmap only as a hint,
// without MAP_FIXED (heaplayers/source.h:21-22), so with ASLR off (brk there) or another mapping in
// the way the kernel places the zone elsewhere. The mapping that holds the heap's first block,
// read from /proc/self/maps, is the zone.
// Prints "ok <checks>" and exits 0, or names the failing check and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cinttypes>

#include "gallocy/allocators/internal.h"
#include "gallocy/utils/constants.h"
#include "gdsm.h"

// constants.cpp:7 declares `extern char* main;`, rejected by g++ >= 11: the Makefile compiles it
// with -Dmain=__gallocy_main_anchor and this is the renamed variable's definition (unused here).
extern "C" {
char* __gallocy_main_anchor;
}

static int g_checks = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    ++g_checks;                                                             \
    if (!(cond)) {                                                          \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static uintptr_t g_zone_lo = 0, g_zone_hi = 0;

// [lo, hi) of the mapping in /proc/self/maps that holds p; false if none does
static bool mapping_of(const void* p, uintptr_t* lo, uintptr_t* hi) {
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  char line[512];
  bool found = false;
  while (!found && fgets(line, sizeof line, f)) {
    uintmax_t l = 0, h = 0;
    if (sscanf(line, "%jx-%jx", &l, &h) == 2 && a >= l && a < h) {
      *lo = (uintptr_t)l;
      *hi = (uintptr_t)h;
      found = true;
    }
  }
  fclose(f);
  return found;
}

static bool in_internal_zone(const void* p) {
  const uintptr_t q = reinterpret_cast<uintptr_t>(p);
  return q >= g_zone_lo && q < g_zone_hi;
}

static void check_owned(char* s) {
  CHECK(s != nullptr);
  CHECK(in_internal_zone(s));
  CHECK(internal_malloc_usable_size(s) >= strlen(s) + 1);
}

int main() {
  {  // the zone: the one shared anonymous mapping of ZONE_SZ bytes that holds a heap block
    void* first = internal_malloc(16);
    CHECK(first != nullptr);
    uintptr_t lo = 0, hi = 0;
    CHECK(mapping_of(first, &lo, &hi));
    CHECK(hi - lo >= (uintptr_t)ZONE_SZ && hi - lo < (uintptr_t)ZONE_SZ + 4096);
    g_zone_lo = lo;
    g_zone_hi = hi;
    internal_free(first);
  }
  CHECK(gdsm_set_allocator(internal_malloc, internal_free) == 0);

  {  // test_diff.cpp:10-20 DiffTinyTest
    char* a1 = NULL;
    char* a2 = NULL;
    CHECK(diff("GGAATGG", 7, a1, "ATG", 3, a2) == 0);
    CHECK(strcmp(a1, "GGAATGG") == 0);
    CHECK(strcmp(a2, "---AT-G") == 0);
    check_owned(a1);
    check_owned(a2);
    internal_free(a1);
    internal_free(a2);
  }
  {  // test_diff.cpp:23-35 DiffGeneral_1
    const char* s1 = "FOO BOP BOOP";
    const char* s2 = "FOOO BOOP BOP";
    char* a1 = NULL;
    char* a2 = NULL;
    CHECK(diff(s1, strlen(s1), a1, s2, strlen(s2), a2) == 0);
    CHECK(strcmp(a1, "F-OO B-OP BOOP") == 0);
    CHECK(strcmp(a2, "FOOO BOOP B-OP") == 0);
    check_owned(a1);
    check_owned(a2);
    // first-fit reuse: the freed block serves the next request of the same size
    const size_t sz = internal_malloc_usable_size(a1);
    internal_free(a1);
    char* again = static_cast<char*>(internal_malloc(sz));
    CHECK(again == a1);
    internal_free(again);
    internal_free(a2);
  }
  {  // test_diff.cpp:38-57 DiffGeneral_2 (inputs from the internal heap too)
    const int mem_sz = 512;
    char* s1 = static_cast<char*>(internal_malloc(mem_sz));
    char* s2 = static_cast<char*>(internal_malloc(mem_sz));
    srand(2026);
    for (int i = 0; i < mem_sz; i++) s1[i] = (char)(1 + rand() % 254);  // no NUL: strlen below
    memcpy(s2, s1, mem_sz);
    int subs = 0;
    for (int i = 0; i < mem_sz; i++)
      if (rand() % 10 == 1) {
        const char c = (char)(1 + rand() % 254);
        subs += c != s2[i];
        s2[i] = c;
      }
    char* a1 = NULL;
    char* a2 = NULL;
    CHECK(diff(s1, mem_sz, a1, s2, mem_sz, a2) == 0);
    check_owned(a1);
    check_owned(a2);
    CHECK(strlen(a1) == strlen(a2));
    CHECK(strlen(a1) >= (size_t)mem_sz);
    internal_free(a1);
    internal_free(a2);
    internal_free(s1);
    internal_free(s2);
    (void)subs;
  }
  {  // many calls: every output goes back to the zone, which therefore never runs out
    for (int r = 0; r < 2000; ++r) {
      char* a1 = NULL;
      char* a2 = NULL;
      CHECK(diff("GATTACA", 7, a1, "GCATGCU", 7, a2) == 0);
      if (r == 0) {
        check_owned(a1);
        check_owned(a2);
      }
      internal_free(a1);
      internal_free(a2);
    }
  }
  printf("ok %d\n", g_checks);
  return 0;
}
