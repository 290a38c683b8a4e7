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
//   3. every output checked to lie inside the internal heap's 32 MiB zone
//      (get_heap_location(PURPOSE_INTERNAL_HEAP), utils/constants.cpp:36-54), to have an
//      internal_malloc_usable_size covering the string, and released with internal_free; the
//      freed space is handed out again by the next internal_malloc (first-fit reuse,
//      test/test_internal_allocator.cpp:105-138).
// Prints "ok <checks>" and exits 0, or names the failing check and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

static bool in_internal_zone(const void* p) {
  const char* base = static_cast<const char*>(get_heap_location(PURPOSE_INTERNAL_HEAP));
  const char* q = static_cast<const char*>(p);
  return q >= base && q < base + ZONE_SZ;
}

static void check_owned(char* s) {
  CHECK(s != nullptr);
  CHECK(in_internal_zone(s));
  CHECK(internal_malloc_usable_size(s) >= strlen(s) + 1);
}

int main() {
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
