// TEST INFRASTRUCTURE ONLY. Driver for the REFERENCE application heap, compiled by oracle/Makefile
// straight from the sources under /root/reference into oracle/_ref/ref_layout_driver. No
// reference source is copied here.
//
// Linked with gallocy/libgallocy.cpp (custom_malloc, libgallocy.cpp:33-35, over the
// `ApplicationHeapType heap` of heaplayers/application.h:20-29) and allocators/internal.cpp, with
// the reference's own vendored sqlite3 header directory on the include path (external/sqlite3:
// libgallocy.h reaches sqlite.h), as SURVEY §8c's recipe does.
//
//   ref_layout_driver <NDIM>
// makes test_mmult's allocations in its order (test/test_mmult.cpp:31-37 init_matrix for a, b,
// c: a row-pointer array then NDIM rows of NDIM doubles; :152 threads = n pthread_t; :154
// arg = n parm; n = 4) through the reference's custom_malloc, and prints each object's ZONE
// OFFSET, one per line: "a_rp <off>", "a_row <i> <off>" ..., "threads <off>", "args <off>",
// then "zone_used_min <off of the last object's end>". The zone is the mapping the heap's
// first block lies in (read from /proc/self/maps): SourceMmapHeap passes its address to mmap
// only as a hint (heaplayers/source.h:21-22). When the 32 MiB zone runs out the reference prints
// ---ENOMEM--- and aborts (source.h:23-24, 35-36), which is what NDIM 1022 does.
#include <pthread.h>

#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "libgallocy.h"

// constants.cpp:7 declares `extern char* main;`, which g++ >= 11 rejects; the Makefile compiles
// it with -Dmain=__gallocy_main_anchor and this is the renamed variable's definition.
extern "C" {
char* __gallocy_main_anchor;
}

typedef struct {  // test_mmult.cpp:23-28
  int id;
  int noproc;
  int dim;
  double(**a), (**b), (**c);
} parm;

static uintptr_t g_base = 0;

static uintptr_t mapping_start(const void* p) {
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  char line[512];
  uintptr_t found = 0;
  while (!found && fgets(line, sizeof line, f)) {
    uintmax_t l = 0, h = 0;
    if (sscanf(line, "%jx-%jx", &l, &h) == 2 && a >= l && a < h) found = (uintptr_t)l;
  }
  fclose(f);
  return found;
}

static uintptr_t off(const void* p) {
  if (!g_base) g_base = mapping_start(p);
  return reinterpret_cast<uintptr_t>(p) - g_base;
}

static void matrix(const char* name, int ndim) {
  double** m = static_cast<double**>(custom_malloc(sizeof(double*) * ndim));
  printf("%s_rp %" PRIuPTR "\n", name, off(m));
  for (int i = 0; i < ndim; i++) {
    m[i] = static_cast<double*>(custom_malloc(sizeof(double) * ndim));
    printf("%s_row %d %" PRIuPTR "\n", name, i, off(m[i]));
  }
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s NDIM\n", argv[0]);
    return 2;
  }
  const int ndim = atoi(argv[1]);
  const int n = 4;
  setvbuf(stdout, nullptr, _IOFBF, 1 << 20);
  matrix("a", ndim);
  matrix("b", ndim);
  matrix("c", ndim);
  pthread_t* threads = static_cast<pthread_t*>(custom_malloc(n * sizeof(pthread_t)));
  printf("threads %" PRIuPTR "\n", off(threads));
  parm* arg = static_cast<parm*>(custom_malloc(sizeof(parm) * n));
  printf("args %" PRIuPTR "\n", off(arg));
  printf("zone_used_min %" PRIuPTR "\n", off(arg) + sizeof(parm) * n);
  return 0;
}
