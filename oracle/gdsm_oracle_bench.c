/*
 * CPU baseline driver over the oracle — TEST / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's
 * cpu_baseline leg). OpenMP threads, each on its own sample of the workload, time repeated
 * diff + apply passes of the C restatement (or_diff_pages + or_apply, docs/SPEC.md §3-4) in C.
 */
#define _POSIX_C_SOURCE 200809L
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#include "gdsm_oracle.h"

int or_bench_diff_apply(uint64_t n, int mode, uint32_t ppm, uint64_t seed, double seconds,
                        int threads, uint64_t* pages, double* elapsed, int* ok) {
  if (n == 0 || threads < 1) return -22;
  uint64_t total = 0;
  double slowest = 0.0;
  int all_ok = 1, failed = 0;
#pragma omp parallel num_threads(threads) reduction(+ : total) reduction(max : slowest) \
    reduction(&& : all_ok) reduction(|| : failed)
  {
    const uint64_t first = (uint64_t)omp_get_thread_num() * n;
    uint8_t* twin = malloc(n * OR_PAGE_SZ);
    uint8_t* cur = malloc(n * OR_PAGE_SZ);
    uint8_t* rep = malloc(n * OR_PAGE_SZ);
    uint64_t* rec_off = malloc((n + 1) * sizeof(uint64_t));
    uint8_t* data = NULL;
    uint64_t cap = 0, reps = 0;
    double t0 = 0.0, dt = 0.0;
    const int have = twin && cur && rep && rec_off;
    if (have) {
      or_gen_pages(twin, cur, rep, first, 1, n, seed, mode, ppm);
      cap = or_diff_pages(twin, cur, NULL, n, rec_off, NULL, 0);  // sizes the stream
      data = malloc(cap ? cap : 1);
    }
    failed = !(have && data);
#pragma omp barrier
    if (!failed) {
      t0 = omp_get_wtime();
      do {
        or_diff_pages(twin, cur, NULL, n, rec_off, data, cap);
        if (or_apply(rep, NULL, n, rec_off, data)) failed = 1;
        ++reps;
        dt = omp_get_wtime() - t0;
      } while (dt < seconds && !failed);
      all_ok = memcmp(rep, cur, n * OR_PAGE_SZ) == 0;
    }
    total = reps * n;
    slowest = dt;
    free(twin);
    free(cur);
    free(rep);
    free(rec_off);
    free(data);
  }
  *pages = total;
  *elapsed = slowest;
  *ok = all_ok && !failed;
  return failed ? -12 : 0;
}
