/*
 * CPU baseline driver over the oracle — TEST / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's
 * cpu_baseline leg). OpenMP threads, each on its own sample of the workload, time repeated
 * diff + apply passes of the C restatement (or_diff_pages + or_apply, docs/SPEC.md §3-4) in C.
 */
#define _POSIX_C_SOURCE 200809L
#include <omp.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

/* Batched coherence (or_coherence, docs/SPEC.md §5) over `threads` disjoint page ranges of one
 * sorted batch: thread t folds the events of pages [t*n_pages/threads, (t+1)*n_pages/threads)
 * (its slice of `page_off`, the batch's per-page event offsets) into the shared page table,
 * repeatedly for `seconds`. Pages never cross threads, so the fold is the sequential one. */
int or_bench_coherence(const uint64_t* events, const uint64_t* page_off, uint64_t n_pages,
                       uint32_t n_nodes, double seconds, int threads, uint64_t* done,
                       double* elapsed) {
  if (n_pages == 0 || threads < 1) return -22;
  uint32_t* state = malloc(n_pages * sizeof(uint32_t));
  uint32_t* faults = malloc(n_pages * sizeof(uint32_t));
  if (!state || !faults) {
    free(state);
    free(faults);
    return -12;
  }
  or_coh_init(state, faults, n_pages, n_nodes);
  uint64_t total = 0;
  double slowest = 0.0;
  int failed = 0;
#pragma omp parallel num_threads(threads) reduction(+ : total) reduction(max : slowest) \
    reduction(|| : failed)
  {
    const uint64_t t = (uint64_t)omp_get_thread_num(), nt = (uint64_t)omp_get_num_threads();
    const uint64_t p0 = t * n_pages / nt, p1 = (t + 1) * n_pages / nt;
    const uint64_t e0 = page_off[p0], ne = page_off[p1] - e0;
    uint64_t tot[10], reps = 0;
    double dt = 0.0;
#pragma omp barrier
    const double t0 = omp_get_wtime();
    do {
      if (or_coherence(state, faults, n_pages, n_nodes, events + e0, ne, tot)) failed = 1;
      ++reps;
      dt = omp_get_wtime() - t0;
    } while (dt < seconds && !failed);
    total = reps * ne;
    slowest = dt;
  }
  free(state);
  free(faults);
  *done = total;
  *elapsed = slowest;
  return failed ? -22 : 0;
}

int64_t or_check_stream(const uint64_t* rec_off, const uint8_t* data, uint64_t first,
                        uint64_t n, uint64_t seed, int mode, uint32_t ppm, int threads) {
  if (threads < 1) threads = 1;
  const uint64_t kB = 4096;  // pages per work item
  const uint64_t nitems = (n + kB - 1) / kB;
  int64_t bad = -1;
  int failed = 0;
  if (n && rec_off[0] != 0) return 0;
#pragma omp parallel num_threads(threads) reduction(|| : failed)
  {
    uint8_t* twin = malloc(kB * OR_PAGE_SZ);
    uint8_t* cur = malloc(kB * OR_PAGE_SZ);
    uint64_t* ro = malloc((kB + 1) * sizeof(uint64_t));
    uint8_t* buf = NULL;
    uint64_t bcap = 0;
    if (!twin || !cur || !ro) failed = 1;
#pragma omp for schedule(dynamic, 1)
    for (uint64_t it = 0; it < nitems; ++it) {
      if (failed) continue;
      const uint64_t p0 = it * kB, m = n - p0 < kB ? n - p0 : kB;
      or_gen_pages(twin, cur, NULL, first + p0, 1, m, seed, mode, ppm);
      const uint64_t need = or_diff_pages(twin, cur, NULL, m, ro, NULL, 0);
      if (need > bcap) {
        free(buf);
        bcap = need;
        buf = malloc(bcap ? bcap : 1);
        if (!buf) {
          failed = 1;
          continue;
        }
      }
      or_diff_pages(twin, cur, NULL, m, ro, buf, bcap);
      for (uint64_t i = 0; i < m; ++i) {
        const uint64_t a = rec_off[p0 + i], b = rec_off[p0 + i + 1];
        if (b - a != ro[i + 1] - ro[i] || b < a ||
            memcmp(data + a, buf + ro[i], (size_t)(ro[i + 1] - ro[i])) != 0) {
#pragma omp critical
          {
            if (bad < 0 || (int64_t)(p0 + i) < bad) bad = (int64_t)(p0 + i);
          }
          break;
        }
      }
    }
    free(twin);
    free(cur);
    free(ro);
    free(buf);
  }
  return failed ? -2 : bad;
}

/* Config 5 (the test_mmult trace) on one host thread, the whole round loop in C: per round the
 * coherence batch (or_coherence), the twin of the pages the round writes, the row writes, the diff
 * of those pages (or_diff_pages) and its apply to the home copy (or_apply). `nodes` node views
 * of the zone sit side by side in twin / cur (page t * zone_pages + p). The plan is precomputed
 * by the caller (bench.py): round r's events are events[ev_off[r], ev_off[r+1]), its written
 * pages ids / home[ids_off[r], ids_off[r+1]) (node view index / home copy index), its row writes
 * (cur byte offset row_dst[k] <- rowvals row row_src[k], row_bytes each) k in
 * [row_off[r], row_off[r+1]). Timed with CLOCK_MONOTONIC around the loop only; totals are the
 * sums over rounds. Returns 0, -12 (allocation) or the first failing call's code. */

int or_bench_mmult(uint32_t* state, uint32_t* faults, uint64_t zone_pages, uint32_t nodes,
                   uint8_t* twin, uint8_t* cur, uint8_t* rep, uint64_t rounds,
                   const uint64_t* events, const uint64_t* ev_off, const uint32_t* ids,
                   const uint32_t* home, const uint64_t* ids_off, const uint64_t* row_dst,
                   const uint32_t* row_src, const uint64_t* row_off, const uint8_t* rowvals,
                   uint64_t row_bytes, uint64_t* totals, double* elapsed, int retwin) {
  uint64_t max_ids = 0;
  for (uint64_t r = 0; r < rounds; ++r)
    if (ids_off[r + 1] - ids_off[r] > max_ids) max_ids = ids_off[r + 1] - ids_off[r];
  /* the largest record: 4 + 2048 run headers + 4096 payload bytes */
  const uint64_t cap = (max_ids ? max_ids : 1) * (4 + 4 * 2048 + OR_PAGE_SZ);
  uint64_t* rec_off = malloc((max_ids + 1) * sizeof(uint64_t));
  uint8_t* data = malloc(cap);
  if (!rec_off || !data) {
    free(rec_off);
    free(data);
    return -12;
  }
  memset(rec_off, 0, (max_ids + 1) * sizeof(uint64_t));  /* first touches outside the clock */
  memset(data, 0, cap);
  for (int k = 0; k < 10; ++k) totals[k] = 0;
  uint64_t tot[10];
  int rc = 0;
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (uint64_t r = 0; r < rounds && !rc; ++r) {
    rc = or_coherence(state, faults, zone_pages, nodes, events + ev_off[r],
                      ev_off[r + 1] - ev_off[r], tot);
    for (int k = 0; k < 10; ++k) totals[k] += tot[k];
    const uint64_t n = ids_off[r + 1] - ids_off[r];
    const uint32_t* id = ids + ids_off[r];
    if (!retwin) or_twin(twin, cur, id, n);
    for (uint64_t k = row_off[r]; k < row_off[r + 1]; ++k)
      memcpy(cur + row_dst[k], rowvals + (uint64_t)row_src[k] * row_bytes, row_bytes);
    or_diff_pages(twin, cur, id, n, rec_off, data, cap);
    if (!rc) rc = or_apply(rep, home + ids_off[r], n, rec_off, data);
    /* gdsm_release's re-twin: TWIN := CURRENT for the released pages, the dirty bytes only
       (the stream applied to the twin views) */
    if (!rc && retwin) rc = or_apply(twin, id, n, rec_off, data);
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  *elapsed = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
  free(rec_off);
  free(data);
  return rc;
}
