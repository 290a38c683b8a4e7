/*
 * gdsm oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the DSM hot path, used as the parity checker for the HIP
 * engine. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (libgdsm.so) never links or calls it.
 *
 * Pinning:
 *   - or_nw_diff restates the reference diff() (gallocy/utils/diff.cpp:73-167) and is checked
 *     against the reference's own golden strings (test/test_diff.cpp:13-16,29-31) and against
 *     vectors produced by the reference itself compiled here (oracle/_ref, tests/golden/).
 *   - Twin / run-diff / apply / coherence have no reference implementation and no reference
 *     test: they follow docs/SPEC.md. PARITY UNPINNED by the reference, except for the one
 *     bridge checked in tests: for equal-length substitution-only inputs where the reference
 *     NW alignment is gap-free, {i : out1[i] != out2[i]} equals the union of our runs.
 */
#ifndef GDSM_ORACLE_H_
#define GDSM_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_PAGE_SZ 4096u

uint64_t or_mix64(uint64_t z);
uint64_t or_hash3(uint64_t s, uint64_t a, uint64_t b);

/* SPEC §6. Arena page i is global page first_page + i * stride. Any arena may be NULL. */
void or_gen_pages(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t first_page,
                  uint64_t stride, uint64_t n, uint64_t seed, int mode, uint32_t ppm);

/* SPEC §3. ids == NULL means identity (ids[i] = i). Returns rec_off[n] (bytes required);
 * data bytes at or past cap are not written. */
uint64_t or_diff_pages(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                       uint64_t n, uint64_t* rec_off, uint8_t* data, uint64_t cap);

/* SPEC §4. Returns 0, or -22 (EINVAL) on a malformed record. */
int or_apply(uint8_t* target, const uint32_t* ids, uint64_t n, const uint64_t* rec_off,
             const uint8_t* data);

/* SPEC §2. */
void or_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n);

/* Restatement of the reference NW diff() (gallocy/utils/diff.cpp:73-167).
 * out1/out2 must hold n1+n2+1 bytes. Writes the alignment (NUL terminated) and its length. */
int or_nw_diff(const char* m1, size_t n1, const char* m2, size_t n2, char* out1, char* out2,
               size_t* out_len);

/* SPEC §5. */
void or_coh_init(uint32_t* state, uint32_t* faults, uint64_t n_pages, uint32_t n_nodes);
/* totals[0] = invalidations, totals[1] = transfers, totals[2..10) = node faults.
 * Returns 0, or -22 if the batch is not sorted by page or names a page >= n_pages or a node
 * >= n_nodes (the state is then partly folded). */
int or_coherence(uint32_t* state, uint32_t* faults, uint64_t n_pages, uint32_t n_nodes,
                 const uint64_t* events, uint64_t n_events, uint64_t* totals);

/* SPEC §6 event fill from per-page counts; offsets = exclusive scan of counts (n+1). */
void or_gen_events(uint64_t* events, const uint64_t* offsets, uint64_t first_page, uint64_t n,
                   uint64_t seed, uint32_t n_nodes, uint32_t write_pct);

/* bench.py's CPU baseline only (gdsm_oracle_bench.c): `threads` OpenMP threads, thread t on
 * pages [t*n, (t+1)*n) of the SPEC §6 workload, repeat diff + apply passes for `seconds`.
 * *pages = pages processed by all threads, *elapsed = the slowest thread's seconds, *ok = every
 * replica equals its current arena. Returns 0, -12 (allocation) or -22. */
int or_bench_diff_apply(uint64_t n, int mode, uint32_t ppm, uint64_t seed, double seconds,
                        int threads, uint64_t* pages, double* elapsed, int* ok);
/* Tests only: the stream (rec_off[n + 1], data) of the SPEC §6 workload's pages [first, first + n)
 * equals the oracle's, record by record (each record's size and bytes), regenerating the pages
 * 4096 at a time on `threads` OpenMP threads. Returns -1 when every record matches, the first
 * mismatching page index otherwise, -2 on an allocation failure. */
int64_t or_check_stream(const uint64_t* rec_off, const uint8_t* data, uint64_t first,
                        uint64_t n, uint64_t seed, int mode, uint32_t ppm, int threads);
int or_bench_coherence(const uint64_t* events, const uint64_t* page_off, uint64_t n_pages,
                       uint32_t n_nodes, double seconds, int threads, uint64_t* done,
                       double* elapsed);
/* bench.py's config-5 CPU baseline (gdsm_oracle_bench.c): the mmult trace's round loop on one
 * thread, timed in C. */
int or_bench_mmult(uint32_t* state, uint32_t* faults, uint64_t zone_pages, uint32_t nodes,
                   uint8_t* twin, uint8_t* cur, uint8_t* rep, uint64_t rounds,
                   const uint64_t* events, const uint64_t* ev_off, const uint32_t* ids,
                   const uint32_t* home, const uint64_t* ids_off, const uint64_t* row_dst,
                   const uint32_t* row_src, const uint64_t* row_off, const uint8_t* rowvals,
                   uint64_t row_bytes, uint64_t* totals, double* elapsed, int retwin);

#ifdef __cplusplus
}
#endif
#endif
