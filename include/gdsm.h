/*
 * gdsm — MI355X-native engine for gallocy's DSM hot path (page twin / run diff / apply /
 * batched coherence). C ABI: plain pointers and sizes, no torch or HIP types in signatures.
 * Semantics are frozen in docs/SPEC.md.
 *
 * Where each entry point sits in the reference (/root/reference, gallocy 0.0.438):
 *   - The reference has no plugin or operator registry; its hot-path "interface" is the leaf
 *     utility `int diff(const char*, size_t, char*&, const char*, size_t, char*&)`
 *     (gallocy/include/gallocy/utils/diff.h:9-11, gallocy/utils/diff.cpp:73-167) plus the
 *     page-tracking hooks of the allocator stack that were never written:
 *     `PageTableHeap<Super>` (gallocy/include/gallocy/heaplayers/pagetableheap.h:12-29, only a
 *     LOG_DEBUG) and the per-page record `ApplicationMemory`
 *     (gallocy/include/gallocy/models.h:171-213, declared, never defined).
 *   - gdsm_diff / gdsm_apply / gdsm_twin replace the twin/diff/apply steps of the
 *     fault → negotiate → "copy over the latest contents" flow that the reference describes but
 *     does not implement (resources/NUTSHELL.md:59-69, resources/IMPLEMENTATION.md:246-249);
 *     the run record is the (offset, bytes) edit of print_diff (gallocy/utils/diff.cpp:43-70).
 *   - gdsm_coh_* replace the ApplicationMemory table (`dirty, owner, permissions, faults`,
 *     models.h:171-213) and the missing page-table application step of Raft's `try_apply`
 *     (gallocy/consensus/state.cpp:308-316).
 *   - gdsm_nw_diff is the reference diff() with the alignment length returned (the reference
 *     drops it, diff.h:9-11); the unchanged legacy C++ symbol `diff` is declared at the bottom.
 *   - The allocator hooks gdsm_set_allocator mirror internal_malloc/internal_free
 *     (gallocy/include/gallocy/allocators/internal.h:75-82), which own diff()'s outputs.
 *
 * Conventions: every function returns 0 or a negative errno (-EINVAL -22, -ENOMEM -12,
 * -EIO -5 for a HIP failure, -ENOSPC -28, -ENODEV -19, -EOVERFLOW -75 for a fixed-budget exchange
 * stream over its budget, -ETIMEDOUT -110 for a loopback rank that never arrived) and never
 * aborts. Device work is
 * enqueued on the context's HIP stream and is asynchronous unless the comment says it
 * synchronises. One context per host thread, or external synchronisation.
 */
#ifndef GDSM_H_
#define GDSM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GDSM_PAGE_SZ 4096u
#define GDSM_MAX_RUNS 2048u
#define GDSM_MAX_NODES 8u
/* Largest page table gdsm_coh_init accepts: page ids of coherence events fit 28 bits (1 TiB of
 * 4 KiB pages, beyond any one GPU's HBM). */
#define GDSM_MAX_COH_PAGES (1ull << 28)
/* Largest record: 4 + 4*2048 + 2048 (alternating bytes), SPEC §3. */
#define GDSM_MAX_RECORD 10244u

enum gdsm_arena_kind { GDSM_TWIN = 0, GDSM_CURRENT = 1, GDSM_REPLICA = 2 };
enum gdsm_gen_mode { GDSM_GEN_UNIFORM = 0, GDSM_GEN_CLUSTERED = 1 };
/* gdsm_init flags: which arenas the context allocates (all three when 0). */
enum gdsm_init_flags {
  GDSM_WANT_TWIN = 1u << 0,
  GDSM_WANT_CURRENT = 1u << 1,
  GDSM_WANT_REPLICA = 1u << 2,
  GDSM_NO_ARENAS = 1u << 31, /* page-table-only context */
};
/* Per-kernel stages timed by gdsm_prof_* (HIP events on the context stream). */
enum gdsm_prof_stage {
  GDSM_PROF_DIFF = 0,   /* diff_single_kernel: the dominant kernel of the hot path */
  GDSM_PROF_APPLY,      /* apply_kernel */
  GDSM_PROF_TWIN,       /* twin_kernel */
  GDSM_PROF_COH_FOLD,   /* coh_fold_kernel: the coherence batch */
  GDSM_PROF_COH_REDUCE, /* the batch totals */
  GDSM_PROF_NW_FILL,    /* GPU diff(): DP fill */
  GDSM_PROF_NW_TRACE,   /* GPU diff(): traceback + alignment strings */
  GDSM_PROF_EXCHANGE,   /* gdsm_exchange: the transfer of the record streams (RCCL group) */
  GDSM_PROF_ROUTE,      /* gdsm_route_events / gdsm_coherence_notify: the transfers */
  GDSM_PROF_EXCHANGE_WAIT, /* gdsm_exchange: the transfer plus the wait for the peers' streams */
  GDSM_PROF_STAGES
};

typedef struct gdsm_ctx gdsm_ctx;

/* A diff stream (SPEC §3). All pointers are device pointers. */
typedef struct gdsm_runs {
  uint64_t n;        /* records in the stream (set by gdsm_diff) */
  uint64_t* rec_off; /* n + 1 */
  uint8_t* data;     /* cap bytes */
  uint64_t cap;      /* data capacity in bytes */
  uint64_t n_cap;    /* record capacity: rec_off holds n_cap + 1 entries */
  uint32_t owned;    /* 1 if allocated by gdsm_runs_alloc */
  uint32_t _pad;
} gdsm_runs;

/* ---- context ------------------------------------------------------------------------- */
int gdsm_device_count(int* count);
/* Allocates the arenas (n_pages × 4 KiB each) on `device` and one HIP stream. */
int gdsm_init(gdsm_ctx** out, int device, uint64_t n_pages, uint32_t flags);
int gdsm_fini(gdsm_ctx* ctx);
int gdsm_arena(gdsm_ctx* ctx, int which, void** dev_ptr);
uint64_t gdsm_n_pages(const gdsm_ctx* ctx);
/* The context's hipStream_t, as an opaque pointer. */
void* gdsm_stream(gdsm_ctx* ctx);
/* Waits for all enqueued work; reports a device-side failure recorded since the last sync. */
int gdsm_sync(gdsm_ctx* ctx);
/* Synchronous host <-> arena copies of pages [first, first+n). */
int gdsm_upload(gdsm_ctx* ctx, int which, uint64_t first, uint64_t n, const void* host);
int gdsm_download(gdsm_ctx* ctx, int which, uint64_t first, uint64_t n, void* host);
/* Pre-sizes the context's diff and coherence workspaces so later calls never reallocate (a
 * reallocation synchronises the device). */
int gdsm_reserve(gdsm_ctx* ctx, uint64_t diff_pages, uint64_t coh_events);
/* Device scratch owned by the context (freed by gdsm_fini). */
int gdsm_dev_alloc(gdsm_ctx* ctx, uint64_t bytes, void** dev_ptr);
int gdsm_dev_free(gdsm_ctx* ctx, void* dev_ptr);
int gdsm_memcpy_h2d(gdsm_ctx* ctx, void* dev, const void* host, uint64_t bytes);
int gdsm_memcpy_d2h(gdsm_ctx* ctx, void* host, const void* dev, uint64_t bytes);
/* Asynchronous device-to-device copy on the context stream. */
int gdsm_memcpy_d2d(gdsm_ctx* ctx, void* dst, const void* src, uint64_t bytes);
/* n device-to-device copies in one launch on the context stream: desc (device, 3n u64) holds
 * (dst, src, bytes) per copy; the copies must not overlap each other. E.g. the application
 * writes of one DSM round replayed at once (gallocy_amd/replay.py). */
int gdsm_memcpy_batch(gdsm_ctx* ctx, const uint64_t* desc, uint64_t n);

/* HIP graphs: record a launch-bound sequence once and replay it with one launch.
 * - Between gdsm_capture_begin(ctx) and gdsm_capture_end(ctx, &g), the asynchronous calls on ctx
 *   are recorded, not run: gdsm_twin, gdsm_diff, gdsm_apply, gdsm_memcpy_d2d / _batch,
 *   gdsm_coherence_batch_async and the generators.
 * - gdsm_capture_join(ctx, other) adds a second context on the same device. Its asynchronous
 *   calls are recorded into the same graph, ordered after what ctx had recorded when it joined.
 *   ctx's recording waits for them at gdsm_capture_end.
 * - Size the workspaces beforehand with gdsm_reserve: a call that would grow one fails with
 *   -EBUSY, and so does gdsm_sync on a recording context. Other calls that synchronise the host
 *   fail too.
 * - gdsm_graph_launch enqueues the whole graph on ctx's stream; gdsm_sync reports its
 *   device-side failures as usual. Every recorded pointer must stay valid while the graph
 *   lives.
 * - A caller may also capture gdsm_stream(ctx) itself (hipStreamBeginCapture): every call checks
 *   hipStreamIsCapturing and then records the forms that replay correctly (a zeroing launch
 *   before each short diff / small coherence batch instead of the one-launch chained forms,
 *   whose per-launch epoch a replay would repeat). The same sizing rule applies. */
typedef struct gdsm_graph gdsm_graph;
int gdsm_capture_begin(gdsm_ctx* ctx);
int gdsm_capture_join(gdsm_ctx* ctx, gdsm_ctx* other);
int gdsm_capture_end(gdsm_ctx* ctx, gdsm_graph** out);
int gdsm_graph_launch(gdsm_ctx* ctx, const gdsm_graph* g);
int gdsm_graph_destroy(gdsm_graph* g);

/* Per-kernel timing: when enabled, every kernel the context launches is bracketed by HIP events
 * on its stream; gdsm_prof_read synchronises and returns the summed milliseconds and launch
 * counts per stage (arrays of GDSM_PROF_STAGES), then clears them. */
int gdsm_prof_enable(gdsm_ctx* ctx, int on);
int gdsm_prof_read(gdsm_ctx* ctx, double* ms, uint64_t* launches);

/* Box ceilings (measurement support for bench.py, gdsm_probe.hip; no reference counterpart): how
 * fast this GPU streams given page arenas, `reps` launches timed by HIP events on ctx's stream
 * (best and median ms per launch). GDSM_PROBE_READ: arenas a and b (n_pages each) read once, the
 * diff's input pattern; GDSM_PROBE_COPY: dst := a over n_pages pages (dst is overwritten), the
 * fastest of three copy shapes (`reps` launches each). */
#define GDSM_PROBE_READ 0
#define GDSM_PROBE_COPY 1
int gdsm_probe_ceiling(gdsm_ctx* ctx, int kind, const void* a, const void* b, void* dst,
                       uint64_t n_pages, int reps, float* best_ms, float* median_ms);

/* ---- DSM rounds on the device ------------------------------------------------------------
 * n_rounds release rounds of one DSM run, each: a coherence batch of fault events on `pt`'s page
 * table (as gdsm_coherence_batch_async, totals row r = totals + 10 r), the application's writes
 * of the round on `data` (copy descriptors as gdsm_memcpy_batch) and the release of the pages
 * written (as gdsm_release with GDSM_RELEASE_RETWIN: diff of list entries ids, applied to
 * REPLICA at home, TWIN := CURRENT), round after round. Instead of three calls per round, ONE
 * persistent launch per context: the page-table rounds on pt's stream, the page-data rounds on
 * data's stream, a device-wide barrier between rounds where the launches had their boundaries.
 * Round r = events [ev_off[r], ev_off[r+1]), list entries [id_off[r], id_off[r+1]) of ids / home,
 * descriptors [desc_off[r], desc_off[r+1]) of desc (3 u64 each). The offset arrays are HOST
 * arrays of n_rounds + 1 entries from 0 (copied to the device by the call); events, totals, ids,
 * home, desc are device pointers. A round's writes are laid onto its released pages by the
 * release itself (no separate copy step), so they must be 8-B aligned (dst, src and bytes) and lie
 * inside the pages that round releases, each page listed once per round; otherwise gdsm_sync on
 * data reports -EINVAL. Limits: <= 2048 pages and <= 2^20 events per round, runs sized for the
 * largest round; data and pt distinct contexts of one device. runs ends holding the last round's
 * stream. Asynchronous on both streams; gdsm_sync on each reports failures (-ETIMEDOUT: a device
 * barrier gave up, never expected). Replaces gallocy_amd/native/replay.cpp's per-round
 * calls for config 5 (test/test_mmult.cpp:51-64's rounds). */
int gdsm_rounds(gdsm_ctx* data, gdsm_ctx* pt, uint32_t n_rounds, const uint64_t* events,
                const int64_t* ev_off, uint64_t* totals, const uint32_t* ids,
                const uint32_t* home, const int64_t* id_off, const uint64_t* desc,
                const int64_t* desc_off, gdsm_runs* runs);

/* ---- DSM rounds on the device ------------------------------------------------------------
 * n_rounds release rounds of one DSM run, each: a coherence batch of fault events on `pt`'s page
 * table (as gdsm_coherence_batch_async, totals row r = totals + 10 r), the application's writes
 * of the round on `data` (copy descriptors as gdsm_memcpy_batch) and the release of the pages
 * written (as gdsm_release with GDSM_RELEASE_RETWIN: diff of list entries ids, applied to
 * REPLICA at home, TWIN := CURRENT), round after round. Instead of three calls per round, ONE
 * persistent launch per context: the page-table rounds on pt's stream, the page-data rounds on
 * data's stream, a device-wide barrier between rounds where the launches had their boundaries.
 * Round r = events [ev_off[r], ev_off[r+1]), list entries [id_off[r], id_off[r+1]) of ids / home,
 * descriptors [desc_off[r], desc_off[r+1]) of desc (3 u64 each). The offset arrays are HOST
 * arrays of n_rounds + 1 entries from 0 (copied to the device by the call); events, totals, ids,
 * home, desc are device pointers. A round's writes are laid onto its released pages by the
 * release itself (no separate copy step), so they must be 8-B aligned (dst, src and bytes) and lie
 * inside the pages that round releases, each page listed once per round; otherwise gdsm_sync on
 * data reports -EINVAL. Limits: <= 2048 pages and <= 2^20 events per round, runs sized for the
 * largest round; data and pt distinct contexts of one device. runs ends holding the last round's
 * stream. Asynchronous on both streams; gdsm_sync on each reports failures (-ETIMEDOUT: a device
 * barrier gave up, never expected). Replaces gallocy_amd/native/replay.cpp's per-round
 * calls for config 5 (test/test_mmult.cpp:51-64's rounds). */
int gdsm_rounds(gdsm_ctx* data, gdsm_ctx* pt, uint32_t n_rounds, const uint64_t* events,
                const int64_t* ev_off, uint64_t* totals, const uint32_t* ids,
                const uint32_t* home, const int64_t* id_off, const uint64_t* desc,
                const int64_t* desc_off, gdsm_runs* runs);

/* ---- synthetic inputs (SPEC §6) ------------------------------------------------------- */
/* Fills the arenas named in `arenas` (bit 1<<GDSM_TWIN | 1<<GDSM_CURRENT | 1<<GDSM_REPLICA,
 * 0 = all) for every page; arena page i has global id first_global + i * stride (stride 0 = 1).
 * REPLICA gets the page's TWIN content. */
int gdsm_gen_pages(gdsm_ctx* ctx, uint32_t arenas, uint64_t first_global, uint64_t stride,
                   uint64_t seed, int mode, uint32_t ppm);
int gdsm_gen_pages_raw(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t n,
                       uint64_t first_global, uint64_t stride, uint64_t seed, int mode,
                       uint32_t ppm, void* stream);

/* ---- twin / diff / apply (SPEC §2-4) ------------------------------------------------- */
/* `ids` is a device array of n page ids, or NULL for the identity range [0, n). */
int gdsm_twin(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n);
/* Allocates a stream for n records with `cap` data bytes (cap 0: worst case n*10244). */
int gdsm_runs_alloc(gdsm_ctx* ctx, uint64_t n, uint64_t cap, gdsm_runs* out);
int gdsm_runs_free(gdsm_ctx* ctx, gdsm_runs* runs);
/* Diffs TWIN against CURRENT for the listed pages into `out` (n <= out->n_cap; out->n is set
 * to n). Asynchronous; use gdsm_runs_total to learn the size. */
int gdsm_diff(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out);
/* gdsm_diff, and the same runs applied to arena `target` (GDSM_REPLICA: a home copy on this
 * GPU, indexed by the same ids) by the same kernel: each dirty 16-B chunk's changed bytes, which
 * are exactly the bytes its runs cover (SPEC §4), are stored from the registers that found them,
 * so the stream is not read back. Equivalent to gdsm_diff + gdsm_apply(ctx, target, ids, out),
 * except that every page is applied even when the stream overflows out->cap (-ENOSPC from
 * gdsm_runs_total). Replaces the local-home half of gallocy's described release
 * (resources/NUTSHELL.md:59-69): the home applies what the writer diffed. */
int gdsm_diff_apply(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out, int target);
/* gdsm_diff_apply with the home copy indexed differently: list entry i (page ids[i] of TWIN and
 * CURRENT) is applied to page target_ids[i] of arena `target` (device, n entries; out-of-range
 * ids are reported by the next gdsm_sync and write nothing). For writers whose pages sit at other
 * indices than their home copies on the same GPU (e.g. several nodes' views of one zone, each
 * at its own offset, and one home copy of it). */
int gdsm_diff_apply_ids(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out,
                        int target, const uint32_t* target_ids);
/* A whole release of a writer's pages on this GPU: gdsm_diff of the listed pages into `out`;
 * with target >= 0 the runs are applied to arena `target` as gdsm_diff_apply_ids does
 * (target_ids NULL: the same page ids); with GDSM_RELEASE_RETWIN, TWIN := CURRENT afterwards for
 * every listed page whose record fit out->cap (a page whose record did not fit stays dirty, so
 * redoing the release with a larger stream ships it), i.e. the next interval's diff starts clean
 * without a gdsm_twin step. ids must be unique. A short release (<= 16 pages) is one kernel
 * launch, re-twin included. Replaces the twin taken at the next write fault
 * (resources/NUTSHELL.md:52-69: twin on the first write, diff at release). */
#define GDSM_RELEASE_RETWIN 1u
int gdsm_release(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out, int target,
                 const uint32_t* target_ids, uint32_t flags);
/* One diff launch for a release with several destinations: arena pages [bounds[d],
 * bounds[d+1]) are diffed into out[d] (G <= 8 streams, each with its own buffers; record i of
 * out[d] is page bounds[d] + i; out[d].n is set). Every stream is exactly what gdsm_diff of that
 * range would write, but the G ranges share one launch instead of G (gdsm_exchange's per-home
 * streams). */
int gdsm_diff_split(gdsm_ctx* ctx, const uint64_t* bounds, uint32_t G, gdsm_runs* out);
/* Synchronises, returns rec_off[n] in *total; -ENOSPC if it exceeded runs->cap. */
int gdsm_runs_total(gdsm_ctx* ctx, const gdsm_runs* runs, uint64_t* total);
/* Applies `in` to arena `target` (normally GDSM_REPLICA) for the listed pages (ids unique). */
int gdsm_apply(gdsm_ctx* ctx, int target, const uint32_t* ids, const gdsm_runs* in);
/* As gdsm_apply, on the context's second stream: it runs concurrently with the gdsm_diff calls
 * that follow (double-buffered releases: diff k+1 overlaps apply k). A later gdsm_diff into the
 * same `in` waits for this apply; every other call on the context is ordered after it.
 * Malformed records are reported by the next gdsm_sync. */
int gdsm_apply_async(gdsm_ctx* ctx, int target, const uint32_t* ids, const gdsm_runs* in);

/* ---- raw entry points (caller-owned device memory, e.g. tensors; stream = hipStream_t) ---- */
uint64_t gdsm_diff_workspace_bytes(uint64_t n);
int gdsm_diff_raw(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                  uint64_t* rec_off, uint8_t* data, uint64_t cap, void* workspace,
                  uint64_t workspace_bytes, void* stream);
int gdsm_diff_apply_raw(const uint8_t* twin, const uint8_t* cur, uint8_t* target,
                        const uint32_t* ids, uint64_t n, uint64_t* rec_off, uint8_t* data,
                        uint64_t cap, void* workspace, uint64_t workspace_bytes, void* stream);
/* err: caller-owned device word, OR-ed with 1 on a malformed record (NULL: not reported). */
int gdsm_apply_raw(uint8_t* target, const uint32_t* ids, uint64_t n, const uint64_t* rec_off,
                   const uint8_t* data, uint32_t* err, void* stream);
int gdsm_twin_raw(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                  void* stream);

/* ---- batched coherence (SPEC §5) ------------------------------------------------------- */
/* Allocates and initialises the page table (state + faults) for n_nodes <= 8; -EINVAL for a
 * context of more than GDSM_MAX_COH_PAGES pages. */
int gdsm_coh_init(gdsm_ctx* ctx, uint32_t n_nodes);
/* Applies one batch of page-sorted events (device array). Synchronises and writes
 * totals[10] = {invalidations, transfers, node_faults[8]}; -EINVAL if the batch is not sorted
 * by page or names a page/node out of range (the page table is then unspecified). */
int gdsm_coherence_batch(gdsm_ctx* ctx, const uint64_t* events, uint64_t n_events,
                         uint64_t* totals);
/* Asynchronous variant: totals stay on the device (10 x u64, written at the end). */
int gdsm_coherence_batch_async(gdsm_ctx* ctx, const uint64_t* events, uint64_t n_events,
                               uint64_t* totals_dev);
int gdsm_coh_download(gdsm_ctx* ctx, uint32_t* state, uint32_t* faults);
int gdsm_coh_upload(gdsm_ctx* ctx, const uint32_t* state, const uint32_t* faults);
/* Fills events from per-page counts: offsets is a device array of n+1 exclusive-scan offsets. */
int gdsm_gen_events(gdsm_ctx* ctx, uint64_t* events, const uint64_t* offsets, uint64_t first_page,
                    uint64_t n, uint64_t seed, uint32_t n_nodes, uint32_t write_pct);

/* ---- reference diff() (NW alignment), CPU ----------------------------------------------- */
/* out1/out2 are allocated with the installed allocator (default malloc); *len = alignment
 * length, which the legacy symbol cannot return. */
int gdsm_nw_diff(const char* mem1, size_t mem1_len, char** out1, const char* mem2,
                 size_t mem2_len, char** out2, size_t* len);
/* Installs the allocator used for diff()/gdsm_nw_diff outputs: gallocy passes
 * internal_malloc/internal_free so callers keep freeing with internal_free. */
int gdsm_set_allocator(void* (*alloc_fn)(size_t), void (*free_fn)(void*));

/* ---- reference diff() on the GPU: batched NW alignment --------------- */
/* Aligns n pairs (a_i, b_i) exactly like diff() / gdsm_nw_diff (same scores, tie-break and
 * traceback, gallocy/utils/diff.cpp:73-167), on the context's GPU. Device pointers: a and b hold
 * the concatenated inputs, a_off/b_off[n+1] their exclusive offsets; every |a_i|, |b_i| must be
 * <= max_len (-EINVAL otherwise). Pair i's alignment (L_i bytes + NUL) is written at
 * out1/out2 + a_off[i] + b_off[i] + i, so each output buffer needs a_off[n] + b_off[n] + n
 * bytes; out_len[i] = L_i. Synchronises (it checks the device error word). */
int gdsm_nw_diff_batch(gdsm_ctx* ctx, const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                       const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                       uint8_t* out2, uint64_t* out_len);
/* Routes the legacy diff() symbol (and gdsm_nw_diff) through gdsm_nw_diff_batch on ctx when
 * mem1_len * mem2_len >= min_cells; ctx == NULL restores the CPU path (the default). Outputs
 * still come from the installed allocator. The caller keeps ctx alive while it is installed and
 * does not use it for other work meanwhile: offloaded calls stage through its stream and buffers
 * (concurrent diff() calls are serialised on an internal lock; the CPU path stays reentrant). */
int gdsm_set_diff_device(gdsm_ctx* ctx, uint64_t min_cells);

/* ---- Host write-fault capture (the step before the diff). The reference
 * describes protecting shared pages and faulting on access (resources/NUTSHELL.md:52-69,
 * resources/IMPLEMENTATION.md:246-249) but never implements it; its only mprotect use is the
 * thread-stack guard (gallocy/threads.cpp:53-58). A tracker protects a page-aligned host region
 * read-only; the first write to a page in an interval is caught by a SIGSEGV handler, which
 * copies the page to the tracker's twin and makes it writable. CPU only (no GPU needed) except
 * gdsm_track_diff. Faults outside every tracked region go to the previously installed handler. */
typedef struct gdsm_tracker gdsm_tracker;
int gdsm_track_begin(gdsm_tracker** out, void* base, uint64_t n_pages);
/* Sorted ids of the pages written since begin / the last rearm; *n_out = their count. With
 * ids == NULL only the count is returned; -ENOSPC if cap < count. */
int gdsm_track_dirty(gdsm_tracker* t, uint32_t* ids, uint64_t cap, uint64_t* n_out);
/* The twin buffer (n_pages x 4 KiB; page p valid while p is dirty): p's contents before the
 * interval's first write to it. */
int gdsm_track_twin(gdsm_tracker* t, const void** twin);
/* Write faults taken so far (all intervals). */
int gdsm_track_faults(gdsm_tracker* t, uint64_t* faults);
/* Release point: re-protects the dirty pages and empties the dirty list. No thread may write
 * the region during the call. */
int gdsm_track_rearm(gdsm_tracker* t);
/* Unprotects the region and frees the tracker once no fault handler is still inside it. Only
 * write faults are claimed by a tracker; any other fault goes to the previous handler. */
int gdsm_track_end(gdsm_tracker* t);
/* Packs the dirty pages' twin and current contents, uploads them (synchronous w.r.t. the host
 * region: it may be written again once this returns) and diffs them on the GPU into `out`, one
 * record per dirty page in id order; ids_dev (>= count entries, device) receives the sorted ids,
 * so gdsm_apply(ctx, GDSM_REPLICA, ids_dev, out) applies the interval to a replica indexed by
 * page id. *n_out = count. */
int gdsm_track_diff(gdsm_ctx* ctx, gdsm_tracker* t, gdsm_runs* out, uint32_t* ids_dev,
                    uint64_t* n_out);

/* ---- diff wire format (docs/SPEC.md §7): a diff stream as a Raft log command text --------
 * The step after the diff: gallocy replicates Command{string}
 * (gallocy/include/gallocy/consensus/log.h:18-27) inside append-entries JSON
 * (consensus/client.cpp:133-142) and applies committed entries in try_apply
 * (consensus/state.cpp:308-316). The text is "GDSM1:" + base64(frame): printable, no NUL, no
 * JSON escapes. Framing, checksum and base64 run on the GPU. */
/* Length of the command text (without its NUL) for n records carrying data_bytes. */
uint64_t gdsm_wire_size(uint64_t n, uint64_t data_bytes);
/* Encodes the stream `runs` of pages ids[0..runs->n) (device; NULL = pages 0..n-1) into `out`
 * (host, cap bytes including the NUL); *len = text length. -ENOSPC (and *len = the length
 * needed) when cap is too small. Synchronises. */
int gdsm_wire_encode(gdsm_ctx* ctx, const uint32_t* ids, const gdsm_runs* runs, char* out,
                     uint64_t cap, uint64_t* len);
/* Decodes and verifies a command text (host, len bytes, no NUL needed) into device ids_out
 * (>= n entries) and `out` (n <= out->n_cap, data <= out->cap); *n_out = n. -EINVAL for any
 * malformed text (SPEC §7), -ENOSPC when out is too small. Synchronises. */
int gdsm_wire_decode(gdsm_ctx* ctx, const char* text, uint64_t len, uint32_t* ids_out,
                     gdsm_runs* out, uint64_t* n_out);
/* Follower side of try_apply: decodes, verifies (including page ids < the arena's pages) and
 * applies the command's records to arena `target`; nothing is applied when the text is rejected
 * (-EINVAL); a malformed record inside a well-formed frame fails during the apply (SPEC §7).
 * *n_out = records applied. Synchronises. */
int gdsm_wire_apply(gdsm_ctx* ctx, int target, const char* text, uint64_t len, uint64_t* n_out);

/* ---- multi-GPU diff propagation over RCCL / xGMI -------------------------------
 * One process and one context per GPU; pages are sharded by home rank. At a release, each rank
 * diffs the pages it wrote, grouped by home rank d, into one stream per destination (send[d]);
 * gdsm_exchange ships every stream to its home and applies what arrives to the home's arena.
 * This replaces the reference's page-update transport, an HTTP POST per peer fanned out with
 * std::async (gallocy/http/client.cpp:39-91, driven by gallocy/consensus/client.cpp:15-42).
 * RCCL is bound at run time (the librccl already loaded in the process, e.g. by torch, else
 * librccl.so.1); without it gdsm_comm_* return -ENOSYS. */
typedef struct gdsm_comm gdsm_comm;
#define GDSM_COMM_ID_BYTES 128
/* ncclGetUniqueId: call on ONE rank and hand the 128 bytes to every rank (Raft, HTTP, env). */
int gdsm_comm_unique_id(uint8_t* id);
/* Collective over the nranks processes (ncclCommInitRank on ctx's device). */
int gdsm_comm_init(gdsm_comm** out, gdsm_ctx* ctx, int nranks, int rank, const uint8_t* id);
int gdsm_comm_fini(gdsm_comm* comm);
int gdsm_comm_size(const gdsm_comm* comm, int* nranks, int* rank);
/* Test transport: nranks communicators over nranks contexts of ONE process (normally all on one
 * GPU), comms[r] bound to ctxs[r] and driven by its own host thread. Every collective below makes
 * the same calls at the same points as over RCCL; the moves become device-to-device copies on
 * the contexts' streams, ordered by HIP events (a receiver copies after the sender's stream
 * reached the send; the sender's stream continues after every receiver copied). It lets the
 * multi-rank code paths run on a one-GPU box. RCCL stays the transport of gdsm_comm_init. */
int gdsm_comm_init_loopback(gdsm_comm** comms, gdsm_ctx* const* ctxs, int nranks);
/* Collective, synchronous (after the work enqueued on ctx): *value becomes the maximum of every
 * rank's *value. The ranks' agreement on what to do next, e.g. whether to redo a release whose
 * fixed budget overflowed (-EOVERFLOW on some rank, below). */
int gdsm_comm_agree(gdsm_comm* comm, gdsm_ctx* ctx, uint64_t* value);

/* gdsm_exchange flags */
enum gdsm_exchange_flags {
  /* No host synchronisation: every record count and byte count is fixed by the caller.
   * send[d] ships exactly send[d].n records and send[d].cap data bytes (cap is the byte budget:
   * the stream's real size, rec_off[n], must not exceed it; the bytes past it are padding);
   * recv[s].n and recv[s].cap must equal what rank s ships here. A stream found larger than its
   * budget is not applied (its offsets are zeroed) and the next gdsm_sync of the home AND of the
   * sender reports -EOVERFLOW (when nothing else went wrong). Nothing of the release is lost
   * that the same release redone without the flag does not restore: gdsm_comm_agree on the
   * verdict, then re-diff and exchange with exact sizes (diff streams are idempotent). Without
   * the flag the library learns the sizes with one device all-to-all of (records, bytes) and
   * one host read, and agrees on capacity with every rank (all return -ENOSPC when any stream
   * is too small). */
  GDSM_XCHG_FIXED = 1u << 0,
  /* Measurement: before the transfer, a device-side barrier (a one-word all-to-all on the
   * exchange stream), so the transfer starts once every rank's streams are ready. With profiling
   * on, GDSM_PROF_EXCHANGE then times the RCCL group alone (the link) and
   * GDSM_PROF_EXCHANGE_WAIT the group plus the wait for the peers; without the flag both time the
   * group from when this rank's own streams are ready. */
  GDSM_XCHG_TIMED = 1u << 1,
};
/* Collective: every rank of `comm` calls it with arrays of nranks entries.
 *   send[d], send_ids[d]: this rank's stream for home rank d and, per record, the page's index
 *                         in rank d's arena `target` (device, send[d].n entries);
 *   recv[s], recv_ids[s]: where the stream from rank s lands (capacity recv[s].n_cap records,
 *                         recv[s].cap bytes; recv_ids[s] >= that many entries); recv[s].n is set.
 *                         recv[rank] / recv_ids[rank] are unused: the own stream is applied in
 *                         place from send[rank].
 * Runs on the context's second stream after everything enqueued on the main stream (the diffs
 * that produced send[]); it overlaps the gdsm_diff calls that follow, and a later gdsm_diff into
 * one of the send streams waits for it (as gdsm_apply_async). Every stream (the own one too) is
 * checked whole before it is applied: offsets from 0, non-decreasing, 4-aligned, within the
 * budget, every page index < the arena's pages; a stream failing any check is not applied at
 * all and the next gdsm_sync reports -EINVAL (-EOVERFLOW when the budget was the only fault);
 * a malformed record inside a well-formed stream is caught by the apply (SPEC §4). */
int gdsm_exchange(gdsm_ctx* ctx, gdsm_comm* comm, const gdsm_runs* send,
                  const uint32_t* const* send_ids, gdsm_runs* recv, uint32_t* const* recv_ids,
                  int target, uint32_t flags);

/* ---- coherence across GPUs (docs/SPEC.md §5b) ----------------------------------
 * Rank r of the communicator is DSM node r and the home of the page block
 * [r * per, (r+1) * per), per = ceil(total_pages / nranks) (SPEC §5's initial home); its page-table
 * context holds that block (local page = global page - base). A batch of faults is handled in two
 * collective, host-synchronising steps (every rank calls both, in this order, with its own data):
 *   1. gdsm_route_events: each node's fault events go to their pages' homes, where the sources'
 *      lists are merged into one page-sorted batch;
 *   2. gdsm_coherence_notify: each home folds its batch into its page-table shard (SPEC §5) and
 *      sends every node whose access to a page changed a notice, the "negotiate access / copy over
 *      the latest contents / update protections" step of resources/NUTSHELL.md:61-69 that the
 *      reference only describes (its transport would be gallocy/http/client.cpp:39-91).
 * The shards then equal the sequential fold of all nodes' events in (page, seq) order. */
#define GDSM_STAMP_PAGE_SHIFT 36
/* A node's fault event, stamped: (page << 36) | (seq << 4) | (node << 1) | rw, page < 2^28 the
 * GLOBAL page, seq < 2^32 the event's position in the batch's global order (a logical clock; unique
 * per page), node = the calling rank. A node's list is sorted ascending (by page, then seq). */
/* Routes this node's n stamped events (device) to the homes; on return *n_batch events of this
 * rank's home block, from every node, merged by (page, seq) and packed as SPEC §5 events with the
 * LOCAL page, are being written to `batch` (device, cap entries) on ctx's stream. All ranks return
 * -EINVAL if any node's list is unsorted or names a page >= total_pages or a node >= nranks, and
 * -ENOSPC if any home's cap is too small; nothing moves then. A rank whose own step fails after
 * the arguments were accepted (a workspace it cannot allocate, a launch error) returns that error
 * and every other rank -ECANCELED, together; nothing moves either. */
int gdsm_route_events(gdsm_ctx* ctx, gdsm_comm* comm, const uint64_t* events, uint64_t n,
                      uint64_t total_pages, uint64_t* batch, uint64_t cap, uint64_t* n_batch);
/* Home side: folds `batch` (n events, local pages, e.g. from gdsm_route_events) into ctx's page
 * table (gdsm_coh_init'd, pages [base, base + n_pages)) with its totals into totals_dev (10 x u64,
 * as gdsm_coherence_batch_async), then sends each node its notices. On return *n_notices notices
 * for THIS rank as a node, from every home, sorted by page, are being written to `notices`
 * (device, cap entries) on ctx's stream. A notice (u64) for page p and node d:
 *   bits 0-31 global page | 32-33 d's access before the batch | 34-35 d's access after |
 *   40-47 owner before | 48-55 owner after
 * with access 0 none, 1 read (d in the copyset), 2 write (EXCLUSIVE and d the owner); d gets one
 * iff its access changed or it is the old or the new owner of a page whose owner changed, so a
 * node never gets more notices than there are distinct pages in all homes' batches: every rank
 * returns -ENOSPC, before any page table changes, when some node's cap is below that count. All
 * ranks return -EINVAL if any home's batch was rejected by the fold (that page table is then
 * unspecified, as after a rejected gdsm_coherence_batch). A rank whose own step fails (a workspace
 * it cannot allocate, a launch error) returns that error and every other rank -ECANCELED,
 * together: before the fold (every workspace is sized then) no page table changes; a launch
 * failure of the fold itself leaves the page tables unspecified, as above. Only this fold's
 * rejection counts: an error bit an earlier unsynchronised batch left is kept for gdsm_sync. */
int gdsm_coherence_notify(gdsm_ctx* ctx, gdsm_comm* comm, const uint64_t* batch, uint64_t n,
                          uint64_t base, uint64_t* totals_dev, uint64_t* notices, uint64_t cap,
                          uint64_t* n_notices);

const char* gdsm_version(void);
/* Process-wide kernel-variant knobs for measurement (every value produces the same results):
 * "diff_variant" 0..8 (diff geometry), "apply_variant" 0..7, "diff_solo_max" 0..16 and
 * "diff_chain" 0..4 (short lists: one-workgroup / chained forms), "coh_variant" 0..2,
 * "coh_chain" 0|1 (small coherence batches without the zeroing launch), "coh_span" 1|2|4 (their
 * span, in 64-event chunks). Returns 0, or -EINVAL
 * for an unknown key or value. */
int gdsm_tune(const char* key, int64_t value);
/* Test hook: the nth next growth of one of ctx's internal workspaces fails with -ENOMEM (0 = off).
 * Used to show that a collective call refuses on every rank together when one rank fails. */
int gdsm_debug_fail_alloc(gdsm_ctx* ctx, int nth);

#ifdef __cplusplus
}  /* extern "C" */

/* Legacy drop-in, C++ linkage, mangled _Z4diffPKcmRPcS0_mS2_ exactly like
 * gallocy/include/gallocy/utils/diff.h:9-11. Bit-exact with the reference for
 * mem1_len, mem2_len <= 1180 (the reference crashes beyond). Always returns 0. */
int diff(const char* mem1, size_t mem1_len, char*& mem1_alignment, const char* mem2,
         size_t mem2_len, char*& mem2_alignment);
#endif

#endif /* GDSM_H_ */
