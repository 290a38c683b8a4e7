// Host-side launchers for the gdsm kernels (internal; the public ABI is include/gdsm.h).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "gdsm_prof.h"

namespace gdsm {

// Workspace of one diff of n list entries (ticket counter + one look-back granule per unit).
uint64_t diff_workspace_bytes(uint64_t n);
// Kernel variant knobs (see gdsm_tune); returns -1 for an unknown key.
int tune(const char* key, int64_t value);
int coh_tune(const char* key, int64_t value);

hipError_t launch_gen_pages(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t n,
                            uint64_t first_global, uint64_t stride, uint64_t seed, int mode,
                            uint32_t ppm, hipStream_t s);
// With a caller list, n_pages / err guard it in the kernel (ids >= n_pages -> the guard page
// n_pages, err |= 8); the defaults leave the list unchecked (raw entry points).
hipError_t launch_twin(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       hipStream_t s, Prof* prof = nullptr, uint64_t n_pages = ~0ull,
                       uint32_t* err = nullptr);
// Full diff of n pages in one pass: rec_off[n+1], data[cap]. With `target`, the runs are also
// applied to target by the same kernel, page tids[i] for list entry i (tids NULL: the same page
// ids). bpp_hint: stream bytes per page the caller saw last time (0 = unknown); it only picks
// the geometry.
// Caller page-id lists checked by the diff launch itself (in the launch that zeroes its
// workspace): safe_ids[i] = ids[i] if < n_pages, else n_pages (the guard page), the same for
// tids, err |= 8 when any id was out of range. A null list is not checked.
// Device error bit of a persistent grid's barrier that never completed (gdsm_rounds).
constexpr uint32_t kErrRoundsBarrier = 64;
// ... and of a round's writes that were not 8-B aligned or fell outside its released pages.
constexpr uint32_t kErrRoundsWrites = 128;
struct IdGuard {
  const uint32_t* ids;
  const uint32_t* tids;
  uint32_t* safe_ids;
  uint32_t* safe_tids;
  uint64_t n_pages;
  uint32_t* err;
};
// A context's chain of zero-free diff launches: lists of at most kDiffChainUnits pages (one-page
// units) take one launch, no workspace-zeroing launch before it. ws (diff_chain_bytes(), device)
// holds two ticket counters and one epoch-tagged look-back granule per unit; it is zeroed once
// (epoch 0: by the next launch, then epoch 1). Launch E draws its tickets from counter E & 1 and
// zeroes counter (E + 1) & 1 for launch E + 1; a granule counts only when it carries E. Not for
// graph capture (a replayed launch would repeat its epoch).
constexpr uint64_t kDiffChainUnits = 2048;
struct DiffChain {
  uint64_t* ws = nullptr;
  uint32_t epoch = 0;  // the next launch's epoch, 1 .. 2^30 - 1; 0 = zero ws first
};
uint64_t diff_chain_bytes();
// With `guard`, the kernel reads guard->safe_ids / safe_tids in place of ids / tids.
hipError_t launch_diff(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                       uint64_t* rec_off, uint8_t* data, uint64_t cap, uint8_t* ws,
                       uint64_t ws_bytes, hipStream_t s, Prof* prof = nullptr,
                       uint8_t* target = nullptr, uint32_t bpp_hint = 0,
                       const uint32_t* tids = nullptr, const IdGuard* guard = nullptr,
                       uint8_t* retwin = nullptr, DiffChain* chain = nullptr);
// retwin (gdsm_release's GDSM_RELEASE_RETWIN; must be the `twin` arena): after the diff, TWIN :=
// CURRENT for every listed page whose record fits the capacity (inside the one-workgroup kernel
// of a short release, by a second launch otherwise).
// The diff kernel's output streams: list entries [first[d], first[d+1]) go to stream d (record
// i of stream d = entry first[d] + i); ustart: the first work unit of each stream (set by the
// launcher). One launch serves them all, each stream with its own look-back chain.
constexpr uint32_t kMaxSplit = 8;
struct DiffSplit {
  uint64_t* rec_off[kMaxSplit];
  uint8_t* data[kMaxSplit];
  uint64_t cap[kMaxSplit];
  uint64_t first[kMaxSplit + 1];
  uint64_t ustart[kMaxSplit + 1];
  uint32_t G;
  uint32_t epoch;  // a DiffChain launch's epoch (set by the launcher)
};
// One diff launch over arena pages [first[0], first[G]) (ids = identity) into sp's G streams.
hipError_t launch_copy_batch(const uint64_t* desc, uint64_t n, hipStream_t s);
// DSM rounds on the device (gdsm_rounds): the page-data side, one persistent launch of `grid`
// workgroups: per round the release of list entries [off[r], off[r+1]) of ids (home indices tids
// into target, re-twin) with its copy descriptors [doff[r], doff[r+1]) of desc laid onto the
// pages, then a grid barrier. off / doff on the device; look-back granules in chain_ws
// (DiffChain layout) with epochs epoch0 + r; bar: kRoundsBarBytes zeroed by the launcher.
// xcd: the rounds run on a one-XCD team of the grid (xcd_team: about grid / 8 members).
hipError_t launch_rounds_data(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids,
                              const uint32_t* tids, const int64_t* off, const uint64_t* desc,
                              const int64_t* doff, uint32_t n_rounds, uint32_t grid,
                              uint64_t* rec_off, uint8_t* data, uint64_t cap, uint64_t* chain_ws,
                              uint8_t* target, uint64_t n_pages, uint32_t* err, uint32_t epoch0,
                              uint32_t* bar, bool xcd, hipStream_t s, Prof* prof = nullptr);
const void* rounds_data_kernel_ptr(bool xcd);  // (for the occupancy query)
constexpr uint64_t kRoundsBarBytes = 256;      // a rounds grid's barrier and team words
hipError_t launch_diff_split(const uint8_t* twin, const uint8_t* cur, DiffSplit sp, uint8_t* ws,
                             uint64_t ws_bytes, hipStream_t s, Prof* prof, uint32_t bpp_hint);
hipError_t launch_apply(uint8_t* target, const uint32_t* ids, uint64_t n,
                        const uint64_t* rec_off, const uint8_t* data, uint32_t* err,
                        hipStream_t s, Prof* prof = nullptr);
// A stream about to be applied by gdsm_exchange: checked whole (offsets from 0, non-decreasing,
// 4-aligned, rec_off[n] <= budget; page indices < n_pages, copied to safe[n]). A rejected stream
// has every offset zeroed (nothing applied); err |= 16 (malformed offsets), 32 (over budget),
// 8 (bad page index). `verdict` is one device word of scratch.
hipError_t launch_xchg_guard(uint64_t* rec_off, const uint32_t* ids, uint64_t n, uint64_t budget,
                             uint64_t n_pages, uint32_t* safe, uint32_t* verdict, uint32_t* err,
                             hipStream_t s);
// err |= 32 when rec_off[n] > budget (a fixed-budget stream its sender shipped over budget).
hipError_t launch_budget_check(const uint64_t* rec_off, uint64_t n, uint64_t budget,
                               uint32_t* err, hipStream_t s);
// Caller page-id lists at the context level: safe[i] = ids[i] if < n_pages, else n_pages (the
// arenas' guard page), and err |= 8 when any id was out of range.
hipError_t launch_check_ids(const uint32_t* ids, uint64_t n, uint64_t n_pages, uint32_t* safe,
                            uint32_t* err, hipStream_t s);

// Coherence (SPEC §5).
uint64_t coh_workspace_bytes(uint64_t n_events);
// Page table: one u64 per page, state | faults << 32.
hipError_t launch_coh_init(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes, hipStream_t s);
// A context's chain of zero-free small coherence batches (as DiffChain): ws (coh_chain_bytes(),
// device) holds two sets of ticket counters, totals rows and completion counters, then
// epoch-tagged status granules; zeroed once (epoch 0: by the next launch). Not for graph capture.
struct CohChainState {
  uint64_t* ws = nullptr;
  uint32_t epoch = 0;
};
uint64_t coh_chain_bytes();
// Events naming a page >= n_pages or a node >= n_nodes reject the batch (err |= 2).
hipError_t launch_coherence(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                            const uint64_t* events, uint64_t n_events, uint64_t* totals,
                            uint8_t* ws, uint64_t ws_bytes, uint32_t* err, hipStream_t s,
                            Prof* prof = nullptr, CohChainState* chain = nullptr);
// DSM rounds on the device (gdsm_rounds): the page-table side, one persistent launch of `grid`
// workgroups over n_rounds rounds (eoff: device, n_rounds + 1 event offsets; totals: 10 u64 per
// round). Uses the chain's ws with epochs of its own; the chain restarts (zeroed) afterwards.
// bar: kRoundsBarBytes zeroed by the launcher; xcd: a one-XCD team (as launch_rounds_data).
// lds: instead `grid` workgroups (<= kRoundsLdsMaxWGs) with the page table in LDS slices of
// ceil(n_pages / grid) <= kRoundsLdsPages pages (every round <= kRoundsLdsEvents events, n_rounds
// <= kRoundsLdsRounds; chain and bar unused).
constexpr uint64_t kRoundsLdsPages = 8192;    // 64 KiB of page-table words per workgroup
constexpr uint32_t kRoundsLdsMaxWGs = 16;     // workgroups (page-table slices) of the LDS form
constexpr uint64_t kRoundsLdsWGEvents = 4096; // a round's events per workgroup the host aims at
constexpr uint64_t kRoundsLdsEvents = 16384;  // 64 KiB of a round's staged events
constexpr uint32_t kRoundsLdsRounds = 2048;   // 16 KiB of event offsets
// (gdsm_rounds takes the LDS form whenever it fits: config 5, same box, against the grid fold,
// 1 / 2 / 4 / 8 nodes on 1 / 1 / 2 / 4 workgroups: +12 % / tied / +12 % / +5 %; one workgroup
// alone at 4 and 8 nodes was the slower form, -10 % / -25 %, profiles/r06_rounds_lds_ab.txt)
hipError_t launch_rounds_fold(uint64_t* pt, uint64_t n_pages, uint32_t n_nodes,
                              const uint64_t* events, const int64_t* eoff, uint32_t n_rounds,
                              uint32_t grid, uint64_t* totals, uint32_t* err, CohChainState* chain,
                              uint32_t* bar, bool xcd, bool lds, hipStream_t s,
                              Prof* prof = nullptr);
const void* rounds_fold_kernel_ptr(bool xcd);  // (for the occupancy query)
hipError_t launch_gen_events(uint64_t* events, const uint64_t* offsets, uint64_t first_page,
                             uint64_t n, uint64_t seed, uint32_t n_nodes, uint32_t write_pct,
                             hipStream_t s);

// Coherence across GPUs (SPEC §5b; gdsm_route.hip).
// A node's stamped events: validation (bad |= 1), per-home bounds[G+1] and counts[G] (u64).
hipError_t launch_route_split(const uint64_t* ev, uint64_t n, uint64_t total_pages, uint64_t per,
                              uint32_t G, uint64_t* counts, uint64_t* bounds, uint32_t* bad,
                              hipStream_t s);
// G sorted runs (host offsets off[G+1] into `runs`) merged into one page-sorted local batch.
hipError_t launch_route_merge(const uint64_t* runs, const uint64_t* off, uint32_t G, uint64_t base,
                              uint64_t* out, hipStream_t s);
uint64_t notice_blocks(uint64_t n);
// pre[i] = the page-table word at each page's first event; *heads = the batch's distinct pages.
hipError_t launch_notice_pre(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                             uint64_t n, uint32_t* pre, uint64_t* heads, hipStream_t s);
// blk: notice_blocks(n) x 8 u32; blk_off the same in u64; dest_total / dest_base: G u64 each.
hipError_t launch_notice_count(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                               uint64_t n, const uint32_t* pre, uint32_t G, uint32_t* blk,
                               uint64_t* blk_off, uint64_t* dest_total, uint64_t* dest_base,
                               hipStream_t s);
hipError_t launch_notice_emit(const uint64_t* pt, uint64_t n_pages, const uint64_t* batch,
                              uint64_t n, const uint32_t* pre, uint32_t G, uint64_t base,
                              const uint64_t* blk_off, const uint64_t* dest_base, uint64_t* out,
                              hipStream_t s);

// GPU NW alignment (legacy diff()): workspace per pair and the fill + trace launches.
uint64_t nw_pair_ws_bytes(uint32_t max_len);
hipError_t launch_nw(const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                     const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                     uint8_t* out2, uint64_t* out_len, uint8_t* ws, uint64_t ws_bytes,
                     uint32_t* err, hipStream_t s, Prof* prof = nullptr);

// Diff wire format (SPEC §7).
uint64_t wire_frame_bytes(uint64_t n, uint64_t data_bytes);
hipError_t launch_wire_sum(const uint8_t* frame, uint64_t F, uint64_t* sum, hipStream_t s);
// dst[i] = i for i < n (identity page-id lists on the device).
hipError_t launch_iota(uint32_t* dst, uint64_t n, hipStream_t s);
hipError_t launch_b64_encode(const uint8_t* frame, uint64_t F, uint8_t* text, hipStream_t s);
hipError_t launch_b64_decode(const uint8_t* text, uint64_t T, uint32_t pad, uint8_t* frame,
                             uint64_t F, uint32_t* err, hipStream_t s);
hipError_t launch_wire_check(const uint32_t* ids, const uint64_t* rec_off, uint64_t n,
                             uint64_t D, uint64_t n_pages, uint32_t* err, hipStream_t s);

}  // namespace gdsm
