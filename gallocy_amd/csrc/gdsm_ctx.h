// The context object behind the C ABI and the host helpers shared by the .cpp files that
// implement include/gdsm.h (internal header).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <map>
#include <set>
#include <vector>

#include "gdsm.h"
#include "gdsm_launch.h"
#include "gdsm_prof.h"

struct gdsm_ctx {
  int device = 0;
  uint64_t n_pages = 0;
  hipStream_t stream = nullptr;
  uint8_t* arena[3] = {nullptr, nullptr, nullptr};
  uint32_t* err = nullptr;       // device error word (bit 0: malformed record, bit 1: bad events)
  // error bits taken off the device word by a call that must not see them (gdsm_coherence_notify
  // and an earlier batch's rejection); gdsm_sync reports them with the device word's
  uint32_t err_held = 0;
  uint8_t* diff_ws = nullptr;    // diff workspace
  uint64_t diff_ws_bytes = 0;
  gdsm::DiffChain chain;         // short releases without a zeroing launch (allocated by gdsm_init)
  uint8_t* coh_ws = nullptr;
  uint64_t coh_ws_bytes = 0;
  uint64_t* coh_pt = nullptr;      // page table: state | faults << 32 per page
  uint64_t* coh_totals = nullptr;  // device 10 x u64
  gdsm::CohChainState coh_chain;   // small batches without a zeroing launch (allocated by gdsm_init)
  uint32_t n_nodes = 0;
  // gdsm_rounds: the rounds' offset arrays on the device and the grid-barrier word
  uint8_t* rounds_ws = nullptr;
  uint64_t rounds_ws_bytes = 0;
  uint32_t diff_bpp = 0;         // stream bytes per page the host last learned (diff geometry)
  std::set<void*> allocs;        // gdsm_dev_alloc / gdsm_runs_alloc blocks
  // gdsm_apply_async: applies run on `aux`, ordered after everything enqueued on `stream` before
  // them; every other operation joins `aux` first, except gdsm_diff, which only waits for the
  // apply still reading its output stream (runs_busy) or writing an arena it reads.
  hipStream_t aux = nullptr;
  hipEvent_t ev_main = nullptr, ev_aux = nullptr;
  bool aux_pending = false;
  uint32_t aux_targets = 0;                      // arenas written by pending async applies
  std::map<const void*, hipEvent_t> runs_busy;   // rec_off -> last async apply reading it
  gdsm::Prof prof;
  gdsm::Prof* P() { return prof.on ? &prof : nullptr; }
  // gdsm_track_diff staging: pinned host and device, 2 x n x 4 KiB pages + n ids
  uint8_t* track_host = nullptr;
  uint64_t track_host_bytes = 0;
  uint8_t* track_dev = nullptr;
  uint64_t track_dev_bytes = 0;
  // gdsm_nw_diff_batch: traceback workspace; host-offloaded diff() staging (device)
  uint8_t* nw_ws = nullptr;
  uint64_t nw_ws_bytes = 0;
  uint8_t* nw_stage = nullptr;
  uint64_t nw_stage_bytes = 0;
  // gdsm_wire_*: text + frame + checksum word
  uint8_t* wire_ws = nullptr;
  uint64_t wire_ws_bytes = 0;
  uint64_t wire_hdr[4] = {};  // host staging of the frame header
  // checked copies of caller page-id lists (launch_check_ids): one per stream, so an async
  // apply's list is never overwritten by a call on the main stream
  // [2]: the target-page list of gdsm_diff_apply_ids (main stream, beside [0])
  uint32_t* ids_safe[3] = {nullptr, nullptr, nullptr};
  uint64_t ids_safe_bytes[3] = {0, 0, 0};
  // graph capture (gdsm_capture_*): open on this context's stream (or joined into another's)
  bool capturing = false;
  bool capture_origin = false;  // this context began the capture (only it may end it)
  std::vector<gdsm_ctx*> capture_joined;
  std::vector<hipEvent_t> capture_events;
  // gdsm_debug_fail_alloc: the fail_alloc-th next workspace growth fails with -ENOMEM (tests of
  // the collective refusals); 0 = off
  mutable int fail_alloc = 0;
};

namespace gdsm {
namespace detail {

// Bits of the device error word (gdsm_ctx::err).
constexpr uint32_t kErrRecord = 1;       // malformed record (apply)
constexpr uint32_t kErrEvents = 2;       // coherence batch not sorted / out of range
constexpr uint32_t kErrNw = 4;           // GPU NW input out of range
constexpr uint32_t kErrIds = 8;          // page id / index out of range
constexpr uint32_t kErrStream = 16;      // exchanged stream with malformed offsets
constexpr uint32_t kErrOverBudget = 32;  // fixed-budget exchanged stream over its budget
static_assert(gdsm::kErrRoundsBarrier == 64, "gdsm_rounds: a barrier that never completed");

int map_err(hipError_t e);
// ctx->stream is being recorded into a graph (gdsm_capture_* or a caller's own capture of it).
bool recording(const gdsm_ctx* ctx);
// hipMalloc-backed buffer that only grows (contents are not kept); -EBUSY while ctx (the owner of
// the buffer, or NULL) is recording a graph.
int ensure(const gdsm_ctx* ctx, uint8_t** buf, uint64_t* have, uint64_t need);
// Makes ctx->stream wait for every pending operation on ctx->aux.
int join_aux(gdsm_ctx* ctx);
// Creates ctx->aux and its events on first use.
int ensure_aux(gdsm_ctx* ctx);
// A caller's device id list checked against the arenas into buffer `which` (0 and 2 on the main
// stream, 1 on aux).
int safe_ids(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, int which, const uint32_t** out);
// Only the buffer `which` for n checked ids (for a launch that checks the list itself).
int safe_buf(gdsm_ctx* ctx, uint64_t n, int which, uint32_t** out);
int check_and_clear_err(gdsm_ctx* ctx);
// Records the stream density (bytes / pages) the host learned, for the diff's geometry choice
// (stored + 1, so 0 stays "unknown"). Lists of at most kDiffShortList pages take the short-list
// geometry anyway and do not count.
constexpr uint64_t kDiffShortList = 32768;
void note_density(gdsm_ctx* ctx, uint64_t bytes, uint64_t pages);

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Device guard for an operation on the context's stream: ordered after pending async work.
struct CtxGuard : DeviceGuard {
  int rc;
  explicit CtxGuard(gdsm_ctx* c) : DeviceGuard(c->device), rc(join_aux(c)) {}
};

}  // namespace detail
}  // namespace gdsm

#define GDSM_TRY(expr)                                              \
  do {                                                              \
    hipError_t e_ = (expr);                                         \
    if (e_ != hipSuccess) return ::gdsm::detail::map_err(e_);       \
  } while (0)
