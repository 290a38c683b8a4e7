// C-ABI of libgdsm.so (include/gdsm.h): context, arenas, streams, error mapping.
// Host C++ only; kernels are launched through gdsm_launch.h.
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <vector>

#include "gdsm.h"
#include "gdsm_ctx.h"
#include "gdsm_launch.h"
#include "gdsm_track.h"

namespace gdsm {
namespace detail {

int map_err(hipError_t e) {
  switch (e) {
    case hipSuccess: return 0;
    case hipErrorOutOfMemory: return -ENOMEM;
    case hipErrorInvalidValue: return -EINVAL;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice: return -ENODEV;
    default: return -EIO;
  }
}

// Makes `stream` wait for every pending operation on the aux stream (async applies, exchanges).
int join_aux(gdsm_ctx* ctx) {
  if (!ctx->aux_pending) return 0;
  GDSM_TRY(hipEventRecord(ctx->ev_aux, ctx->aux));
  GDSM_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_aux, 0));
  ctx->aux_pending = false;
  ctx->aux_targets = 0;
  return 0;
}

int ensure_aux(gdsm_ctx* ctx) {
  if (ctx->aux) return 0;
  GDSM_TRY(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
  GDSM_TRY(hipEventCreateWithFlags(&ctx->ev_main, hipEventDisableTiming));
  GDSM_TRY(hipEventCreateWithFlags(&ctx->ev_aux, hipEventDisableTiming));
  return 0;
}

// The context's stream is being recorded into a graph: by gdsm_capture_begin / _join, or by a
// caller that captures gdsm_stream() itself (hipStreamBeginCapture). A recorded launch replays
// with the arguments it was recorded with, so the chained forms (one epoch per launch, DiffChain /
// CohChainState) are not used then: the zeroing forms replay correctly.
bool recording(const gdsm_ctx* ctx) {
  if (ctx->capturing) return true;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(ctx->stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone;
}

// A context whose calls are being recorded (gdsm_capture_begin / _join) may not move its
// workspaces, since the recorded kernels keep their addresses; other contexts are unaffected.
int ensure(const gdsm_ctx* ctx, uint8_t** buf, uint64_t* have, uint64_t need) {
  if (*have >= need) return 0;
  if (ctx && recording(ctx)) return -EBUSY;  // size workspaces with gdsm_reserve before capturing
  if (ctx && ctx->fail_alloc > 0 && --ctx->fail_alloc == 0) return -ENOMEM;  // test hook
  // kernels queued on the context's streams (main or aux, e.g. an exchange's applies reading the
  // checked id lists) may still use the old buffer: drain them before it goes (stated here rather
  // than left to hipFree's own synchronisation)
  if (*buf && ctx) {
    if (ctx->stream) GDSM_TRY(hipStreamSynchronize(ctx->stream));
    if (ctx->aux) GDSM_TRY(hipStreamSynchronize(ctx->aux));
  }
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  GDSM_TRY(hipMalloc(reinterpret_cast<void**>(buf), need));
  *have = need;
  return 0;
}

// The buffer `which` of checked ids, grown to n.
int safe_buf(gdsm_ctx* ctx, uint64_t n, int which, uint32_t** out) {
  uint8_t* buf = reinterpret_cast<uint8_t*>(ctx->ids_safe[which]);
  int rc = ensure(ctx, &buf, &ctx->ids_safe_bytes[which], 4 * n);
  ctx->ids_safe[which] = reinterpret_cast<uint32_t*>(buf);
  *out = ctx->ids_safe[which];
  return rc;
}

// A caller's device id list, checked against the arenas on stream `which` (0 main, 1 aux):
// returns the list the kernels may use (out-of-range ids -> the guard page n_pages).
int safe_ids(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, int which, const uint32_t** out) {
  *out = ids;
  if (!ids || n == 0) return 0;
  uint32_t* buf = nullptr;
  int rc = safe_buf(ctx, n, which, &buf);
  if (rc) return rc;
  GDSM_TRY(gdsm::launch_check_ids(ids, n, ctx->n_pages, buf, ctx->err,
                                  which == 1 ? ctx->aux : ctx->stream));
  *out = buf;
  return 0;
}

void note_density(gdsm_ctx* ctx, uint64_t bytes, uint64_t pages) {
  if (pages) ctx->diff_bpp = (uint32_t)(bytes / pages > 0xFFFFFFFEull ? 0xFFFFFFFEull : bytes / pages) + 1;
}

int check_and_clear_err(gdsm_ctx* ctx) {
  uint32_t h = 0;
  GDSM_TRY(hipMemcpyAsync(&h, ctx->err, 4, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipMemsetAsync(ctx->err, 0, 4, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  h |= ctx->err_held;
  ctx->err_held = 0;
  if (h && getenv("GDSM_DEBUG_ERR")) fprintf(stderr, "gdsm err word 0x%x\n", h);
  // a fixed-budget exchange stream over its budget, and nothing else: the release can be redone
  // with exact sizes (gdsm.h GDSM_XCHG_FIXED)
  if (h == kErrOverBudget) return -EOVERFLOW;
  if (h & gdsm::kErrRoundsBarrier) return -ETIMEDOUT;  // gdsm_rounds: a grid barrier gave up
  return h ? -EINVAL : 0;
}

}  // namespace detail
}  // namespace gdsm

using namespace gdsm::detail;

extern "C" {

int gdsm_track_diff(gdsm_ctx* ctx, gdsm_tracker* t, gdsm_runs* out, uint32_t* ids_dev,
                    uint64_t* n_out) {
  if (!ctx || !t || !out || !out->rec_off || !n_out) return -EINVAL;
  uint64_t n = 0;
  int rc = gdsm_track_dirty(t, nullptr, 0, &n);
  if (rc) return rc;
  if (n && !ids_dev) return -EINVAL;
  if (out->n_cap ? n > out->n_cap : (out->owned && n > out->n)) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  const uint64_t bytes = n * 2 * GDSM_PAGE_SZ + n * sizeof(uint32_t);
  if (bytes > ctx->track_host_bytes) {
    if (ctx->track_host) (void)hipHostFree(ctx->track_host);
    ctx->track_host = nullptr;
    ctx->track_host_bytes = 0;
    GDSM_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->track_host), bytes));
    ctx->track_host_bytes = bytes;
  }
  rc = ensure(ctx, &ctx->track_dev, &ctx->track_dev_bytes, bytes ? bytes : 1);
  if (rc) return rc;
  uint8_t* h_twin = ctx->track_host;
  uint8_t* h_cur = h_twin + n * GDSM_PAGE_SZ;
  uint32_t* h_ids = reinterpret_cast<uint32_t*>(h_cur + n * GDSM_PAGE_SZ);
  uint64_t m = 0;
  rc = gdsm::track_pack(t, h_twin, h_cur, h_ids, n, &m);
  if (rc) return rc;
  if (m != n) return -EINVAL;  // written concurrently: the interval is not quiescent
  if (n) {
    GDSM_TRY(hipMemcpyAsync(ctx->track_dev, ctx->track_host, bytes, hipMemcpyHostToDevice,
                            ctx->stream));
    GDSM_TRY(hipMemcpyAsync(ids_dev, ctx->track_dev + 2 * n * GDSM_PAGE_SZ, n * sizeof(uint32_t),
                            hipMemcpyDeviceToDevice, ctx->stream));
  }
  rc = ensure(ctx, &ctx->diff_ws, &ctx->diff_ws_bytes, gdsm::diff_workspace_bytes(n));
  if (rc) return rc;
  out->n = n;
  GDSM_TRY(gdsm::launch_diff(ctx->track_dev, ctx->track_dev + n * GDSM_PAGE_SZ, nullptr, n,
                             out->rec_off, out->data, out->cap, ctx->diff_ws, ctx->diff_ws_bytes,
                             ctx->stream, ctx->P()));
  // the pinned staging is reused by the next call: wait for the upload now
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  *n_out = n;
  return 0;
}

const char* gdsm_version(void) { return "gdsm 0.1.0 (gfx950)"; }

int gdsm_tune(const char* key, int64_t value) {
  if (!key) return -EINVAL;
  return gdsm::tune(key, value) == 0 ? 0 : -EINVAL;
}

int gdsm_device_count(int* count) {
  if (!count) return -EINVAL;
  *count = 0;
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return -ENODEV;
  }
  return 0;
}

int gdsm_init(gdsm_ctx** out, int device, uint64_t n_pages, uint32_t flags) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return -ENODEV;
  if (device < 0 || device >= count) return -EINVAL;
  if (flags == 0) flags = GDSM_WANT_TWIN | GDSM_WANT_CURRENT | GDSM_WANT_REPLICA;
  if (flags & GDSM_NO_ARENAS) flags = 0;
  gdsm_ctx* ctx = new (std::nothrow) gdsm_ctx();
  if (!ctx) return -ENOMEM;
  ctx->device = device;
  ctx->n_pages = n_pages;
  DeviceGuard g(device);
  int rc = 0;
  do {
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      rc = -EIO;
      break;
    }
    if (hipMalloc(reinterpret_cast<void**>(&ctx->err), 256) != hipSuccess) {
      rc = -ENOMEM;
      break;
    }
    // on the context's own stream: a non-blocking stream does not wait for the null stream,
    // so a hipMemset there could land after the first read of the word (a recycled allocation
    // still holding an earlier context's error bits)
    if (hipMemsetAsync(ctx->err, 0, 256, ctx->stream) != hipSuccess) {
      rc = -EIO;
      break;
    }
    // the chained forms' workspaces (short releases, small coherence batches; zeroed by their
    // first launch): allocated here, so that no later call allocates outside ensure()
    if (hipMalloc(reinterpret_cast<void**>(&ctx->chain.ws), gdsm::diff_chain_bytes()) !=
            hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&ctx->coh_chain.ws), gdsm::coh_chain_bytes()) !=
            hipSuccess) {
      rc = -ENOMEM;
      break;
    }
    for (int a = 0; a < 3 && !rc; ++a) {
      if (!(flags & (1u << a)) || n_pages == 0) continue;
      // + one guard page (index n_pages): where a checked id list sends out-of-range ids
      if (hipMalloc(reinterpret_cast<void**>(&ctx->arena[a]), (n_pages + 1) * GDSM_PAGE_SZ) !=
          hipSuccess)
        rc = -ENOMEM;
    }
  } while (0);
  if (rc) {
    gdsm_fini(ctx);
    return rc;
  }
  *out = ctx;
  return 0;
}

int gdsm_fini(gdsm_ctx* ctx) {
  if (!ctx) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& a : ctx->arena)
    if (a) (void)hipFree(a);
  for (void* p : ctx->allocs) (void)hipFree(p);
  if (ctx->err) (void)hipFree(ctx->err);
  if (ctx->diff_ws) (void)hipFree(ctx->diff_ws);
  if (ctx->chain.ws) (void)hipFree(ctx->chain.ws);
  if (ctx->coh_chain.ws) (void)hipFree(ctx->coh_chain.ws);
  if (ctx->coh_ws) (void)hipFree(ctx->coh_ws);
  if (ctx->rounds_ws) (void)hipFree(ctx->rounds_ws);
  if (ctx->coh_pt) (void)hipFree(ctx->coh_pt);
  if (ctx->coh_totals) (void)hipFree(ctx->coh_totals);
  if (ctx->track_dev) (void)hipFree(ctx->track_dev);
  if (ctx->track_host) (void)hipHostFree(ctx->track_host);
  if (ctx->nw_ws) (void)hipFree(ctx->nw_ws);
  if (ctx->nw_stage) (void)hipFree(ctx->nw_stage);
  if (ctx->wire_ws) (void)hipFree(ctx->wire_ws);
  for (auto* p : ctx->ids_safe)
    if (p) (void)hipFree(p);
  for (auto& kv : ctx->runs_busy) (void)hipEventDestroy(kv.second);
  if (ctx->ev_main) (void)hipEventDestroy(ctx->ev_main);
  if (ctx->ev_aux) (void)hipEventDestroy(ctx->ev_aux);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return 0;
}

int gdsm_arena(gdsm_ctx* ctx, int which, void** dev_ptr) {
  if (!ctx || !dev_ptr || which < 0 || which > 2 || !ctx->arena[which]) return -EINVAL;
  *dev_ptr = ctx->arena[which];
  return 0;
}

uint64_t gdsm_n_pages(const gdsm_ctx* ctx) { return ctx ? ctx->n_pages : 0; }

void* gdsm_stream(gdsm_ctx* ctx) {
  if (!ctx) return nullptr;
  DeviceGuard g(ctx->device);
  (void)join_aux(ctx);  // the caller may enqueue anything on it
  return reinterpret_cast<void*>(ctx->stream);
}

int gdsm_sync(gdsm_ctx* ctx) {
  if (!ctx) return -EINVAL;
  if (ctx->capturing) return -EBUSY;  // a recording stream cannot be waited for
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return check_and_clear_err(ctx);
}

// ---- HIP graphs ---------------------------------------------------------------------------
struct gdsm_graph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int device = 0;
};

int gdsm_capture_begin(gdsm_ctx* ctx) {
  if (!ctx || ctx->capturing) return -EINVAL;
  CtxGuard g(ctx);  // pending async applies join the main stream before the capture opens
  if (g.rc) return g.rc;
  GDSM_TRY(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
  ctx->capturing = true;
  ctx->capture_origin = true;
  return 0;
}

int gdsm_capture_join(gdsm_ctx* ctx, gdsm_ctx* other) {
  if (!ctx || !other || !ctx->capturing || other == ctx || other->capturing ||
      other->device != ctx->device || other->aux_pending)
    return -EINVAL;
  DeviceGuard g(ctx->device);
  hipEvent_t e = nullptr;
  GDSM_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (hipEventRecord(e, ctx->stream) != hipSuccess ||
      hipStreamWaitEvent(other->stream, e, 0) != hipSuccess) {
    (void)hipEventDestroy(e);
    return -EIO;
  }
  ctx->capture_events.push_back(e);
  ctx->capture_joined.push_back(other);
  other->capturing = true;
  return 0;
}

int gdsm_capture_end(gdsm_ctx* ctx, gdsm_graph** out) {
  // only the context that began the capture ends it (a joined one has no capture of its own)
  if (!ctx || !out || !ctx->capturing || !ctx->capture_origin) return -EINVAL;
  DeviceGuard g(ctx->device);
  int rc = 0;
  for (gdsm_ctx* o : ctx->capture_joined) {  // the joined streams rejoin before the capture ends
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(e, o->stream) != hipSuccess ||
        hipStreamWaitEvent(ctx->stream, e, 0) != hipSuccess)
      rc = -EIO;
    if (e) ctx->capture_events.push_back(e);
    o->capturing = false;
  }
  hipGraph_t graph = nullptr;
  const hipError_t ee = hipStreamEndCapture(ctx->stream, &graph);
  ctx->capturing = false;
  ctx->capture_origin = false;
  for (hipEvent_t e : ctx->capture_events) (void)hipEventDestroy(e);
  ctx->capture_events.clear();
  ctx->capture_joined.clear();
  if (ee != hipSuccess || !graph || rc) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc ? rc : map_err(ee) ? map_err(ee) : -EIO;
  }
  gdsm_graph* gg = new (std::nothrow) gdsm_graph;
  if (!gg) {
    (void)hipGraphDestroy(graph);
    return -ENOMEM;
  }
  gg->graph = graph;
  gg->device = ctx->device;
  if (hipGraphInstantiate(&gg->exec, graph, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGraphDestroy(graph);
    delete gg;
    return -EIO;
  }
  *out = gg;
  return 0;
}

int gdsm_graph_launch(gdsm_ctx* ctx, const gdsm_graph* gg) {
  if (!ctx || !gg || ctx->capturing || gg->device != ctx->device) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipGraphLaunch(gg->exec, ctx->stream));
  return 0;
}

int gdsm_graph_destroy(gdsm_graph* gg) {
  if (!gg) return -EINVAL;
  DeviceGuard g(gg->device);
  if (gg->exec) (void)hipGraphExecDestroy(gg->exec);
  if (gg->graph) (void)hipGraphDestroy(gg->graph);
  delete gg;
  return 0;
}

static int page_copy(gdsm_ctx* ctx, int which, uint64_t first, uint64_t n, void* host, bool up) {
  if (!ctx || which < 0 || which > 2 || !ctx->arena[which] || (!host && n)) return -EINVAL;
  if (first > ctx->n_pages || n > ctx->n_pages - first) return -EINVAL;
  if (n == 0) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  uint8_t* dev = ctx->arena[which] + first * GDSM_PAGE_SZ;
  const uint64_t bytes = n * GDSM_PAGE_SZ;
  if (up)
    GDSM_TRY(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  else
    GDSM_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gdsm_upload(gdsm_ctx* ctx, int which, uint64_t first, uint64_t n, const void* host) {
  return page_copy(ctx, which, first, n, const_cast<void*>(host), true);
}

int gdsm_download(gdsm_ctx* ctx, int which, uint64_t first, uint64_t n, void* host) {
  return page_copy(ctx, which, first, n, host, false);
}

int gdsm_reserve(gdsm_ctx* ctx, uint64_t diff_pages, uint64_t coh_events) {
  if (!ctx) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  int rc = 0;
  if (diff_pages) {
    rc = ensure(ctx, &ctx->diff_ws, &ctx->diff_ws_bytes, gdsm::diff_workspace_bytes(diff_pages));
    // checked copies of the id lists of diff / twin / apply on the main stream
    if (!rc) {
      for (int w : {0, 2}) {  // the diff's page list and gdsm_diff_apply_ids' target list
        uint8_t* buf = reinterpret_cast<uint8_t*>(ctx->ids_safe[w]);
        if (!rc) rc = ensure(ctx, &buf, &ctx->ids_safe_bytes[w], 4 * diff_pages);
        ctx->ids_safe[w] = reinterpret_cast<uint32_t*>(buf);
      }
    }
  }
  if (!rc && coh_events)
    rc = ensure(ctx, &ctx->coh_ws, &ctx->coh_ws_bytes, gdsm::coh_workspace_bytes(coh_events));
  return rc;
}

int gdsm_dev_alloc(gdsm_ctx* ctx, uint64_t bytes, void** dev_ptr) {
  if (!ctx || !dev_ptr) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  void* p = nullptr;
  GDSM_TRY(hipMalloc(&p, bytes ? bytes : 16));
  ctx->allocs.insert(p);
  *dev_ptr = p;
  return 0;
}

int gdsm_dev_free(gdsm_ctx* ctx, void* dev_ptr) {
  if (!ctx || !dev_ptr || !ctx->allocs.count(dev_ptr)) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  (void)hipStreamSynchronize(ctx->stream);
  ctx->allocs.erase(dev_ptr);
  GDSM_TRY(hipFree(dev_ptr));
  return 0;
}

int gdsm_memcpy_h2d(gdsm_ctx* ctx, void* dev, const void* host, uint64_t bytes) {
  if (!ctx || (bytes && (!dev || !host))) return -EINVAL;
  if (!bytes) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gdsm_memcpy_d2h(gdsm_ctx* ctx, void* host, const void* dev, uint64_t bytes) {
  if (!ctx || (bytes && (!dev || !host))) return -EINVAL;
  if (!bytes) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gdsm_prof_enable(gdsm_ctx* ctx, int on) {
  if (!ctx) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  ctx->prof.resolve();
  ctx->prof.clear();
  ctx->prof.on = on != 0;
  return 0;
}

int gdsm_debug_fail_alloc(gdsm_ctx* ctx, int nth) {
  if (!ctx || nth < 0) return -EINVAL;
  ctx->fail_alloc = nth;
  return 0;
}

int gdsm_prof_read(gdsm_ctx* ctx, double* ms, uint64_t* launches) {
  if (!ctx || !ms || !launches) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  ctx->prof.resolve();
  for (int i = 0; i < GDSM_PROF_STAGES; ++i) {
    ms[i] = ctx->prof.ms[i];
    launches[i] = ctx->prof.launches[i];
  }
  ctx->prof.clear();
  return 0;
}

int gdsm_memcpy_batch(gdsm_ctx* ctx, const uint64_t* desc, uint64_t n) {
  if (!ctx || (n && !desc)) return -EINVAL;
  if (!n) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(gdsm::launch_copy_batch(desc, n, ctx->stream));
  return 0;
}

int gdsm_memcpy_d2d(gdsm_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  if (!ctx || (bytes && (!dst || !src))) return -EINVAL;
  if (!bytes) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return 0;
}

int gdsm_gen_pages(gdsm_ctx* ctx, uint32_t arenas, uint64_t first_global, uint64_t stride,
                   uint64_t seed, int mode, uint32_t ppm) {
  if (!ctx) return -EINVAL;
  if (arenas == 0) arenas = 7u;
  if (arenas & ~7u) return -EINVAL;
  for (int a = 0; a < 3; ++a)
    if ((arenas & (1u << a)) && !ctx->arena[a]) return -EINVAL;
  if (mode != GDSM_GEN_UNIFORM && mode != GDSM_GEN_CLUSTERED) return -EINVAL;
  if (ppm > 1000000u) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  auto pick = [&](int a) { return (arenas & (1u << a)) ? ctx->arena[a] : nullptr; };
  GDSM_TRY(gdsm::launch_gen_pages(pick(GDSM_TWIN), pick(GDSM_CURRENT), pick(GDSM_REPLICA),
                                  ctx->n_pages, first_global, stride, seed, mode, ppm,
                                  ctx->stream));
  return 0;
}

int gdsm_gen_pages_raw(uint8_t* twin, uint8_t* cur, uint8_t* replica, uint64_t n,
                       uint64_t first_global, uint64_t stride, uint64_t seed, int mode,
                       uint32_t ppm, void* stream) {
  if (mode != GDSM_GEN_UNIFORM && mode != GDSM_GEN_CLUSTERED) return -EINVAL;
  if (ppm > 1000000u) return -EINVAL;
  GDSM_TRY(gdsm::launch_gen_pages(twin, cur, replica, n, first_global, stride, seed, mode, ppm,
                                  static_cast<hipStream_t>(stream)));
  return 0;
}

int gdsm_twin(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n) {
  if (!ctx || !ctx->arena[GDSM_TWIN] || !ctx->arena[GDSM_CURRENT]) return -EINVAL;
  if (!ids && n > ctx->n_pages) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  // the kernel guards the list itself (no check launch: config 5 twins every round)
  GDSM_TRY(gdsm::launch_twin(ctx->arena[GDSM_TWIN], ctx->arena[GDSM_CURRENT], ids, n,
                             ctx->stream, ctx->P(), ctx->n_pages, ctx->err));
  return 0;
}

int gdsm_runs_alloc(gdsm_ctx* ctx, uint64_t n, uint64_t cap, gdsm_runs* out) {
  if (!ctx || !out) return -EINVAL;
  if (cap == 0) cap = n * (uint64_t)GDSM_MAX_RECORD;
  cap = (cap + 15) & ~15ull;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  memset(out, 0, sizeof(*out));
  void* ro = nullptr;
  void* d = nullptr;
  GDSM_TRY(hipMalloc(&ro, (n + 1) * sizeof(uint64_t)));
  if (hipMalloc(&d, cap ? cap : 16) != hipSuccess) {
    (void)hipFree(ro);
    return -ENOMEM;
  }
  ctx->allocs.insert(ro);
  ctx->allocs.insert(d);
  out->n = n;
  out->n_cap = n;
  out->rec_off = static_cast<uint64_t*>(ro);
  out->data = static_cast<uint8_t*>(d);
  out->cap = cap;
  out->owned = 1;
  return 0;
}

int gdsm_runs_free(gdsm_ctx* ctx, gdsm_runs* runs) {
  if (!ctx || !runs || !runs->owned) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  (void)hipStreamSynchronize(ctx->stream);
  auto it = ctx->runs_busy.find(runs->rec_off);
  if (it != ctx->runs_busy.end()) {
    (void)hipEventDestroy(it->second);
    ctx->runs_busy.erase(it);
  }
  for (void* p : {static_cast<void*>(runs->rec_off), static_cast<void*>(runs->data)}) {
    if (ctx->allocs.erase(p)) (void)hipFree(p);
  }
  memset(runs, 0, sizeof(*runs));
  return 0;
}

static int diff_impl(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out,
                     int target, const uint32_t* tids = nullptr, bool retwin = false) {
  if (!ctx || !out || !out->rec_off || (!out->data && out->cap)) return -EINVAL;
  if (!ctx->arena[GDSM_TWIN] || !ctx->arena[GDSM_CURRENT]) return -EINVAL;
  if (target >= 0 && (target > 2 || target == GDSM_TWIN || target == GDSM_CURRENT ||
                      !ctx->arena[target]))
    return -EINVAL;
  if (!ids && n > ctx->n_pages) return -EINVAL;
  if (out->n_cap ? n > out->n_cap : (out->owned && n > out->n)) return -EINVAL;
  DeviceGuard g(ctx->device);
  uint32_t touched = (1u << GDSM_TWIN) | (1u << GDSM_CURRENT);
  if (target >= 0) touched |= 1u << target;
  if (ctx->aux_targets & touched) {
    int rc = join_aux(ctx);  // a pending apply writes an arena this call reads or writes
    if (rc) return rc;
  }
  auto busy = ctx->runs_busy.find(out->rec_off);
  if (busy != ctx->runs_busy.end()) GDSM_TRY(hipStreamWaitEvent(ctx->stream, busy->second, 0));
  int rc = ensure(ctx, &ctx->diff_ws, &ctx->diff_ws_bytes, gdsm::diff_workspace_bytes(n));
  // the caller's lists are checked into ids_safe[0] / [2] by the diff launch's prep kernel
  gdsm::IdGuard guard{ids, tids, nullptr, nullptr, ctx->n_pages, ctx->err};
  if (!rc && ids && n) rc = safe_buf(ctx, n, 0, &guard.safe_ids);
  if (!rc && tids && n) rc = safe_buf(ctx, n, 2, &guard.safe_tids);
  if (rc) return rc;
  if (!n) guard.ids = guard.tids = nullptr;
  // a short list outside graph capture: the chained one-launch form (its granules and counters
  // allocated by gdsm_init)
  gdsm::DiffChain* chain = nullptr;
  if (n && n <= gdsm::kDiffChainUnits && ctx->chain.ws && !recording(ctx)) chain = &ctx->chain;
  out->n = n;
  GDSM_TRY(gdsm::launch_diff(ctx->arena[GDSM_TWIN], ctx->arena[GDSM_CURRENT], ids, n,
                             out->rec_off, out->data, out->cap, ctx->diff_ws, ctx->diff_ws_bytes,
                             ctx->stream, ctx->P(), target >= 0 ? ctx->arena[target] : nullptr,
                             ctx->diff_bpp, tids, &guard,
                             retwin ? ctx->arena[GDSM_TWIN] : nullptr, chain));
  return 0;
}

int gdsm_release(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out, int target,
                 const uint32_t* target_ids, uint32_t flags) {
  if (flags & ~(uint32_t)GDSM_RELEASE_RETWIN) return -EINVAL;
  if (target < 0 && target_ids) return -EINVAL;
  return diff_impl(ctx, ids, n, out, target, target_ids, (flags & GDSM_RELEASE_RETWIN) != 0);
}

int gdsm_diff_apply_ids(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out,
                        int target, const uint32_t* target_ids) {
  if (target < 0 || (n && !target_ids)) return -EINVAL;
  return diff_impl(ctx, ids, n, out, target, target_ids);
}

int gdsm_diff(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out) {
  return diff_impl(ctx, ids, n, out, -1);
}

int gdsm_diff_apply(gdsm_ctx* ctx, const uint32_t* ids, uint64_t n, gdsm_runs* out,
                    int target) {
  if (target < 0) return -EINVAL;
  return diff_impl(ctx, ids, n, out, target);
}

int gdsm_diff_split(gdsm_ctx* ctx, const uint64_t* bounds, uint32_t G, gdsm_runs* out) {
  if (!ctx || !bounds || !out || G < 1 || G > gdsm::kMaxSplit) return -EINVAL;
  if (!ctx->arena[GDSM_TWIN] || !ctx->arena[GDSM_CURRENT]) return -EINVAL;
  if (bounds[G] > ctx->n_pages) return -EINVAL;
  gdsm::DiffSplit sp{};
  sp.G = G;
  for (uint32_t d = 0; d < G; ++d) {
    gdsm_runs& o = out[d];
    if (bounds[d + 1] < bounds[d] || !o.rec_off || (!o.data && o.cap)) return -EINVAL;
    const uint64_t n = bounds[d + 1] - bounds[d];
    if (o.n_cap ? n > o.n_cap : (o.owned && n > o.n)) return -EINVAL;
    for (uint32_t e = 0; e < d; ++e)
      if (out[e].rec_off == o.rec_off) return -EINVAL;  // every stream its own buffers
    sp.rec_off[d] = o.rec_off;
    sp.data[d] = o.data;
    sp.cap[d] = o.cap;
    sp.first[d] = bounds[d];
  }
  sp.first[G] = bounds[G];
  DeviceGuard g(ctx->device);
  if (ctx->aux_targets & ((1u << GDSM_TWIN) | (1u << GDSM_CURRENT))) {
    int rc = join_aux(ctx);  // a pending apply writes an arena this call reads
    if (rc) return rc;
  }
  for (uint32_t d = 0; d < G; ++d) {
    auto busy = ctx->runs_busy.find(out[d].rec_off);
    if (busy != ctx->runs_busy.end()) GDSM_TRY(hipStreamWaitEvent(ctx->stream, busy->second, 0));
  }
  int rc = ensure(ctx, &ctx->diff_ws, &ctx->diff_ws_bytes,
                  gdsm::diff_workspace_bytes(bounds[G] - bounds[0]));
  if (rc) return rc;
  for (uint32_t d = 0; d < G; ++d) out[d].n = bounds[d + 1] - bounds[d];
  GDSM_TRY(gdsm::launch_diff_split(ctx->arena[GDSM_TWIN], ctx->arena[GDSM_CURRENT], sp,
                                   ctx->diff_ws, ctx->diff_ws_bytes, ctx->stream, ctx->P(),
                                   ctx->diff_bpp));
  return 0;
}

int gdsm_runs_total(gdsm_ctx* ctx, const gdsm_runs* runs, uint64_t* total) {
  if (!ctx || !runs || !total || !runs->rec_off) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  uint64_t t = 0;
  GDSM_TRY(hipMemcpyAsync(&t, runs->rec_off + runs->n, 8, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  *total = t;
  if (runs->n > kDiffShortList) note_density(ctx, t, runs->n);
  return t > runs->cap ? -ENOSPC : 0;
}

int gdsm_apply(gdsm_ctx* ctx, int target, const uint32_t* ids, const gdsm_runs* in) {
  if (!ctx || !in || target < 0 || target > 2 || !ctx->arena[target]) return -EINVAL;
  if (!ids && in->n > ctx->n_pages) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  int rc = safe_ids(ctx, ids, in->n, 0, &ids);
  if (rc) return rc;
  GDSM_TRY(gdsm::launch_apply(ctx->arena[target], ids, in->n, in->rec_off, in->data, ctx->err,
                              ctx->stream, ctx->P()));
  return 0;
}

int gdsm_apply_async(gdsm_ctx* ctx, int target, const uint32_t* ids, const gdsm_runs* in) {
  if (!ctx || !in || target < 0 || target > 2 || !ctx->arena[target]) return -EINVAL;
  if (!ids && in->n > ctx->n_pages) return -EINVAL;
  DeviceGuard g(ctx->device);
  int rc0 = ensure_aux(ctx);
  if (rc0) return rc0;
  hipEvent_t& busy = ctx->runs_busy[in->rec_off];
  if (!busy) GDSM_TRY(hipEventCreateWithFlags(&busy, hipEventDisableTiming));
  GDSM_TRY(hipEventRecord(ctx->ev_main, ctx->stream));  // after the diff that produced `in`
  GDSM_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_main, 0));
  int rc = safe_ids(ctx, ids, in->n, 1, &ids);
  if (rc) return rc;
  GDSM_TRY(gdsm::launch_apply(ctx->arena[target], ids, in->n, in->rec_off, in->data, ctx->err,
                              ctx->aux, ctx->P()));
  GDSM_TRY(hipEventRecord(busy, ctx->aux));
  ctx->aux_pending = true;
  ctx->aux_targets |= 1u << target;
  return 0;
}

uint64_t gdsm_diff_workspace_bytes(uint64_t n) { return gdsm::diff_workspace_bytes(n); }

int gdsm_diff_raw(const uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                  uint64_t* rec_off, uint8_t* data, uint64_t cap, void* workspace,
                  uint64_t workspace_bytes, void* stream) {
  if (!twin || !cur || !rec_off || !workspace || (!data && cap)) return -EINVAL;
  GDSM_TRY(gdsm::launch_diff(twin, cur, ids, n, rec_off, data, cap,
                             static_cast<uint8_t*>(workspace), workspace_bytes,
                             static_cast<hipStream_t>(stream)));
  return 0;
}

int gdsm_diff_apply_raw(const uint8_t* twin, const uint8_t* cur, uint8_t* target,
                        const uint32_t* ids, uint64_t n, uint64_t* rec_off, uint8_t* data,
                        uint64_t cap, void* workspace, uint64_t workspace_bytes, void* stream) {
  if (!twin || !cur || !target || !rec_off || !workspace || (!data && cap)) return -EINVAL;
  GDSM_TRY(gdsm::launch_diff(twin, cur, ids, n, rec_off, data, cap,
                             static_cast<uint8_t*>(workspace), workspace_bytes,
                             static_cast<hipStream_t>(stream), nullptr, target));
  return 0;
}

int gdsm_apply_raw(uint8_t* target, const uint32_t* ids, uint64_t n, const uint64_t* rec_off,
                   const uint8_t* data, uint32_t* err, void* stream) {
  if (!target || !rec_off || (!data && n)) return -EINVAL;
  // unreported errors land in a sink word on the stream's own device (one per device)
  static std::map<int, uint32_t*> sinks;
  static std::mutex mu;
  if (!err) {
    int dev = -1;
    if (!stream || hipStreamGetDevice(static_cast<hipStream_t>(stream), &dev) != hipSuccess)
      GDSM_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    uint32_t*& sink = sinks[dev];
    if (!sink) {
      DeviceGuard g(dev);
      GDSM_TRY(hipMalloc(reinterpret_cast<void**>(&sink), 4));
    }
    err = sink;
  }
  GDSM_TRY(gdsm::launch_apply(target, ids, n, rec_off, data, err,
                              static_cast<hipStream_t>(stream)));
  return 0;
}

int gdsm_twin_raw(uint8_t* twin, const uint8_t* cur, const uint32_t* ids, uint64_t n,
                  void* stream) {
  if (!twin || !cur) return -EINVAL;
  GDSM_TRY(gdsm::launch_twin(twin, cur, ids, n, static_cast<hipStream_t>(stream)));
  return 0;
}

// ---- coherence -------------------------------------------------------------------------
int gdsm_coh_init(gdsm_ctx* ctx, uint32_t n_nodes) {
  if (!ctx || n_nodes == 0 || n_nodes > GDSM_MAX_NODES) return -EINVAL;
  // the fold kernel reads page ids from the events' low dwords (SPEC §5: page < 2^28)
  if (ctx->n_pages > GDSM_MAX_COH_PAGES) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  if (!ctx->coh_pt) {
    GDSM_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->coh_pt),
                       (ctx->n_pages ? ctx->n_pages : 1) * 8));
    GDSM_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->coh_totals), 10 * sizeof(uint64_t)));
  }
  ctx->n_nodes = n_nodes;
  GDSM_TRY(gdsm::launch_coh_init(ctx->coh_pt, ctx->n_pages, n_nodes, ctx->stream));
  return 0;
}

int gdsm_coherence_batch_async(gdsm_ctx* ctx, const uint64_t* events, uint64_t n_events,
                               uint64_t* totals_dev) {
  if (!ctx || !ctx->coh_pt || !totals_dev || (!events && n_events)) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  int rc = ensure(ctx, &ctx->coh_ws, &ctx->coh_ws_bytes, gdsm::coh_workspace_bytes(n_events));
  if (rc) return rc;
  // (outside graph capture, see launch_coherence; allocated by gdsm_init)
  gdsm::CohChainState* chain = nullptr;
  if (ctx->coh_chain.ws && !recording(ctx)) chain = &ctx->coh_chain;
  GDSM_TRY(gdsm::launch_coherence(ctx->coh_pt, ctx->n_pages, ctx->n_nodes, events, n_events,
                                  totals_dev, ctx->coh_ws, ctx->coh_ws_bytes, ctx->err,
                                  ctx->stream, ctx->P(), chain));
  return 0;
}

// ---- DSM rounds on the device ----------------------------------------------------------------
namespace {
// offsets (host, n + 1) checked: non-decreasing from 0; the largest step
bool check_offsets(const int64_t* off, uint32_t n, uint64_t* max_step) {
  if (!off || off[0] != 0) return false;
  uint64_t m = 0;
  for (uint32_t r = 0; r < n; ++r) {
    if (off[r + 1] < off[r]) return false;
    m = std::max<uint64_t>(m, (uint64_t)(off[r + 1] - off[r]));
  }
  *max_step = m;
  return true;
}

// The largest grid of 256-thread workgroups of `kern` that is resident at once (0 on failure).
uint64_t resident_grid(const void* kern) {
  int dev = 0, ncu = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, 0) != hipSuccess)
    return 0;
  return (uint64_t)std::max(ncu, 0) * (uint64_t)std::max(occ, 0);
}
}  // namespace

int gdsm_rounds(gdsm_ctx* data, gdsm_ctx* pt, uint32_t n_rounds, const uint64_t* events,
                const int64_t* ev_off, uint64_t* totals, const uint32_t* ids,
                const uint32_t* home, const int64_t* id_off, const uint64_t* desc,
                const int64_t* desc_off, gdsm_runs* runs) {
  if (!data || !pt || data == pt || data->device != pt->device || !runs || !runs->rec_off ||
      (!runs->data && runs->cap))
    return -EINVAL;
  if (!data->arena[GDSM_TWIN] || !data->arena[GDSM_CURRENT] || !data->arena[GDSM_REPLICA] ||
      !pt->coh_pt || !data->chain.ws || !pt->coh_chain.ws)
    return -EINVAL;
  uint64_t max_ev = 0, max_ids = 0, max_desc = 0;
  if (!check_offsets(ev_off, n_rounds, &max_ev) || !check_offsets(id_off, n_rounds, &max_ids) ||
      !check_offsets(desc_off, n_rounds, &max_desc))
    return -EINVAL;
  if ((ev_off[n_rounds] && !events) || (id_off[n_rounds] && (!ids || !home)) ||
      (desc_off[n_rounds] && !desc) || (n_rounds && !totals))
    return -EINVAL;
  // a round's pages: one look-back granule each; its events: the streaming fold's spans
  if (max_ids > gdsm::kDiffChainUnits || max_ev > (1u << 20)) return -EINVAL;
  if (runs->n_cap ? max_ids > runs->n_cap : (runs->owned && max_ids > runs->n)) return -EINVAL;
  if (n_rounds == 0) return 0;
  if (recording(data) || recording(pt)) return -EBUSY;  // (epochs per launch: not replayable)
  CtxGuard gd(data);
  if (gd.rc) return gd.rc;
  CtxGuard gp(pt);
  if (gp.rc) return gp.rc;
  // the offsets on the device (behind them the grid-barrier word, 256-B aligned)
  const uint64_t ob = 8ull * (n_rounds + 1);
  const uint64_t bar_at = (2 * ob + 255) & ~255ull;
  int rc = ensure(data, &data->rounds_ws, &data->rounds_ws_bytes, bar_at + gdsm::kRoundsBarBytes);
  if (!rc) rc = ensure(pt, &pt->rounds_ws, &pt->rounds_ws_bytes, bar_at + gdsm::kRoundsBarBytes);
  if (rc) return rc;
  GDSM_TRY(hipMemcpyAsync(data->rounds_ws, id_off, ob, hipMemcpyHostToDevice, data->stream));
  GDSM_TRY(hipMemcpyAsync(data->rounds_ws + ob, desc_off, ob, hipMemcpyHostToDevice, data->stream));
  GDSM_TRY(hipMemcpyAsync(pt->rounds_ws, ev_off, ob, hipMemcpyHostToDevice, pt->stream));
  // grids: a workgroup per page of the largest round (data), a wave per 256-event span of
  // the largest round (page table); both far below what is resident at once, which the barriers
  // need (checked)
  const uint64_t gd_n = std::min<uint64_t>(std::max<uint64_t>(max_ids, 1), 256);
  const uint64_t gp_n = std::min<uint64_t>(std::max<uint64_t>((max_ev + 1023) / 1024, 1), 256);
  // small rounds (every round's workgroups fit one XCD, one per CU) run on one-XCD teams: a grid of
  // 8x the workgroups, the members being those on the first one's XCD (about 1 in 8), their
  // hand-offs meeting in that XCD's L2. GDSM_ROUNDS_XCD=0 / 1 forces the choice (A/B runs).
  const char* xe = getenv("GDSM_ROUNDS_XCD");  // (read per call: tests switch it)
  const int xcd_env = xe && *xe ? (xe[0] == '1' ? 1 : 0) : -1;
  const bool xcd = xcd_env == 1 || (xcd_env < 0 && gd_n <= 32 && gp_n <= 32);
  const uint64_t gd_grid = xcd ? 8 * gd_n : gd_n, gp_grid = xcd ? 8 * gp_n : gp_n;
  // a page table and rounds this small fold on a few workgroups that keep slices of the table in
  // LDS (no grid barrier, no gathers, no hand-off); GDSM_ROUNDS_LDS=0 / 1 forces the choice
  const char* le = getenv("GDSM_ROUNDS_LDS");  // (read per call: tests switch it)
  // its workgroups: one per kRoundsLdsWGEvents of the largest round, and enough that every slice
  // of the table fits (GDSM_ROUNDS_LDS_WG forces the count: A/B runs)
  const char* lw = getenv("GDSM_ROUNDS_LDS_WG");
  uint64_t lds_wg = std::max<uint64_t>(
      std::max<uint64_t>((max_ev + gdsm::kRoundsLdsWGEvents - 1) / gdsm::kRoundsLdsWGEvents, 1),
      (pt->n_pages + gdsm::kRoundsLdsPages - 1) / gdsm::kRoundsLdsPages);
  if (lw && *lw) lds_wg = std::max<uint64_t>((uint64_t)atoll(lw), 1);
  const bool lds_fits = lds_wg <= gdsm::kRoundsLdsMaxWGs &&
                        (pt->n_pages + lds_wg - 1) / lds_wg <= gdsm::kRoundsLdsPages &&
                        max_ev <= gdsm::kRoundsLdsEvents && n_rounds <= gdsm::kRoundsLdsRounds;
  const bool lds = lds_fits && !(le && *le == '0');
  if (le && *le == '1' && !lds_fits) return -EINVAL;
  if (gd_grid > resident_grid(gdsm::rounds_data_kernel_ptr(xcd)) ||
      (!lds && gp_grid > resident_grid(gdsm::rounds_fold_kernel_ptr(xcd))))
    return -EINVAL;
  gdsm::DiffChain& ch = data->chain;
  if (ch.epoch == 0 || ch.epoch + n_rounds >= (1u << 30)) {
    GDSM_TRY(hipMemsetAsync(ch.ws, 0, gdsm::diff_chain_bytes(), data->stream));
    ch.epoch = 1;
  }
  const uint32_t epoch0 = ch.epoch;
  ch.epoch = 0;  // the next chained release zeroes the workspace again (its ticket sets restart)
  GDSM_TRY(gdsm::launch_rounds_fold(
      pt->coh_pt, pt->n_pages, pt->n_nodes, events,
      reinterpret_cast<const int64_t*>(pt->rounds_ws), n_rounds,
      (uint32_t)(lds ? lds_wg : gp_grid), totals,
      pt->err, &pt->coh_chain, reinterpret_cast<uint32_t*>(pt->rounds_ws + bar_at), xcd, lds,
      pt->stream, pt->P()));
  runs->n = (uint64_t)(id_off[n_rounds] - id_off[n_rounds - 1]);
  GDSM_TRY(gdsm::launch_rounds_data(
      data->arena[GDSM_TWIN], data->arena[GDSM_CURRENT], ids, home,
      reinterpret_cast<const int64_t*>(data->rounds_ws), desc,
      reinterpret_cast<const int64_t*>(data->rounds_ws + ob), n_rounds, (uint32_t)gd_grid,
      runs->rec_off, runs->data, runs->cap, ch.ws, data->arena[GDSM_REPLICA], data->n_pages,
      data->err, epoch0, reinterpret_cast<uint32_t*>(data->rounds_ws + bar_at), xcd,
      data->stream, data->P()));
  return 0;
}

int gdsm_coherence_batch(gdsm_ctx* ctx, const uint64_t* events, uint64_t n_events,
                         uint64_t* totals) {
  if (!ctx || !totals) return -EINVAL;
  int rc = gdsm_coherence_batch_async(ctx, events, n_events, ctx->coh_totals);
  if (rc) return rc;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(hipMemcpyAsync(totals, ctx->coh_totals, 10 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          ctx->stream));
  return gdsm_sync(ctx);
}

// The page table is interleaved on the device (u64 = state | faults << 32); these copy the two
// word columns to / from the caller's separate arrays with strided (2-D) copies.
int gdsm_coh_download(gdsm_ctx* ctx, uint32_t* state, uint32_t* faults) {
  if (!ctx || !ctx->coh_pt) return -EINVAL;
  if (ctx->n_pages == 0) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  const uint32_t* base = reinterpret_cast<const uint32_t*>(ctx->coh_pt);
  if (state)
    GDSM_TRY(hipMemcpy2DAsync(state, 4, base, 8, 4, ctx->n_pages, hipMemcpyDeviceToHost,
                              ctx->stream));
  if (faults)
    GDSM_TRY(hipMemcpy2DAsync(faults, 4, base + 1, 8, 4, ctx->n_pages, hipMemcpyDeviceToHost,
                              ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gdsm_coh_upload(gdsm_ctx* ctx, const uint32_t* state, const uint32_t* faults) {
  if (!ctx || !ctx->coh_pt) return -EINVAL;
  if (ctx->n_pages == 0) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  uint32_t* base = reinterpret_cast<uint32_t*>(ctx->coh_pt);
  if (state)
    GDSM_TRY(hipMemcpy2DAsync(base, 8, state, 4, 4, ctx->n_pages, hipMemcpyHostToDevice,
                              ctx->stream));
  if (faults)
    GDSM_TRY(hipMemcpy2DAsync(base + 1, 8, faults, 4, 4, ctx->n_pages, hipMemcpyHostToDevice,
                              ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int gdsm_gen_events(gdsm_ctx* ctx, uint64_t* events, const uint64_t* offsets, uint64_t first_page,
                    uint64_t n, uint64_t seed, uint32_t n_nodes, uint32_t write_pct) {
  if (!ctx || (n && (!events || !offsets)) || n_nodes == 0 || n_nodes > GDSM_MAX_NODES ||
      write_pct > 100)
    return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  GDSM_TRY(gdsm::launch_gen_events(events, offsets, first_page, n, seed, n_nodes, write_pct,
                                   ctx->stream));
  return 0;
}

// ---- GPU NW (legacy diff()) ---------------------------------------------------------------
int gdsm_nw_diff_batch(gdsm_ctx* ctx, const uint8_t* a, const uint64_t* a_off, const uint8_t* b,
                       const uint64_t* b_off, uint64_t n, uint32_t max_len, uint8_t* out1,
                       uint8_t* out2, uint64_t* out_len) {
  if (!ctx || !a_off || !b_off || (n && (!out1 || !out2 || !out_len))) return -EINVAL;
  if (max_len > (1u << 20)) return -EINVAL;  // scores travel as 24-bit fields
  if (!n) return 0;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  // Up to 4 GiB of checkpoint / row workspace per chunk of pairs, at least one pair.
  const uint64_t per = gdsm::nw_pair_ws_bytes(max_len);
  uint64_t pairs = (4ull << 30) / per;
  if (pairs < 1) pairs = 1;
  if (pairs > n) pairs = n;
  int rc = ensure(ctx, &ctx->nw_ws, &ctx->nw_ws_bytes, pairs * per);
  if (rc) return rc;
  GDSM_TRY(gdsm::launch_nw(a, a_off, b, b_off, n, max_len, out1, out2, out_len, ctx->nw_ws,
                           pairs * per, ctx->err, ctx->stream, ctx->P()));
  return check_and_clear_err(ctx);
}

// ---- diff wire format (SPEC §7) -------------------------------------------------------------
}  // extern "C"

namespace {
constexpr char kWirePrefix[] = "GDSM1:";
constexpr uint64_t kWirePrefixLen = 6;
constexpr uint32_t kWireMagic = 0x4D534447u;  // "GDSM"

uint64_t up16(uint64_t v) { return (v + 15) & ~15ull; }
uint64_t ids_bytes(uint64_t n) { return 4 * ((n + 1) & ~1ull); }

// Host base64 of the first 44 characters (the 32-byte header); false on a bad character.
bool b64_head(const char* t, uint8_t* out32) {
  uint8_t buf[33];
  for (int q = 0; q < 11; ++q) {
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const unsigned char c = (unsigned char)t[4 * q + k];
      uint32_t x;
      if (c >= 'A' && c <= 'Z') x = c - 'A';
      else if (c >= 'a' && c <= 'z') x = c - 'a' + 26;
      else if (c >= '0' && c <= '9') x = c - '0' + 52;
      else if (c == '+') x = 62;
      else if (c == '/') x = 63;
      else return false;
      v = (v << 6) | x;
    }
    buf[3 * q] = (uint8_t)(v >> 16);
    buf[3 * q + 1] = (uint8_t)(v >> 8);
    buf[3 * q + 2] = (uint8_t)v;
  }
  memcpy(out32, buf, 32);
  return true;
}

struct WireFrame {
  uint64_t n = 0, D = 0, F = 0;
  uint8_t* frame = nullptr;  // device
  const uint32_t* ids() const { return reinterpret_cast<const uint32_t*>(frame + 32); }
  const uint64_t* rec_off() const {
    return reinterpret_cast<const uint64_t*>(frame + 32 + ids_bytes(n));
  }
  const uint8_t* data() const { return frame + 32 + ids_bytes(n) + 8 * (n + 1); }
};

// Decodes and verifies a command text into the context's wire workspace (SPEC §7 "Decode").
int wire_decode_frame(gdsm_ctx* ctx, const char* text, uint64_t len, uint64_t n_pages,
                      WireFrame* wf) {
  if (!text || len < kWirePrefixLen || memcmp(text, kWirePrefix, kWirePrefixLen)) return -EINVAL;
  const char* body = text + kWirePrefixLen;
  const uint64_t T = len - kWirePrefixLen;
  if (T % 4 || T < 44) return -EINVAL;
  const uint32_t pad = body[T - 1] == '=' ? (body[T - 2] == '=' ? 2 : 1) : 0;
  const uint64_t F = T / 4 * 3 - pad;
  uint8_t hdr[32];
  if (F % 8 || !b64_head(body, hdr)) return -EINVAL;
  uint32_t magic;
  uint16_t ver, flags;
  uint64_t n, D, sum;
  memcpy(&magic, hdr, 4);
  memcpy(&ver, hdr + 4, 2);
  memcpy(&flags, hdr + 6, 2);
  memcpy(&n, hdr + 8, 8);
  memcpy(&D, hdr + 16, 8);
  memcpy(&sum, hdr + 24, 8);
  if (magic != kWireMagic || ver != 1 || flags != 0 || D % 4 || n >= (1ull << 32) ||
      D > F || gdsm::wire_frame_bytes(n, D) != F)
    return -EINVAL;
  int rc = ensure(ctx, &ctx->wire_ws, &ctx->wire_ws_bytes, up16(T) + up16(F) + 16);
  if (rc) return rc;
  uint8_t* dtext = ctx->wire_ws;
  uint8_t* frame = dtext + up16(T);
  uint64_t* dsum = reinterpret_cast<uint64_t*>(frame + up16(F));
  GDSM_TRY(hipMemcpyAsync(dtext, body, T, hipMemcpyHostToDevice, ctx->stream));
  GDSM_TRY(gdsm::launch_b64_decode(dtext, T, pad, frame, F, ctx->err, ctx->stream));
  GDSM_TRY(gdsm::launch_wire_sum(frame, F, dsum, ctx->stream));
  wf->n = n;
  wf->D = D;
  wf->F = F;
  wf->frame = frame;
  GDSM_TRY(gdsm::launch_wire_check(wf->ids(), wf->rec_off(), n, D, n_pages, ctx->err,
                                   ctx->stream));
  uint64_t got = 0;
  GDSM_TRY(hipMemcpyAsync(&got, dsum, 8, hipMemcpyDeviceToHost, ctx->stream));
  rc = check_and_clear_err(ctx);  // synchronises
  if (rc) return rc;
  return got == sum ? 0 : -EINVAL;
}
}  // namespace

extern "C" {

uint64_t gdsm_wire_size(uint64_t n, uint64_t data_bytes) {
  const uint64_t F = gdsm::wire_frame_bytes(n, (data_bytes + 3) & ~3ull);
  return kWirePrefixLen + 4 * ((F + 2) / 3);
}

int gdsm_wire_encode(gdsm_ctx* ctx, const uint32_t* ids, const gdsm_runs* runs, char* out,
                     uint64_t cap, uint64_t* len) {
  if (!ctx || !runs || !runs->rec_off || !len || (cap && !out)) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  const uint64_t n = runs->n;
  uint64_t D = 0;
  GDSM_TRY(hipMemcpyAsync(&D, runs->rec_off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  if (D % 4 || D > runs->cap) return -EINVAL;
  const uint64_t F = gdsm::wire_frame_bytes(n, D);
  const uint64_t T = 4 * ((F + 2) / 3);
  *len = kWirePrefixLen + T;
  if (cap < kWirePrefixLen + T + 1) return -ENOSPC;
  int rc = ensure(ctx, &ctx->wire_ws, &ctx->wire_ws_bytes, up16(T) + up16(F) + 16);
  if (rc) return rc;
  uint8_t* dtext = ctx->wire_ws;
  uint8_t* frame = dtext + up16(T);
  uint64_t* dsum = reinterpret_cast<uint64_t*>(frame + up16(F));
  const uint64_t ib = ids_bytes(n);
  ctx->wire_hdr[0] = (uint64_t)kWireMagic | (1ull << 32);  // magic, version 1, flags 0
  ctx->wire_hdr[1] = n;
  ctx->wire_hdr[2] = D;
  ctx->wire_hdr[3] = 0;
  GDSM_TRY(hipMemcpyAsync(frame, ctx->wire_hdr, 32, hipMemcpyHostToDevice, ctx->stream));
  if (n & 1) GDSM_TRY(hipMemsetAsync(frame + 32 + ib - 4, 0, 4, ctx->stream));  // odd-n padding
  // Every frame write is ordered on ctx->stream (the identity list is filled on the device).
  if (n && ids)
    GDSM_TRY(hipMemcpyAsync(frame + 32, ids, 4 * n, hipMemcpyDeviceToDevice, ctx->stream));
  else if (n)
    GDSM_TRY(gdsm::launch_iota(reinterpret_cast<uint32_t*>(frame + 32), n, ctx->stream));
  uint8_t* dro = frame + 32 + ib;
  GDSM_TRY(hipMemcpyAsync(dro, runs->rec_off, 8 * (n + 1), hipMemcpyDeviceToDevice, ctx->stream));
  uint8_t* ddata = dro + 8 * (n + 1);
  if (D) GDSM_TRY(hipMemcpyAsync(ddata, runs->data, D, hipMemcpyDeviceToDevice, ctx->stream));
  if (D % 8) GDSM_TRY(hipMemsetAsync(ddata + D, 0, 4, ctx->stream));
  GDSM_TRY(gdsm::launch_wire_sum(frame, F, dsum, ctx->stream));
  GDSM_TRY(hipMemcpyAsync(frame + 24, dsum, 8, hipMemcpyDeviceToDevice, ctx->stream));
  GDSM_TRY(gdsm::launch_b64_encode(frame, F, dtext, ctx->stream));
  memcpy(out, kWirePrefix, kWirePrefixLen);
  GDSM_TRY(hipMemcpyAsync(out + kWirePrefixLen, dtext, T, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  out[kWirePrefixLen + T] = 0;
  return 0;
}

int gdsm_wire_decode(gdsm_ctx* ctx, const char* text, uint64_t len, uint32_t* ids_out,
                     gdsm_runs* out, uint64_t* n_out) {
  if (!ctx || !out || !out->rec_off || !n_out) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  WireFrame wf;
  int rc = wire_decode_frame(ctx, text, len, ~0ull, &wf);
  if (rc) return rc;
  const uint64_t ncap = out->n_cap ? out->n_cap : out->n;
  if (wf.n > ncap || wf.D > out->cap) return -ENOSPC;
  if (wf.n && !ids_out) return -EINVAL;
  if (wf.n)
    GDSM_TRY(hipMemcpyAsync(ids_out, wf.ids(), 4 * wf.n, hipMemcpyDeviceToDevice, ctx->stream));
  GDSM_TRY(hipMemcpyAsync(out->rec_off, wf.rec_off(), 8 * (wf.n + 1), hipMemcpyDeviceToDevice,
                          ctx->stream));
  if (wf.D)
    GDSM_TRY(hipMemcpyAsync(out->data, wf.data(), wf.D, hipMemcpyDeviceToDevice, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  out->n = wf.n;
  *n_out = wf.n;
  return 0;
}

int gdsm_wire_apply(gdsm_ctx* ctx, int target, const char* text, uint64_t len, uint64_t* n_out) {
  if (!ctx || target < 0 || target > 2 || !ctx->arena[target] || !n_out) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  WireFrame wf;
  int rc = wire_decode_frame(ctx, text, len, ctx->n_pages, &wf);
  if (rc) return rc;
  GDSM_TRY(gdsm::launch_apply(ctx->arena[target], wf.ids(), wf.n, wf.rec_off(), wf.data(),
                              ctx->err, ctx->stream, ctx->P()));
  rc = check_and_clear_err(ctx);
  if (rc) return rc;
  *n_out = wf.n;
  return 0;
}

}  // extern "C"

namespace gdsm {
// diff() offload (legacy_diff.cpp): one pair staged through the context. `alloc` allocates the
// two L+1-byte outputs (the installed allocator).
int nw_host(gdsm_ctx* ctx, const char* m1, size_t n1, const char* m2, size_t n2,
            void* (*alloc)(size_t), void (*release)(void*), char** o1, char** o2, size_t* len) {
  if (n1 > (1u << 20) || n2 > (1u << 20)) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  auto up16 = [](uint64_t v) { return (v + 15) & ~15ull; };
  const uint64_t out_bytes = n1 + n2 + 1;
  const uint64_t need = up16(n1 + 1) + up16(n2 + 1) + 64 + 2 * up16(out_bytes) + 16;
  int rc = ensure(ctx, &ctx->nw_stage, &ctx->nw_stage_bytes, need);
  if (rc) return rc;
  uint8_t* da = ctx->nw_stage;
  uint8_t* db = da + up16(n1 + 1);
  uint64_t* offs = reinterpret_cast<uint64_t*>(db + up16(n2 + 1));
  uint8_t* d1 = reinterpret_cast<uint8_t*>(offs) + 64;
  uint8_t* d2 = d1 + up16(out_bytes);
  uint64_t* dlen = reinterpret_cast<uint64_t*>(d2 + up16(out_bytes));
  const uint64_t h_off[4] = {0, n1, 0, n2};
  if (n1) GDSM_TRY(hipMemcpyAsync(da, m1, n1, hipMemcpyHostToDevice, ctx->stream));
  if (n2) GDSM_TRY(hipMemcpyAsync(db, m2, n2, hipMemcpyHostToDevice, ctx->stream));
  GDSM_TRY(hipMemcpyAsync(offs, h_off, sizeof h_off, hipMemcpyHostToDevice, ctx->stream));
  const uint32_t max_len = (uint32_t)(n1 > n2 ? n1 : n2);
  rc = gdsm_nw_diff_batch(ctx, da, offs, db, offs + 2, 1, max_len, d1, d2, dlen);
  if (rc) return rc;
  uint64_t L = 0;  // on the context's stream: the null stream does not wait for a non-blocking one
  GDSM_TRY(hipMemcpyAsync(&L, dlen, 8, hipMemcpyDeviceToHost, ctx->stream));
  GDSM_TRY(hipStreamSynchronize(ctx->stream));
  char* a1 = static_cast<char*>(alloc(L + 1));
  char* a2 = static_cast<char*>(alloc(L + 1));
  if (!a1 || !a2) {
    if (a1) release(a1);
    if (a2) release(a2);
    return -ENOMEM;
  }
  hipError_t e = hipMemcpyAsync(a1, d1, L + 1, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(a2, d2, L + 1, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    release(a1);
    release(a2);
    return map_err(e);
  }
  *o1 = a1;
  *o2 = a2;
  if (len) *len = L;
  return 0;
}
}  // namespace gdsm
