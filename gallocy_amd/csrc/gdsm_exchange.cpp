// Multi-GPU diff propagation (include/gdsm.h gdsm_comm_* / gdsm_exchange).
//
// The reference moves page updates (had it implemented them) over HTTP: one POST per peer,
// fanned out with std::async and joined for a majority (gallocy/http/client.cpp:39-91, called
// from gallocy/consensus/client.cpp:15-42). Here the records a shard produced for pages homed on
// other GPUs travel GPU-to-GPU over xGMI in one grouped RCCL transfer per release, and the home
// applies them with the same apply kernel as a local release.
//
// Per release, on the context's second stream (after the diffs on the main stream):
//   sizes   exact mode: (records, bytes) per destination -> ncclAllToAll -> one host read, then
//           an ncclAllReduce(max) of a "some receive stream is too small" flag so that every rank
//           agrees to go on or to return -ENOSPC (nobody is left waiting in a send);
//           GDSM_XCHG_FIXED: sizes are the caller's (send[d].n / .cap, recv[s].n / .cap), so the
//           release never synchronises the host; received streams are guarded on the device.
//   move    ncclGroupStart; per peer: send ids, rec_off, data / recv the same; ncclGroupEnd.
//   apply   per source (own stream in place): checked ids, then the apply kernel (SPEC §4).
// RCCL is resolved with dlopen at first use: the librccl the process already has (torch's,
// "librccl.so") or the system one (librccl.so.1), so one RCCL instance serves the process.
#include <dlfcn.h>
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <new>
#include <vector>

#include "gdsm.h"
#include "gdsm_ctx.h"
#include "gdsm_launch.h"

namespace {

struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllToAll) AllToAll = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so", "librccl.so.1"})
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
#define GDSM_SYM(field, sym) r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, #sym))
    GDSM_SYM(GetUniqueId, ncclGetUniqueId);
    GDSM_SYM(CommInitRank, ncclCommInitRank);
    GDSM_SYM(CommDestroy, ncclCommDestroy);
    GDSM_SYM(AllToAll, ncclAllToAll);
    GDSM_SYM(AllReduce, ncclAllReduce);
    GDSM_SYM(Send, ncclSend);
    GDSM_SYM(Recv, ncclRecv);
    GDSM_SYM(GroupStart, ncclGroupStart);
    GDSM_SYM(GroupEnd, ncclGroupEnd);
#undef GDSM_SYM
    r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.AllToAll && r.AllReduce &&
           r.Send && r.Recv && r.GroupStart && r.GroupEnd;
  });
  return r;
}

#define GDSM_NCCL(expr)                        \
  do {                                         \
    if ((expr) != ncclSuccess) return -EIO;    \
  } while (0)

}  // namespace

struct gdsm_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  uint64_t* cnt_dev = nullptr;   // [2G] sent (records, bytes) + [2G] received + flag word
  uint64_t* cnt_host = nullptr;  // pinned mirror
  uint32_t* ids_chk = nullptr;   // checked page indices of one received stream
  uint64_t ids_chk_bytes = 0;
};

using namespace gdsm::detail;

extern "C" {

int gdsm_comm_unique_id(uint8_t* id) {
  if (!id) return -EINVAL;
  const Rccl& R = rccl();
  if (!R.ok) return -ENOSYS;
  ncclUniqueId u;
  GDSM_NCCL(R.GetUniqueId(&u));
  memcpy(id, u.internal, GDSM_COMM_ID_BYTES);
  return 0;
}

int gdsm_comm_init(gdsm_comm** out, gdsm_ctx* ctx, int nranks, int rank, const uint8_t* id) {
  if (!out || !ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
  *out = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return -ENOSYS;
  DeviceGuard g(ctx->device);
  gdsm_comm* c = new (std::nothrow) gdsm_comm;
  if (!c) return -ENOMEM;
  c->nranks = nranks;
  c->rank = rank;
  c->device = ctx->device;
  const size_t words = 4 * (size_t)nranks + 2;
  if (hipMalloc(reinterpret_cast<void**>(&c->cnt_dev), words * 8) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->cnt_host), words * 8) != hipSuccess) {
    gdsm_comm_fini(c);
    return -ENOMEM;
  }
  ncclUniqueId u;
  memcpy(u.internal, id, GDSM_COMM_ID_BYTES);
  if (R.CommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
    c->comm = nullptr;
    gdsm_comm_fini(c);
    return -EIO;
  }
  *out = c;
  return 0;
}

int gdsm_comm_fini(gdsm_comm* c) {
  if (!c) return -EINVAL;
  DeviceGuard g(c->device);
  if (c->comm) (void)rccl().CommDestroy(c->comm);
  if (c->cnt_dev) (void)hipFree(c->cnt_dev);
  if (c->cnt_host) (void)hipHostFree(c->cnt_host);
  if (c->ids_chk) (void)hipFree(c->ids_chk);
  delete c;
  return 0;
}

int gdsm_comm_size(const gdsm_comm* c, int* nranks, int* rank) {
  if (!c) return -EINVAL;
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  return 0;
}

int gdsm_exchange(gdsm_ctx* ctx, gdsm_comm* c, const gdsm_runs* send,
                  const uint32_t* const* send_ids, gdsm_runs* recv, uint32_t* const* recv_ids,
                  int target, uint32_t flags) {
  if (!ctx || !c || !send || !send_ids || !recv || !recv_ids) return -EINVAL;
  if (target < 0 || target > 2 || !ctx->arena[target] || (flags & ~GDSM_XCHG_FIXED)) return -EINVAL;
  if (c->device != ctx->device) return -EINVAL;
  const int G = c->nranks, me = c->rank;
  const bool fixed = flags & GDSM_XCHG_FIXED;
  for (int d = 0; d < G; ++d) {
    if (send[d].n && (!send[d].rec_off || !send_ids[d] || (!send[d].data && send[d].cap)))
      return -EINVAL;
    if (d != me && (!recv[d].rec_off || (!recv[d].data && recv[d].cap))) return -EINVAL;
  }
  const Rccl& R = rccl();
  if (!R.ok) return -ENOSYS;
  DeviceGuard g(ctx->device);
  int rc = ensure_aux(ctx);
  if (rc) return rc;
  hipStream_t s = ctx->aux;
  // ordered after the diffs that produced send[] (and anything else on the main stream)
  GDSM_TRY(hipEventRecord(ctx->ev_main, ctx->stream));
  GDSM_TRY(hipStreamWaitEvent(s, ctx->ev_main, 0));

  std::vector<uint64_t> rn(G), rb(G), sb(G);  // received records / bytes, sent bytes
  if (fixed) {
    for (int d = 0; d < G; ++d) {
      sb[d] = send[d].cap;
      rn[d] = d == me ? 0 : recv[d].n;
      rb[d] = d == me ? 0 : recv[d].cap;
      if (d != me && rn[d] > (recv[d].n_cap ? recv[d].n_cap : recv[d].n)) return -EINVAL;
    }
  } else {
    // (records, bytes) per destination -> all-to-all -> host
    uint64_t* h = c->cnt_host;
    for (int d = 0; d < G; ++d) h[2 * d] = send[d].n;
    GDSM_TRY(hipMemcpyAsync(c->cnt_dev, h, 16 * G, hipMemcpyHostToDevice, s));
    for (int d = 0; d < G; ++d) {
      if (send[d].rec_off)
        GDSM_TRY(hipMemcpyAsync(c->cnt_dev + 2 * d + 1, send[d].rec_off + send[d].n, 8,
                                hipMemcpyDeviceToDevice, s));
      else
        GDSM_TRY(hipMemsetAsync(c->cnt_dev + 2 * d + 1, 0, 8, s));
    }
    GDSM_NCCL(R.AllToAll(c->cnt_dev, c->cnt_dev + 2 * G, 2, ncclUint64, c->comm, s));
    GDSM_TRY(hipMemcpyAsync(h, c->cnt_dev, 32 * G, hipMemcpyDeviceToHost, s));
    GDSM_TRY(hipStreamSynchronize(s));
    uint64_t too_small = 0;
    for (int d = 0; d < G; ++d) {
      sb[d] = h[2 * d + 1];
      too_small |= sb[d] > send[d].cap;  // that diff overflowed its stream (-ENOSPC)
      if (d == me) continue;
      rn[d] = h[2 * G + 2 * d];
      rb[d] = h[2 * G + 2 * d + 1];
      const uint64_t ncap = recv[d].n_cap ? recv[d].n_cap : recv[d].n;
      too_small |= rn[d] > ncap || rb[d] > recv[d].cap;
    }
    // every rank must agree before anyone posts a send
    h[4 * G] = too_small;
    GDSM_TRY(hipMemcpyAsync(c->cnt_dev + 4 * G, h + 4 * G, 8, hipMemcpyHostToDevice, s));
    GDSM_NCCL(R.AllReduce(c->cnt_dev + 4 * G, c->cnt_dev + 4 * G + 1, 1, ncclUint64, ncclMax,
                          c->comm, s));
    GDSM_TRY(hipMemcpyAsync(h + 4 * G + 1, c->cnt_dev + 4 * G + 1, 8, hipMemcpyDeviceToHost, s));
    GDSM_TRY(hipStreamSynchronize(s));
    if (h[4 * G + 1]) return -ENOSPC;
  }

  // ---- move: one grouped point-to-point transfer per peer pair
  {
    gdsm::ProfScope ps(ctx->P(), GDSM_PROF_EXCHANGE, s);
    GDSM_NCCL(R.GroupStart());
    for (int p = 0; p < G; ++p) {
      if (p == me) continue;
      const uint64_t ns = send[p].n;
      GDSM_NCCL(R.Send(send[p].rec_off, 8 * (ns + 1), ncclUint8, p, c->comm, s));
      if (ns) GDSM_NCCL(R.Send(send_ids[p], 4 * ns, ncclUint8, p, c->comm, s));
      if (sb[p]) GDSM_NCCL(R.Send(send[p].data, sb[p], ncclUint8, p, c->comm, s));
      GDSM_NCCL(R.Recv(recv[p].rec_off, 8 * (rn[p] + 1), ncclUint8, p, c->comm, s));
      if (rn[p]) GDSM_NCCL(R.Recv(recv_ids[p], 4 * rn[p], ncclUint8, p, c->comm, s));
      if (rb[p]) GDSM_NCCL(R.Recv(recv[p].data, rb[p], ncclUint8, p, c->comm, s));
    }
    GDSM_NCCL(R.GroupEnd());
  }
  for (int p = 0; p < G; ++p)
    if (p != me) recv[p].n = rn[p];

  // ---- apply every source's stream to the home arena (own stream in place)
  for (int p = 0; p < G; ++p) {
    const gdsm_runs& in = p == me ? send[p] : recv[p];
    const uint64_t n = p == me ? send[p].n : rn[p];
    if (n == 0) continue;
    if (p != me && fixed)
      GDSM_TRY(gdsm::launch_guard_stream(in.rec_off, n, rb[p], ctx->err, s));
    const uint32_t* ids = p == me ? send_ids[p] : recv_ids[p];
    uint8_t* buf = reinterpret_cast<uint8_t*>(c->ids_chk);
    rc = ensure(&buf, &c->ids_chk_bytes, 4 * n);
    c->ids_chk = reinterpret_cast<uint32_t*>(buf);
    if (rc) return rc;
    GDSM_TRY(gdsm::launch_check_ids(ids, n, ctx->n_pages, c->ids_chk, ctx->err, s));
    GDSM_TRY(gdsm::launch_apply(ctx->arena[target], c->ids_chk, n, in.rec_off, in.data, ctx->err,
                                s, ctx->P()));
  }
  // a later gdsm_diff into a send stream waits for this exchange; everything else joins aux
  for (int d = 0; d < G; ++d) {
    if (!send[d].rec_off) continue;
    hipEvent_t& busy = ctx->runs_busy[send[d].rec_off];
    if (!busy) GDSM_TRY(hipEventCreateWithFlags(&busy, hipEventDisableTiming));
    GDSM_TRY(hipEventRecord(busy, s));
  }
  ctx->aux_pending = true;
  ctx->aux_targets |= 1u << target;
  return 0;
}

}  // extern "C"
