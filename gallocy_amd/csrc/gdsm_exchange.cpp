// Multi-GPU diff propagation (include/gdsm.h gdsm_comm_* / gdsm_exchange).
//
// The reference moves page updates (had it implemented them) over HTTP: one POST per peer,
// fanned out with std::async and joined for a majority (gallocy/http/client.cpp:39-91, called
// from gallocy/consensus/client.cpp:15-42). Here the records a shard produced for pages homed on
// other GPUs travel GPU-to-GPU over xGMI in one grouped RCCL transfer per release, and the home
// applies them with the same apply kernel as a local release.
//
// Per release, on the context's second stream (after the diffs on the main stream):
//   sizes   exact mode: (records, bytes) per destination -> all-to-all -> one host read, then
//           an agreement (all-reduce max) on "some stream is too small" so that every rank goes
//           on or returns -ENOSPC together (nobody is left waiting in a send);
//           GDSM_XCHG_FIXED: sizes are the caller's (send[d].n / .cap, recv[s].n / .cap), so the
//           release never synchronises the host; every stream is checked on the device.
//   move    group start; per peer: send rec_off, ids, data / recv the same; group end.
//   apply   per source (own stream in place): the whole stream checked (offsets, budget, page
//           indices; a rejected stream is emptied, never partly applied), then the apply kernel.
//
// The data movement goes through a Transport: RCCL (the product: ncclAllToAll / ncclAllReduce /
// grouped ncclSend+ncclRecv over xGMI), or Loopback (tests: several ranks as threads of one
// process on one GPU, the same calls at the same points become device-to-device copies ordered
// by HIP events). RCCL is resolved with dlopen at first use: the librccl the process already has
// (torch's, "librccl.so") or the system one (librccl.so.1), so one RCCL instance serves the
// process.
#include <dlfcn.h>
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
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

// The collective operations the exchange and the event routing are built from.
struct Transport {
  virtual ~Transport() = default;
  // recv[p * per .. +per) = what rank p sent to this rank from its send[me * per .. +per)
  // (device u64 arrays of nranks * per words), ordered on stream s.
  virtual int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t per, hipStream_t s) = 0;
  // Synchronous: *v = max over ranks (after everything enqueued on s).
  virtual int agree_max(uint64_t* v, hipStream_t s) = 0;
  virtual int group_start() = 0;
  virtual int send(const void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual int recv(void* buf, size_t bytes, int peer, hipStream_t s) = 0;
  virtual int group_end(hipStream_t s) = 0;
};

// ---- RCCL (product transport)
struct RcclTransport final : Transport {
  ncclComm_t comm = nullptr;
  uint64_t* scratch_dev = nullptr;   // 2 words: agree_max in / out
  uint64_t* scratch_host = nullptr;  // pinned mirror
  ~RcclTransport() override {
    if (comm) (void)rccl().CommDestroy(comm);
    if (scratch_dev) (void)hipFree(scratch_dev);
    if (scratch_host) (void)hipHostFree(scratch_host);
  }
  int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t per, hipStream_t s) override {
    GDSM_NCCL(rccl().AllToAll(send, recv, per, ncclUint64, comm, s));
    return 0;
  }
  int agree_max(uint64_t* v, hipStream_t s) override {
    scratch_host[0] = *v;
    GDSM_TRY(hipMemcpyAsync(scratch_dev, scratch_host, 8, hipMemcpyHostToDevice, s));
    GDSM_NCCL(rccl().AllReduce(scratch_dev, scratch_dev + 1, 1, ncclUint64, ncclMax, comm, s));
    GDSM_TRY(hipMemcpyAsync(scratch_host + 1, scratch_dev + 1, 8, hipMemcpyDeviceToHost, s));
    GDSM_TRY(hipStreamSynchronize(s));
    *v = scratch_host[1];
    return 0;
  }
  int group_start() override {
    GDSM_NCCL(rccl().GroupStart());
    return 0;
  }
  int send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
    GDSM_NCCL(rccl().Send(buf, bytes, ncclUint8, peer, comm, s));
    return 0;
  }
  int recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
    GDSM_NCCL(rccl().Recv(buf, bytes, ncclUint8, peer, comm, s));
    return 0;
  }
  int group_end(hipStream_t) override {
    GDSM_NCCL(rccl().GroupEnd());
    return 0;
  }
};

// ---- Loopback (tests): nranks ranks as host threads of one process. A group's sends are posted
// with an event recorded on the sender's stream; after a barrier every receiver copies its
// messages (device to device, on its own stream, after the sender's event), records its own
// event, and after a second barrier every sender's stream waits for the receivers' copies, so the
// sender's later work cannot overwrite a buffer still being read: the ordering an RCCL
// ncclGroupEnd gives on both streams. Matching is RCCL's: the k-th recv from p takes p's k-th send
// to this rank, and the sizes must agree (-EIO otherwise).
struct LoopGroup {
  struct Msg {
    const void* buf;
    size_t bytes;
    int peer;
  };
  struct Post {
    std::vector<Msg> sends;
    hipEvent_t ready = nullptr, done = nullptr;
    uint64_t value = 0;
  };
  int nranks = 0;
  int refs = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  bool broken = false;
  std::vector<Post> post;

  // All ranks meet here; a rank missing for 60 s breaks the group (-ETIMEDOUT, then -EIO for
  // every later call) instead of hanging the test that drives it.
  int barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return -EIO;
    const uint64_t gen = generation;
    if (++arrived == nranks) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return 0;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60),
                     [&] { return generation != gen || broken; })) {
      broken = true;
      cv.notify_all();
      return -ETIMEDOUT;
    }
    return broken ? -EIO : 0;
  }
};

struct LoopbackTransport final : Transport {
  LoopGroup* g = nullptr;
  int rank = 0;
  std::vector<LoopGroup::Msg> sends, recvs;
  ~LoopbackTransport() override {
    if (!g) return;  // never joined a group
    LoopGroup::Post& me = g->post[rank];
    if (me.ready) (void)hipEventDestroy(me.ready);
    if (me.done) (void)hipEventDestroy(me.done);
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      last = --g->refs == 0;
    }
    if (last) delete g;
  }
  int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t per, hipStream_t s) override {
    int rc = group_start();
    for (int p = 0; p < g->nranks && !rc; ++p) {
      rc = this->send(send + p * per, 8 * per, p, s);
      if (!rc) rc = this->recv(recv + p * per, 8 * per, p, s);
    }
    const int rc2 = group_end(s);
    return rc ? rc : rc2;
  }
  int agree_max(uint64_t* v, hipStream_t s) override {
    GDSM_TRY(hipStreamSynchronize(s));
    g->post[rank].value = *v;
    int rc = g->barrier();
    if (rc) return rc;
    uint64_t m = 0;
    for (const auto& p : g->post) m = p.value > m ? p.value : m;
    rc = g->barrier();  // nobody posts the next value before everyone has read this one
    if (rc) return rc;
    *v = m;
    return 0;
  }
  int group_start() override {
    sends.clear();
    recvs.clear();
    return 0;
  }
  int send(const void* buf, size_t bytes, int peer, hipStream_t) override {
    if (peer < 0 || peer >= g->nranks) return -EINVAL;
    sends.push_back({buf, bytes, peer});
    return 0;
  }
  int recv(void* buf, size_t bytes, int peer, hipStream_t) override {
    if (peer < 0 || peer >= g->nranks) return -EINVAL;
    recvs.push_back({buf, bytes, peer});
    return 0;
  }
  int group_end(hipStream_t s) override {
    LoopGroup::Post& me = g->post[rank];
    me.sends = sends;
    GDSM_TRY(hipEventRecord(me.ready, s));
    int rc = g->barrier();
    if (rc) return rc;
    int err = 0;
    std::vector<size_t> taken(g->nranks, 0);  // sends of peer p to this rank matched so far
    for (const auto& r : recvs) {
      const LoopGroup::Post& from = g->post[r.peer];
      const LoopGroup::Msg* m = nullptr;
      for (size_t k = 0, seen = 0; k < from.sends.size(); ++k)
        if (from.sends[k].peer == rank && seen++ == taken[r.peer]) {
          m = &from.sends[k];
          break;
        }
      ++taken[r.peer];
      if (!m || m->bytes != r.bytes) {
        err = -EIO;
        continue;
      }
      if (!r.bytes) continue;
      if (hipStreamWaitEvent(s, from.ready, 0) != hipSuccess ||
          hipMemcpyAsync(const_cast<void*>(r.buf), m->buf, r.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
        err = -EIO;
    }
    if (hipEventRecord(me.done, s) != hipSuccess) err = -EIO;
    rc = g->barrier();
    if (rc) return rc;
    std::vector<bool> waited(g->nranks, false);
    for (const auto& m : sends)
      if (!waited[m.peer]) {
        waited[m.peer] = true;
        if (hipStreamWaitEvent(s, g->post[m.peer].done, 0) != hipSuccess) err = -EIO;
      }
    sends.clear();
    recvs.clear();
    return err;
  }
};

}  // namespace

struct gdsm_comm {
  Transport* xp = nullptr;
  int nranks = 0, rank = 0, device = 0;
  uint64_t* cnt_dev = nullptr;   // exchange: [2G] sent (records, bytes) + [2G] received
  uint64_t* cnt_host = nullptr;  // pinned mirror
  uint32_t* verdict = nullptr;   // one word per source: its stream's check (launch_xchg_guard)
  uint32_t* ids_chk = nullptr;   // checked page indices of every source's stream, back to back
  uint64_t ids_chk_bytes = 0;
  // coherence routing (gdsm_route_events / gdsm_coherence_notify): [G] sent, [G] received,
  // [G+1] bounds or bases, flag word; pinned mirror; scratch
  uint64_t* rcnt_dev = nullptr;
  uint64_t* rcnt_host = nullptr;
  uint8_t* route_buf = nullptr;  // received stamped events, back to back by source
  uint64_t route_bytes = 0;
  uint8_t* pre = nullptr;        // page-table words before the fold, at each page's first event
  uint64_t pre_bytes = 0;
  uint8_t* blk = nullptr;        // notice counts per (block, node)
  uint64_t blk_bytes = 0;
  uint8_t* blk_off = nullptr;    // their exclusive offsets
  uint64_t blk_off_bytes = 0;
  uint8_t* staging = nullptr;    // this home's notices, destination-major
  uint64_t staging_bytes = 0;
};

using namespace gdsm::detail;

namespace {

int comm_alloc(gdsm_comm* c) {
  const size_t words = 4 * (size_t)c->nranks + 2;
  if (hipMalloc(reinterpret_cast<void**>(&c->cnt_dev), words * 8) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->cnt_host), words * 8) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&c->rcnt_dev), words * 8) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->rcnt_host), words * 8) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&c->verdict), 4 * (size_t)c->nranks) != hipSuccess)
    return -ENOMEM;
  return 0;
}

}  // namespace

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
  RcclTransport* xp = new (std::nothrow) RcclTransport;
  if (!c || !xp) {
    delete c;
    delete xp;
    return -ENOMEM;
  }
  c->xp = xp;
  c->nranks = nranks;
  c->rank = rank;
  c->device = ctx->device;
  if (comm_alloc(c) || hipMalloc(reinterpret_cast<void**>(&xp->scratch_dev), 16) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&xp->scratch_host), 16) != hipSuccess) {
    gdsm_comm_fini(c);
    return -ENOMEM;
  }
  ncclUniqueId u;
  memcpy(u.internal, id, GDSM_COMM_ID_BYTES);
  if (R.CommInitRank(&xp->comm, nranks, u, rank) != ncclSuccess) {
    xp->comm = nullptr;
    gdsm_comm_fini(c);
    return -EIO;
  }
  *out = c;
  return 0;
}

int gdsm_comm_init_loopback(gdsm_comm** comms, gdsm_ctx* const* ctxs, int nranks) {
  if (!comms || !ctxs || nranks < 1) return -EINVAL;
  for (int r = 0; r < nranks; ++r) {
    comms[r] = nullptr;
    if (!ctxs[r]) return -EINVAL;
  }
  LoopGroup* grp = new (std::nothrow) LoopGroup;
  if (!grp) return -ENOMEM;
  grp->nranks = nranks;
  grp->post.resize(nranks);
  int rc = 0, joined = 0;  // joined: transports holding a reference to grp
  for (int r = 0; r < nranks && !rc; ++r) {
    DeviceGuard g(ctxs[r]->device);
    gdsm_comm* c = new (std::nothrow) gdsm_comm;
    LoopbackTransport* xp = new (std::nothrow) LoopbackTransport;
    if (!c || !xp) {
      delete c;
      delete xp;
      rc = -ENOMEM;
      break;
    }
    xp->g = grp;
    xp->rank = r;
    {
      std::lock_guard<std::mutex> lk(grp->mu);
      ++grp->refs;
    }
    ++joined;
    c->xp = xp;
    c->nranks = nranks;
    c->rank = r;
    c->device = ctxs[r]->device;
    comms[r] = c;
    if (comm_alloc(c) ||
        hipEventCreateWithFlags(&grp->post[r].ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&grp->post[r].done, hipEventDisableTiming) != hipSuccess)
      rc = -ENOMEM;
  }
  if (rc) {
    // the last transport's destructor deletes grp; with none joined nobody else will
    for (int r = 0; r < nranks; ++r)
      if (comms[r]) {
        gdsm_comm_fini(comms[r]);
        comms[r] = nullptr;
      }
    if (joined == 0) delete grp;
  }
  return rc;
}

int gdsm_comm_fini(gdsm_comm* c) {
  if (!c) return -EINVAL;
  DeviceGuard g(c->device);
  delete c->xp;
  if (c->cnt_dev) (void)hipFree(c->cnt_dev);
  if (c->cnt_host) (void)hipHostFree(c->cnt_host);
  if (c->verdict) (void)hipFree(c->verdict);
  if (c->ids_chk) (void)hipFree(c->ids_chk);
  if (c->rcnt_dev) (void)hipFree(c->rcnt_dev);
  if (c->rcnt_host) (void)hipHostFree(c->rcnt_host);
  for (uint8_t* p : {c->route_buf, c->pre, c->blk, c->blk_off, c->staging})
    if (p) (void)hipFree(p);
  delete c;
  return 0;
}

int gdsm_comm_size(const gdsm_comm* c, int* nranks, int* rank) {
  if (!c) return -EINVAL;
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  return 0;
}

int gdsm_comm_agree(gdsm_comm* c, gdsm_ctx* ctx, uint64_t* value) {
  if (!c || !ctx || !value || c->device != ctx->device) return -EINVAL;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  return c->xp->agree_max(value, ctx->stream);
}

int gdsm_exchange(gdsm_ctx* ctx, gdsm_comm* c, const gdsm_runs* send,
                  const uint32_t* const* send_ids, gdsm_runs* recv, uint32_t* const* recv_ids,
                  int target, uint32_t flags) {
  if (!ctx || !c || !send || !send_ids || !recv || !recv_ids) return -EINVAL;
  if (target < 0 || target > 2 || !ctx->arena[target] ||
      (flags & ~(GDSM_XCHG_FIXED | GDSM_XCHG_TIMED)))
    return -EINVAL;
  if (c->device != ctx->device) return -EINVAL;
  const int G = c->nranks, me = c->rank;
  const bool fixed = flags & GDSM_XCHG_FIXED;
  for (int d = 0; d < G; ++d) {
    if (send[d].n && (!send[d].rec_off || !send_ids[d] || (!send[d].data && send[d].cap)))
      return -EINVAL;
    if (d != me && (!recv[d].rec_off || (!recv[d].data && recv[d].cap))) return -EINVAL;
    if (d != me && !recv_ids[d] && (fixed ? recv[d].n : recv[d].n_cap)) return -EINVAL;
  }
  Transport* xp = c->xp;
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
    rc = xp->all_to_all_u64(c->cnt_dev, c->cnt_dev + 2 * G, 2, s);
    if (rc) return rc;
    GDSM_TRY(hipMemcpyAsync(h, c->cnt_dev, 32 * G, hipMemcpyDeviceToHost, s));
    GDSM_TRY(hipStreamSynchronize(s));
    uint64_t too_small = 0, sent_bytes = 0, sent_recs = 0;
    for (int d = 0; d < G; ++d) {
      sb[d] = h[2 * d + 1];
      sent_bytes += sb[d];
      sent_recs += send[d].n;
      too_small |= sb[d] > send[d].cap;  // that diff overflowed its stream (-ENOSPC)
      if (d == me) continue;
      rn[d] = h[2 * G + 2 * d];
      rb[d] = h[2 * G + 2 * d + 1];
      const uint64_t ncap = recv[d].n_cap ? recv[d].n_cap : recv[d].n;
      too_small |= rn[d] > ncap || rb[d] > recv[d].cap;
    }
    if (sent_recs / G > kDiffShortList) note_density(ctx, sent_bytes, sent_recs);
    // every rank must agree before anyone posts a send
    rc = xp->agree_max(&too_small, s);
    if (rc) return rc;
    if (too_small) return -ENOSPC;
  }

  // ---- move: one grouped point-to-point transfer per peer pair
  {
    gdsm::Prof* P = ctx->P();
    hipEvent_t w0 = P ? P->mark(s) : nullptr;  // this rank's streams are ready
    if (flags & GDSM_XCHG_TIMED) {
      // every rank's streams are ready once this one-word all-to-all completes (the exchange
      // counters are free here: exact mode read them back above)
      rc = xp->all_to_all_u64(c->cnt_dev, c->cnt_dev + G, 1, s);
      if (rc) {
        if (P) P->span(GDSM_PROF_EXCHANGE_WAIT, w0, nullptr);
        return rc;
      }
    }
    int rc2 = 0;
    {
      gdsm::ProfScope ps(P, GDSM_PROF_EXCHANGE, s);
      rc = xp->group_start();
      for (int p = 0; p < G && !rc; ++p) {
        if (p == me) continue;
        const uint64_t ns = send[p].n;
        rc = xp->send(send[p].rec_off, 8 * (ns + 1), p, s);
        if (!rc && ns) rc = xp->send(send_ids[p], 4 * ns, p, s);
        if (!rc && sb[p]) rc = xp->send(send[p].data, sb[p], p, s);
        if (!rc) rc = xp->recv(recv[p].rec_off, 8 * (rn[p] + 1), p, s);
        if (!rc && rn[p]) rc = xp->recv(recv_ids[p], 4 * rn[p], p, s);
        if (!rc && rb[p]) rc = xp->recv(recv[p].data, rb[p], p, s);
      }
      rc2 = xp->group_end(s);
    }
    if (P) P->span(GDSM_PROF_EXCHANGE_WAIT, w0, P->mark(s));
    if (rc || rc2) return rc ? rc : rc2;
  }
  for (int p = 0; p < G; ++p)
    if (p != me) recv[p].n = rn[p];
  if (fixed)  // the sender learns of its own over-budget streams too (the home rejects them)
    for (int p = 0; p < G; ++p)
      if (p != me && send[p].n)
        GDSM_TRY(gdsm::launch_budget_check(send[p].rec_off, send[p].n, send[p].cap, ctx->err, s));

  // ---- apply every source's stream to the home arena (own stream in place), each one checked
  // whole first; the checked index lists sit back to back in one scratch buffer
  uint64_t total = 0;
  for (int p = 0; p < G; ++p) total += p == me ? send[p].n : rn[p];
  uint8_t* buf = reinterpret_cast<uint8_t*>(c->ids_chk);
  rc = ensure(ctx, &buf, &c->ids_chk_bytes, 4 * (total ? total : 1));
  c->ids_chk = reinterpret_cast<uint32_t*>(buf);
  if (rc) return rc;
  uint64_t at = 0;
  for (int p = 0; p < G; ++p) {
    const gdsm_runs& in = p == me ? send[p] : recv[p];
    const uint64_t n = p == me ? send[p].n : rn[p];
    if (n == 0) continue;
    const uint64_t budget = p == me ? send[p].cap : rb[p];
    const uint32_t* ids = p == me ? send_ids[p] : recv_ids[p];
    uint32_t* chk = c->ids_chk + at;
    at += n;
    GDSM_TRY(gdsm::launch_xchg_guard(in.rec_off, ids, n, budget, ctx->n_pages, chk,
                                     c->verdict + p, ctx->err, s));
    GDSM_TRY(gdsm::launch_apply(ctx->arena[target], chk, n, in.rec_off, in.data, ctx->err, s,
                                ctx->P()));
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

// ---- coherence across GPUs (SPEC §5b) ----------------------------------------------------
// Both calls are collective: once the arguments are accepted, a rank's own failure (a workspace it
// cannot allocate, a launch error) is folded into the next agreement instead of being returned
// alone, so no peer is left waiting in a transfer. Every workspace is grown before the agreement
// that precedes its use.
namespace {
constexpr uint64_t kVerdictLocal = 4;  // some rank failed on its own (bits 0-1: the call's own)
inline int refused(int local) { return local ? local : -ECANCELED; }
}  // namespace

int gdsm_route_events(gdsm_ctx* ctx, gdsm_comm* c, const uint64_t* events, uint64_t n,
                      uint64_t total_pages, uint64_t* batch, uint64_t cap, uint64_t* n_batch) {
  if (!ctx || !c || !n_batch || (n && !events) || (cap && !batch)) return -EINVAL;
  if (c->device != ctx->device || c->nranks > (int)GDSM_MAX_NODES || total_pages == 0 ||
      total_pages > GDSM_MAX_COH_PAGES)
    return -EINVAL;
  const int G = c->nranks, me = c->rank;
  Transport* xp = c->xp;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  hipStream_t s = ctx->stream;
  const uint64_t per = (total_pages + G - 1) / G;
  const uint64_t base = (uint64_t)me * per < total_pages ? (uint64_t)me * per : total_pages;
  uint64_t* cnt = c->rcnt_dev;  // [0,G) sent, [G,2G) received, [2G,3G+1) bounds, [4G] flag
  uint32_t* flag = reinterpret_cast<uint32_t*>(cnt + 4 * G);
  int local = 0;
  {
    hipError_t e = hipMemsetAsync(flag, 0, 8, s);
    if (e == hipSuccess)
      e = gdsm::launch_route_split(events, n, total_pages, per, (uint32_t)G, cnt, cnt + 2 * G,
                                   flag, s);
    if (e != hipSuccess) {  // send nothing; the agreement below refuses everywhere
      local = map_err(e);
      (void)hipMemsetAsync(cnt, 0, 8 * (4 * (size_t)G + 1), s);
    }
  }
  int rc = xp->all_to_all_u64(cnt, cnt + G, 1, s);
  if (rc) return rc;
  uint64_t* h = c->rcnt_host;
  GDSM_TRY(hipMemcpyAsync(h, cnt, 8 * (4 * (size_t)G + 1), hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipStreamSynchronize(s));
  std::vector<uint64_t> off(G + 1, 0);
  for (int p = 0; p < G; ++p) off[p + 1] = off[p] + h[G + p];
  const bool fits = off[G] <= cap;
  if (!local && fits) local = ensure(ctx, &c->route_buf, &c->route_bytes, 8 * (off[G] ? off[G] : 1));
  // every rank agrees before anything moves: 4 = some rank failed, 2 = some node's events are
  // invalid, 1 = some home's batch buffer is too small
  uint64_t verdict = (local ? kVerdictLocal : 0u) |
                     ((reinterpret_cast<uint32_t*>(h + 4 * G)[0] & 1u) ? 2u : 0u) | (fits ? 0u : 1u);
  rc = xp->agree_max(&verdict, s);
  if (rc) return rc;
  if (verdict & kVerdictLocal) return refused(local);
  if (verdict & 2) return -EINVAL;
  if (verdict & 1) return -ENOSPC;
  uint64_t* runs = reinterpret_cast<uint64_t*>(c->route_buf);
  {
    gdsm::ProfScope ps(ctx->P(), GDSM_PROF_ROUTE, s);
    rc = xp->group_start();
    for (int p = 0; p < G && !rc; ++p) {
      if (p == me) continue;
      if (h[p]) rc = xp->send(events + h[2 * G + p], 8 * h[p], p, s);
      if (!rc && h[G + p]) rc = xp->recv(runs + off[p], 8 * h[G + p], p, s);
    }
    const int rc2 = xp->group_end(s);
    if (rc || rc2) return rc ? rc : rc2;
  }
  if (h[me])
    GDSM_TRY(hipMemcpyAsync(runs + off[me], events + h[2 * G + me], 8 * h[me],
                            hipMemcpyDeviceToDevice, s));
  GDSM_TRY(gdsm::launch_route_merge(runs, off.data(), (uint32_t)G, base, batch, s));
  *n_batch = off[G];
  return 0;
}

int gdsm_coherence_notify(gdsm_ctx* ctx, gdsm_comm* c, const uint64_t* batch, uint64_t n,
                          uint64_t base, uint64_t* totals_dev, uint64_t* notices, uint64_t cap,
                          uint64_t* n_notices) {
  if (!ctx || !c || !ctx->coh_pt || !totals_dev || !n_notices || (n && !batch) ||
      (cap && !notices))
    return -EINVAL;
  if (c->device != ctx->device || c->nranks > (int)GDSM_MAX_NODES) return -EINVAL;
  const int G = c->nranks, me = c->rank;
  Transport* xp = c->xp;
  CtxGuard g(ctx);
  if (g.rc) return g.rc;
  hipStream_t s = ctx->stream;
  const uint64_t nb = gdsm::notice_blocks(n);
  uint32_t* pre = nullptr;
  uint64_t* cnt = c->rcnt_dev;  // [0,G) notices per node, [G,2G) received, [2G,3G) bases
  uint64_t* h = c->rcnt_host;
  // every workspace of the call, the fold's included, before the first agreement
  int local = ensure(ctx, &c->pre, &c->pre_bytes, 4 * (n ? n : 1));
  if (!local) local = ensure(ctx, &c->blk, &c->blk_bytes, 4 * GDSM_MAX_NODES * (nb ? nb : 1));
  if (!local)
    local = ensure(ctx, &c->blk_off, &c->blk_off_bytes, 8 * GDSM_MAX_NODES * (nb ? nb : 1));
  if (!local) local = ensure(ctx, &ctx->coh_ws, &ctx->coh_ws_bytes, gdsm::coh_workspace_bytes(n));
  pre = reinterpret_cast<uint32_t*>(c->pre);
  // capacity first, before the page table changes: a node gets at most one notice per page that
  // any home's batch touches, so every node needs cap >= the sum of the homes' distinct pages
  if (!local) {
    const hipError_t e = gdsm::launch_notice_pre(ctx->coh_pt, ctx->n_pages, batch, n, pre,
                                                 cnt + 4 * G, s);
    if (e != hipSuccess) local = map_err(e);
  }
  GDSM_TRY(hipMemcpyAsync(h + 4 * G, cnt + 4 * G, 8, hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipMemcpyAsync(h + 4 * G + 1, ctx->err, 4, hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipStreamSynchronize(s));
  const uint64_t distinct = local ? 0 : h[4 * G];
  // an error bit an earlier batch left: only this fold's rejection may refuse the call, so the bit
  // moves to the host-held word, which gdsm_sync reports whatever way this call ends
  const uint32_t stale = reinterpret_cast<uint32_t*>(h + 4 * G + 1)[0] & gdsm::detail::kErrEvents;
  if (stale) {
    ctx->err_held |= stale;
    reinterpret_cast<uint32_t*>(h + 4 * G + 1)[0] &= ~stale;
    GDSM_TRY(hipMemcpyAsync(ctx->err, h + 4 * G + 1, 4, hipMemcpyHostToDevice, s));
  }
  for (int p = 0; p < G; ++p) h[p] = distinct;
  GDSM_TRY(hipMemcpyAsync(cnt, h, 8 * (size_t)G, hipMemcpyHostToDevice, s));
  int rc = xp->all_to_all_u64(cnt, cnt + G, 1, s);
  if (rc) return rc;
  GDSM_TRY(hipMemcpyAsync(h + G, cnt + G, 8 * (size_t)G, hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipStreamSynchronize(s));
  uint64_t bound = 0;
  for (int p = 0; p < G; ++p) bound += h[G + p];
  // this home sends at most one notice per (distinct page of its batch, node): the staging is
  // sized for that worst case (G notices of 8 B per distinct page) before the agreement, since
  // the real count is known only after the fold; it only grows
  if (!local) local = ensure(ctx, &c->staging, &c->staging_bytes, 8 * G * (distinct ? distinct : 1));
  uint64_t verdict = (local ? kVerdictLocal : 0u) | (bound > cap ? 1u : 0u);
  rc = xp->agree_max(&verdict, s);
  if (rc) return rc;
  if (verdict & kVerdictLocal) return refused(local);
  if (verdict & 1) return -ENOSPC;
  // from here a failure leaves the page tables unspecified (as a rejected batch does)
  local = gdsm_coherence_batch_async(ctx, batch, n, totals_dev);
  uint32_t* blk = reinterpret_cast<uint32_t*>(c->blk);
  uint64_t* blk_off = reinterpret_cast<uint64_t*>(c->blk_off);
  if (!local) {
    const hipError_t e = gdsm::launch_notice_count(ctx->coh_pt, ctx->n_pages, batch, n, pre,
                                                   (uint32_t)G, blk, blk_off, cnt, cnt + 2 * G, s);
    if (e != hipSuccess) local = map_err(e);
  }
  if (local) GDSM_TRY(hipMemsetAsync(cnt, 0, 8 * 3 * (size_t)G, s));
  rc = xp->all_to_all_u64(cnt, cnt + G, 1, s);
  if (rc) return rc;
  GDSM_TRY(hipMemcpyAsync(h, cnt, 8 * 3 * (size_t)G, hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipMemcpyAsync(h + 4 * G, ctx->err, 4, hipMemcpyDeviceToHost, s));
  GDSM_TRY(hipStreamSynchronize(s));
  const uint32_t err_now = reinterpret_cast<uint32_t*>(h + 4 * G)[0];
  std::vector<uint64_t> off(G + 1, 0);
  uint64_t sent = 0;
  for (int p = 0; p < G; ++p) {
    off[p + 1] = off[p] + h[G + p];
    sent += h[p];
  }
  // some home's batch was rejected by this fold (its page table is unspecified): all refuse
  verdict = (local ? kVerdictLocal : 0u) | ((err_now & gdsm::detail::kErrEvents) ? 1u : 0u) |
            (off[G] > cap || sent > (uint64_t)G * (distinct ? distinct : 1) ? 1u : 0u);
  rc = xp->agree_max(&verdict, s);
  if (rc) return rc;
  if (verdict & kVerdictLocal) return refused(local);
  if (verdict) return -EINVAL;
  uint64_t* stg = reinterpret_cast<uint64_t*>(c->staging);
  GDSM_TRY(gdsm::launch_notice_emit(ctx->coh_pt, ctx->n_pages, batch, n, pre, (uint32_t)G, base,
                                    blk_off, cnt + 2 * G, stg, s));
  {
    gdsm::ProfScope ps(ctx->P(), GDSM_PROF_ROUTE, s);
    rc = xp->group_start();
    for (int p = 0; p < G && !rc; ++p) {
      if (p == me) continue;
      if (h[p]) rc = xp->send(stg + h[2 * G + p], 8 * h[p], p, s);
      if (!rc && h[G + p]) rc = xp->recv(notices + off[p], 8 * h[G + p], p, s);
    }
    const int rc2 = xp->group_end(s);
    if (rc || rc2) return rc ? rc : rc2;
  }
  if (h[me])
    GDSM_TRY(hipMemcpyAsync(notices + off[me], stg + h[2 * G + me], 8 * h[me],
                            hipMemcpyDeviceToDevice, s));
  *n_notices = off[G];
  return 0;
}

}  // extern "C"
