"""Diff propagation between page shards: one process per GPU, the records of every release
shipped to their home GPU over RCCL (xGMI) by libgdsm's `gdsm_exchange` (C ABI, include/gdsm.h).

The reference sends its (unimplemented) page updates over HTTP with a per-peer std::async
fan-out (gallocy/http/client.cpp:39-91, gallocy/consensus/client.cpp:15-42).

Layout (G ranks, N pages in all, n = N / G homed per rank):
  home(p)   = p // n                 (contiguous page blocks; REPLICA index p - home·n)
  writer(p) = p mod G                (rank r writes pages r, r+G, r+2G, ...: TWIN/CURRENT arena
                                      index i holds global page i·G + r)
A writer's pages for home d are the arena indices [bounds[d], bounds[d+1]) (dest_bounds), which
it diffs into its own stream send[d]; each record travels with its page's REPLICA index at the
home (send_ids). Protocol per release (gdsm_exchange; `GlooTransport` restates it for CPU tests):
  1. sizes: (records, bytes) per destination, all-to-all (or fixed by the caller: no host sync);
  2. per peer pair: rec_off, ids, data;
  3. the home applies every source's stream to its REPLICA (its own stream in place).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import threading
import time
from errno import EIO, EOVERFLOW

import numpy as np

from . import gdsm
from ._lib import GdsmRuns, check

XCHG_FIXED = 1
XCHG_TIMED = 2  # a device barrier before each transfer: the exchange stage times the link alone


def dest_bounds(rank: int, world: int, n: int) -> list[int]:
    """Writer-local arena index ranges per destination: [bounds[d], bounds[d+1])."""
    b = []
    for d in range(world + 1):
        # smallest i with i*G + rank >= d*n
        b.append(max(0, min(n, -(-(d * n - rank) // world))))
    return b


def send_ids(rank: int, world: int, n: int) -> list[np.ndarray]:
    """Per destination d: the REPLICA index at rank d of each page rank `rank` sends there."""
    b = dest_bounds(rank, world, n)
    return [(np.arange(b[d], b[d + 1], dtype=np.int64) * world + rank - d * n).astype(np.uint32)
            for d in range(world)]


def budget(nbytes: int) -> int:
    """Fixed-size exchange byte budget for a stream of `nbytes` (same formula on both sides)."""
    return ((nbytes + nbytes // 32 + 4096) + 255) // 256 * 256


# ---------------------------------------------------------------- CPU restatement (tests)
class GlooTransport:
    """The gdsm_exchange protocol restated over torch.distributed (gloo, CPU tensors): the
    checker for multi-rank runs without GPUs (tests/test_exchange.py) and the transport of the
    one-GPU multi-rank rehearsal (several ranks cannot share a GPU under RCCL)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group

    def exchange(self, send: list) -> list:
        """send[d] = (rec_off uint64[n+1], ids uint32[n], data uint8[>= rec_off[n]]) for every
        destination d. Returns recv[s] = (rec_off, ids, data) as rank s sent them (recv[rank] is
        send[rank] itself)."""
        import torch
        dist, g = self.dist, self.group
        world, me = dist.get_world_size(g), dist.get_rank(g)
        sizes = torch.tensor([[len(s[1]), int(s[0][-1])] for s in send], dtype=torch.int64)
        got = torch.empty_like(sizes)
        dist.all_to_all_single(got, sizes, group=g)                     # 1. sizes
        rn, rb = got[:, 0].tolist(), got[:, 1].tolist()

        def a2a(parts, recv_lens, dtype):
            inp = torch.from_numpy(np.concatenate(parts).astype(dtype, copy=False))
            out = torch.empty(sum(recv_lens), dtype=inp.dtype)
            dist.all_to_all_single(out, inp, output_split_sizes=recv_lens,
                                   input_split_sizes=[len(p) for p in parts], group=g)
            return torch.split(out, recv_lens)
        ro = a2a([s[0].astype(np.int64) for s in send], [x + 1 for x in rn], np.int64)  # 2.
        ids = a2a([s[1].astype(np.int32) for s in send], rn, np.int32)
        data = a2a([np.asarray(s[2][:int(s[0][-1])], np.uint8) for s in send], rb, np.uint8)
        out = []
        for s in range(world):
            if s == me:
                out.append(send[s])
            else:
                out.append((ro[s].numpy().astype(np.uint64), ids[s].numpy().astype(np.uint32),
                            data[s].numpy()))
        return out


# ---------------------------------------------------------------- deadlines
class Watchdog:
    """Ends the process when a phase of a multi-rank run overruns its deadline: a peer that died
    or hangs leaves the others blocked inside a collective (ncclCommInitRank, an RCCL group, a
    gloo barrier) with no error to return, so the launcher would only ever see a timeout. A
    daemon thread prints which phase overran to stderr and calls os._exit(code): the process
    ends non-zero, and torch.distributed.run then stops the other ranks. Nothing is re-executed
    (a process that has touched the GPU must never exec).

    arm(seconds, what) (re)starts the clock for a phase; disarm() stops it. GDSM_DEADLINE_S
    overrides the seconds of every phase (0 = off)."""

    def __init__(self, rank: int = 0, code: int = 3):
        self.rank, self.code = rank, code
        self._cv = threading.Condition()
        self._due = None
        self._what = ""
        self._thread = None

    def arm(self, seconds: float, what: str):
        env = os.environ.get("GDSM_DEADLINE_S")
        if env is not None:
            seconds = float(env)
        with self._cv:
            self._due = time.monotonic() + seconds if seconds > 0 else None
            self._what = what
            if self._thread is None and self._due is not None:
                self._thread = threading.Thread(target=self._watch, name="gdsm-watchdog",
                                                daemon=True)
                self._thread.start()
            self._cv.notify_all()
        return self

    def disarm(self):
        with self._cv:
            self._due = None
            self._cv.notify_all()

    def _watch(self):
        with self._cv:
            while True:
                if self._due is None:
                    self._cv.wait()
                    continue
                left = self._due - time.monotonic()
                if left > 0:
                    self._cv.wait(left)
                    continue
                msg = (f"gdsm: rank {self.rank}: deadline passed in '{self._what}' (a peer "
                       f"died or hangs); exiting with status {self.code}")
                print(msg, file=sys.stderr, flush=True)
                os._exit(self.code)


# ---------------------------------------------------------------- the GPU shard
class Comm:
    """A communicator owned by libgdsm (gdsm_comm_*). RCCL (the product transport): bootstrapped
    with a torch.distributed group (any backend) that carries the 128-byte unique id. Loopback
    (`Comm.loopback`, tests): several ranks as threads of one process on one GPU."""

    def __init__(self, ctx: gdsm.Context, rank: int, world: int, group=None, handle=None,
                 deadline_s: float = 0):
        """deadline_s > 0: the unique-id broadcast and gdsm_comm_init (ncclCommInitRank, which
        blocks until every rank joins) must finish within it, else the process exits non-zero
        (Watchdog)."""
        self.rank, self.world = rank, world
        if handle is not None:
            self.handle = handle
            return
        wd = Watchdog(rank).arm(deadline_s, "communicator setup") if deadline_s > 0 else None
        try:
            self._init(ctx, rank, world, group)
        finally:
            if wd is not None:
                wd.disarm()

    def _init(self, ctx, rank, world, group):
        import torch
        import torch.distributed as dist
        L = gdsm.lib()
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            check(L.gdsm_comm_unique_id(uid), "gdsm_comm_unique_id")
        t = torch.tensor(list(uid), dtype=torch.uint8)
        if world > 1:
            obj = [bytes(t.tolist())]
            dist.broadcast_object_list(obj, src=0, group=group)
            uid = (C.c_uint8 * 128)(*obj[0])
        h = C.c_void_p()
        check(L.gdsm_comm_init(C.byref(h), ctx.handle, world, rank, uid), "gdsm_comm_init")
        self.handle = h.value

    @classmethod
    def loopback(cls, ctxs: list) -> list:
        """gdsm_comm_init_loopback: one communicator per context, rank r bound to ctxs[r]; each
        must then be driven by its own thread (every collective blocks until all ranks call it)."""
        G = len(ctxs)
        hs = (C.c_void_p * G)()
        cs = (C.c_void_p * G)(*[c.handle for c in ctxs])
        check(gdsm.lib().gdsm_comm_init_loopback(hs, cs, G), "gdsm_comm_init_loopback")
        return [cls(ctxs[r], r, G, handle=hs[r]) for r in range(G)]

    def size(self) -> tuple[int, int]:
        """gdsm_comm_size: (ranks, this rank) as the communicator itself reports them."""
        nr, me = C.c_int(0), C.c_int(-1)
        check(gdsm.lib().gdsm_comm_size(self.handle, C.byref(nr), C.byref(me)), "gdsm_comm_size")
        return nr.value, me.value

    def agree(self, ctx: gdsm.Context, value: int) -> int:
        """gdsm_comm_agree: the maximum of every rank's value (collective, synchronous)."""
        v = C.c_uint64(value)
        check(gdsm.lib().gdsm_comm_agree(self.handle, ctx.handle, C.byref(v)), "gdsm_comm_agree")
        return v.value

    def close(self):
        if self.handle:
            gdsm.lib().gdsm_comm_fini(self.handle)
            self.handle = None


def exchange_runs(ctx: gdsm.Context, comm: Comm, send: list, send_ids: list, recv: list,
                  recv_ids: list, flags: int = 0, target=gdsm.REPLICA):
    """gdsm_exchange over lists of G Runs / device id pointers; updates recv[s].n."""
    G = comm.world
    s_arr = (GdsmRuns * G)(*[r.s for r in send])
    r_arr = (GdsmRuns * G)(*[r.s for r in recv])
    sid = (C.c_void_p * G)(*send_ids)
    rid = (C.c_void_p * G)(*recv_ids)
    check(gdsm.lib().gdsm_exchange(ctx.handle, comm.handle, s_arr, sid, r_arr, rid, target, flags),
          "gdsm_exchange")
    for s in range(G):
        recv[s].s.n = r_arr[s].n


def exchange_gloo(ctx: gdsm.Context, gloo: GlooTransport, send: list, send_ids: list,
                  counts: list, rank: int):
    """The same release over GlooTransport with host staging (one-GPU multi-rank rehearsal):
    every source's stream is applied to ctx's REPLICA. Returns (sent_remote, received) bytes."""
    parts = []
    for d, r in enumerate(send):
        if counts[d]:
            h = r.to_host()
            ids = send_ids[d].download(np.uint32, counts[d])
        else:
            h = gdsm.HostRuns(np.zeros(1, np.uint64), np.zeros(0, np.uint8))
            ids = np.zeros(0, np.uint32)
        parts.append((h.rec_off, ids, h.data))
    got = gloo.exchange(parts)
    for ro, ids, data in got:
        if len(ids) == 0:
            continue
        runs = gdsm.Runs.from_host(ctx, gdsm.HostRuns(ro, data))
        d_ids = ctx.ids(ids)
        ctx.apply(runs, "replica", d_ids)
        ctx.sync()
        runs.free()
        d_ids.free()
    sent_remote = sum(int(p[0][-1]) for d, p in enumerate(parts) if d != rank)
    return sent_remote, sum(int(g[0][-1]) for g in got)


class Shard:
    """One rank's release pipeline: per-destination diffs -> exchange -> apply at the homes.

    `n` arena pages per rank (TWIN/CURRENT: the pages this rank writes; REPLICA: its home block).
    Two sets of per-destination send streams alternate, so diff k+1 (main stream) overlaps the
    exchange and home-side apply of release k (the context's second stream); a diff into set b
    waits on the device for the exchange that last read it (libgdsm orders that itself).

    transport "rccl": gdsm_exchange (RCCL inside libgdsm). After `calibrate()`, releases use
    GDSM_XCHG_FIXED byte budgets: no host synchronisation at all per release. A release whose
    stream outgrew its budget is rejected whole at the home (and reported on both ends as
    -EOVERFLOW); `drain()` has the ranks agree on it (gdsm_comm_agree) and redoes the release with
    exact sizes, then re-calibrates. The twin is never refreshed inside the Shard, so one exact
    release of the current state restores every home.
    transport "loopback": the same calls through a `Comm.loopback` communicator (`comm=`): ranks
    are threads of one process on one GPU (tests of the multi-rank C++ path).
    transport "gloo": the GlooTransport restatement with host staging (rehearsal of several ranks
    on one GPU as processes); not a measurement."""

    def __init__(self, ctx: gdsm.Context, rank: int, world: int, n: int, cap_per_page: int,
                 transport: str = "rccl", group=None, sets: int = 2, comm: "Comm" = None):
        if n % world:
            raise ValueError("pages per rank must be a multiple of the rank count")
        self.ctx, self.rank, self.world, self.n = ctx, rank, world, n
        self.L = gdsm.lib()
        self.bounds = dest_bounds(rank, world, n)
        self.counts = [self.bounds[d + 1] - self.bounds[d] for d in range(world)]
        self.iota = ctx.ids(np.arange(n, dtype=np.uint32))             # arena index lists
        self.sids = [ctx.ids(x) for x in send_ids(rank, world, n)]    # REPLICA index at home
        self.send = [[gdsm.Runs(ctx, max(1, c), cap=max(4096, c * cap_per_page))
                      for c in self.counts] for _ in range(sets)]
        for st in self.send:
            for d, r in enumerate(st):
                r.s.n = self.counts[d]
        rmax = max(self.counts) + 1  # records from any source: n/G or n/G + 1
        # receive streams per source (the own stream is applied in place: a stub)
        self.recv = [gdsm.Runs(ctx, rmax, cap=max(4096, rmax * cap_per_page)) if s != rank
                     else gdsm.Runs(ctx, 1, cap=16) for s in range(world)]
        self.rids = [ctx.buffer(4 * rmax if s != rank else 4) for s in range(world)]
        self.transport = transport
        if transport == "loopback" and comm is None:
            raise ValueError("transport loopback needs comm= (Comm.loopback)")
        self.comm = comm if comm is not None else (
            Comm(ctx, rank, world, group) if transport == "rccl" else None)
        self.own_comm = comm is None
        self.gloo = GlooTransport(group) if transport == "gloo" else None
        self.flags = 0
        self.sent_remote = self.received = self.moved_remote = 0
        self.k = 0
        self.recoveries = 0

    # -- one release
    def diff(self, k: int):
        """The release's per-destination streams: one launch for all of them (gdsm_diff_split;
        one launch per destination cost 9 % more at 8 GPUs' shard shape, scripts/dev/split_diff.py)."""
        st = self.send[k % len(self.send)]
        if self.world <= 8:
            self.ctx.diff_split(self.bounds, st)
            return
        for d in range(self.world):
            c = self.counts[d]
            if c:
                self.ctx.diff(self.iota.ptr + 4 * self.bounds[d], n=c, out=st[d])

    def exchange(self, k: int):
        st = self.send[k % len(self.send)]
        if self.comm is not None:
            exchange_runs(self.ctx, self.comm, st, [b.ptr for b in self.sids], self.recv,
                          [b.ptr for b in self.rids], self.flags)
        else:
            self._exchange_gloo(st)

    def _exchange_gloo(self, st):
        self.sent_remote, self.received = exchange_gloo(self.ctx, self.gloo, st, self.sids,
                                                        self.counts, self.rank)

    def step(self, k: int):
        self.diff(k)
        self.exchange(k)

    def run(self, steps: int, pipelined: bool = True):
        """`steps` releases, enqueued in order diff k -> exchange k -> diff k+1 -> ... Pipelined:
        the two send sets alternate, so diff k+1 (main stream) runs while exchange + home-side
        apply k run on the second stream (gdsm_exchange waits only for what the main stream
        holds when it is called: diff k). Serial: one send set, so diff k+1 waits on the device
        for the exchange that read it. Neither synchronises the host (RCCL transport)."""
        for k in range(steps):
            j = self.k + k if pipelined else 0
            self.diff(j)
            self.exchange(j)
            if self.comm is None:
                self.ctx.sync()
        self.k += steps

    def calibrate(self):
        """After an exact-size release: fixes every stream's byte budget (budget()) on both
        sides so later releases exchange with GDSM_XCHG_FIXED (no host synchronisation)."""
        self.ctx.sync()
        sent = [r.total() if self.counts[d] else 0 for d, r in enumerate(self.send[0])]
        for st in self.send:
            for d, r in enumerate(st):
                r.s.cap = min(r.cap_alloc, budget(sent[d]))
        recvd = []
        for s, r in enumerate(self.recv):
            if s == self.rank:
                recvd.append(0)
                continue
            t = np.empty(1, np.uint64)
            check(self.L.gdsm_memcpy_d2h(self.ctx.handle, t.ctypes.data, r.s.rec_off + 8 * r.s.n,
                                         8), "d2h")
            recvd.append(int(t[0]))
            r.s.cap = min(r.cap_alloc, budget(int(t[0])))
        self.sent_remote = sum(b for d, b in enumerate(sent) if d != self.rank)
        self.received = sum(recvd) + sent[self.rank]
        # what the transport carries to the peers per fixed-budget release
        self.moved_remote = sum(8 * (c + 1) + 4 * c + self.send[0][d].s.cap
                                for d, c in enumerate(self.counts) if d != self.rank)
        self.flags = XCHG_FIXED

    def drain(self):
        """Waits for both streams. With a communicator the ranks then agree on the outcome
        (gdsm_comm_agree: 0 ok, 1 some fixed-budget stream overflowed, 2 anything else): on 1
        every rank redoes the release with exact sizes and re-calibrates (`recoveries` counts
        them); on 2 every rank raises."""
        rc = self.L.gdsm_sync(self.ctx.handle)
        if self.comm is None:
            check(rc, "gdsm_sync")
            return
        verdict = 0 if rc == 0 else (1 if rc == -EOVERFLOW else 2)
        agreed = self.comm.agree(self.ctx, verdict)
        if agreed >= 2:
            check(rc if rc else -EIO, "gdsm_sync (a rank failed its release)")
        if agreed == 1:
            self.recover()

    def recover(self):
        """Redoes the release with exact sizes (TWIN vs CURRENT is unchanged, so the streams
        carry everything the rejected fixed-budget releases did; the apply is idempotent), then
        fixes new budgets."""
        self.flags = 0
        for r in [x for st in self.send for x in st] + self.recv:
            r.s.cap = r.cap_alloc  # budgets off: the whole allocation again
        self.diff(0)
        self.exchange(0)
        check(self.L.gdsm_sync(self.ctx.handle), "gdsm_sync (recovery release)")
        self.calibrate()
        self.recoveries += 1

    def verify(self, seed: int, mode: int, ppm: int) -> bool:
        """REPLICA (home block) == CURRENT content of those pages, generated independently."""
        n, L = self.n, self.L
        scratch = self.ctx.buffer(n * 4096)
        if L.gdsm_gen_pages_raw(None, scratch.ptr, None, n, self.rank * n, 1, seed, mode, ppm,
                                self.ctx.stream):
            return False
        chk = gdsm.Runs(self.ctx, n, cap=1 << 20)
        ws = self.ctx.buffer(L.gdsm_diff_workspace_bytes(n))
        rc = L.gdsm_diff_raw(self.ctx.arena_ptr("replica"), scratch.ptr, None, n, chk.s.rec_off,
                             chk.s.data, chk.cap, ws.ptr, ws.nbytes, self.ctx.stream)
        ok = rc == 0 and chk.total() == 0
        for x in (scratch, ws):
            x.free()
        chk.free()
        return ok

    def close(self):
        if self.comm is not None and self.own_comm:
            self.comm.close()


# ---------------------------------------------------------------- coherence across GPUs
def route_events(ctx: gdsm.Context, comm: Comm, events: int, n: int, total_pages: int,
                 batch: int, cap: int) -> int:
    """gdsm_route_events (SPEC §5b): this node's n stamped events (device pointer) to their
    homes; returns how many events of this rank's home block land in `batch` (device, cap)."""
    nb = C.c_uint64(0)
    check(gdsm.lib().gdsm_route_events(ctx.handle, comm.handle, events, n, total_pages, batch,
                                       cap, C.byref(nb)), "gdsm_route_events")
    return nb.value


def coherence_notify(ctx: gdsm.Context, comm: Comm, batch: int, n: int, base: int, totals: int,
                     notices: int, cap: int) -> int:
    """gdsm_coherence_notify (SPEC §5b): fold this home's batch into ctx's page-table shard and
    exchange the notices; returns how many notices for this node land in `notices`."""
    nn = C.c_uint64(0)
    check(gdsm.lib().gdsm_coherence_notify(ctx.handle, comm.handle, batch, n, base, totals,
                                           notices, cap, C.byref(nn)), "gdsm_coherence_notify")
    return nn.value
