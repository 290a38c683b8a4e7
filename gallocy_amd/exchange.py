"""Diff propagation between page shards: one process per GPU, RCCL all-to-all over xGMI.

The reference sends its (unimplemented) page updates over HTTP with a per-peer std::async
fan-out (gallocy/http/client.cpp:39-91, gallocy/consensus/client.cpp:15-42); here the records a
shard produces for pages whose home is another rank travel in one all-to-all per step.

Layout (SURVEY §8e, config 3 shape, weak scaling): G ranks, n pages homed per rank, N = G·n.
  home(p)   = p // n                 (contiguous page blocks, REPLICA arena index p - home·n)
  writer(p) = p mod G                (rank r writes pages r, r+G, r+2G, ...: TWIN/CURRENT arena
                                      index i holds global page i·G + r)
A writer's page list is increasing in p, so its records for one home are one contiguous slice
of its canonical diff stream (docs/SPEC.md §3); rank d receives from every source s the n/G
records of pages p ≡ s (mod G) of its block, in increasing p, i.e. REPLICA indices s, s+G, ...

`exchange_stream` is device-agnostic (CUDA tensors over RCCL, or CPU tensors over gloo in the
tests); `Shard` wires it to a gdsm Context on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist


def dest_bounds(rank: int, world: int, n: int) -> list[int]:
    """Writer-local record index ranges per destination: [bounds[d], bounds[d+1])."""
    b = []
    for d in range(world + 1):
        # smallest i with i*G + rank >= d*n
        b.append(max(0, min(n, -(-(d * n - rank) // world))))
    return b


def recv_ids(world: int, n: int) -> np.ndarray:
    """REPLICA indices of the received records, in (source, page) order."""
    return np.concatenate([np.arange(s, n, world, dtype=np.uint32) for s in range(world)])


def exchange_stream(rec_off: torch.Tensor, data: torch.Tensor, bounds: list[int], world: int,
                    group=None):
    """All-to-all of a canonical diff stream split by destination.

    rec_off: int64[n+1] (the stream's offsets), data: uint8[>= rec_off[n]]. Returns the received
    (rec_off int64[m+1], data uint8[rec_off[m]]) with the sources' records concatenated in rank
    order. Two small collectives (byte counts, record sizes) and one payload all-to-all."""
    dev = rec_off.device
    bt = torch.tensor(bounds, dtype=torch.int64, device=dev)
    edges = rec_off.index_select(0, bt)
    send_bytes = (edges[1:] - edges[:-1]).contiguous()
    recv_bytes = torch.empty_like(send_bytes)
    dist.all_to_all_single(recv_bytes, send_bytes, group=group)
    sizes = (rec_off[1:] - rec_off[:-1]).to(torch.int32)
    send_recs = [bounds[d + 1] - bounds[d] for d in range(world)]
    recv_recs_t = torch.tensor(send_recs, dtype=torch.int64, device=dev)
    recv_recs_o = torch.empty_like(recv_recs_t)
    dist.all_to_all_single(recv_recs_o, recv_recs_t, group=group)
    counts = torch.stack([send_bytes, recv_bytes, recv_recs_o]).cpu().tolist()  # one host sync
    sb, rb, rr = counts
    recv_sizes = torch.empty(sum(rr), dtype=torch.int32, device=dev)
    dist.all_to_all_single(recv_sizes, sizes, output_split_sizes=rr, input_split_sizes=send_recs,
                           group=group)
    total_in = int(sum(sb))
    recv_data = torch.empty(max(1, sum(rb)), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv_data[:sum(rb)], data[:total_in], output_split_sizes=rb,
                           input_split_sizes=sb, group=group)
    out_off = torch.zeros(len(recv_sizes) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(recv_sizes.to(torch.int64), 0, out=out_off[1:])
    return out_off, recv_data, int(sum(sb) - sb[dist.get_rank(group)]), int(sum(rb))


class Shard:
    """One rank's release pipeline: diff -> exchange -> apply to REPLICA.

    The diff runs on the context's stream, the exchange (RCCL) and the apply of the received
    records on a second stream, with the diff stream double-buffered: diff k+1 is enqueued
    before exchange k, so the all-to-all and the home-side apply of step k overlap the diff of
    step k+1 (the only host synchronisation, the byte counts of exchange k, then waits for
    diff k alone). Buffer b is reused by diff k+2 only after exchange k has read it."""

    def __init__(self, ctx, runs, rank: int, world: int, n: int):
        from . import gdsm
        if n % world:
            raise ValueError("pages per rank must be a multiple of the rank count")
        runs = list(runs) if isinstance(runs, (list, tuple)) else [runs]
        self.ctx, self.runs, self.rank, self.world, self.n = ctx, runs, rank, world, n
        self.lib = gdsm.lib()
        dev = torch.device("cuda", torch.cuda.current_device())
        self.stream = torch.cuda.ExternalStream(ctx.stream, device=dev)   # diff
        self.comm = torch.cuda.Stream(device=dev)                          # exchange + apply
        self.bounds = dest_bounds(rank, world, n)
        # Tensors aliasing the diff streams that libgdsm writes (device memory owned by ctx).
        self.views = [(_tensor_at(r.s.rec_off, (n + 1,), torch.int64, dev),
                       _tensor_at(r.s.data, (r.cap,), torch.uint8, dev)) for r in runs]
        self.ready = [torch.cuda.Event() for _ in runs]      # diff into buffer b done
        self.consumed = [None for _ in runs]                  # exchange of buffer b done
        with torch.cuda.stream(self.comm):
            self.recv_ids = torch.from_numpy(recv_ids(world, n)).to(dev)
            self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.sent_remote = 0
        self.received = 0

    def _diff(self, k: int):
        b = k % len(self.runs)
        if self.consumed[b] is not None:
            self.stream.wait_event(self.consumed[b])
        self.ctx.diff(out=self.runs[b])
        self.ready[b].record(self.stream)

    def _exchange_apply(self, k: int):
        b = k % len(self.runs)
        rec_off, data = self.views[b]
        self.comm.wait_event(self.ready[b])
        with torch.cuda.stream(self.comm):
            off, rdata, sent_remote, received = exchange_stream(rec_off, data, self.bounds,
                                                               self.world)
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self.consumed[b] = ev
            rc = self.lib.gdsm_apply_raw(self.ctx.arena_ptr("replica"), self.recv_ids.data_ptr(),
                                         self.n, off.data_ptr(), rdata.data_ptr(),
                                         self.err.data_ptr(), self.comm.cuda_stream)
            if rc:
                raise RuntimeError(f"gdsm_apply_raw: {rc}")
        self.sent_remote, self.received = sent_remote, received

    def run(self, steps: int):
        """`steps` releases, pipelined as described above; returns with work still in flight."""
        if steps <= 0:
            return
        self._diff(0)
        for k in range(steps):
            if k + 1 < steps:
                self._diff(k + 1)
            self._exchange_apply(k)

    def exchange_and_apply(self):
        """One unpipelined step (the diff already enqueued on the context stream)."""
        self.ready[0].record(self.stream)
        self._exchange_apply(0)

    def drain(self):
        """Waits for both streams; raises if an apply found a malformed record."""
        self.comm.synchronize()
        self.stream.synchronize()
        if int(self.err.item()) != 0:
            raise RuntimeError("apply: malformed record in the received stream")

    def verify(self) -> bool:
        """REPLICA (home block) == CURRENT content of those pages, generated independently."""
        from . import gdsm
        n = self.n
        scratch = self.ctx.buffer(n * 4096)
        seedinfo = getattr(self, "gen_args", None)
        if seedinfo is None:
            return False
        seed, mode, ppm = seedinfo
        L = self.lib
        if L.gdsm_gen_pages_raw(None, scratch.ptr, None, n, self.rank * n, 1, seed, mode, ppm,
                                self.ctx.stream):
            return False
        chk = gdsm.Runs(self.ctx, n, cap=1 << 20)
        ws = self.ctx.buffer(L.gdsm_diff_workspace_bytes(n))
        rc = L.gdsm_diff_raw(self.ctx.arena_ptr("replica"), scratch.ptr, None, n, chk.s.rec_off,
                             chk.s.data, chk.cap, ws.ptr, ws.nbytes, self.ctx.stream)
        ok = rc == 0 and chk.total() == 0
        scratch.free()
        ws.free()
        chk.free()
        return ok


def _tensor_at(ptr: int, shape, dtype, device) -> torch.Tensor:
    """A torch tensor viewing existing device memory (no copy, not owned)."""
    itemsize = torch.empty((), dtype=dtype).element_size()

    class _Iface:
        pass

    holder = _Iface()
    typestr = {torch.int64: "<i8", torch.uint8: "|u1", torch.int32: "<i4"}[dtype]
    holder.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr,
                                       "data": (int(ptr), False), "version": 2, "strides": None}
    t = torch.as_tensor(holder, device=device)
    assert t.data_ptr() == int(ptr) and t.element_size() == itemsize
    return t
