"""The multi-GPU release machinery on one real GPU: libgdsm's own RCCL communicator
(gdsm_comm_*) and gdsm_exchange through the C ABI on one rank, exchange.Shard's pipelined
per-destination releases, and bench.py's N > 1 step rehearsed with several ranks on cuda:0 over
gloo (RCCL cannot put two ranks on one GPU). N > 1 RCCL runs in the driver's multi-GPU bench;
tests/test_exchange.py covers 2-4 ranks of the same protocol over gloo on CPU."""
import os
import socket

import pytest
import gallocy_amd as ga
from gallocy_amd import exchange

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_exchange_c_abi_single_rank_rccl():
    """gdsm_comm_* + gdsm_exchange through the C ABI on one RCCL rank: the exact-size path (device
    all-to-all of (records, bytes), host read, all-reduce of the capacity verdict) and the
    fixed-budget path both land the stream in the home REPLICA, which must equal CURRENT."""
    import ctypes as C

    import numpy as np

    from gallocy_amd._lib import GdsmRuns
    L = ga.gdsm.lib()
    n = 1 << 14
    with ga.Context(n) as ctx:
        comm = exchange.Comm(ctx, 0, 1)
        try:
            nr = C.c_int(0)
            me = C.c_int(-1)
            assert L.gdsm_comm_size(comm.handle, C.byref(nr), C.byref(me)) == 0
            assert (nr.value, me.value) == (1, 0)
            for fixed in (0, exchange.XCHG_FIXED):
                ctx.gen_pages(seed=5 + fixed, mode=ga.GEN_CLUSTERED, ppm=100000)
                ids = ctx.ids(np.arange(n, dtype=np.uint32))
                runs = ctx.diff(ids, n=n, cap=n * 1024)
                send = (GdsmRuns * 1)(runs.s)
                recv = (GdsmRuns * 1)(GdsmRuns())
                sid = (C.c_void_p * 1)(ids.ptr)
                rid = (C.c_void_p * 1)(None)
                assert L.gdsm_exchange(ctx.handle, comm.handle, send, sid, recv, rid, ga.REPLICA,
                                       fixed) == 0
                ctx.sync()
                assert np.array_equal(ctx.download("replica"), ctx.download("current"))
                # a later diff into the same stream is ordered after the exchange that read it
                ctx.diff(ids, n=n, out=runs)
                ctx.sync()
                runs.free()
        finally:
            comm.close()


@pytest.mark.parametrize("mode,ppm", [(0, 10000), (1, 100000)])
def test_shard_pipelined_single_rank_rccl(mode, ppm):
    """exchange.Shard on one RCCL rank: release 0 with exact sizes, calibrate() fixes the byte
    budgets, then pipelined releases (diff k+1 on the main stream overlaps exchange + apply k on
    the second stream, two send sets alternating) with no host synchronisation; the home REPLICA
    must equal CURRENT."""
    n = 1 << 14
    with ga.Context(n) as ctx:
        ctx.gen_pages(seed=6, mode=mode, ppm=ppm, first_global=0, stride=1,
                      arenas=("twin", "current"))
        ctx.gen_pages(seed=6, mode=mode, ppm=ppm, first_global=0, stride=1, arenas=("replica",))
        shard = exchange.Shard(ctx, 0, 1, n, 1024)
        try:
            shard.run(1, pipelined=False)
            shard.calibrate()
            assert shard.flags == exchange.XCHG_FIXED and shard.received > 0
            ctx.prof_enable(True)
            shard.run(5)
            shard.drain()
            prof = ctx.prof_read()
            assert prof["diff"][1] == 5 and prof["apply"][1] == 5
            assert shard.verify(6, mode, ppm)
        finally:
            shard.close()


@pytest.mark.parametrize("ranks,overlap", [(2, "on"), (3, "off"), (8, "on")])
def test_bench_multi_rank_rehearsal_gloo(ranks, overlap):
    """bench.py's N > 1 step end to end with `ranks` processes sharing cuda:0 and exchanging over
    gloo (GDSM_BENCH_BACKEND=gloo, a rehearsal of the RCCL path: the same per-destination diffs,
    Shard, barriers, max-over-ranks timing; the strong-scaling default at a small total): every
    rank's home REPLICA must equal CURRENT afterwards."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, GDSM_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1", "--master-port",
           str(_port()), str(root / "bench.py"), "--gpus", str(ranks), "--steps", "3",
           "--warmup", "1", "--total-pages", str(ranks * ranks * 8192), "--no-cpu", "--overlap",
           overlap]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == ranks and d["replica_equals_current"] is True
    assert d["exchange"]["received_bytes_per_step"] > 0
    assert d["pipelined"] is (overlap == "on")
    assert d["scaling"] == "strong" and d["config"]["total_pages"] == ranks * ranks * 8192
    # the same sweep's N = 1 reference (rank 0 alone, after the N-rank run) and the efficiency
    # from it; the box ceilings beside the spec fraction
    same = d["same_run_reference"]
    assert same["pages"] == ranks * ranks * 8192 and same["ms_per_step"] > 0
    assert d["efficiency_same_run"] > 0
    roof = d["roofline"]
    assert roof["box_read_gbs"] > 0 and roof["box_copy_gbs"] > 0 and roof["frac_of_box"] > 0


def _bench_no_launcher(args, backend="gloo"):
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GDSM_BENCH_BACKEND"] = backend
    r = subprocess.run([sys.executable, str(root / "bench.py"), *args], cwd=root, env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    return json.loads(line[0])


def test_bench_gpus_2_without_launcher():
    """`bench.py --gpus 2` with no launcher (how a user or the driver may call it): the GPU-free
    parent spawns the two ranks itself, and rank 0's line reports n_gpus 2 (ranks share cuda:0
    over the gloo rehearsal transport here; RCCL on a multi-GPU node)."""
    d = _bench_no_launcher(["--gpus", "2", "--steps", "2", "--warmup", "1", "--total-pages",
                            str(4 * 8192), "--no-cpu"])
    assert d["n_gpus"] == 2 and d["replica_equals_current"] is True
    assert d["config"]["total_pages"] == 4 * 8192 and d["config"]["pages_per_gpu"] == 2 * 8192


def test_bench_coherence_sharded_gpus_2_without_launcher():
    """The coherence workload at N = 2: the page table sharded by home, each rank folding its own
    pages' batch; one line with n_gpus 2 and the events of both shards."""
    d = _bench_no_launcher(["--gpus", "2", "--workload", "coherence", "--coh-pages",
                            str(1 << 20), "--events", str(1 << 22), "--steps", "2", "--warmup",
                            "1", "--no-cpu"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["value"] > 0 and "sharded over 2 GPUs" in d["config"]["workload"]


def test_bench_gpus_2_hung_rank_exits_nonzero_within_the_deadline():
    """A rank that hangs in its setup (GDSM_BENCH_HANG_RANK=1, test hook) leaves its peer blocked
    in the first release's exchange. With --deadline 20 both ranks' watchdogs end their processes
    non-zero, torch.distributed.run stops and returns non-zero: the job ends in about the
    deadline instead of hanging (gloo rehearsal on one GPU)."""
    import subprocess
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(GDSM_BENCH_BACKEND="gloo", GDSM_BENCH_HANG_RANK="1")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--total-pages", str(4 * 8192), "--no-cpu",
                        "--deadline", "20"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=110)
    took = time.monotonic() - t0
    assert r.returncode != 0
    assert "deadline passed" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert took < 100, took
