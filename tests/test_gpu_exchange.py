"""The multi-GPU step machinery on one real GPU: a 1-rank RCCL (torch 'nccl') group drives
gallocy_amd.exchange.Shard — device tensors aliasing libgdsm buffers, the context stream as
torch's current stream, all_to_all_single, gdsm_apply_raw — and the home REPLICA must end equal
to CURRENT. (N > 1 runs in the driver's multi-GPU bench; tests/test_exchange.py covers 2-4 ranks
of the same code over gloo.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import gallocy_amd as ga
from gallocy_amd import exchange

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_step_single_rank_rccl():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 1 << 14
        with ga.Context(n) as ctx:
            ctx.gen_pages(seed=5, mode=ga.GEN_CLUSTERED, ppm=100000, first_global=0, stride=1,
                          arenas=("twin", "current"))
            ctx.gen_pages(seed=5, mode=ga.GEN_CLUSTERED, ppm=100000, first_global=0, stride=1,
                          arenas=("replica",))
            runs = ga.Runs(ctx, n, cap=n * 1024)
            shard = exchange.Shard(ctx, runs, 0, 1, n)
            shard.gen_args = (5, ga.GEN_CLUSTERED, 100000)
            for _ in range(2):
                ctx.diff(out=runs)
                shard.exchange_and_apply()
            ctx.sync()
            torch.cuda.synchronize()
            assert shard.received == runs.total() > 0
            assert shard.verify()
    finally:
        dist.destroy_process_group()


def test_shard_pipelined_run_single_rank_rccl():
    """Shard.run: diff k+1 on the context stream overlaps exchange + apply k on the comm
    stream, two run buffers alternating; the replica must still end equal to CURRENT."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 1 << 14
        with ga.Context(n) as ctx:
            ctx.gen_pages(seed=6, mode=ga.GEN_UNIFORM, ppm=10000, first_global=0, stride=1,
                          arenas=("twin", "current"))
            ctx.gen_pages(seed=6, mode=ga.GEN_UNIFORM, ppm=10000, first_global=0, stride=1,
                          arenas=("replica",))
            runs = [ga.Runs(ctx, n, cap=n * 256) for _ in range(2)]
            shard = exchange.Shard(ctx, runs, 0, 1, n)
            shard.gen_args = (6, ga.GEN_UNIFORM, 10000)
            shard.run(5)
            shard.drain()
            ctx.sync()
            assert shard.received == runs[0].total() == runs[1].total() > 0
            assert shard.verify()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ranks,overlap", [(2, "on"), (3, "off")])
def test_bench_multi_rank_rehearsal_gloo(ranks, overlap):
    """bench.py's N > 1 step end to end with `ranks` processes sharing cuda:0 and exchanging over
    gloo (GDSM_BENCH_BACKEND=gloo, a rehearsal of the RCCL path: same Shard pipeline, barriers,
    max-over-ranks timing): every rank's home REPLICA must equal CURRENT afterwards."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, GDSM_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1", "--master-port",
           str(_port()), str(root / "bench.py"), "--gpus", str(ranks), "--steps", "3",
           "--warmup", "1", "--pages", str(ranks * 16384), "--no-cpu", "--overlap", overlap]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == ranks and d["replica_equals_current"] is True
    assert d["exchange"]["received_bytes_per_step"] > 0
    assert d["pipelined"] is (overlap == "on")
