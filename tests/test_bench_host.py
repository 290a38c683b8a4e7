"""bench.py's host-side pieces that need no GPU: the CPU baseline leg (the C oracle, one thread
and all-core, every sample's REPLICA checked equal to CURRENT inside the leg) and the diff-stream
payload count used for the roofline bytes."""
from pathlib import Path

import numpy as np
import pytest

import bench
from oracle import oracle

ROOT = Path(__file__).resolve().parents[1]


def test_cpu_baseline_single_and_all_core(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    out = bench.cpu_baseline(0, 10000, 7, 0.4)
    assert out["kind"] == "port" and out["unit"] == "pages/s"
    assert out["cores"] == min(2, len(__import__("os").sched_getaffinity(0)))
    assert out["value"] > 0 and out["single_thread"]["value"] > 0
    assert out["single_thread"]["cores"] == 1


def test_payload_bytes_matches_run_lengths():
    twin, cur = oracle.gen_pages(64, seed=3, mode=0, ppm=10000)
    ro, data = oracle.diff_pages(twin, cur)
    want = 0
    w = data.view("<u4")
    for i in range(64):
        a = int(ro[i]) // 4
        if ro[i + 1] > ro[i]:
            want += sum(int(h) >> 16 for h in w[a + 1:a + 1 + int(w[a])])
    assert bench.payload_bytes(ro, data) == want
    assert want == int(np.count_nonzero(twin != cur))  # runs cover exactly the changed bytes


def test_cpu_baseline_reports_host(monkeypatch):
    """BASELINE.md timing rules: nproc, the CPU model and the host RAM next to CPU numbers; the
    thread count is the process's CPU share (OMP_NUM_THREADS), with no fixed cap."""
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_threads() == min(3, len(__import__("os").sched_getaffinity(0)))
    h = bench.host_info()
    assert h["nproc"] >= 1 and h["host_ram_gib"] > 0 and h["host_cpu"]


def _bench(args, env_extra):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(bench.ROOT / "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=120)


def test_gpus_mismatch_with_launcher_exits_nonzero():
    """Under a launcher (WORLD_SIZE set) --gpus must equal the rank count: a mismatch exits
    non-zero before anything touches a GPU, instead of printing a line for the wrong N."""
    r = _bench(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "--gpus 1" in r.stderr and "WORLD_SIZE" in r.stderr
    r = _bench(["--gpus", "8", "--steps", "1"], {"WORLD_SIZE": "4", "RANK": "0"})
    assert r.returncode != 0
    r = _bench(["--gpus", "0"], {})
    assert r.returncode != 0


def test_gpus_n_without_launcher_spawns_n_ranks(monkeypatch):
    """`bench.py --gpus N` with no launcher: the parent (no GPU call) starts torch.distributed.run
    with N processes on 127.0.0.1 and returns their exit code; --gpus 1 runs in-process."""
    import argparse
    import subprocess
    calls = []

    class R:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        calls.append((cmd, env))
        return R()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(bench.sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert bench.launch_ranks(argparse.Namespace(gpus=4)) == 7
    cmd, env = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and cmd[-5].endswith("bench.py")
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.launch_ranks(argparse.Namespace(gpus=1)) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_ranks(argparse.Namespace(gpus=4)) is None  # already a rank


def test_mmult_cpu_baseline_replays_the_trace():
    """Config 5's CPU baseline: the test_mmult trace through the C oracle round by round; the
    home copies equal the product zone afterwards."""
    out = bench.mmult_cpu_baseline(96, 3, 7)
    assert out["home_copy_equals_product"] is True
    assert out["value"] > 0 and out["unit"] == "rounds/s" and out["kind"] == "port"


@pytest.mark.parametrize("disarm", [False, True])
def test_watchdog_ends_the_process_or_stays_quiet(disarm):
    """exchange.Watchdog: a phase that overruns its deadline ends the process with status 3 and
    names the phase on stderr; a disarmed one lets the process finish normally."""
    import subprocess
    import sys
    code = ("import time\nfrom gallocy_amd.exchange import Watchdog\n"
            "w = Watchdog(rank=5).arm(0.5, 'a test phase')\n"
            + ("w.disarm()\n" if disarm else "") + "time.sleep(3)\nprint('finished')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    if disarm:
        assert r.returncode == 0 and "finished" in r.stdout
    else:
        assert r.returncode == 3 and "finished" not in r.stdout
        assert "rank 5: deadline passed in 'a test phase'" in r.stderr


@pytest.mark.parametrize("nodes", [1, 3])
def test_mmult_cpu_baseline_c_loop_and_python_loop_agree(nodes):
    """Config 5's CPU baseline: the round loop in C (oracle or_bench_mmult over the precomputed
    plan) and the same loop driven from Python both end with the home copy equal to the product
    (test_mmult.cpp's c = a x b), and the line is labelled as timed in C."""
    out = bench.mmult_cpu_baseline(48, nodes, 3, min_seconds=0.01)
    assert out["home_copy_equals_product"] is True
    assert out["python_driven"]["home_copy_equals_product"] is True
    assert out["timed_in"].startswith("C") and out["value"] > 0 and out["cores"] == 1
    # the per-round twin work matches the GPU line's (gdsm_release re-twins after the diff), and
    # the other workflow is timed beside it, also ending at the product
    assert out["twin_workflow"] == "re-twin after the diff"
    assert out["other_twin_workflow"]["twin_workflow"] == "twin before the writes"
    assert out["other_twin_workflow"]["home_copy_equals_product"] is True
    assert out["other_twin_workflow"]["value"] > 0
