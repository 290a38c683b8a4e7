#!/usr/bin/env python3
"""Benchmark of the DSM hot path: pages diffed + applied per second (4 KiB pages).

One step = diff of every page of the shard (TWIN vs CURRENT -> canonical run stream, SPEC §3)
+ apply of that stream to the REPLICA arena (SPEC §4). On one GPU the step is serial (diff k+1
starts after apply k): it is HBM-bound and an overlapped apply only takes bandwidth from the
diff. For N > 1 each rank diffs its pages into one stream per home GPU and libgdsm's
gdsm_exchange ships them over RCCL (xGMI) and applies them at the homes
(gallocy_amd/exchange.py); releases are double-buffered (the exchange and home-side apply of k
run on a second stream while k+1 is diffed) and, after the first release has fixed every
stream's byte budget, never synchronise the host. Every step is complete when the clock stops.

Workloads (`--config`): the default at EVERY N is the north_star target, 16M x 4 KiB pages in all
(64 GiB per copy) with 1 % random 8-byte word writes, strong-scaled: N = 1 holds all 16M pages
on one GPU (three arenas, 192 GiB), N > 1 holds 16M/N per GPU, so the driver's N = 1..8 lines
are one workload. `--config 2` is BASELINE configs[1] (1M pages per GPU, 1 % words, weak);
`--config 3` is configs[2] (16M pages in all, clustered 10 %, strong).
Synthetic inputs (SPEC §6), resident in HBM before the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement); everything else -> stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["northstar", "2", "3"], default="northstar",
                    help="northstar (default): 16M pages in all, 1 %% word writes, strong scaling "
                         "at every N; 2: BASELINE configs[1], 1M pages per GPU, 1 %% words, weak; "
                         "3: configs[2], 16M pages in all, clustered 10 %%, strong")
    ap.add_argument("--pages", type=int, default=None, help="pages per GPU (weak scaling)")
    ap.add_argument("--total-pages", type=int, default=None, help="pages in all (strong scaling)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None)
    ap.add_argument("--mode", choices=["uniform", "clustered"], default=None)
    ap.add_argument("--ppm", type=int, default=None, help="write density in parts per million")
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="double-buffered steps (exchange/apply k overlaps diff k+1); auto = on "
                         "for N > 1 (hides the RCCL exchange), off on one GPU (HBM-bound)")
    ap.add_argument("--fuse", choices=["on", "off"], default="off",
                    help="N = 1: on = gdsm_diff_apply (the diff kernel applies each page's runs "
                         "to its home copy from the registers that found them); off = gdsm_diff "
                         "then gdsm_apply of the stream")
    ap.add_argument("--compare-overlap", action="store_true",
                    help="also time the other overlap mode (reported beside the measured one)")
    ap.add_argument("--workload", choices=["pages", "coherence", "mmult", "nw", "twin"],
                    default="pages",
                    help="pages: BASELINE configs[1]/[2] (the headline); coherence: configs[3]; "
                         "mmult: configs[4] trace replay; nw: the reference diff() (NW alignment) "
                         "on the GPU over configs[0]-shaped page pairs; twin: the twin step "
                         "(TWIN := CURRENT) of the north-star pages, beside the writer-side "
                         "re-twin of only the dirty bytes (the release's stream applied to TWIN)")
    ap.add_argument("--nw-pairs", type=int, default=2048,
                    help="nw: 4 KiB page pairs per batch (2048: 8 fill waves per SIMD, the "
                         "fill's serial max3 chain needs them; 512 left it at 4)")
    ap.add_argument("--ndim", type=int, default=1000, help="mmult: matrix size (<= 1021)")
    ap.add_argument("--nodes", type=int, default=4, help="mmult: simulated DSM nodes (1-8)")
    ap.add_argument("--retwin", choices=["on", "off"], default="on",
                    help="mmult: on = each release re-twins its pages (gdsm_release, no twin step "
                         "per round); off = a twin launch before the round's writes (round 4)")
    ap.add_argument("--graph", action="store_true",
                    help="mmult: replay one HIP graph of every round instead of eager launches")
    ap.add_argument("--driver", choices=["device", "native", "native2", "python"],
                    default="device",
                    help="mmult: every round on the device (gdsm_rounds: one persistent launch "
                         "per context, a barrier between rounds; the default, faster at 1-8 "
                         "nodes: DESIGN §4), or rounds issued by the C++ loop over the C ABI "
                         "(gallocy_amd/native/replay.cpp; native2: two host threads, one per "
                         "context), or from Python")
    ap.add_argument("--events", type=int, default=1 << 30, help="coherence: events per batch")
    ap.add_argument("--coh-pages", type=int, default=16 << 20, help="coherence: pages")
    ap.add_argument("--dist", choices=["zipf", "uniform"], default="zipf")
    ap.add_argument("--coh-nodes", type=int, default=8,
                    help="coherence: DSM nodes of the batch (BASELINE config 4: 8)")
    ap.add_argument("--same-run-ref", choices=["on", "off"], default="on",
                    help="pages workload, N > 1: after the N-rank run rank 0 times the N = 1 step "
                         "of the same total workload on its own GPU (outside `value`) and reports "
                         "efficiency_same_run")
    ap.add_argument("--deadline", type=float, default=300.0,
                    help="N > 1: seconds each phase may take before a rank exits non-zero (a "
                         "peer died or hangs; exchange.Watchdog). The pages workload re-arms it "
                         "per phase (setup + first release, the timed releases, the link timing, "
                         "verification, the same-run N = 1 reference, teardown); the other "
                         "workloads arm it once for their whole run. 0 = off")
    return ap.parse_args()


def payload_bytes(rec_off: np.ndarray, data: np.ndarray) -> int:
    """Sum of run lengths (|P|) of a host diff stream, vectorised."""
    sizes = np.diff(rec_off)
    dirty = np.flatnonzero(sizes)
    if len(dirty) == 0:
        return 0
    w = data.view("<u4") if len(data) % 4 == 0 else np.frombuffer(data.tobytes(), "<u4")
    starts = (rec_off[dirty] // 4).astype(np.int64)
    nr = w[starts].astype(np.int64)
    first_hdr = np.repeat(starts + 1, nr)
    within = np.arange(nr.sum()) - np.repeat(np.cumsum(nr) - nr, nr)
    return int((w[first_hdr + within] >> 16).astype(np.int64).sum())


CONFIGS = {  # --config -> (scaling, mode, ppm, pages: in all when strong, per GPU when weak)
    "northstar": ("strong", "uniform", 10000, 16 << 20),
    "2": ("weak", "uniform", 10000, 1 << 20),
    "3": ("strong", "clustered", 100000, 16 << 20),
}


def workload_shape(args, world: int):
    """(scaling, mode name, ppm, pages per GPU) of the pages workload: --config, then overrides."""
    scaling, mode_name, ppm, pages = CONFIGS[args.config]
    scaling = args.scaling or scaling
    mode_name = args.mode or mode_name
    if args.mode and args.ppm is None:
        ppm = 10000 if mode_name == "uniform" else 100000
    ppm = args.ppm if args.ppm is not None else ppm
    if scaling == "strong":
        total = args.total_pages or (args.pages * world if args.pages else pages)
        if total % (world * world):
            raise SystemExit("the total page count must be a multiple of GPUs^2")
        return scaling, mode_name, ppm, total // world
    n = args.pages or (args.total_pages // world if args.total_pages else pages)
    if n % world:
        raise SystemExit("--pages must be a multiple of the GPU count")
    return scaling, mode_name, ppm, n


def efficiency_ref(pages_total: int, mode: str, ppm: int):
    """The same workload's N = 1 line committed under profiles/ (newest first): (ms_per_step,
    file name), or (None, None). Parallel efficiency at N is ref_ms / (N * ms_per_step_N)."""
    for p in sorted((ROOT / "profiles").glob("*bench*n1*.json"), reverse=True):
        try:
            j = json.loads(p.read_text().strip().splitlines()[-1])
        except Exception:  # noqa: BLE001
            continue
        c = j.get("config", {})
        if (j.get("n_gpus") == 1 and c.get("total_pages") == pages_total
                and c.get("mode") == mode and c.get("ppm") == ppm):
            return j.get("ms_per_step"), p.name
    return None, None


XGMI_LINK_GBS = 153.0  # per xGMI link, one direction (MI355X_MICROARCH.md); 7 links per GPU


def host_info() -> dict:
    """nproc, the CPU model and the host RAM (BASELINE.md timing rules), next to CPU numbers."""
    out = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        out["host_cpu"] = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t")
    except Exception:  # noqa: BLE001
        pass
    try:
        kb = int([ln for ln in open("/proc/meminfo") if ln.startswith("MemTotal")][0].split()[1])
        out["host_ram_gib"] = round(kb / (1 << 20), 1)
    except Exception:  # noqa: BLE001
        pass
    return out


def cpu_threads() -> int:
    """The CPU share this process may use: OMP_NUM_THREADS when set (the GPU box exports its
    share there; os.cpu_count() is the whole machine), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(int(env), aff) if env and env.isdigit() else aff)


def cpu_baseline(mode: int, ppm: int, seed: int, seconds: float):
    """The C oracle (oracle/liboracle.so, -O3, OpenMP, timed in C) on a bounded sample of the
    workload: one thread, then all of this process's CPU share (single-core and
    all-core), each thread repeating diff + apply passes over its own sample."""
    from oracle import oracle
    n1, nper = 32768, 16384
    pages1, dt1, ok1 = oracle.bench_diff_apply(n1, mode, ppm, seed, seconds / 2, 1)
    assert ok1
    nt = cpu_threads()
    pages, dt, ok = oracle.bench_diff_apply(nper, mode, ppm, seed, seconds / 2, nt)
    assert ok
    out = {"value": round(pages / dt, 1), "unit": "pages/s", "cores": nt, "kind": "port",
           "sample": f"{nt} OpenMP threads x {nper} pages each (thread t: pages [t*{nper}, "
                     f"(t+1)*{nper}) of the workload, seed {seed}), repeated diff+apply passes "
                     f"for {seconds / 2:.1f} s, oracle/gdsm_oracle.c -O3, timed in C",
           "single_thread": {"value": round(pages1 / dt1, 1), "cores": 1,
                             "sample": f"{n1} pages x {pages1 // n1} passes, {dt1:.1f} s"}}
    drv = oracle.REF_DRIVER
    if drv.exists():
        try:
            r = subprocess.run([str(drv), "time", "1024", "3"], capture_output=True, text=True,
                               timeout=120, check=True).stdout.split()
            s, cells = float(r[0]), int(r[1])
            out["reference_nw_diff"] = {
                "cells_per_s": round(cells / s, 1), "n": 1024, "seconds_per_call": s,
                "extrapolated_seconds_per_4KiB_page": round(4096 * 4096 / (cells / s), 4),
                "note": "reference diff() (gallocy/utils/diff.cpp:73-167) compiled -O0 from its "
                        "sources (oracle/_ref); extrapolated, the reference crashes at 4 KiB"}
        except Exception as e:  # noqa: BLE001
            out["reference_nw_diff"] = {"error": str(e)[:200]}
    out.update(host_info())
    return out


DIFF_KERNEL = "gdsm::diff_single_kernel"


def read_traffic(pages: int, mode: str, ppm: int, fused: bool):
    """Per-launch HBM bytes of the diff kernel (the instance with the apply fused in, or not)
    from the newest committed PMC summary that measured it on this workload
    (profiles/*traffic*.json, scripts/gpu_prof.sh), else None. Summaries without a workload tag
    are for the default config-2 workload."""
    flag = ", true" if fused else ", false"  # the kApply template argument
    default = {"pages": 1 << 20, "mode": "uniform", "ppm": 10000}
    for p in sorted((ROOT / "profiles").glob("*traffic*.json"), reverse=True):
        try:
            j = json.loads(p.read_text())
        except Exception:  # noqa: BLE001
            continue
        if (str(j.get("diff_kernel", "")).startswith(DIFF_KERNEL)
                and flag in str(j.get("diff_kernel", ""))
                and j.get("workload", default) == {"pages": pages, "mode": mode, "ppm": ppm}):
            return j.get("diff_kernel_bytes_per_launch"), p.name
    return None, None


def read_kernel_traffic(prefix: str, workload: dict):
    """Per-launch HBM bytes of kernel family `prefix` from the newest committed PMC summary of
    this workload (profiles/*traffic*.json written by scripts/pmc_summary.py with a kernel
    prefix), else (None, None)."""
    for p in sorted((ROOT / "profiles").glob("*traffic*.json"), reverse=True):
        try:
            j = json.loads(p.read_text())
        except Exception:  # noqa: BLE001
            continue
        if (j.get("workload") == workload and j.get("main_kernel_bytes_per_launch")
                and str(j.get("main_kernel", "")).startswith(prefix)):
            return j["main_kernel_bytes_per_launch"], p.name
    return None, None


def read_coh_traffic(dist: str, pages: int, events: int):
    """Per-launch HBM bytes of the coherence fold kernel from the newest committed PMC summary of
    the same batch shape (profiles/*coh_traffic*.json, scripts/coh_traffic.sh), else None."""
    want = {"workload": "coherence", "dist": dist, "pages": pages, "events": events}
    for p in sorted((ROOT / "profiles").glob("*coh_traffic*.json"), reverse=True):
        try:
            j = json.loads(p.read_text())
        except Exception:  # noqa: BLE001
            continue
        if (j.get("workload") == want and j.get("main_kernel_bytes_per_launch")
                and str(j.get("main_kernel", "")).startswith("gdsm::coh_fold_kernel")):
            return j["main_kernel_bytes_per_launch"], p.name
    return None, None


def box_ceilings(ctx, n: int, read=None, copy=None, reps: int = 5) -> dict:
    """This GPU's own streaming ceilings over the workload's arenas, measured in this process
    before the timed region (gdsm_probe_ceiling, gallocy_amd/csrc/gdsm_probe.hip): `read` = two
    device pointers of n pages each read once (the diff's input), `copy` = (src, dst) n pages
    copied (dst is overwritten: the caller regenerates it). Best of `reps` launches (HIP events);
    the medians beside. A line's frac_of_box = achieved / the matching ceiling: the kernel's
    fraction of the box it ran on, where frac is against the 8 TB/s spec."""
    import ctypes as C

    import gallocy_amd as ga
    L = ga.gdsm.lib()
    out = {}
    for key, kind, args in (("read", 0, read), ("copy", 1, copy)):
        if args is None:
            continue
        a, b, dst = (args[0], args[1], None) if kind == 0 else (args[0], None, args[1])
        best, med = C.c_float(), C.c_float()
        rc = L.gdsm_probe_ceiling(ctx.handle, kind, a, b, dst, n, reps, C.byref(best),
                                  C.byref(med))
        if rc:
            raise RuntimeError(f"gdsm_probe_ceiling({key}) {rc}")
        moved = 2 * n * 4096  # read: both arenas; copy: read + write of one
        out[f"box_{key}_gbs"] = round(moved / (best.value * 1e-3) / 1e9, 1)
        out[f"box_{key}_gbs_median"] = round(moved / (med.value * 1e-3) / 1e9, 1)
    out["box_probe"] = (f"gdsm_probe_ceiling over this run's own arenas ({n} pages), best of "
                        f"{reps} launches: read = two page arenas read once with 16-B "
                        f"nontemporal loads (the diff's input), copy = the fastest of a flat "
                        f"16-B copy and two page-shaped copies; "
                        f"frac_of_box = achieved / the ceiling matching the kernel")
    return out


def with_box(roof: dict, box: dict, which: str) -> dict:
    """roofline + the box ceilings and the kernel's fraction of the `which` ceiling."""
    if not box:
        return roof
    r = dict(roof, **box)
    r["frac_of_box"] = round(roof["achieved"] / box[f"box_{which}_gbs"], 4)
    r["frac_of_box_against"] = f"box_{which}_gbs"
    return r


def n1_reference(args, total: int, mode: int, ppm: int, device: int) -> dict:
    """--gpus N > 1, after the N-rank run (its arenas freed): rank 0 times the N = 1 step of the
    SAME total workload on its own GPU (all `total` pages in one shard, diff + apply, serial, as
    bench.py --gpus 1 runs it), so parallel efficiency comes from one sweep and one box. Outside
    `value`. Skipped when the three arenas do not fit the free HBM."""
    import torch

    import gallocy_amd as ga
    cap_pp = 128 if mode == ga.GEN_UNIFORM else 1024
    need = 3 * (total + 1) * 4096 + total * cap_pp + 16 * (total + 1) + (2 << 30)
    free, _ = torch.cuda.mem_get_info(device)
    if free < need:
        return {"skipped": f"{need / 2**30:.1f} GiB needed for the N = 1 arenas, "
                           f"{free / 2**30:.1f} GiB free"}
    ctx = ga.Context(total, device=device)
    try:
        ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=0, stride=1,
                      arenas=("twin", "current"))
        ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=0, stride=1,
                      arenas=("replica",))
        runs = ga.Runs(ctx, total, cap=total * cap_pp)
        for _ in range(args.warmup):
            ctx.diff(out=runs)
            ctx.apply(runs)
        ctx.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.diff(out=runs)
            ctx.apply(runs)
        ctx.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        runs.free()
    finally:
        ctx.close()
    return {"ms_per_step": round(dt / args.steps * 1e3, 4), "pages": total,
            "steps": args.steps, "warmup": args.warmup}


def watchdog(args, rank: int, world: int, what: str):
    """N > 1: (re)arms the rank's deadline for the phase `what` (exchange.Watchdog: a rank
    blocked on a dead or hung peer exits non-zero instead of hanging the job)."""
    global WATCHDOG
    if world <= 1 or args.deadline <= 0:
        return
    if WATCHDOG is None:
        from gallocy_amd.exchange import Watchdog
        WATCHDOG = Watchdog(rank)
    WATCHDOG.arm(args.deadline, what)
    hang = os.environ.get("GDSM_BENCH_HANG_RANK")  # test hook: this rank hangs in its setup
    if hang is not None and int(hang) == rank and what.startswith("setup"):
        log(f"bench.py: rank {rank} hangs (GDSM_BENCH_HANG_RANK)")
        time.sleep(1e9)


WATCHDOG = None


def ranks_setup(args):
    """(rank, world, local device) under a launcher (gloo carries barriers and the max-over-ranks
    time; nothing of the data path), or (0, 1, 0). N > 1: the whole run has --deadline."""
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        watchdog(args, rank, world, "setup and run")
    return rank, world, local


def max_over_ranks(dt: float, world: int) -> float:
    if world == 1:
        return dt
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def run_coherence(args):
    """BASELINE configs[3]: batched coherence, 16M pages, 8 nodes, 1B events (Zipf 0.8 or
    uniform pages, 20 % writes), one GPU. A step = one whole batch through the page table.
    N > 1 GPUs: the page table is sharded by home (SPEC §5b: rank r holds pages [r n/N,
    (r+1) n/N)) and every home folds the batch of its own pages (n/N pages, E/N events, the
    events as gdsm_route_events delivers them); no collective in the timed region (strong
    scaling, the same 16M pages and 1B events in all)."""
    import torch

    import gallocy_amd as ga
    from gallocy_amd.workloads import event_counts
    rank, world, local = ranks_setup(args)
    if args.coh_pages % world or args.events % world:
        raise SystemExit("--coh-pages and --events must be multiples of the GPU count")
    n, E = args.coh_pages // world, args.events // world
    counts = event_counts(n, E, args.dist, seed=args.seed + rank)
    ctx = ga.Context(n, arenas=(), device=local)
    nn = args.coh_nodes
    if not 1 <= nn <= 8:
        raise SystemExit("--coh-nodes must be 1-8")
    ev = ctx.gen_events(counts, seed=args.seed + rank, n_nodes=nn, write_pct=20)
    touched = int((counts > 0).sum())
    # this box's read ceiling over the event buffer itself (its two halves as the probe's arenas)
    half = (ev.count * 8) // 2 // 4096
    box = box_ceilings(ctx, half, read=(ev.ptr, ev.ptr + half * 4096)) if half else {}
    ctx.coh_init(nn)
    tot_dev = ctx.buffer(80)
    L = ga.gdsm.lib()

    def step():
        rc = L.gdsm_coherence_batch_async(ctx.handle, ev.ptr, ev.count, tot_dev.ptr)
        if rc:
            raise RuntimeError(f"gdsm_coherence_batch_async {rc}")

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier(world)
    ctx.prof_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world)
    prof = ctx.prof_read()
    totals = tot_dev.download(np.uint64, 10)
    main_ms = max_over_ranks(prof["coh_fold"][0] / max(1, prof["coh_fold"][1]), world)
    alg = ev.count * 8 + touched * 16  # events read + state/faults words read and written
    achieved = alg / (main_ms * 1e-3) / 1e9
    traffic, traffic_src = read_coh_traffic(args.dist, n, E)
    stages = {k: {"ms_per_launch": round(v[0] / v[1], 4), "launches": v[1]} for k, v in prof.items() if v[1]}
    all_events = ev.count
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([ev.count, touched], dtype=torch.int64)
        dist.all_reduce(t)
        all_events = int(t[0])
    if rank != 0:
        ctx.close()
        barrier(world)
        return
    res = {"metric": "coherence events/sec", "value": round(all_events * args.steps / dt, 1),
           "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "u64",
           "data": f"synthetic ({args.dist} page popularity, SPEC §6 events)",
           "config": {"workload": f"{n * world} pages, {nn} nodes, {all_events} events/batch, "
                                  f"{args.dist}, 20% writes"
                                  + (f", page table sharded over {world} GPUs (rank 0's shard: "
                                     f"{n} pages, {ev.count} events)" if world > 1 else ""),
                      "touched_pages": touched},
           "roofline": with_box({"bound": "hbm", "kernel": "gdsm::coh_fold_kernel",
                                 "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                 "traffic": traffic, "traffic_source": traffic_src,
                                 "algorithmic_bytes_per_launch": int(alg),
                                 "avg_launch_ms": round(main_ms, 4)}, box, "read"),
           "stages": stages,
           "last_batch_totals": {"invalidations": int(totals[0]), "transfers": int(totals[1]),
                                 "node_faults": [int(x) for x in totals[2:]]},
           "cpu_baseline": None}
    if not args.no_cpu and world == 1:
        from oracle import oracle
        m = 1 << 20
        sub = event_counts(m, 1 << 26, args.dist, seed=args.seed)
        hev = oracle.gen_events(sub, seed=args.seed)
        nt = cpu_threads()
        d1, t1 = oracle.bench_coherence(sub, hev, args.cpu_seconds / 2, 1)
        dn, tn = oracle.bench_coherence(sub, hev, args.cpu_seconds / 2, nt)
        res["cpu_baseline"] = {
            "value": round(dn / tn, 1), "unit": "events/s", "cores": nt, "kind": "port",
            "sample": f"{len(hev)} events over {m} pages ({args.dist}); {nt} OpenMP threads, "
                      f"each folding its own contiguous page range of the batch, repeated for "
                      f"{args.cpu_seconds / 2:.1f} s, oracle or_coherence -O3, timed in C",
            "single_thread": {"value": round(d1 / t1, 1), "cores": 1,
                              "sample": f"the same batch, {d1 // max(1, len(hev))} passes, "
                                        f"{t1:.1f} s"}, **host_info()}
    print(json.dumps(res), flush=True)
    ctx.close()
    barrier(world)


def run_twin(args):
    """The twin step of north_star ("page twin/diff creation") on the north-star pages (16M x 4
    KiB, 1 % word writes), one GPU per rank (replicas at N > 1, weak scaling). A step =
    gdsm_twin of every page (TWIN := CURRENT, the copy that opens a write interval: 8192 B of
    HBM per page). Reported beside it: the writer-side re-twin a release can do instead, the
    release's own diff stream applied to TWIN (gdsm_apply, |D| + |P| bytes per page), which
    leaves TWIN == CURRENT too (checked)."""
    import torch

    import gallocy_amd as ga
    rank, world, local = ranks_setup(args)
    n = args.pages or (16 << 20)
    mode = ga.GEN_UNIFORM if (args.mode or "uniform") == "uniform" else ga.GEN_CLUSTERED
    ppm = args.ppm if args.ppm is not None else (10000 if mode == ga.GEN_UNIFORM else 100000)
    ctx = ga.Context(n, device=local, arenas=("twin", "current"))
    # this box's ceilings over the two arenas (the copy probe writes TWIN: generated after it)
    box = box_ceilings(ctx, n, read=(ctx.arena_ptr("twin"), ctx.arena_ptr("current")),
                       copy=(ctx.arena_ptr("current"), ctx.arena_ptr("twin")))
    ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=rank * n,
                  arenas=("twin", "current"))
    runs = ctx.diff(cap=n * (128 if mode == ga.GEN_UNIFORM else 1024))
    total = runs.total()
    host = runs.to_host()
    pay = payload_bytes(host.rec_off, host.data)
    del host

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        ctx.sync()
        torch.cuda.synchronize()
        barrier(world)
        ctx.prof_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        ctx.sync()
        torch.cuda.synchronize()
        dt = max_over_ranks(time.perf_counter() - t0, world)
        return dt, ctx.prof_read()

    dt, prof = timed(lambda: ctx.twin())
    twin_ms = max_over_ranks(prof["twin"][0] / max(1, prof["twin"][1]), world)
    ok_full = ctx.diff(cap=1 << 20).total() == 0
    # re-twin by the stream: TWIN back to its generated state, then the stream applied to it
    ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=rank * n, arenas=("twin",))
    dt_a, prof_a = timed(lambda: ctx.apply(runs, "twin"))
    apply_ms = max_over_ranks(prof_a["apply"][0] / max(1, prof_a["apply"][1]), world)
    ok_apply = ctx.diff(cap=1 << 20).total() == 0
    alg = 8192 * n
    achieved = alg / (twin_ms * 1e-3) / 1e9
    traffic, traffic_src = read_kernel_traffic("gdsm::twin_kernel", {"workload": "twin", "pages": n})
    res = None
    if rank == 0:
        res = {"metric": "pages twinned/sec (4 KiB)", "value": round(world * n * args.steps / dt, 1),
               "unit": "pages/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8",
               "data": "synthetic (counter-hash pages, docs/SPEC.md §6)",
               "config": {"workload": f"{n} x 4 KiB pages per GPU, gdsm_twin of every page"
                                      + (f", {world} replicas" if world > 1 else ""),
                          "pages_per_gpu": n, "seed": args.seed},
               "roofline": with_box({"bound": "hbm", "kernel": "gdsm::twin_kernel",
                                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                     "traffic": traffic, "traffic_source": traffic_src,
                                     "algorithmic_bytes_per_launch": alg,
                                     "avg_launch_ms": round(twin_ms, 4)}, box, "copy"),
               "twin_equals_current": bool(ok_full),
               "retwin_by_stream": {
                   "kernel": "gdsm::apply_flat_kernel (target TWIN)",
                   "ms_per_launch": round(apply_ms, 4),
                   "algorithmic_bytes_per_launch": int(total + pay),
                   "achieved_gbs": round((total + pay) / (apply_ms * 1e-3) / 1e9, 1),
                   "speedup_vs_full_twin": round(twin_ms / apply_ms, 2),
                   "twin_equals_current": bool(ok_apply),
                   "note": "the release's diff stream applied to the writer's TWIN re-twins only "
                           "the dirty bytes; it needs the stream the release computes anyway"},
               "cpu_baseline": None}
        if not args.no_cpu and world == 1:
            m = 1 << 18
            src = np.random.default_rng(args.seed).integers(0, 256, (m, 4096), dtype=np.uint8)
            dst = np.empty_like(src)
            reps, t1 = 0, time.perf_counter()
            while time.perf_counter() - t1 < min(args.cpu_seconds, 6.0) or reps == 0:
                np.copyto(dst, src)
                reps += 1
            ct = time.perf_counter() - t1
            res["cpu_baseline"] = {"value": round(reps * m / ct, 1), "unit": "pages/s", "cores": 1,
                                   "kind": "port",
                                   "sample": f"{m} pages (1 GiB) copied {reps} times with "
                                             "numpy.copyto (memcpy), one thread (or_twin's "
                                             "per-page memcpy, oracle/gdsm_oracle.c)",
                                   **host_info()}
        print(json.dumps(res), flush=True)
    runs.free()
    ctx.close()
    barrier(world)


def mmult_cpu_baseline(ndim: int, nodes: int, seed: int, min_seconds: float = 2.0,
                       retwin: bool = True) -> dict:
    """Config 5 on the host: the same trace replayed round by round on one thread through the C
    oracle (or_coherence of the round's events, the row writes, or_diff_pages of the written
    pages, or_apply of the stream to the home copies), P node views side by side as on the GPU.
    The per-round twin work matches the GPU line's: with `retwin` (gdsm_release, the default)
    the round's stream is applied to the twin views after the diff (only the dirty bytes move,
    as in the release), else the written pages are twinned before the writes (round 4's
    workflow). The other workflow is timed beside it. The round loop runs in C
    (oracle/gdsm_oracle_bench.c:or_bench_mmult, CLOCK_MONOTONIC around the loop) over a plan
    precomputed here; the same loop driven from Python (numpy + ctypes per round) is reported
    beside it, labelled. The home copies are checked against the product afterwards."""
    from gallocy_amd.trace import PAGE_SZ, MmultTrace, c_row_values, mmult_layout, zone_image
    from oracle import oracle
    L = mmult_layout(ndim)
    T = MmultTrace(L, nodes, seed)
    Z = L.n_pages
    img = zone_image(L).reshape(Z, PAGE_SZ)
    rowvals = np.stack([c_row_values(L, i) for i in range(L.ndim)]).view(np.uint8)
    rb = 8 * ndim
    plan = []
    for r in range(T.rounds):
        rows = T.round_rows(r)
        ids, home = [], []
        for t, i in rows:
            wp = np.arange(int(L.c_rows[i]) // PAGE_SZ, (int(L.c_rows[i]) + rb - 1) // PAGE_SZ + 1)
            ids.append(t * Z + wp)
            home.append(wp)
        plan.append((np.asarray(T.round_events(r), np.uint64), rows,
                     np.concatenate(ids).astype(np.uint32), np.concatenate(home).astype(np.uint32)))
    z = img.copy().reshape(-1)
    f64 = z.view("<f8")
    for i in range(ndim):
        o = int(L.c_rows[i]) // 8
        f64[o:o + ndim] = c_row_values(L, i)

    def fresh():
        cur = np.tile(img, (nodes, 1))
        st, fl = oracle.coh_init(Z, nodes)
        return cur, cur.copy(), img.copy(), st, fl

    # 1. the round loop in C
    flat_plan = {
        "events": np.concatenate([p[0] for p in plan]),
        "ev_off": np.concatenate([[0], np.cumsum([len(p[0]) for p in plan])]).astype(np.uint64),
        "ids": np.concatenate([p[2] for p in plan]),
        "home": np.concatenate([p[3] for p in plan]),
        "ids_off": np.concatenate([[0], np.cumsum([len(p[2]) for p in plan])]).astype(np.uint64),
        "row_dst": np.array([t * Z * PAGE_SZ + int(L.c_rows[i]) for p in plan for t, i in p[1]],
                            np.uint64),
        "row_src": np.array([i for p in plan for _, i in p[1]], np.uint32),
        "row_off": np.concatenate([[0], np.cumsum([len(p[1]) for p in plan])]).astype(np.uint64),
    }
    # the trace is short (tens of ms): replayed from a fresh state until min_seconds of C time
    def c_loop(rt: bool, seconds: float):
        dt_c, reps, ok_c = 0.0, 0, True
        while (dt_c < seconds and reps < 500) or reps == 0:
            cur, twin, rep, st, fl = fresh()
            dt, _ = oracle.bench_mmult(st, fl, nodes, twin, cur, rep, flat_plan, rowvals,
                                       retwin=rt)
            dt_c += dt
            reps += 1
            ok_c = ok_c and bool(np.array_equal(rep.reshape(-1), z))
        return dt_c, reps, ok_c

    dt_c, reps, ok_c = c_loop(retwin, min_seconds)
    dt_o, reps_o, ok_o = c_loop(not retwin, min_seconds / 2)
    # 2. the same loop driven from Python, per round
    cur, twin, rep, st, fl = fresh()
    flat = cur.reshape(-1)
    t0 = time.perf_counter()
    for ev, rows, ids, home in plan:
        oracle.coherence(st, fl, ev, n_nodes=nodes)
        twin[ids] = cur[ids]
        for t, i in rows:
            o = t * Z * PAGE_SZ + int(L.c_rows[i])
            flat[o:o + rb] = rowvals[i]
        ro, data = oracle.diff_pages(twin, cur, ids, cap=len(ids) * 10244)
        oracle.apply(rep, ro, data, home)
    dt_py = time.perf_counter() - t0
    ok_py = bool(np.array_equal(rep.reshape(-1), z))
    return {"value": round(reps * T.rounds / dt_c, 1), "unit": "rounds/s", "cores": 1,
            "kind": "port",
            "sample": f"the whole NDIM={ndim} trace ({T.rounds} rounds, {nodes} nodes) replayed "
                      f"{reps} times from a fresh state through the C oracle (coherence, "
                      + ("row writes, diff, apply, re-twin of the dirty bytes (the stream "
                         "applied to the twin views, as gdsm_release)" if retwin else
                         "twin, row writes, diff, apply")
                      + f"), the round loop in C over a precomputed plan (or_bench_mmult), "
                        f"{dt_c:.3f} s timed in C",
            "twin_workflow": "re-twin after the diff" if retwin else "twin before the writes",
            "other_twin_workflow": {
                "twin_workflow": "twin before the writes" if retwin else "re-twin after the diff",
                "value": round(reps_o * T.rounds / dt_o, 1), "unit": "rounds/s",
                "home_copy_equals_product": ok_o},
            "timed_in": "C (CLOCK_MONOTONIC)",
            "python_driven": {"value": round(T.rounds / dt_py, 1), "unit": "rounds/s",
                              "note": "the same loop with Python numpy/ctypes per round "
                                      "(round 4's figure)", "seconds": round(dt_py, 4),
                              "home_copy_equals_product": ok_py},
            "home_copy_equals_product": ok_c and ok_py and ok_o, **host_info()}


def run_mmult_ranks(args, rank: int, world: int):
    """BASELINE configs[4] at N > 1: one process (GPU) per DSM node of the trace
    (gallocy_amd.replay.MmultRankReplay): each node's fault events routed to the page-table shards
    at the homes and the access-change notices returned (gdsm_route_events /
    gdsm_coherence_notify), the per-round diffs shipped to the home GPUs with gdsm_exchange, all
    over RCCL. Strong scaling: the same NDIM = 1000 product. (Several ranks on one GPU are
    rehearsed by tests/test_gpu_replay.py with the loopback communicator.)"""
    import torch
    import torch.distributed as dist

    from gallocy_amd.replay import MmultRankReplay
    if os.environ.get("GDSM_BENCH_BACKEND", "nccl") != "nccl":
        raise SystemExit("--workload mmult at N > 1 runs on RCCL only")
    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    watchdog(args, rank, world, "setup and run")
    R = MmultRankReplay(rank, world, ndim=args.ndim, seed=args.seed, device=local)
    dist.barrier()
    dt = R.run()
    ok = torch.tensor([1 if np.array_equal(R.home_block(), R.final_block()) else 0],
                      dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    tot = torch.tensor(R.totals.tolist(), dtype=torch.int64)
    dist.all_reduce(tot)
    ev = torch.tensor([R.events_total, R.pages_diffed], dtype=torch.int64)
    dist.all_reduce(ev)
    if rank == 0:
        res = {"metric": "mmult trace replay rounds/sec", "value": round(R.T.rounds / dt, 1),
               "unit": "rounds/s", "n_gpus": world, "steps": R.T.rounds, "warmup": 0,
               "ms_per_step": round(dt / R.T.rounds * 1e3, 4), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "u8/u64",
               "data": "test_mmult trace from the reference heap layout (gallocy_amd/trace.py)",
               "config": {"workload": f"NDIM={args.ndim}, {world} DSM nodes = {world} GPUs, "
                                      f"{R.Z} zone pages, events routed to page-table shards + notices back + "
                                      f"diff exchange, RCCL",
                          "rows": args.ndim, "events": int(ev[0]), "pages_diffed": int(ev[1])},
               "seconds_total": round(dt, 4), "rows_per_s": round(args.ndim / dt, 1),
               "home_copy_equals_product": bool(ok.item()),
               "totals": {"invalidations": int(tot[0]), "transfers": int(tot[1]),
                          "node_faults": [int(x) for x in tot[2:]]}}
        print(json.dumps(res), flush=True)
    R.close()
    dist.barrier()
    dist.destroy_process_group()


def run_mmult(args):
    """BASELINE configs[4]: the test_mmult trace (reference heap layout, NDIM=1000) replayed end
    to end: per round one coherence batch + twin/write/diff/apply of every row written. One GPU
    simulates --nodes nodes; under torch.distributed.run every rank is one node on its own GPU
    (run_mmult_ranks)."""
    import torch

    from gallocy_amd.replay import MmultReplay
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        return run_mmult_ranks(args, int(os.environ.get("RANK", "0")), world)
    torch.cuda.set_device(0)
    if args.driver == "device" and (args.graph or args.retwin == "off"):
        args.driver = "native"  # (gdsm_rounds runs the re-twinning release, eagerly)
    # warmup: with --warmup W > 0, one untimed replay of the whole trace on a fresh state first
    # (the kernels' code objects loaded and the host paths warm: a cold first replay in a fresh
    # process takes ~1.5x as long per round); the timed replay starts from a fresh state again
    warm_rounds = 0
    def replay(driver):
        return MmultReplay(ndim=args.ndim, nodes=args.nodes, seed=args.seed,
                           retwin=args.retwin == "on", driver=driver)

    if args.warmup > 0:
        R0 = replay(args.driver)
        R0.run(graph=args.graph)
        warm_rounds = R0.T.rounds
        R0.close()
    R = replay(args.driver)
    dt = R.run(graph=args.graph)
    # the same replay (warm, fresh state) with every round issued from Python, reported beside
    other = None
    if not args.graph and args.driver != "python":
        R3 = replay("python")
        dt3 = R3.run()
        ok3 = bool(np.array_equal(R3.home_copy(), R3.final_image()))
        R3.close()
        other = {"value": round(R.T.rounds / dt3, 1), "unit": "rounds/s",
                 "note": "the same warm replay with each round's calls issued from Python "
                         "(MmultReplay.round, ~1 us of interpreter per call)",
                 "home_copy_equals_product": ok3}
    # the other C++/device issue mode on the same box, same warm state: the per-round calls of the
    # C++ loop against gdsm_rounds (every round in one persistent launch per context)
    alt = None
    if not args.graph and args.driver in ("native", "device") and args.retwin == "on":
        other_driver = "device" if args.driver == "native" else "native"
        R4 = replay(other_driver)
        dt4 = R4.run()
        ok4 = bool(np.array_equal(R4.home_copy(), R4.final_image()))
        R4.close()
        alt = {"driver": other_driver, "value": round(R.T.rounds / dt4, 1), "unit": "rounds/s",
               "home_copy_equals_product": ok4}
    ok = bool(np.array_equal(R.home_copy(), R.final_image()))
    # latency breakdown: the same replay again on a fresh state with per-launch HIP events (a
    # separate run, so the events do not weigh on `value`)
    R2 = replay(args.driver)
    R2.data.prof_enable(True)
    R2.pt.prof_enable(True)
    dt2 = R2.run(graph=False)
    pd, pp = R2.data.prof_read(), R2.pt.prof_read()
    R2.close()
    rounds = R.T.rounds
    stages = {}
    for k, v in list(pd.items()) + list(pp.items()):
        if v[1]:
            stages[k] = {"ms_per_launch": round(v[0] / v[1], 5),
                         "launches_per_round": round(v[1] / rounds, 2)}
    kern_ms = sum(v[0] for v in pd.values()) + sum(v[0] for v in pp.values())
    launches = sum(v[1] for v in pd.values()) + sum(v[1] for v in pp.values())
    copies = sum(len(R.rows[r]) for r in range(rounds))  # rows written per round
    device = args.driver == "device"
    latency = {"bound": "latency",
               "kernel_launches_per_round": round(launches / rounds, 4),
               "copy_launches_per_round": 0 if device else 1,
               "rows_written_per_round": round(copies / rounds, 2),
               "host_syncs_per_round": 0,
               "kernel_ms_per_round": round(kern_ms / rounds, 5),
               "wall_ms_per_round_profiled": round(dt2 / rounds * 1e3, 5),
               "stages": stages,
               "note": ("a round is ~10 dense pages (~500 runs each) and ~8000 fault events: "
                        "every operation is a few microseconds of dependent latency. "
                        + ("gdsm_rounds: two launches for the whole trace (stages: ms per launch "
                           "= all rounds), a round is the longer of the page-data loop (the "
                           "release with the round's writes laid on, then a device barrier) and "
                           "the page-table loop (the fold, then a device barrier)" if device else
                           "The round is the longer of two streams (page data: the row writes' "
                           "batched copy, then one release launch that diffs, applies to the "
                           "home copies and re-twins; page table: one coherence fold launch) or "
                           "the host's issue time for the three calls")
                        + ". No HBM or MFMA roofline applies.")}
    res = {"metric": "mmult trace replay rounds/sec", "value": round(R.T.rounds / dt, 1),
           "unit": "rounds/s", "n_gpus": 1, "steps": R.T.rounds, "warmup": warm_rounds,
           "ms_per_step": round(dt / R.T.rounds * 1e3, 4), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u8/u64",
           "data": "test_mmult trace from the reference heap layout (gallocy_amd/trace.py)",
           "config": {"workload": f"NDIM={args.ndim}, {args.nodes} simulated nodes, "
                                  f"{R.Z} zone pages", "rows": args.ndim,
                      "events": R.events_total, "pages_diffed": R.pages_diffed},
           "seconds_total": round(dt, 4),
           "launch": f"one HIP graph of every round (recorded in {R.graph_build_s:.2f} s, untimed)"
                     if args.graph else ("eager, two streams, rounds issued by the C++ loop over "
                                         "the C ABI (gallocy_amd/native/replay.cpp)"
                                         if args.driver == "native" else
                                         "eager, two streams, rounds issued by two C++ threads, one "
                                         "per context (gallocy_amd/native/replay.cpp)"
                                         if args.driver == "native2" else
                                         "one persistent launch per stream for every round "
                                         "(gdsm_rounds), a device-wide barrier between rounds"
                                         if args.driver == "device" else
                                         "eager, two streams, rounds issued from Python"),
           "python_rounds": other,
           "driver": args.driver,
           "other_driver_rounds": alt,
           "round": ("coherence batch | the round's row writes (one batched copy), the release "
                     "applying its runs to the home copies and re-twinning its pages "
                     "(gdsm_release)") if args.retwin == "on" else
                    ("coherence batch | twin, the round's row writes (one batched copy), diff "
                     "applying its runs to the home copies (gdsm_diff_apply_ids)"),
           "events_per_s": round(R.events_total / dt, 1),
           "rows_per_s": round(args.ndim / dt, 1),
           "home_copy_equals_product": ok,
           "totals": {"invalidations": int(R.totals[0]), "transfers": int(R.totals[1]),
                      "node_faults": [int(x) for x in R.totals[2:]]},
           "roofline": None, "latency": latency,
           "cpu_baseline": None if args.no_cpu else mmult_cpu_baseline(args.ndim, args.nodes,
                                                                       args.seed,
                                                                       retwin=args.retwin == "on")}
    print(json.dumps(res), flush=True)
    R.close()


VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9  # lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes/clk (MICROARCH)
NW_OPS_PER_CELL = 3.5  # 28 VALU per step of 8 cells: gdsm_nw.hip fill_block (cmp, addc, max3 per cell)


def run_nw(args):
    """The reference diff() (gallocy/utils/diff.cpp:73-167) on the GPU: a batch of 4 KiB page
    pairs (twin, current with 1 % of 8-byte words rewritten: BASELINE configs[0]'s shape, which
    the reference itself cannot align: it crashes from 1181 bytes) through gdsm_nw_diff_batch.
    A step = one batch: DP fill + traceback + alignment strings. VALU-bound (no HBM or MFMA
    roofline applies: 2 bits of traceback per cell are the only HBM traffic). N > 1 GPUs:
    replicas only (every rank aligns its own batch; nothing is exchanged), weak scaling."""
    import torch

    import gallocy_amd as ga
    from gallocy_amd import _lib
    rank, world, local = ranks_setup(args)
    n, ln = args.nw_pairs, 4096
    rng = np.random.default_rng(args.seed + rank)
    a = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    b = a.copy()
    b.reshape(n, -1, 8)[rng.random((n, ln // 8)) < 0.01] ^= 0x5A
    off = np.arange(n + 1, dtype=np.uint64) * ln
    ctx = ga.Context(1, arenas=(), device=local)
    da, doff, db = (ctx.buffer(x.nbytes).upload(x) for x in (a, off, b))
    ob = 2 * n * ln + n
    o1, o2, ol = ctx.buffer(ob), ctx.buffer(ob), ctx.buffer(8 * n)
    L = _lib.load()

    def step():
        _lib.check(L.gdsm_nw_diff_batch(ctx.handle, da.ptr, doff.ptr, db.ptr, doff.ptr, n, ln,
                                        o1.ptr, o2.ptr, ol.ptr), "gdsm_nw_diff_batch")

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier(world)
    ctx.prof_enable(True)
    ctx.prof_read()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world)
    prof = ctx.prof_read()
    cells = n * (ln + 1) ** 2
    fill_ms = max_over_ranks(prof["nw_fill"][0] / max(1, prof["nw_fill"][1]), world)
    # spot check against the oracle (first pair)
    from oracle import oracle
    L0 = int(ol.download(np.uint64, 1)[0])
    g1 = o1.download(np.uint8, L0)
    want = oracle.nw_diff(a[0].tobytes(), b[0].tobytes())
    assert g1.tobytes() == want[0], "GPU alignment differs from the oracle"
    if rank != 0:
        ctx.close()
        barrier(world)
        return
    achieved = cells * NW_OPS_PER_CELL / (fill_ms * 1e-3) / 1e12
    peak = VALU_PEAK_OPS / 1e12
    stages = {k: {"ms_per_launch": round(v[0] / v[1], 4), "launches": v[1]}
              for k, v in prof.items() if v[1]}
    res = {"metric": "NW alignment DP cells/sec (reference diff() on GPU)",
           "value": round(world * cells * args.steps / dt, 1), "unit": "cells/s",
           "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "i32",
           "data": "synthetic 4 KiB page pairs, 1 % of 8-byte words rewritten",
           "config": {"workload": f"{n} pairs x 4096 x 4096 bytes per GPU, diff() alignment"
                                  + (f", {world} replicas" if world > 1 else ""),
                      "pairs_per_s": round(world * n * args.steps / dt, 1)},
           "roofline": {"bound": "valu", "kernel": "gdsm::nw_fill_kernel",
                        "achieved": round(achieved, 2), "peak": round(peak, 1),
                        "unit": "Tops/s", "frac": round(achieved / peak, 4), "traffic": None,
                        "ops_per_cell": NW_OPS_PER_CELL, "cells_per_launch": cells,
                        "avg_launch_ms": round(fill_ms, 4)},
           "stages": stages, "cpu_baseline": None}
    if not args.no_cpu and world == 1:
        base = {}
        drv = oracle.REF_DRIVER
        if drv.exists():
            r = subprocess.run([str(drv), "time", "1024", "3"], capture_output=True, text=True,
                               timeout=120, check=True).stdout.split()
            s, c = float(r[0]), int(r[1])
            base = {"value": round(c / s, 1), "unit": "cells/s", "cores": 1,
                    "kind": "reference",
                    "sample": "reference diff() compiled -O0 from its sources (oracle/_ref), "
                              "1024 x 1024 bytes (its largest size before the 1181-byte crash), "
                              f"{s:.3f} s per call"}
        reps, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < min(args.cpu_seconds, 5.0) or reps == 0:
            oracle.nw_diff(a[reps % n].tobytes(), b[reps % n].tobytes())
            reps += 1
        ct = time.perf_counter() - t1
        port = {"value": round(reps * (ln + 1) ** 2 / ct, 1), "unit": "cells/s", "cores": 1,
                "kind": "port", "sample": f"{reps} 4 KiB pairs through oracle or_nw_diff"}
        res["cpu_baseline"] = base or port
        if base:
            res["cpu_baseline"]["oracle_port"] = port
    print(json.dumps(res), flush=True)
    ctx.close()
    barrier(world)


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: this GPU-free parent starts the N ranks itself
    (torch.distributed.run on 127.0.0.1, one process per GPU), before anything touches a GPU,
    and returns their exit code; rank 0's JSON line goes to this process's stdout. Under a
    launcher (WORLD_SIZE set) --gpus must equal the rank count. None: run here as one rank."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} "
                             f"ranks (WORLD_SIZE)")
        return None
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus == 1:
        return None
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           str(ROOT / "bench.py"), *sys.argv[1:]]
    log("bench.py: launching", args.gpus, "ranks:", " ".join(cmd[2:]))
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.workload == "coherence":
        return run_coherence(args)
    if args.workload == "nw":
        return run_nw(args)
    if args.workload == "mmult":
        return run_mmult(args)
    if args.workload == "twin":
        return run_twin(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    # The control plane (barriers, max-over-ranks time, the RCCL unique id) runs over gloo; the
    # page data goes GPU to GPU over RCCL inside libgdsm (gdsm_exchange). GDSM_BENCH_BACKEND=gloo:
    # REHEARSAL ONLY of the N > 1 step (several ranks may share one GPU, the records go through
    # host memory); the line it prints is not a measurement.
    backend = os.environ.get("GDSM_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit("GDSM_BENCH_BACKEND must be nccl or gloo")
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    elif local >= torch.cuda.device_count():
        # RCCL takes one rank per GPU ("Duplicate GPU detected" otherwise)
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local}, but {torch.cuda.device_count()} "
                         f"GPU(s) are visible: --gpus N runs one rank per GPU over RCCL "
                         f"(GDSM_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs)")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")
        watchdog(args, rank, world, "setup: communicator and the first release")
    import gallocy_amd as ga
    from gallocy_amd import exchange

    scaling, mode_name, ppm, n = workload_shape(args, world)
    mode = ga.GEN_UNIFORM if mode_name == "uniform" else ga.GEN_CLUSTERED
    ctx = ga.Context(n, device=local)
    # writer(p) = p mod G, home(p) = p // n (gallocy_amd/exchange.py); N = 1 is the identity
    ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=rank, stride=world,
                  arenas=("twin", "current"))
    ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=rank * n, stride=1,
                  arenas=("replica",))
    # stream bytes per page reserved (uniform 1 %: ~66 B records; <= 128 B per page lets the
    # diff take 64 pages per wave, gdsm_pages.hip diff_variant)
    cap_pp = 128 if mode == ga.GEN_UNIFORM else 1024
    shard = None
    if world > 1:
        shard = exchange.Shard(ctx, rank, world, n, cap_pp,
                               transport="gloo" if backend == "gloo" else "rccl")
        runs = None
    else:
        # Two diff streams: release k+1 may be diffed while release k is applied
        runs = [ga.Runs(ctx, n, cap=n * cap_pp) for _ in range(2)]

    # this box's read and copy ceilings over the shard's own arenas (REPLICA is the copy's
    # destination, then generated again)
    box = box_ceilings(ctx, n, read=(ctx.arena_ptr("twin"), ctx.arena_ptr("current")),
                       copy=(ctx.arena_ptr("current"), ctx.arena_ptr("replica")))
    ctx.gen_pages(seed=args.seed, mode=mode, ppm=ppm, first_global=rank * n, stride=1,
                  arenas=("replica",))

    def steps(k: int, pipelined: bool):
        if shard is not None:
            shard.run(k, pipelined)
            return
        for i in range(k):
            r = runs[i % 2] if pipelined else runs[0]
            if fused:
                ctx.diff(out=r, apply_to="replica")
                continue
            ctx.diff(out=r)
            (ctx.apply_async if pipelined else ctx.apply)(r)

    def drain():
        if shard is not None:
            shard.drain()
        ctx.sync()

    pipelined = args.overlap == "on" or (args.overlap == "auto" and world > 1)
    fused = shard is None and args.fuse == "on" and not pipelined
    if shard is not None:
        # release 0 with exact sizes (one host read), then fixed byte budgets: no host sync
        shard.run(1, pipelined=False)
        drain()
        if shard.transport == "rccl":
            shard.calibrate()
        steps(max(0, args.warmup - 1), pipelined)
        total = sum(r.total() for d, r in enumerate(shard.send[0]) if shard.counts[d])
        host = None
        pay = 0
        for d, r in enumerate(shard.send[0]):
            if shard.counts[d]:
                h = r.to_host()
                pay += payload_bytes(h.rec_off, h.data)
    else:
        steps(args.warmup, pipelined)
        total = runs[0].total()  # raises ENOSPC if the capacity was too small
        assert not pipelined or args.warmup < 2 or runs[1].total() == total
        host = runs[0].to_host()
        pay = payload_bytes(host.rec_off, host.data)
    drain()
    del host

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(pipelined: bool, prof: bool):
        barrier()
        drain()
        torch.cuda.synchronize()
        barrier()
        if prof:
            ctx.prof_enable(True)
        t0 = time.perf_counter()
        steps(args.steps, pipelined)
        drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        p = ctx.prof_read() if prof else None
        if prof:
            ctx.prof_enable(False)
        dt = t1 - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, p

    # optionally the other mode first, for reference, then the measured run (same K steps); by
    # default only the measured mode runs, so a rocprofv3 summary of this command averages the
    # same launches the HIP events time
    watchdog(args, rank, world, "timed releases")
    dt_other = timed(not pipelined, False)[0] if args.compare_overlap else None
    dt, prof = timed(pipelined, True)
    watchdog(args, rank, world, "link timing")
    # The xGMI link alone: the same releases again (untimed for `value`) with GDSM_XCHG_TIMED, a
    # device-side barrier before each transfer, so the exchange stage starts once every rank's
    # streams are ready and times the RCCL group, not the wait for the peers' diffs.
    link = None
    if shard is not None and shard.comm is not None:
        shard.flags |= exchange.XCHG_TIMED
        try:
            _, plink = timed(pipelined, True)
        finally:
            shard.flags &= ~exchange.XCHG_TIMED
        link = [plink["exchange"][0] / args.steps, plink["exchange_wait"][0] / args.steps]
        watchdog(args, rank, world, "link timing: the stats all-reduce")
        t = torch.tensor(link, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        link = t.tolist()

    # correctness of the measured work: REPLICA == CURRENT afterwards (diff of the two is empty)
    watchdog(args, rank, world, "verification and the stats all-reduces")
    if shard is None:
        chk = ga.Runs(ctx, n, cap=1 << 20)
        ws = ctx.buffer(ga.gdsm.lib().gdsm_diff_workspace_bytes(n))
        rc = ga.gdsm.lib().gdsm_diff_raw(ctx.arena_ptr("replica"), ctx.arena_ptr("current"), None,
                                         n, chk.s.rec_off, chk.s.data, chk.cap, ws.ptr, ws.nbytes,
                                         ctx.stream)
        replica_ok = rc == 0 and chk.total() == 0
    else:
        replica_ok = shard.verify(args.seed, mode, ppm)
        t = torch.tensor([1 if replica_ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)  # every rank's home block, one flag
        replica_ok = bool(t.item())

    # The diff runs as one launch per destination per step: bytes per launch and time per launch
    # are both averaged over the step's launches.
    diff_ms, diff_launches = prof["diff"]
    avg_diff_ms = diff_ms / max(1, diff_launches)
    per_step = max(1, diff_launches // args.steps)
    # algorithmic per launch: twin + current read, records written (+ the payload bytes stored
    # to the home copy when the apply is fused into the diff)
    diff_bytes = (n * 8192 + total + (pay if fused else 0)) / per_step
    achieved = diff_bytes / (avg_diff_ms * 1e-3) / 1e9
    # B_page summed; the fused step does not read the stream back
    step_bytes = n * 8192 + (1 if fused else 2) * total + pay
    ms_step = dt / args.steps * 1e3
    value = world * n * args.steps / dt
    traffic, traffic_src = read_traffic(n, mode_name, ppm, fused)

    # per-stage time per step, max over ranks (HIP events on the stream each stage runs on)
    stage_ms = {k: prof[k][0] / args.steps for k in ("diff", "exchange", "apply")}
    if world > 1:
        t = torch.tensor([stage_ms[k] for k in ("diff", "exchange", "apply")], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        stage_ms = dict(zip(("diff", "exchange", "apply"), t.tolist()))
    xgmi = None
    if link is not None and link[0] > 0:
        moved = shard.moved_remote  # bytes this rank's exchange hands the transport per step
        ach = moved / (link[0] * 1e-3) / 1e9
        peak_node, peak_used = 7 * XGMI_LINK_GBS, (world - 1) * XGMI_LINK_GBS
        xgmi = {"bound": "xgmi", "achieved": round(ach, 2), "unit": "GB/s",
                "peak": peak_node, "frac": round(ach / peak_node, 4),
                "peak_links_used": peak_used, "frac_links_used": round(ach / peak_used, 4),
                "bytes_per_step": int(moved),
                "link_ms_per_step": round(link[0], 4),
                "exchange_ms_incl_wait": round(stage_ms["exchange"], 4),
                "timed_run_exchange_ms_incl_wait": round(link[1], 4),
                "note": "bytes one rank sends to its N-1 peers per step (rec_off + page indices + "
                        "the byte budget of each stream) / link_ms_per_step: the RCCL group's "
                        "time on the exchange stream (HIP events, max over ranks) in a second run "
                        "of the same K releases with GDSM_XCHG_TIMED, where a one-word device "
                        "all-to-all before each transfer makes it start once every rank's "
                        "streams are ready. exchange_ms_incl_wait: the measured run's exchange "
                        "stage, which includes waiting for the peers' diffs. peak: 7 links x 153 "
                        "GB/s (all of an MI355X's xGMI); peak_links_used: the N-1 links one "
                        "rank's peers use"}
    ref_ms, ref_src = efficiency_ref(world * n, mode_name, ppm) if world > 1 else (None, None)
    exch = None if shard is None else {
        "transport": shard.transport, "fixed_budgets": bool(shard.flags),
        "comm_ranks": shard.comm.size()[0] if shard.comm is not None else None,
        "recoveries": shard.recoveries,
        "sent_remote_bytes_per_step": shard.sent_remote,
        "received_bytes_per_step": shard.received}
    same = None
    if world > 1 and args.same_run_ref == "on":
        # the N-rank run's arenas and communicator go first, then rank 0 alone runs the N = 1
        # step of the same total workload (the other ranks wait at the barrier)
        watchdog(args, rank, world, "teardown of the N-rank run")
        shard.close()
        shard = None
        ctx.close()
        ctx = None
        barrier()
        watchdog(args, rank, world, "the same-run N = 1 reference")
        if rank == 0:
            same = n1_reference(args, world * n, mode, ppm, local)
            if "ms_per_step" in same:
                same["efficiency"] = round(same["ms_per_step"] / (world * ms_step), 4)
            same["note"] = ("rank 0 alone, after the N-rank run and its teardown: the N = 1 step "
                            "(diff + apply of all pages on one GPU) of the same total workload; "
                            "efficiency = ms_per_step(N = 1) / (N x ms_per_step(N))")
        barrier()

    if rank == 0:
        stages = {k: {"ms_per_launch": round(v[0] / v[1], 4), "launches": v[1]}
                  for k, v in prof.items() if v[1]}
        if scaling == "strong":
            workload = (f"{world * n} x 4 KiB pages in all, {n} per GPU, {mode_name} "
                        f"{ppm / 1e4:g}% {'8-B word' if mode == ga.GEN_UNIFORM else '64-B cluster'}"
                        f" writes, diff+apply" + (", RCCL exchange to home GPUs" if world > 1 else ""))
        else:
            workload = (f"{n} x 4 KiB pages per GPU, {mode_name} {ppm / 1e4:g}% "
                        f"{'8-B word' if mode == ga.GEN_UNIFORM else '64-B cluster'} writes, "
                        f"diff+apply" + (", RCCL exchange to home GPUs" if world > 1 else ""))
        res = {
            "metric": "pages diffed+applied/sec (4 KiB)",
            "value": round(value, 1),
            "unit": "pages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-hash pages, docs/SPEC.md §6)",
            "config": {"workload": workload, "config": args.config, "mode": mode_name,
                       "ppm": ppm, "pages_per_gpu": n, "total_pages": world * n,
                       "seed": args.seed, "parallelism": f"page-shard x{world}",
                       "diff_bytes_per_step": int(total), "payload_bytes_per_step": int(pay),
                       **({"backend": "gloo (REHEARSAL, not a measurement)"}
                          if world > 1 and backend == "gloo" else {})},
            "step_hbm_gbs": round(step_bytes * args.steps / dt / 1e9, 1),
            "pipelined": pipelined,
            "fused_apply": fused,
            ("serial_ms_per_step" if pipelined else "pipelined_ms_per_step"):
                None if dt_other is None else round(dt_other / args.steps * 1e3, 4),
            "roofline": with_box({"bound": "hbm", "kernel": DIFF_KERNEL,
                                  "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                  "traffic": traffic, "traffic_source": traffic_src,
                                  "algorithmic_bytes_per_launch": int(diff_bytes),
                                  "avg_launch_ms": round(avg_diff_ms, 4)}, box, "read"),
            "step_frac_of_box_read": round(step_bytes * args.steps / dt / 1e9
                                           / box["box_read_gbs"], 4),
            "stages": stages,
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
            "exchange": exch,
            **({"roofline_xgmi": xgmi} if xgmi else {}),
            **({"efficiency_ref_ms": ref_ms, "efficiency_ref_source": ref_src,
                "efficiency_same_run": None if same is None else same.get("efficiency"),
                "same_run_reference": same}
               if world > 1 else {}),
            "replica_equals_current": bool(replica_ok),
            "cpu_baseline": None,
        }
        if not args.no_cpu and world == 1:  # the host baseline is a 1-GPU figure (rank 0, N = 1)
            res["cpu_baseline"] = cpu_baseline(mode, ppm, args.seed, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    watchdog(args, rank, world, "teardown")
    if shard is not None:
        shard.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if ctx is not None:
        ctx.close()
    if WATCHDOG is not None:
        WATCHDOG.disarm()


if __name__ == "__main__":
    main()
