"""Config 5 with one process per DSM node (gallocy_amd.replay.MmultRankReplay), launched with
torch.distributed.run; TEST / REHEARSAL DRIVER (uses the C oracle as the checker). Rank 0 prints
one JSON line: ok = every home block equals the product zone, every page-table shard equals the
oracle's fold of the whole trace on its pages, and the totals summed over ranks equal the
oracle's.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \\
        scripts/rank_replay.py --ndim 1000

One GPU per rank (RCCL); several ranks on one GPU: tests/test_gpu_replay.py (loopback)."""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--transport", choices=["rccl"], default="rccl")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from gallocy_amd.replay import MmultRankReplay
    from oracle import oracle
    R = MmultRankReplay(rank, world, ndim=a.ndim, seed=a.seed, device=dev, transport=a.transport)
    try:
        dt = R.run()
        ok = bool(np.array_equal(R.home_block(), R.final_block()))
        st, fl = oracle.coh_init(R.Z, world)
        acc = np.zeros(10, np.int64)
        for r in range(R.T.rounds):
            rc, t, want = oracle.route_round(st, fl, R.T.round_stamped(r), world, R.Z)
            ok &= rc == 0 and bool(np.array_equal(R.notices_of(r), want[rank]))
            acc += [t["invalidations"], t["transfers"], *t["node_faults"]]
        t = {"invalidations": int(acc[0]), "transfers": int(acc[1]),
             "node_faults": [int(x) for x in acc[2:]]}
        if R.nh:
            gst, gfl = R.pt.coh_download()
            ok &= bool(np.array_equal(gst[:R.nh], st[R.base:R.base + R.nh]))
            ok &= bool(np.array_equal(gfl[:R.nh], fl[R.base:R.base + R.nh]))
        tot = torch.tensor(R.totals.tolist(), dtype=torch.int64)
        dist.all_reduce(tot)
        ok &= tot.tolist() == [t["invalidations"], t["transfers"], *t["node_faults"]]
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        tdt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tdt, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps({"ok": bool(flag.item()), "ranks": world, "ndim": a.ndim,
                              "rounds": R.T.rounds, "seconds": round(float(tdt.item()), 4),
                              "transport": a.transport}), flush=True)
    finally:
        R.close()
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
