"""Is config 5's replay bound by the host issuing its launches? The eager replay timed three ways
on fresh states: issue time of the whole round loop (no sync inside) against the time to the end
of the GPU work, and the host time spent in each call of a round (perf_counter around it).

    python scripts/dev/mmult_host_probe.py [nodes] [native]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from gallocy_amd import gdsm  # noqa: E402
from gallocy_amd.replay import MmultReplay  # noqa: E402


def native(nodes):
    """The C++ round loop: time until gdsm_replay_mmult returns (issue) and until both streams
    drain (end)."""
    import ctypes as C

    import numpy as np
    from gallocy_amd.replay import native_driver
    drv = native_driver()
    for rep in range(4):
        R = MmultReplay(ndim=1000, nodes=nodes, seed=1, retwin=True)
        R.data.sync()
        R.pt.sync()
        ev_off = np.ascontiguousarray(R.ev_off, np.int64)
        id_off = np.ascontiguousarray(R.id_off, np.int64)
        desc_off = np.ascontiguousarray(R.desc_off, np.int64)
        t0 = time.perf_counter()
        rc = drv.gdsm_replay_mmult(R.data.handle, R.pt.handle, 0, R.T.rounds, R.d_events.ptr,
                                   ev_off.ctypes.data, R.d_tot.ptr, R.d_ids.ptr, R.d_home.ptr,
                                   id_off.ctypes.data, R.d_desc.ptr, desc_off.ctypes.data,
                                   C.byref(R._runs.s), 1)
        t_issue = time.perf_counter() - t0
        R.data.sync()
        R.pt.sync()
        t_all = time.perf_counter() - t0
        assert rc == 0
        print(json.dumps({"driver": "native", "nodes": nodes, "rep": rep,
                          "issue_us_per_round": round(t_issue / R.T.rounds * 1e6, 2),
                          "end_us_per_round": round(t_all / R.T.rounds * 1e6, 2)}), flush=True)
        R.close()


def main():
    nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    if len(sys.argv) > 2 and sys.argv[2] == "native":
        return native(nodes)
    for rep in range(3):
        R = MmultReplay(ndim=1000, nodes=nodes, seed=1, retwin=True)
        R.data.sync()
        R.pt.sync()
        t0 = time.perf_counter()
        for r in range(R.T.rounds):
            R.round(r)
        t_issue = time.perf_counter() - t0
        R.data.sync()
        R.pt.sync()
        t_all = time.perf_counter() - t0
        rounds = R.T.rounds
        R.close()
        # per-call host time on another fresh state
        R = MmultReplay(ndim=1000, nodes=nodes, seed=1, retwin=True)
        lib = gdsm.lib()
        acc = [0.0, 0.0, 0.0]
        for r in range(R.T.rounds):
            e0, e1 = R.ev_off[r], R.ev_off[r + 1]
            a, b = int(R.id_off[r]), int(R.id_off[r + 1])
            d0, d1 = R.desc_off[r], R.desc_off[r + 1]
            t = time.perf_counter()
            lib.gdsm_coherence_batch_async(R.pt.handle, R.d_events.ptr + 8 * e0, e1 - e0,
                                           R.d_tot.ptr + 80 * r)
            t1 = time.perf_counter()
            lib.gdsm_memcpy_batch(R.data.handle, R.d_desc.ptr + 24 * d0, d1 - d0)
            t2 = time.perf_counter()
            R.data.release(R.d_ids.ptr + 4 * a, n=b - a, out=R._runs, apply_to="replica",
                           target_ids=R.d_home.ptr + 4 * a)
            t3 = time.perf_counter()
            acc[0] += t1 - t
            acc[1] += t2 - t1
            acc[2] += t3 - t2
        R.data.sync()
        R.pt.sync()
        R.close()
        print(json.dumps({"nodes": nodes, "rounds": rounds,
                          "issue_us_per_round": round(t_issue / rounds * 1e6, 2),
                          "end_us_per_round": round(t_all / rounds * 1e6, 2),
                          "host_us_per_call": {"coherence": round(acc[0] / rounds * 1e6, 2),
                                               "memcpy_batch": round(acc[1] / rounds * 1e6, 2),
                                               "release": round(acc[2] / rounds * 1e6, 2)}}),
              flush=True)


if __name__ == "__main__":
    main()
