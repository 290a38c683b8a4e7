"""How much of the coherence fold's time is waiting for its event loads? The fold kernel timed on
batches small enough to stay in the 256 MB Infinity Cache after a first pass (warm: the events
and most page-table words come from MALL/L2) against the same per-event cost on BASELINE
config 4's 1B-event batch (cold: every event from HBM). Uniform pages, 8 nodes, 20 % writes;
the page table is re-initialised before each batch, events per page held at config 4's 64.

    python scripts/dev/coh_warm_probe.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import gallocy_amd as ga  # noqa: E402
from gallocy_amd.workloads import event_counts  # noqa: E402


def fold_ms(n_ev, reps=5):
    pages = max(1, n_ev // 64)
    ctx = ga.Context(pages, arenas=())
    ev = ctx.gen_events(event_counts(pages, n_ev, "uniform", seed=2026), seed=2026, n_nodes=8,
                        write_pct=20)
    ga.gdsm.lib().gdsm_tune(b"coh_variant", 2)  # the single-pass fold at every size
    out = []
    for _ in range(reps):
        ctx.coh_init(8)
        ctx.prof_enable(True)
        ctx.coherence_batch(ev)
        p = ctx.prof_read()
        ctx.prof_enable(False)
        out.append(p["coh_fold"][0] / p["coh_fold"][1])
    ga.gdsm.lib().gdsm_tune(b"coh_variant", 0)
    ctx.close()
    return out


def main():
    for n_ev in (1 << 22, 1 << 23, 1 << 24, 1 << 25, 1 << 30):
        t = fold_ms(n_ev)
        best = min(t[1:])
        print(json.dumps({"events": n_ev, "bytes": 8 * n_ev, "fold_ms": [round(x, 4) for x in t],
                          "ns_per_1k_events_warm": round(best * 1e6 / (n_ev / 1000), 3),
                          "eff_TBps": round(8 * n_ev / (best * 1e-3) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
