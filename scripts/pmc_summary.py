"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel,
with the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB)
reports exactly half of a wide coalesced streaming read, so it is doubled; WRITE_SIZE (KB) is
exact for 16-B-per-lane streaming stores.
Usage: pmc_summary.py <fetch.csv> <write.csv> <out.json> [<source text> [<workload json>]]
       pmc_summary.py <fetch.csv> <write.csv> <out.json> <source text> <kernel prefix> <workload json>
(defaults: the config-2 bench workload and its diff kernel)."""
import csv
import json
import sys
from collections import defaultdict


LAUNCHES = {}


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        LAUNCHES[k] = max(LAUNCHES.get(k, 0), len(v))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
source = (sys.argv[4] if len(sys.argv) > 4 else
          "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, "
          "bench.py --steps 5 --warmup 1 --no-cpu (1M pages, 1% word writes)")
out = {"source": source,
       "correction": "hbm_bytes = 2 * FETCH_SIZE_KB * 1024 + WRITE_SIZE_KB * 1024 (gfx950)",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    out["kernels"][k] = {"fetch_kb_raw": f, "write_kb": w, "launches": LAUNCHES.get(k, 0),
                         "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
def most_launched(prefix):
    """The kernel of this family the run launched most (the timed one, not a warm-up variant)."""
    ks = [k for k in out["kernels"] if k.startswith(prefix)]
    return max(ks, key=lambda k: out["kernels"][k]["launches"]) if ks else None


if len(sys.argv) > 6:
    # another workload's main kernel (e.g. the coherence fold), keyed like bench.py reads it
    k = most_launched(sys.argv[5])
    if k:
        out["main_kernel"] = k
        out["main_kernel_bytes_per_launch"] = out["kernels"][k]["hbm_bytes_per_launch"]
    out["workload"] = json.loads(sys.argv[6])
else:
    # the diff kernel the bench runs (and its workload, when given as argv[5])
    k = most_launched("gdsm::diff_single_kernel")
    if k:
        out["diff_kernel"] = k
        out["diff_kernel_bytes_per_launch"] = out["kernels"][k]["hbm_bytes_per_launch"]
    if len(sys.argv) > 5:
        out["workload"] = json.loads(sys.argv[5])
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
