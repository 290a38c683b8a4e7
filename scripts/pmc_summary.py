"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel,
with the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB)
reports exactly half of a wide coalesced streaming read, so it is doubled; WRITE_SIZE (KB) is
exact for 16-B-per-lane streaming stores.
Usage: pmc_summary.py <fetch.csv> <write.csv> <out.json> [<source text> <kernel prefix> <workload json>]
(defaults: the config-2 bench workload and its diff kernel)."""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name].append(float(r["Counter_Value"]))
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
    out["kernels"][k] = {"fetch_kb_raw": f, "write_kb": w,
                         "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
if len(sys.argv) > 6:
    # another workload's main kernel (e.g. coherence pass C), keyed like bench.py reads it
    for k, d in out["kernels"].items():
        if k.startswith(sys.argv[5]):
            out["main_kernel"] = k
            out["main_kernel_bytes_per_launch"] = d["hbm_bytes_per_launch"]
    out["workload"] = json.loads(sys.argv[6])
else:
    # the diff kernel the bench runs
    for k, d in out["kernels"].items():
        if k.startswith("gdsm::diff_single_kernel"):
            out["diff_kernel"] = k
            out["diff_kernel_bytes_per_launch"] = d["hbm_bytes_per_launch"]
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
