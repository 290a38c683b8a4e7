#!/bin/bash
# rocprofv3 PMC passes over the nw bench (fill and trace kernels), averages per launch.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/nwpmc
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for p in a b; do
  case $p in a) CT=$A;; b) CT=$B;; esac
  timeout -s KILL 120 rocprofv3 --pmc $CT --kernel-trace -d $OUT/$p -o $p --output-format csv -- python3 bench.py --workload nw --steps 3 --warmup 1 --no-cpu > $OUT/$p.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/nwpmc/*/*counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = "fill" if "nw_fill" in r["Kernel_Name"] else "trace" if "nw_trace" in r["Kernel_Name"] else None
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f.split("/")[2], k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
