#!/bin/bash
# rocprofv3 PMC passes (one per counter group) over coherence pass C variants 0 and 1.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/cohpmc
mkdir -p $OUT
for v in ${COH_PMC_VARIANTS:-0 4}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d $OUT/a$v -o a --output-format csv -- python3 scripts/coh_pmc.py 268435456 uniform $v > $OUT/a$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace -d $OUT/b$v -o b --output-format csv -- python3 scripts/coh_pmc.py 268435456 uniform $v > $OUT/b$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/cohpmc/*/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "coh_apply" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: sum(v) / len(v) for k, v in acc.items()})
PY
