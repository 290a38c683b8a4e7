#!/bin/bash
# rocprofv3 PMC passes (one per counter group) over coherence variants (COH_PMC_VARIANTS);
# counts per 64 events.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/cohpmc
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_SMEM"
C="SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for v in ${COH_PMC_VARIANTS:-0}; do
  for d in ${COH_PMC_DISTS:-uniform}; do
    for p in a b c; do
      case $p in a) CT=$A;; b) CT=$B;; c) CT=$C;; esac
      timeout -s KILL 90 rocprofv3 --pmc $CT --kernel-trace -d $OUT/$p$v$d -o $p --output-format csv -- python3 scripts/dev/coh_pmc.py 268435456 $d $v > $OUT/$p$v$d.log 2>&1 || exit 1
    done
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/cohpmc/*/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "coh_stream_kernel" in r["Kernel_Name"] or "coh_fold_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per 64 events (2^28 events per batch)
    print(f.split("/")[2], {k: round(sum(v) / len(v) / 4194304, 2) for k, v in sorted(acc.items())})
PY
