#!/bin/bash
# rocprofv3 PMC passes of the coherence fold for several libgdsm builds (A/B of fold forms):
# SQ counters per 64 events, one pass per counter group, config 4's batch (2^30 events over 16M
# pages). Usage: scripts/dev/coh_lib_pmc.sh OUT DIST LIB...
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
D=$2
shift 2
mkdir -p $OUT
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_SMEM"
C="SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
i=0
for L in "$@"; do
  for p in a b c; do
    case $p in a) CT=$A;; b) CT=$B;; c) CT=$C;; esac
    GDSM_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $CT --kernel-trace -d $OUT/$p$i -o $p --output-format csv -- python3 scripts/dev/coh_pmc.py 1073741824 $D 0 > $OUT/$p$i.log 2>&1 || exit 1
  done
  echo "$i $L" >> $OUT/libs.txt
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
libs = dict(l.split() for l in open(f"{out}/libs.txt"))
for i in sorted(libs):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{out}/[abc]{i}/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "coh_fold_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(libs[i], {k: round(sum(v) / len(v) / 16777216, 2) for k, v in sorted(acc.items())})
PY
