#!/bin/bash
# PMC passes over the diff kernel alone (scripts/dev/ab_diff.py, config-3 density by default), one
# rocprofv3 run per counter group; summaries in gpurun_out/$OUT/. Usage:
#   scripts/dev/diff_pmc.sh OUT [uniform|clustered] [pages]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
MODE=${2:-clustered}
PAGES=${3:-4194304}
mkdir -p $OUT
pass() {
  local name=$1; shift
  echo "=== $name"
  AB_MODE=$MODE AB_PAGES=$PAGES timeout -k 10 150 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o $name --output-format csv -- python3 scripts/dev/ab_diff.py diff_variant 0 > $OUT/$name.log 2>&1
  local rc=$?
  tail -n 2 $OUT/$name.log
  [ $rc -eq 0 ] || { echo "pass $name rc=$rc"; exit $rc; }
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 scripts/dev/pmc_kernel.py gdsm::diff_single $(find $OUT -name "*counter_collection.csv") > $OUT/diff_pmc.json
cat $OUT/diff_pmc.json
