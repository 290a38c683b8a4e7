#!/bin/bash
# PMC passes over the apply kernel alone (scripts/dev/apply_only.py), one rocprofv3 run per counter
# group; summaries in gpurun_out/$OUT/. Usage: scripts/dev/apply_pmc.sh OUT [variants]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
V=${2:-0}
mkdir -p $OUT
pass() {
  local name=$1; shift
  echo "=== $name"
  APPLY_VARIANTS=$V APPLY_REPS=3 timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o $name --output-format csv -- python3 scripts/dev/apply_only.py > $OUT/$name.log 2>&1
  local rc=$?
  tail -n 2 $OUT/$name.log
  [ $rc -eq 0 ] || { echo "pass $name rc=$rc"; exit $rc; }
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 scripts/dev/pmc_kernel.py gdsm::apply $(find $OUT -name "*counter_collection.csv") > $OUT/apply_pmc.json
cat $OUT/apply_pmc.json
