#!/bin/bash
# Coherence pass-C variant check on one box: GPU coherence tests under the candidate variant,
# then in-process A/B (scripts/ab_coh.py) on config 4, uniform and Zipf.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/cohab
mkdir -p $OUT
V=${1:-4}
GDSM_COH_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_coherence.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for d in uniform zipf; do
  timeout -k 10 300 python -u scripts/ab_coh.py 1073741824 $d 0,$V > $OUT/ab_$d.log 2>&1
  rc=$?; cat $OUT/ab_$d.log | tail -4; [ $rc -eq 0 ] || exit $rc
done
