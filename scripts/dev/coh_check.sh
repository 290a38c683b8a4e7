#!/bin/bash
# Coherence fold on one GPU box: parity tests, then the same-box A/B of the fold (variant 0)
# against the four-pass path (variant 1) on BASELINE config 4, uniform and Zipf.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/coh
mkdir -p $OUT
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_gpu_coherence.py -x -v --timeout 300 --timeout-method thread ${COH_K:+-k "$COH_K"}
step ab_uniform 600 python -u scripts/dev/ab_coh.py 1073741824 uniform 0,1
step ab_zipf 600 python -u scripts/dev/ab_coh.py 1073741824 zipf 0,1
echo "=== done"
