#!/bin/bash
# Development round-trip on one GPU box: selected GPU tests (DEV_K: pytest -k expression), the
# config-2 bench fused and unfused (same box), and the coherence fold's PMC instruction mix.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/dev
mkdir -p $OUT
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -n "${DEV_K:-}" ]; then
  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$DEV_K"
fi
if [ -n "${DEV_BENCH:-1}" ]; then
  step bench_fused 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --fuse on
  step bench_unfused 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --fuse off
fi
if [ -n "${DEV_PMC:-}" ]; then
  COH_PMC_VARIANTS=0 bash scripts/dev/coh_pmc.sh > $OUT/cohpmc.log 2>&1; echo "cohpmc rc=$?"; tail -4 $OUT/cohpmc.log
fi
echo "=== done"
