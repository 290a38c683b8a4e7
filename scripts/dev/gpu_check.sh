#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first crash-like exit (fault/abort/segv/timeout); plain test failures (exit 1)
# do not stop the later steps.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench 600 python bench.py --steps 20 --warmup 3
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu
fi
echo "=== done"
