#!/bin/bash
# Round-end GPU evidence on one box: GPU tests + smoke, the bench line, rocprofv3 kernel stats and
# PMC traffic of the bench workload, and the secondary workloads' bench lines. Outputs under
# gpurun_out/ev/; copy what is judged into profiles/. Stops at the first crash-like exit.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/ev
mkdir -p $OUT
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step pytest_gpu 1500 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench 600 python -u bench.py --steps 20 --warmup 3
  step bench_clustered 600 python -u bench.py --steps 10 --warmup 3 --mode clustered --pages 2097152 --no-cpu
  step bench_config3_n1 900 python -u bench.py --steps 5 --warmup 2 --scaling strong --total-pages 16777216 --mode clustered --no-cpu
  step bench_coh_uniform 600 python -u bench.py --workload coherence --dist uniform --steps 5 --warmup 2 --no-cpu
  step bench_coh_zipf 600 python -u bench.py --workload coherence --dist zipf --steps 5 --warmup 2 --no-cpu
  step bench_mmult 300 python -u bench.py --workload mmult
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  step kt 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu
  step fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu
  step write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu
  F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
  W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py "$F" "$W" $OUT/traffic.json > /dev/null && echo "traffic: $OUT/traffic.json"
  step kt_coh 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_coh -o kt --output-format csv -- python3 bench.py --workload coherence --dist uniform --steps 5 --warmup 2 --no-cpu
  step kt_coh_zipf 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_coh_zipf -o kt --output-format csv -- python3 bench.py --workload coherence --dist zipf --steps 5 --warmup 2 --no-cpu
  step coh_traffic 900 bash scripts/coh_traffic.sh
fi
echo "=== done"
