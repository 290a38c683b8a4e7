#!/bin/bash
# Round-end GPU evidence on one box: GPU tests + smoke, the bench lines (north star with its CPU
# baseline, configs 2 and 3, coherence, mmult), rocprofv3 kernel stats and PMC traffic of the
# north-star and config-3 workloads. Outputs under gpurun_out/ev/; copy what is judged into
# profiles/. Stops at the first nonzero exit. Usage: round_evidence.sh [all|tests|bench|prof|coh]
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
  if [ $rc -ne 0 ]; then tail -n 15 "$OUT/$name.err"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
traffic() {  # name, workload json, bench args... (KPREFIX=kernel family for non-diff kernels)
  local name=$1 wl=$2; shift 2
  step ${name}_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/${name}_fetch -o p --output-format csv -- python3 bench.py "$@"
  step ${name}_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/${name}_write -o p --output-format csv -- python3 bench.py "$@"
  local F W
  F=$(find $OUT/${name}_fetch -name "*counter_collection.csv" | head -1)
  W=$(find $OUT/${name}_write -name "*counter_collection.csv" | head -1)
  if [ -n "${KPREFIX:-}" ]; then
    python3 scripts/pmc_summary.py "$F" "$W" $OUT/$name.json \
      "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, bench.py $*" "$KPREFIX" "$wl" > /dev/null
  else
    python3 scripts/pmc_summary.py "$F" "$W" $OUT/$name.json \
      "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, bench.py $*" "$wl" > /dev/null
  fi && echo "traffic: $OUT/$name.json"
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench 600 python -u bench.py
  step bench_config3_n1 600 python -u bench.py --config 3
  step bench_config2 600 python -u bench.py --config 2 --no-cpu
  step bench_mmult 300 python -u bench.py --workload mmult
  step bench_twin 300 python -u bench.py --workload twin --steps 10 --warmup 2
fi
if [ "$WHAT" = all ] || [ "$WHAT" = coh ]; then
  step bench_coh_uniform 600 python -u bench.py --workload coherence --dist uniform --steps 5 --warmup 2
  step bench_coh_zipf 600 python -u bench.py --workload coherence --dist zipf --steps 5 --warmup 2
  step kt_coh 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_coh -o kt --output-format csv -- python3 bench.py --workload coherence --dist uniform --steps 5 --warmup 2 --no-cpu
  step coh_traffic 900 bash scripts/coh_traffic.sh
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  step kt 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --no-cpu
  step kt_c3 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_c3 -o kt --output-format csv -- python3 bench.py --config 3 --no-cpu
  traffic traffic_northstar '{"pages": 16777216, "mode": "uniform", "ppm": 10000}' --steps 5 --warmup 1 --no-cpu
  traffic traffic_clustered '{"pages": 16777216, "mode": "clustered", "ppm": 100000}' --config 3 --steps 5 --warmup 1 --no-cpu
  traffic traffic_config2 '{"pages": 1048576, "mode": "uniform", "ppm": 10000}' --config 2 --steps 5 --warmup 1 --no-cpu
  step kt_twin 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_twin -o kt --output-format csv -- python3 bench.py --workload twin --steps 10 --warmup 2 --no-cpu
  KPREFIX=gdsm::twin_kernel traffic traffic_twin '{"workload": "twin", "pages": 16777216}' --workload twin --steps 5 --warmup 1 --no-cpu
fi
echo "=== done"
