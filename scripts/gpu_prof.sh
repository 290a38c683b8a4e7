#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: TCC slots), summarised per kernel.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --no-cpu"}
run kt 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS
run fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu
run write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu
F=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/write -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_summary.py "$F" "$W" $OUT/traffic.json > /dev/null && echo "traffic summary: $OUT/traffic.json"
find $OUT -name "*stats.csv"
