#!/bin/bash
# HBM bytes per launch of the coherence kernels (config 4) from rocprofv3 PMC: FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), uniform and Zipf batches, summarised per kernel.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/cohtraffic
mkdir -p $OUT
for d in uniform zipf; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/$d-$c -o p --output-format csv -- python3 bench.py --workload coherence --dist $d --steps 3 --warmup 1 --no-cpu > $OUT/$d-$c.log 2>&1 || { tail -5 $OUT/$d-$c.log; exit 1; }
  done
  F=$(find $OUT/$d-FETCH_SIZE -name "*counter_collection.csv" | head -1)
  W=$(find $OUT/$d-WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py "$F" "$W" $OUT/coh_traffic_$d.json \
    "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, bench.py --workload coherence --dist $d --steps 3 --warmup 1 --no-cpu (16M pages, 1B events)" \
    "gdsm::coh_fold_kernel" "{\"workload\": \"coherence\", \"dist\": \"$d\", \"pages\": 16777216, \"events\": 1073741824}" > /dev/null || exit 1
  echo "$d: $OUT/coh_traffic_$d.json"
done
