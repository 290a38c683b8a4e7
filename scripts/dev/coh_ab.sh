#!/bin/bash
# A/B of the coherence variants on config 4 (uniform and Zipf), alternating, same box.
# Usage: scripts/dev/coh_ab.sh OUTDIR ROUNDS
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
for r in $(seq 1 ${2:-2}); do
  for dist in uniform zipf; do
    for v in 0 1; do
      GDSM_COH_VARIANT=$v timeout -k 10 200 python -u bench.py --workload coherence --dist $dist --steps 10 --warmup 2 --no-cpu > $OUT/ab_${dist}_v${v}_r$r.json 2> $OUT/ab_${dist}_v${v}_r$r.err || exit $?
      python -c "import json,sys; d=json.load(open('$OUT/ab_${dist}_v${v}_r$r.json')); print('$dist v$v r$r', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['last_batch_totals']['invalidations'])"
    done
  done
done
