#!/bin/bash
# A/B of the twin kernel geometries (GDSM_TWIN_VARIANT) on the north-star pages, alternating.
set -u
for r in 1 2; do
  for v in 0 1 2 3 4; do
    GDSM_TWIN_VARIANT=$v timeout -k 10 200 python -u bench.py --workload twin --steps 10 --warmup 2 --no-cpu > gpurun_out/twin_v$v.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/twin_v$v.json')); print('v$v r$r', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['twin_equals_current'])"
  done
done
