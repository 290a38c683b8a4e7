#!/bin/bash
# Workgroup count of the LDS rounds fold (GDSM_ROUNDS_LDS_WG) on config 5, one box, alternating.
set -u
out=${1:-r06w}
steps=()
for spec in "2 1" "2 2" "4 2" "4 4" "8 4" "8 8"; do
  set -- $spec
  for rep in a b; do
    steps+=("b$1_w$2_$rep|200|GDSM_ROUNDS_LDS=1 GDSM_ROUNDS_LDS_WG=$2 python -u bench.py --workload mmult --nodes $1 --no-cpu")
  done
done
bash scripts/gpu_steps.sh "$out" "${steps[@]}"
