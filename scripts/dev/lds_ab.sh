#!/bin/bash
# A/B of gdsm_rounds' page-table side (GDSM_ROUNDS_LDS=1: one workgroup with the page table in
# LDS; =0: the persistent grid / one-XCD team) on config 5, one box, alternating.
set -u
out=${1:-r06l}
steps=()
for n in 1 2 4 8; do for x in 0 1 0 1; do
  steps+=("b${n}_l${x}_$RANDOM|200|GDSM_ROUNDS_LDS=$x python -u bench.py --workload mmult --nodes $n --no-cpu")
done; done
for n in 1 4; do for x in 0 1; do
  steps+=("st${n}_l$x|120|GDSM_ROUNDS_LDS=$x GDSM_LIB=gallocy_amd/lib_st/libgdsm.so python -u scripts/dev/rounds_stamps.py $n")
done; done
bash scripts/gpu_steps.sh "$out" "${steps[@]}"
