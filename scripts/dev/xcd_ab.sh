#!/bin/bash
# A/B of gdsm_rounds' two launch forms (GDSM_ROUNDS_XCD=0: the whole grid, write-through hand-offs;
# =1: a one-XCD team, hand-offs in its L2) on one box: round stamps (lib_st) and mmult lines.
set -u
out=${1:-r06n}
steps=()
for x in 0 1; do for n in 1 4; do
  steps+=("st${n}_x$x|120|GDSM_ROUNDS_XCD=$x GDSM_LIB=gallocy_amd/lib_st/libgdsm.so python -u scripts/dev/rounds_stamps.py $n")
done; done
for n in 1 2 4 8; do for x in 0 1 0 1; do
  steps+=("b${n}_x${x}_$RANDOM|200|GDSM_ROUNDS_XCD=$x python -u bench.py --workload mmult --nodes $n --no-cpu")
done; done
bash scripts/gpu_steps.sh "$out" "${steps[@]}"
