#!/bin/bash
# Round stamps of gdsm_rounds in both launch forms (GDSM_ROUNDS_XCD=0 / 1), lib_st build.
set -u
out=${1:-r06o}
steps=()
for n in 1 4; do for x in 0 1; do
  steps+=("st${n}_x$x|120|GDSM_ROUNDS_XCD=$x GDSM_LIB=gallocy_amd/lib_st/libgdsm.so python -u scripts/dev/rounds_stamps.py $n")
done; done
bash scripts/gpu_steps.sh "$out" "${steps[@]}"
