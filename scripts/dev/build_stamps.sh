#!/bin/bash
# Stamp build of libgdsm (-DGDSM_COH_STAMPS: kernel variants with invalid output, selectable
# through gdsm_tune) into ${STAMP_OUT:-gallocy_amd/lib_st}/; load it with GDSM_LIB=${STAMP_OUT:-gallocy_amd/lib_st}/libgdsm.so.
# STAMP_DEFS overrides the define (e.g. STAMP_DEFS=-DGDSM_ROUNDS_STAMPS for gdsm_rounds' stamps),
# STAMP_OUT the output directory.
set -eu
cd "$(dirname "$0")/../.."
mkdir -p ${STAMP_OUT:-gallocy_amd/lib_st}
objs=()
for s in gallocy_amd/csrc/*.hip gallocy_amd/csrc/*.cpp; do
  o=${STAMP_OUT:-gallocy_amd/lib_st}/$(basename "${s%.*}").o
  x=(); [[ $s == *.cpp ]] && x=(-x hip)
  /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -fPIC -std=c++17 ${STAMP_DEFS:--DGDSM_COH_STAMPS} \
    -I include -I gallocy_amd/csrc -c "$s" -o "$o"
  objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ${STAMP_OUT:-gallocy_amd/lib_st}/libgdsm.so "${objs[@]}" -ldl -Wl,--no-undefined
echo ${STAMP_OUT:-gallocy_amd/lib_st}/libgdsm.so
