#!/bin/bash
# Measurement build of libgdsm (-DGDSM_MEASURE: kernel variants with invalid output, selectable
# through gdsm_tune) into gallocy_amd/lib_x/; load it with GDSM_LIB=gallocy_amd/lib_x/libgdsm.so.
set -eu
cd "$(dirname "$0")/../.."
mkdir -p gallocy_amd/lib_x
objs=()
for s in gallocy_amd/csrc/*.hip gallocy_amd/csrc/*.cpp; do
  o=gallocy_amd/lib_x/$(basename "${s%.*}").o
  x=(); [[ $s == *.cpp ]] && x=(-x hip)
  /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DGDSM_MEASURE \
    -I include -I gallocy_amd/csrc -c "$s" -o "$o"
  objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o gallocy_amd/lib_x/libgdsm.so "${objs[@]}" -ldl -Wl,--no-undefined
echo gallocy_amd/lib_x/libgdsm.so
