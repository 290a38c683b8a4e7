#!/bin/bash
# A/B build of libgdsm with extra compile flags into gallocy_amd/<dir>/ (not product code):
#   scripts/dev/build_variant.sh lib_v1 -DGDSM_FOLD_PRIO=1
# Load it with GDSM_LIB=gallocy_amd/<dir>/libgdsm.so (scripts/dev/ab_many.sh).
set -eu
cd "$(dirname "$0")/../.."
d=gallocy_amd/$1
shift
mkdir -p "$d"
objs=()
for s in gallocy_amd/csrc/*.hip gallocy_amd/csrc/*.cpp; do
  o=$d/$(basename "${s%.*}").o
  x=(); [[ $s == *.cpp ]] && x=(-x hip)
  /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" \
    -I include -I gallocy_amd/csrc -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$d/libgdsm.so" "${objs[@]}" -ldl -Wl,--no-undefined
rm -f "$d"/*.o
echo "$d/libgdsm.so"
