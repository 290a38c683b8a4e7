#!/bin/bash
# Same-box A/B of two libgdsm builds (gallocy_amd/lib_ab/libgdsm.so = A, the in-tree build = B)
# on the coherence fold, alternating, 3 rounds: fold-kernel ms per launch from each bench line.
# Usage: scripts/dev/ab_libs.sh [uniform|zipf]
set -u
D=${1:-uniform}
for r in 1 2 3; do
  for L in gallocy_amd/lib_ab/libgdsm.so gallocy_amd/lib/libgdsm.so; do
    GDSM_LIB=$L timeout -k 10 200 python3 bench.py --workload coherence --dist $D --steps 5 --warmup 2 --no-cpu \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', '$D', d['stages']['coh_fold']['ms_per_launch'])" || exit 1
  done
done
