#!/bin/bash
# Same-box A/B: in-tree fold vs +8 SALU / +8 VALU padding per walk step (measurement builds),
# alternating, 3 rounds, uniform config 4.
set -u
for r in 1 2 3; do
  for L in gallocy_amd/lib/libgdsm.so gallocy_amd/lib_salu/libgdsm.so gallocy_amd/lib_valu/libgdsm.so; do
    GDSM_LIB=$L timeout -k 10 200 python3 bench.py --workload coherence --dist uniform --steps 5 --warmup 2 --no-cpu \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', d['stages']['coh_fold']['ms_per_launch'])" || exit 1
  done
done
