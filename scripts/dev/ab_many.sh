#!/bin/bash
# Same-box A/B/C… of libgdsm builds on the coherence fold, alternating, 3 rounds: fold-kernel ms
# per launch from each bench line.  Usage: scripts/dev/ab_many.sh uniform|zipf LIB...
set -u
D=$1
shift
for r in 1 2 3; do
  for L in "$@"; do
    GDSM_LIB=$L timeout -k 10 200 python3 bench.py --workload coherence --dist $D --steps 5 --warmup 2 --no-cpu \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', '$D', d['stages']['coh_fold']['ms_per_launch'])" || exit 1
  done
done
