#!/bin/bash
# Same-box A/B/C… of libgdsm builds on any bench line, alternating, 3 rounds: each stage's ms per
# launch.  Usage: scripts/dev/ab_bench.sh "<bench.py args>" LIB...
set -u
A=$1
shift
for r in 1 2 3; do
  for L in "$@"; do
    GDSM_LIB=$L timeout -k 10 300 python3 bench.py $A \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', {k: v['ms_per_launch'] for k, v in d['stages'].items()}, d['ms_per_step'])" || exit 1
  done
done
