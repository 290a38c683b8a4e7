#!/bin/bash
# Same-box A/B of libraries (gallocy_amd/<dir>/libgdsm.so, the in-tree one first) on the
# coherence workload, uniform and Zipf, alternating, ROUNDS rounds: fold ms per launch.
# Usage: scripts/dev/lib_ab.sh ROUNDS lib_dir...
set -u
R=$1; shift
for r in $(seq 1 $R); do
  for dist in uniform zipf; do
    for L in gallocy_amd/lib/libgdsm.so "$@"; do
      GDSM_LIB=$L timeout -k 10 200 python3 bench.py --workload coherence --dist $dist --steps 10 --warmup 2 --no-cpu \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$dist', '$L', d['roofline']['avg_launch_ms'], d['roofline']['frac'])" || exit 1
    done
  done
done
