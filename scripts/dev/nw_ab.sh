#!/bin/bash
# NW: parity tests on the in-tree library, then nw bench lines alternating the in-tree library
# and the variants given as arguments (gallocy_amd/<dir>/libgdsm.so), 2 rounds.
set -eu
mkdir -p gpurun_out/nw
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nw.py > gpurun_out/nw/pytest.txt 2>&1
for r in 1 2; do
  for L in gallocy_amd/lib/libgdsm.so "$@"; do
    GDSM_LIB=$L timeout -k 10 200 python3 bench.py --workload nw --steps 10 --warmup 2 --no-cpu \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['stages'].items()})"
  done
done
