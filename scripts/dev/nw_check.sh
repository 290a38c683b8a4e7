#!/bin/bash
# NW: GPU parity tests, then the nw bench line and its kernel stats.
set -eu
mkdir -p gpurun_out/nw
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nw.py > gpurun_out/nw/pytest.txt 2>&1
timeout -k 10 200 python3 bench.py --workload nw --steps 10 --warmup 2 --no-cpu > gpurun_out/nw/bench.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/nw/prof -o nw --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw --steps 5 --warmup 1 --no-cpu > /dev/null
