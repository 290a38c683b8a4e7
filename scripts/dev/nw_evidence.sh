#!/bin/bash
# NW evidence: parity tests (NW + coherence), the nw bench line with its CPU baseline, kernel stats.
set -e
mkdir -p gpurun_out/r04nw
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nw.py tests/test_gpu_coherence.py > gpurun_out/r04nw/pytest.txt 2>&1
timeout -k 10 300 python3 bench.py --workload nw --steps 10 --warmup 2 > gpurun_out/r04nw/bench_nw.json 2> gpurun_out/r04nw/bench_nw.err
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04nw/prof -o nw --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw --steps 10 --warmup 2 --no-cpu > /dev/null 2>&1
