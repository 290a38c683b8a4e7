#!/bin/bash
# Round-6 GPU evidence on one box (outputs under gpurun_out/r06ev/): GPU tests + smoke, every bench
# line (north star with its CPU baseline, configs 2 and 3, twin, coherence uniform / Zipf, mmult
# P = 1/2/4/8, NW), the rocprofv3 kernel stats of the north star. Stops at the first failure.
set -u
export TMPDIR=/tmp
W=${1:-all}
S="bash scripts/gpu_steps.sh r06ev"
if [ "$W" = all ] || [ "$W" = tests ]; then
  $S "pytest_gpu|900|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
     "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
fi
if [ "$W" = all ] || [ "$W" = bench ]; then
  $S "bench_northstar|300|python -u bench.py" \
     "bench_config2|300|python -u bench.py --config 2 --no-cpu" \
     "bench_config3|300|python -u bench.py --config 3" \
     "bench_twin|300|python -u bench.py --workload twin --steps 10 --warmup 2" \
     "bench_coh_uniform|300|python -u bench.py --workload coherence --dist uniform --steps 5 --warmup 2" \
     "bench_coh_zipf|300|python -u bench.py --workload coherence --dist zipf --steps 5 --warmup 2" \
     "bench_nw|300|python -u bench.py --workload nw" || exit $?
fi
if [ "$W" = all ] || [ "$W" = mmult ]; then
  $S "bench_mmult_p1|300|python -u bench.py --workload mmult --nodes 1" \
     "bench_mmult_p2|300|python -u bench.py --workload mmult --nodes 2" \
     "bench_mmult_p4|300|python -u bench.py --workload mmult --nodes 4" \
     "bench_mmult_p8|300|python -u bench.py --workload mmult --nodes 8" || exit $?
fi
if [ "$W" = all ] || [ "$W" = prof ]; then
  $S "kt|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r06ev/kt -o kt --output-format csv -- python3 bench.py --no-cpu" || exit $?
fi
echo "=== evidence done"
