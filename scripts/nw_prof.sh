#!/bin/bash
# GPU NW (legacy diff() on the GPU): bench line + rocprofv3 kernel trace of the same command.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload nw --steps 10 --warmup 2 > $OUT/nw_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/nwprof -o nw --output-format csv -- python3 bench.py --workload nw --steps 10 --warmup 2 --no-cpu > $OUT/nwprof.log 2>&1 || exit $?
find $OUT/nwprof -name '*kernel_stats.csv' -exec cp {} $OUT/nw_kernel_stats.csv \;
echo done
