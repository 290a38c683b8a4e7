#!/bin/bash
# A/B of libgdsm builds on the config-4 fold (uniform and Zipf), alternating, same box:
# coh_fold_kernel ms per launch from bench.py's HIP events. Usage:
#   scripts/dev/coh_lib_ab.sh OUTDIR ROUNDS lib_dir [lib_dir ...]   (e.g. gallocy_amd/lib gallocy_amd/lib_w1)
set -u
OUT=gpurun_out/$1; R=$2; shift 2; mkdir -p $OUT
for r in $(seq 1 $R); do
  for dist in uniform zipf; do
    for L in "$@"; do
      n=$(basename $L)_${dist}_r$r
      GDSM_LIB=$L/libgdsm.so timeout -k 10 200 python -u bench.py --workload coherence --dist $dist --steps 10 --warmup 2 --no-cpu > $OUT/$n.json 2> $OUT/$n.err || exit $?
      python -c "import json; d=json.load(open('$OUT/$n.json')); print('$L $dist r$r', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['last_batch_totals']['invalidations'])"
    done
  done
done
