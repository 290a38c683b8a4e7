#!/bin/bash
# REHEARSAL of bench.py's N > 1 path on a one-GPU box: 2 and 4 ranks share cuda:0 and exchange
# over gloo (GDSM_BENCH_BACKEND=gloo), pipelined and serial. Checks the step machinery, the
# barrier / max-over-ranks timing and the all-rank REPLICA check; the timings are not a measurement.
set -u
export TMPDIR=/tmp GDSM_BENCH_BACKEND=gloo
OUT=gpurun_out/multi
mkdir -p $OUT
port=29611
for spec in "2 on" "2 off" "4 on"; do
  set -- $spec
  name=g$1_$2
  echo "=== $name"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $1 --steps 5 --warmup 1 \
    --pages 262144 --no-cpu --overlap $2 > $OUT/$name.log 2>&1
  rc=$?
  echo "=== $name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-400 || tail -n 20 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  port=$((port + 1))
done
