#!/bin/bash
# Runs named GPU steps on the box, each under its own time limit, output under gpurun_out/$OUT/;
# stops at the first crash-like exit (anything but 0 / 1). Usage:
#   scripts/gpu_steps.sh OUTDIR "name|seconds|command" ["name|seconds|command" ...]
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($(date +%T)) $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -n 15 "$OUT/$name.err"; fi
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo "=== done"
