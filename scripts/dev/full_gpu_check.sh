#!/bin/bash
# Whole GPU suite and smoke() on the current tree, as the driver runs them at round end.
set -e
mkdir -p gpurun_out/full
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/full/pytest.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.txt 2>&1
