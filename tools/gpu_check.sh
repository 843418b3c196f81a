#!/bin/bash
# GPU-box check of the tree (run under gpurun from the repo root):
#   pytest -m gpu (one process, per-test timeout), smoke(), the default bench.
#   usage: gpu_check.sh <tag>
set -e -o pipefail
T=${1:-check}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > gpurun_out/${T}_gputest.log 2>&1
tail -n 3 gpurun_out/${T}_gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
echo smoke-ok
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
cat gpurun_out/${T}_bench.json
