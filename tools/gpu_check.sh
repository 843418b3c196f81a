#!/bin/bash
# GPU-box evidence set of the tree (run under gpurun from the repo root), in
# two parts that each fit one call:
#   gpu_check.sh A <tag>   pytest -m gpu (one process, per-test timeout),
#                          smoke(), the default bench line (plain), the same
#                          bench under rocprofv3 --kernel-trace --stats
#   gpu_check.sh B <tag>   B=1 one-trip timelines at 125k / 1M docs (kernel
#                          trace + host marks), the config sweep (C2-C5 stage
#                          2), the MXFP8 bench (config 5's arithmetic)
# Everything lands in gpurun_out/<tag>/; every GPU step has its own time
# limit and the script stops at the first failure.
set -e -o pipefail
P=${1:-A}
T=${2:-check}
O=gpurun_out/$T
mkdir -p "$O"
export TMPDIR=/tmp
if [ "$P" = A ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$O/gputest.log" 2>&1
  tail -n 2 "$O/gputest.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  echo smoke-ok
  timeout -k 10 600 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
  cat "$O/bench.json"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$O/bench_trace" -o bench -- \
    python3 bench.py > "$O/bench_traced.json" 2> "$O/bench_traced.err"
  python3 tools/kernel_table.py "$(find "$O/bench_trace" -name '*kernel_trace.csv' -print -quit)" 3 \
    > "$O/bench_kernel_table.txt"
  cp "$(find "$O/bench_trace" -name '*kernel_stats.csv' -print -quit)" "$O/bench_kernel_stats.csv"
  head -n 12 "$O/bench_kernel_table.txt"
else
  for D in 125000 1000000; do
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d "$O/tl_$D" -o t -- \
      python3 tools/b1_timeline.py --dtype both --docs $D --iters 40 --marks "$O/marks_$D.jsonl" \
      > "$O/b1_timeline_$D.jsonl" 2> "$O/b1_timeline_$D.err"
    python3 tools/b1_timeline.py --parse "$O/tl_$D" --marks "$O/marks_$D.jsonl" > "$O/b1_timeline_${D}_table.txt"
    cat "$O/b1_timeline_$D.jsonl"
  done
  timeout -k 10 600 python3 tools/config_sweep.py --out "$O/config_sweep.jsonl" > "$O/config_sweep.log" 2>&1
  cat "$O/config_sweep.jsonl"
  timeout -k 10 600 python3 -u bench.py --dtype fp8 > "$O/bench_fp8.json" 2> "$O/bench_fp8.err"
  cat "$O/bench_fp8.json"
fi
