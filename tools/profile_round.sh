#!/bin/bash
# GPU-box profiling recipe for one round (run under gpurun from the repo root):
#   kernel trace + stats of the default bench, then one PMC pass per counter
#   over the scan-only workload for bf16 and fp8.  Every GPU step has its own
#   time limit; the script stops at the first failure.
set -e -o pipefail
R=${1:-r01}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench" -o bench -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
for dt in bf16 fp8; do
  for c in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES; do
    timeout -k 10 240 rocprofv3 --pmc $c -f csv -d "$OUT/pmc_${dt}_$c" -o scan -- \
      python3 "$ROOT/tools/profile_scan.py" --dtype $dt > "$OUT/pmc_${dt}_$c.log" 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench_fp8" -o bench -- \
  python3 "$ROOT/bench.py" --dtype fp8 --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline > "$OUT/bench_fp8.json" 2> "$OUT/bench_fp8.err"
echo profile-done
