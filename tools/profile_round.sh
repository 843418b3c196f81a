#!/bin/bash
# GPU-box profiling recipe for one round (run under gpurun from the repo root):
#   usage: profile_round.sh <round tag> ["dtype:docs[:batch] ..."]
#   1. kernel trace + stats of the default bench (and the MXFP8 bench);
#   2. one rocprofv3 PMC pass per counter (FETCH_SIZE, WRITE_SIZE,
#      GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES) over the scan workload the
#      bench runs (cbv2_search top-100) at the N=1 shape and the per-rank
#      shards of N=2/4/8, plus MXFP8 at N=1 and the mid batches B=64 / B=16;
#   3. tools/pmc_summary.py folds each set into gpurun_out/prof_$R/pmc_scan.json
#      (starting from the committed profiles/pmc_scan.json).
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${1:-r02}
SHAPES=${2:-"bf16:1000000 bf16:500000 bf16:250000 bf16:125000 fp8:1000000 bf16:1000000:64 bf16:1000000:16"}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cp "$ROOT/profiles/pmc_scan.json" "$OUT/pmc_scan.json"
if [ -z "$SKIP_TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench" -o bench -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline --no-faithful \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench_fp8" -o bench -- \
    python3 "$ROOT/bench.py" --dtype fp8 --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline \
    > "$OUT/bench_fp8.json" 2> "$OUT/bench_fp8.err"
  echo trace-done
fi
for shape in $SHAPES; do
  IFS=: read -r dt docs bs <<< "$shape"
  bs=${bs:-256}
  variant=unfused   # cbv2_search's default (the fused top-k is an A/B option)
  kern=maxsim_scan16x4_kernel
  [ "$dt" = fp8 ] && kern=maxsim_scan_f8x4_kernel
  ctrs="FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE"
  ctrs="$ctrs SQ_VALU_MFMA_BUSY_CYCLES"
  csvs=""
  for c in $ctrs; do
    d="$OUT/pmc_${dt}_${docs}_${bs}_$c"
    timeout -s KILL 120 rocprofv3 --pmc $c -f csv -d "$d" -o scan -- \
      python3 "$ROOT/tools/profile_scan.py" --dtype $dt --docs $docs --batch $bs --op search > "$d.log" 2>&1
    csvs="$csvs $(find "$d" -name '*counter_collection.csv' -print -quit)"
  done
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_scan.json" $kern $bs $docs $dt $variant $csvs > "$OUT/pmc_${dt}_${docs}_${bs}.summary"
  echo "pmc $dt $docs $bs done"
done
echo profile-done
