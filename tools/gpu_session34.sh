set -o pipefail
# Final-tree kernel stats: the default bench and the fp8 bench under
# rocprofv3 --kernel-trace --stats (bench's in-region scan timing in the same run).
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_r01h
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench" -o bench -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --p50-iters 10 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench_fp8" -o bench -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --dtype fp8 --steps 10 --warmup 3 --p50-iters 10 --no-cpu-baseline > "$OUT/bench_fp8.json" 2> "$OUT/bench_fp8.err" || exit 2
echo done
