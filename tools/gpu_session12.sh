set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_faithful.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests12.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --dtype fp32 --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline > gpurun_out/bench12_fp32.json 2> gpurun_out/bench12_fp32.err || exit 2
echo done
