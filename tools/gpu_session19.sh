set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_faithful.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests19.log 2>&1 || exit 1
mkdir -p gpurun_out/prof19
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof19 -o fp32 -- python3 bench.py --dtype fp32 --steps 5 --warmup 2 --p50-iters 5 --no-cpu-baseline > gpurun_out/prof19/bench.json 2> gpurun_out/prof19/bench.err || exit 3
timeout -k 10 400 python -u bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench19_fp32.json 2> gpurun_out/bench19_fp32.err || exit 2
echo done
