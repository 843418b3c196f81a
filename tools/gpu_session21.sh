set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_faithful.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests21.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/config_sweep.py > gpurun_out/sweep21.log 2>&1 || exit 2
echo done
