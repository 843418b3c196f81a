set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --durations=0 --timeout 180 --timeout-method thread > gpurun_out/gpu_tests15.log 2>&1 || exit 1
echo done
