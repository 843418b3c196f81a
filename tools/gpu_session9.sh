set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests9.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/scan_lab.py --dtype fp8 --docs 1000000 --batch 256 --rounds 5 --variants 10,12,13,14 > gpurun_out/lab9_fp8.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants f0.1t-16,f0.1t-16k1 > gpurun_out/lab9.log 2>&1 || exit 3
echo done
