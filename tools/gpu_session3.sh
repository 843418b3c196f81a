set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dynamic or small_batch or score" > gpurun_out/gpu_tests3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants f0t128,f0.1t64,f0.1t-16,f0.1t-32,f0.15t-16,f0.05t-16 --stamps f0.1t-16 > gpurun_out/lab3_125k.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants f0t128,f0.1t64,f0.1t-16,f0.1t-32,f0.15t-16 --stamps f0.1t-16 > gpurun_out/lab3.log 2>&1 || exit 2
echo done
