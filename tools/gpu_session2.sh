set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants f0t128,f0.05t128,f0.1t128,f0.1t64,f0.15t128,f0.1t256 --stamps f0t128,f0.1t128 > gpurun_out/lab2.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 7 --variants f0t128,f0.1t64,f0.1t128,f0.2t64 --stamps f0t128,f0.1t64 > gpurun_out/lab2_125k.log 2>&1 || exit 3
echo done
