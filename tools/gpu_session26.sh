set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 7 --variants f0.1t-16,f0.1t-16k10 > gpurun_out/lab26_bf16.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --dtype fp8 --docs 1000000 --batch 256 --rounds 7 --variants 10,17 > gpurun_out/lab26_fp8.log 2>&1 || exit 2
echo done
