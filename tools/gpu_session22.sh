set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 16 --rounds 7 --variants f0.1t-16k6,f0.1t-16k7,f0.1t-16k8,f0.1t-16k9 > gpurun_out/lab22_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 64 --rounds 7 --variants f0.1t-16,f0.1t-16k7,f0.1t-16k6,f0.1t-16k1 > gpurun_out/lab22_b64.log 2>&1 || exit 2
echo done
