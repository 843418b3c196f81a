set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants f0.1t-16,f0.1t-16k1,f0.1t-16k2,f0.1t-16k3 > gpurun_out/lab5.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants f0.1t-16,f0.1t-16k1,f0.1t-16k2,f0.1t-16k3 > gpurun_out/lab5_125k.log 2>&1 || exit 3
echo done
