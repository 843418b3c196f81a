set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants f0.1t-16,f0.1t-16k2,f0.1t-16k4,f0.1t-16k5 > gpurun_out/lab11.log 2>&1 || exit 1
echo done
