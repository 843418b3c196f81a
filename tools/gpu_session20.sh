set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants f0.1t-16,f0.2t-16,f0.05t-16,f0.3t-16,f0t128 --stamps f0.1t-16 > gpurun_out/lab20_125k.log 2>&1 || exit 1
echo done
