set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants 11,12 > gpurun_out/lab7.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants 11,12 > gpurun_out/lab7_125k.log 2>&1 || exit 3
echo done
