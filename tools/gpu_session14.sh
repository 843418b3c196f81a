set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 1 --rounds 9 --variants 9,13 > gpurun_out/lab14_b1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 4 --rounds 9 --variants 10,14 > gpurun_out/lab14_b4.log 2>&1 || exit 2
echo done
