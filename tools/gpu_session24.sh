set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --dtype fp8 --docs 1000000 --batch 256 --rounds 7 --variants 10,15,16 > gpurun_out/lab24_fp8.log 2>&1 || exit 1
echo done
