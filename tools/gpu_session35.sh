set -o pipefail
# fp8 lab A/B at B=256, 1M docs: production (shape 0) vs 4-wave workgroups
# (shape 7: 4 queries/wave, 3 WG per CU; shape 8: 8 queries/wave, 2 WG per CU)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --dtype fp8 --docs 1000000 --batch 256 --rounds 7 --variants 10,17,18 > gpurun_out/lab35_fp8.log 2>&1 || exit 1
echo done
