set -o pipefail
# Lab A/B at B=256, 1M docs: production 8 waves x 4 queries (one WG per CU, one
# barrier domain per CU) vs kind 6 = 4 waves x 4 queries, 32-token iterations,
# two WGs per CU (each SIMD runs waves of two WGs with independent barriers).
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 7 --variants f0.1t-16,f0.1t-16k6 > gpurun_out/lab31_b256.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants f0.1t-16,f0.1t-16k6 > gpurun_out/lab31_b256_125k.log 2>&1 || exit 2
echo done
