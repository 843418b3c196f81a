set -o pipefail
# Lab: dynamic-tail fraction for the B=16 shape (tail loss 9.7% at 0.1), 1M and 125k docs
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 16 --rounds 7 --variants f0.1t-16k6,f0.3t-16k6,f0.5t-16k6,f1t-16k6 > gpurun_out/lab41_b16_dyn.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 64 --rounds 5 --variants f0.1t-16,f0.3t-16,f0.5t-16 > gpurun_out/lab41_b64_dyn.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 16 --rounds 9 --variants f0.1t-16k6,f0.3t-16k6,f0.5t-16k6 > gpurun_out/lab41_b16_125k.log 2>&1 || exit 3
echo done
