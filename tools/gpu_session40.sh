set -o pipefail
# Lab: per-workgroup clocks + phase stamps, B=16 (kind 12) and B=256 (kind 0), 1M docs
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 16 --rounds 3 --variants f0.1t-16k6 --stamps f0.1t-16k12 > gpurun_out/lab40_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 3 --variants f0.1t-16 --stamps f0.1t-16 > gpurun_out/lab40_b256.log 2>&1 || exit 2
echo done
