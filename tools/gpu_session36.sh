set -o pipefail
# Lab: per-wave phase cycles (wait / issue / compute) of the production bf16
# B=256 scan from in-kernel s_memtime stamps (STAMPS build), 1M and 125k docs.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 3 --variants f0.1t-16 --stamps f0.1t-16 > gpurun_out/lab36_phases.log 2>&1 || exit 1
echo done
