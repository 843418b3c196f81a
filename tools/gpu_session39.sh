set -o pipefail
# Lab: phase stamps of the B=16 production shape (4 waves x 4 queries, two
# workgroups per CU, 32-token iterations) at 1M docs, next to its timing.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 16 --rounds 5 --variants f0.1t-16k6 --stamps f0.1t-16k12 > gpurun_out/lab39_b16_phases.log 2>&1 || exit 1
echo done
