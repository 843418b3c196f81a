set -o pipefail
# Lab A/B: production bf16 B=256 scan vs SPREAD (next iteration's DMA pieces
# issued one per tile inside the MFMA stream), 1M and 125k docs, then the
# per-wave phase stamps of both (kind 0 / kind 11).
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 7 --variants f0.1t-16,f0.1t-16k10 --stamps f0.1t-16,f0.1t-16k11 > gpurun_out/lab37_spread.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --docs 125000 --batch 256 --rounds 9 --variants f0.1t-16,f0.1t-16k10 > gpurun_out/lab37_spread_125k.log 2>&1 || exit 2
echo done
