set -o pipefail
# Round-1 final profile set r01g: the default bf16 bench and the fp8 bench
# under rocprofv3 --kernel-trace --stats, the 1M-doc PMC passes (bf16, fp8),
# then bf16 PMC passes at the per-rank shard sizes of the N=2/4/8 runs.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/profile_round.sh r01g > gpurun_out/s29_profile.log 2>&1 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_r01g
for docs in 500000 250000 125000; do
  for c in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
    timeout -k 10 120 rocprofv3 --pmc $c -f csv -d "$OUT/pmc_bf16_${docs}_$c" -o scan -- \
      python3 "$GRAFT_REPO_ROOT/tools/profile_scan.py" --dtype bf16 --docs $docs > "$OUT/pmc_bf16_${docs}_$c.log" 2>&1 || exit 2
  done
done
echo done
