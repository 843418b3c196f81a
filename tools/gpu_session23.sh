set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
for dt in bf16 fp8; do
  timeout -s KILL 90 rocprofv3 --pmc $C -f csv -d gpurun_out/pmc23_$dt -o scan -- python3 tools/profile_scan.py --dtype $dt > gpurun_out/pmc23_$dt.log 2>&1 || exit 1
done
echo done
