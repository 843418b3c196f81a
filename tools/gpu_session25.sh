set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_r01f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests25.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/bench_fp8 -o bench -- python3 bench.py --dtype fp8 --steps 5 --warmup 2 --p50-iters 10 --no-cpu-baseline > $OUT/bench_fp8.json 2> $OUT/bench_fp8.err || exit 2
for c in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES; do
  timeout -k 10 240 rocprofv3 --pmc $c -f csv -d $OUT/pmc_fp8_$c -o scan -- python3 tools/profile_scan.py --dtype fp8 > $OUT/pmc_fp8_$c.log 2>&1 || exit 3
done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --pmc $C -f csv -d $OUT/sq_fp8 -o scan -- python3 tools/profile_scan.py --dtype fp8 > $OUT/sq_fp8.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/bench25_fp8.json 2> gpurun_out/bench25_fp8.err || exit 5
echo done
