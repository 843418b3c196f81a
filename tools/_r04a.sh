set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04a
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_loopback.py \
  tests/test_gpu_onetrip.py tests/test_gpu_api.py tests/test_gpu_kernels.py -k "loopback or one_trip or c1_literal or strict or timing" \
  > gpurun_out/r04a/tests.log 2>&1
tail -n 3 gpurun_out/r04a/tests.log
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d gpurun_out/r04a/tl_$dt -o t -- \
    python3 tools/b1_timeline.py --dtype $dt --docs 1000000 --iters 30 > gpurun_out/r04a/tl_$dt.json 2> gpurun_out/r04a/tl_$dt.err
  echo done $dt
done
