set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s33_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/s33_bench.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --dtype fp8 > gpurun_out/s33_bench_fp8.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --dtype fp32 > gpurun_out/s33_bench_fp32.log 2>&1 || exit 4
BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --p50-iters 5 \
  > gpurun_out/s33_rehearse2.json 2> gpurun_out/s33_rehearse2.err || exit 5
echo done
