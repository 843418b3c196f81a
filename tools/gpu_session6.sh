set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "api or sharded or pipeline or kernels" > gpurun_out/gpu_tests6.log 2>&1 || exit 1
BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --docs 250000 --steps 10 --warmup 2 --p50-iters 5 --no-cpu-baseline > gpurun_out/bench_rehearse6.json 2> gpurun_out/bench_rehearse6.err || exit 3
timeout -k 10 300 python bench.py --docs 125000 --steps 30 --no-cpu-baseline > gpurun_out/bench6_125k.json 2> gpurun_out/bench6_125k.err || exit 2
echo done
