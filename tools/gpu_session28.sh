set -o pipefail
# Multi-rank rehearsal on a one-GPU box: 2 and 4 ranks on cuda:0 over gloo
# (the driver's N>1 runs are one rank per GPU over RCCL), bf16 and fp8.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 2 4; do
  BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 2 --p50-iters 5 \
    > gpurun_out/s28_rehearse$n.json 2> gpurun_out/s28_rehearse$n.err || exit $n
done
BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 2 --dtype fp8 --steps 5 --warmup 2 --p50-iters 5 \
  > gpurun_out/s28_rehearse2_fp8.json 2> gpurun_out/s28_rehearse2_fp8.err || exit 5
echo done
