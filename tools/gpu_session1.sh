set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/scan_lab.py --docs 1000000 --batch 256 --rounds 5 --variants 200,201,202,203 --stamps > gpurun_out/lab1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --docs 125000 --steps 30 --no-cpu-baseline > gpurun_out/bench_125k.json 2> gpurun_out/bench_125k.err || exit 2
BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --docs 250000 --steps 5 --warmup 2 --p50-iters 5 --no-cpu-baseline > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err || exit 3
echo done
