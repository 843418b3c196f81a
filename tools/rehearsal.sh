#!/bin/bash
# N>1 rehearsal of the bench line on ONE GPU box (never used by the driver):
# N ranks over gloo, every rank on cuda:0, the full line (faithful leg, checks).
#   usage: rehearsal.sh <N> <tag> [extra bench args]
set -e -o pipefail
N=${1:-2}; T=${2:-rehearsal}; shift 2 || true
mkdir -p gpurun_out
BENCH_BACKEND=gloo BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$N" --steps 3 --warmup 1 \
  --p50-iters 20 "$@" > gpurun_out/${T}_rehearsal_${N}rank_gloo.json 2> gpurun_out/${T}_rehearsal_${N}rank_gloo.err
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['checks'], d.get('latency_path'))" \
  gpurun_out/${T}_rehearsal_${N}rank_gloo.json
