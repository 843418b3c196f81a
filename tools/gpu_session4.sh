set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/scan_lab.py --dtype fp8 --docs 1000000 --batch 256 --rounds 5 --variants 2,1 > gpurun_out/lab4_fp8.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit 3
timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench4_fp8.json 2> gpurun_out/bench4_fp8.err || exit 4
echo done
