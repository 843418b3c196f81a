set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s42_gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s42_smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/s42_bench.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/config_sweep.py > gpurun_out/s42_sweep.log 2>&1 || exit 4
echo done
