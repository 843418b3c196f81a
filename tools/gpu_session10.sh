set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests10.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke10.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/bench10.json 2> gpurun_out/bench10.err || exit 3
bash tools/profile_round.sh r01d || exit 4
echo done
