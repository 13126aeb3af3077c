set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONPATH="$PWD"
timeout -k 10 300 python -u -m pytest tests/test_x11_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/x11_tests.log 2>&1 && tail -2 gpurun_out/x11_tests.log &&
for i in 1 2 3; do timeout -k 10 120 python tools/bench_x11.py --iters 10 || exit 1; done > gpurun_out/x11_bench_new.jsonl && cat gpurun_out/x11_bench_new.jsonl
