#!/bin/bash
# Round 3: the in-kernel hit ring / abort word runtime on the GPU: its own tests first, then every GPU test,
# smoke and the N=1 bench (hashrates must hold within noise of profiles/r3/a_first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3d}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "runtime tests ok" &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
