#!/bin/bash
# Round 3, first GPU call: GPU tests, smoke, the new bench (N=1 JSON with the self-checks), and the launcher's
# refusal of --gpus 2 on this 1-GPU box. Every GPU step has its own limit; the chain stops at the first failure
# except the deliberate --gpus 2 refusal, whose exit code is checked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
O=gpurun_out/r3a
true &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok" &&
{ timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err; rc=$?;
  echo "bench --gpus 2 exit $rc" | tee $O/bench_n2.rc; test $rc -eq 2; }
