#!/bin/bash
# Round 3: start-up phases (native + device process), scrypt per-kernel times new vs pre-abort tree (two polls),
# GPU tests, smoke, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3h}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 120 tools/bin/x11_variants 3 > $O/x11_variants.json 2> $O/x11_variants.err && echo "x11 variants ok" &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "runtime tests ok" &&
for t in new old; do
  if [ $t = new ]; then tree=.; else tree=ab_old; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_scrypt_$t -o run --output-format csv -- python -c "$(python -c 'import tools.ab_kernels as a; print(a.CHILD)')" $PWD/$tree scrypt > $O/prof_scrypt_$t.log 2>&1 || exit 1
done && echo "scrypt prof ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 15 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok" &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
