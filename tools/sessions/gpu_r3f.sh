#!/bin/bash
# Round 3: where the X11 / scrypt kernel-path regressions come from (per-stage / per-kernel times, new tree vs the
# pre-abort tree), then the production entry-point rehearsal again (two-stream GpuMiner, torch-free engine).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3f}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
for t in new old; do
  if [ $t = new ]; then tree=.; else tree=ab_old; fi
  timeout -k 10 120 env PYTHONPATH=$PWD/$tree python $tree/tools/bench_x11.py --iters 8 > $O/x11_stages_$t.json 2>> $O/x11.err || exit 1
done && echo "x11 stages ok" &&
for t in new old; do
  if [ $t = new ]; then tree=.; else tree=ab_old; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_scrypt_$t -o run --output-format csv -- python -c "$(python -c 'import tools.ab_kernels as a; print(a.CHILD)')" $PWD/$tree scrypt > $O/prof_scrypt_$t.log 2>&1 || exit 1
done && echo "scrypt prof ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 20 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok"
