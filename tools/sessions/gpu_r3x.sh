#!/bin/bash
# Round 3: SIMD-512 lane exchange by ds_swizzle (bit-exactness, time, SQ counters), then the per-queue host-memory
# knob sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3x}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 300 python -u -m pytest tests/test_x11_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_x11.txt 2>&1 && echo "x11 tests ok" &&
timeout -k 10 120 tools/bin/x11_variants 5 > $O/x11_variants.json 2> $O/x11_variants.err && echo "x11 variants ok" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --stats -d $O/pmc -o run --output-format csv -- tools/bin/x11_variants 1 > $O/pmc.log 2>&1 && echo "pmc ok" &&
bash tools/sessions/gpu_r3w.sh && echo "knobs ok"
