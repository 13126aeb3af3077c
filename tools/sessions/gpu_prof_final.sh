#!/bin/bash
# Final-state profiles: X11 stages (trace + SQ counters) and the SHA-256d K-variant kernel (trace + SQ counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "runtime_shares or k_variants" --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 && tail -1 gpurun_out/final_tests.log &&
bash tools/gpu_prof_x11.sh x11final &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/shak_trace -o run --output-format csv -- python3 tools/bench_sha_k.py > gpurun_out/shak_trace.log 2>&1 && echo "sha trace ok" &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/shak_pmc -o run --output-format csv -- python3 tools/bench_sha_k.py > gpurun_out/shak_pmc.log 2>&1 && echo "sha pmc ok"
