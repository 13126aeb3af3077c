#!/bin/bash
# rocprofv3 kernel-trace stats + PMC counter passes (counters in their own runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -k 10 300 python tools/experiments/sweep_kernels.py --algo scrypt --grids 512,1024,2048 --gaps 1,2 > gpurun_out/sweep_scrypt.jsonl 2>&1 && echo "sweep scrypt ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 tools/prof_kernels.py both > gpurun_out/prof_trace.log 2>&1 && echo "trace ok" &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof_pmc_sq -o run --output-format csv -- python3 tools/prof_kernels.py both > gpurun_out/prof_pmc_sq.log 2>&1 && echo "pmc sq ok" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_pmc_tcc -o run --output-format csv -- python3 tools/prof_kernels.py scrypt > gpurun_out/prof_pmc_tcc.log 2>&1 && echo "pmc tcc ok"
