#!/bin/bash
# scrypt ROMix A/B on one MI355X: numerics vs hashlib, geometry sweep, memory-path counters for the
# cooperative variant. gap codes: 1/2 per-lane ROMix, 8 lane-cooperative full-line ROMix, 9 per-lane @8 waves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q -k scrypt > gpurun_out/pytest_scrypt.log 2>&1 && echo "scrypt tests ok" &&
timeout -k 10 400 python tools/sweep_kernels.py --algo scrypt --grids 1024,2048 --gaps 1,8,2 > gpurun_out/sweep_ab.jsonl 2>&1 && echo "sweep ok" &&
timeout -k 10 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_ta_g8 -o run --output-format csv -- python3 tools/prof_kernels.py scrypt 8 > gpurun_out/pmc_ta_g8.log 2>&1 && echo "pmc ta ok" &&
timeout -k 10 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_tcp_g8 -o run --output-format csv -- python3 tools/prof_kernels.py scrypt 8 > gpurun_out/pmc_tcp_g8.log 2>&1 && echo "pmc tcp ok"
