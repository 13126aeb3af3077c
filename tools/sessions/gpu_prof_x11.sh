#!/bin/bash
# X11 stage profiles on one MI355X: kernel-trace stats, then SQ counter passes (each its own run).
# Usage (via gpurun): bash tools/gpu_prof_x11.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-x11}
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
run="python3 tools/bench_x11.py --batch 4194304 --iters 3"
timeout -k 10 120 $run > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err && cat gpurun_out/${tag}_bench.json &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run --output-format csv -- $run > gpurun_out/${tag}_trace.log 2>&1 && echo "trace ok" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU -d gpurun_out/${tag}_pmc1 -o run --output-format csv -- $run > gpurun_out/${tag}_pmc1.log 2>&1 && echo "pmc1 ok" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_INT GRBM_GUI_ACTIVE -d gpurun_out/${tag}_pmc2 -o run --output-format csv -- $run > gpurun_out/${tag}_pmc2.log 2>&1 && echo "pmc2 ok"
