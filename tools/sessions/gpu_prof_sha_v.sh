#!/bin/bash
# rocprofv3 evidence for the version-parallel SHA-256d kernel (run on the GPU box from the repo root):
# kernel-trace stats, then one SQ counter pass in its own run. Argument: prof_kernels.py mode (sha_v | sha_v2).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
MODE=${1:-sha_v}
O=gpurun_out/${MODE}_prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/prof_kernels.py $MODE > $O/trace.log 2>&1 && echo "trace ok" &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 tools/prof_kernels.py $MODE > $O/pmc.log 2>&1 && echo "pmc ok"
find $O -name "*.csv" | head -20
