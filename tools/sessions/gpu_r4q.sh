#!/bin/bash
# Round 4, GPU pass q: PMC counters of the production miner's kernels on the final tree (tools/trace_native_miner.py:
# SHA-256d, scrypt, X11 in one process). Pass 1: instruction mix, waves, busy and GPU-active cycles. Pass 2: HBM
# fetch bytes. Each pass in its own run, counters within the per-block limits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1 -o run --output-format csv -- python3 tools/trace_native_miner.py 2 > $O/p1.log 2>&1 && echo "pass 1 ok" && grep -h '^{' $O/p1.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p2 -o run --output-format csv -- python3 tools/trace_native_miner.py 2 > $O/p2.log 2>&1 && echo "pass 2 ok" && grep -h '^{' $O/p2.log
