#!/bin/bash
# HBM bytes of the scrypt ROMix pipeline (cooperative kernel, 4 x 2^20 hashes) and of the X11 stage chain
# (4 x 2^23 nonces): one rocprofv3 pass per TCC counter
# (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2, so they cannot share a pass), plus a kernel-trace pass for durations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
out=gpurun_out/hbm
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/prof_kernels.py scrypt > $out/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 tools/prof_kernels.py scrypt > $out/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 tools/prof_kernels.py scrypt > $out/write.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/x11_trace -o run --output-format csv -- python3 tools/prof_kernels.py x11 > $out/x11_trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/x11_fetch -o run --output-format csv -- python3 tools/prof_kernels.py x11 > $out/x11_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/x11_write -o run --output-format csv -- python3 tools/prof_kernels.py x11 > $out/x11_write.log 2>&1 &&
echo "hbm passes ok"
