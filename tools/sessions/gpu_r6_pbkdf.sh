#!/bin/bash
# Round 6: is otd_scrypt_pbkdf_out work or slot-waiting? Per-kernel VALU instructions and waves
# of the production scrypt miner (staggered halves, the default), then a kernel trace of the same miner with the two
# halves and a single-stream pass (OTEDAMA_SCRYPT_HALVES=0). Each step has its own limit; the chain stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r6_pbkdf}
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES -d "$out/pmc" -o run \
  --output-format csv -- python3 tools/trace_native_miner.py 3 scrypt > "$out/pmc.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$out/trace_halves" -o run --output-format csv \
  -- python3 tools/trace_native_miner.py 3 scrypt > "$out/trace_halves.log" 2>&1 &&
OTEDAMA_SCRYPT_HALVES=0 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$out/trace_single" -o run \
  --output-format csv -- python3 tools/trace_native_miner.py 3 scrypt > "$out/trace_single.log" 2>&1
