#!/bin/bash
# Round 3: rocprofv3 evidence on the latest tree: kernel-trace stats of a short bench.py (all three PoWs), then one SQ
# counter pass of the SHA-256d part (two-chain V kernel + the single-midstate pass at 256 blocks/CU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3ah}
mkdir -p $O
true &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 4 \
  --warmup 1 --scrypt-steps 4 --x11-steps 4 --no-latency > $O/bench_traced.json 2> $O/trace.err && echo "trace ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d $O/pmc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --scrypt-steps 0 --x11-steps 0 \
  --no-latency > $O/bench_pmc.json 2> $O/pmc.err && echo "pmc ok"
