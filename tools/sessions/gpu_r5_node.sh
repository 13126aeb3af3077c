#!/bin/bash
# Round 5 GPU run: the GPU tests, RCCL under a saturating miner, and the node rehearsals on the one GPU.
set -o pipefail
out=gpurun_out/${1:-r5c}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python -m otedama_amd.parallel.comm_probe --seconds 4 --windows 2 > "$out/comm.json" 2> "$out/comm.err" || exit $?
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 400 python tools/node_switch_rehearsal.py --worlds 2,4 --algorithms sha256d \
  > "$out/node_switch.jsonl" 2> "$out/node_switch.err" || exit $?
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python tools/node_switch_rehearsal.py --worlds 2 --algorithms x11,scrypt \
  --switches 4 >> "$out/node_switch.jsonl" 2>> "$out/node_switch.err"
