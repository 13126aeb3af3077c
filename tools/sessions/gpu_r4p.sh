#!/bin/bash
# Round 4, GPU pass p: `otedama node --gpus 4` (gloo, host buffers, all four ranks' device processes on the one GPU)
# soak on the torch-free store: the control plane at world 4 with production miners; 0 rejects, no RSS growth.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 300 python -u tools/soak.py --seconds 150 --protocol sv2 --node 4 --workdir $O/node4 > $O/soak_node4_sv2.jsonl 2>&1 && echo "node4 soak ok" && tail -1 $O/soak_node4_sv2.jsonl | cut -c1-600
