#!/bin/bash
# Round 4, GPU pass n: `otedama node --gpus 2` (gloo, one GPU) soak on the supervisor's torch-free store
# (parallel/kvstore.py), the local pool with a job every 5 s and a block every 45 s: 0 rejects, no RSS growth.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 360 python -u tools/soak.py --seconds 240 --protocol sv2 --node 2 --workdir $O/node2 > $O/soak_node2_sv2.jsonl 2>&1 && echo "node soak ok" && tail -1 $O/soak_node2_sv2.jsonl | cut -c1-600
