#!/bin/bash
# Round 3: `otedama node --gpus 2` (gloo, both ranks on the one MI355X; same op-log / heartbeat control plane as the
# RCCL node) against the churning local pool, then the same with a pool restart mid-run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3ar}
mkdir -p $O
true &&
timeout -k 10 300 python -u tools/soak.py --seconds 120 --protocol sv2 --node 2 --workdir $O/node2 \
  > $O/soak_node2_sv2.jsonl 2>&1 && echo "node soak ok" &&
timeout -k 10 300 python -u tools/soak.py --seconds 120 --protocol sv2 --node 2 --bounce-at 50 --workdir $O/node2_bounce \
  > $O/soak_node2_sv2_bounce.jsonl 2>&1 && echo "node bounce ok"
