#!/bin/bash
# Round 3: node soak again after pairing each remote rank's hashes with its heartbeat's completion time (r3ar's node
# total read 19.66 GH/s median on one GPU that does ~19.4), and `otedama run` for the same pool settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3as}
mkdir -p $O
true &&
timeout -k 10 300 python -u tools/soak.py --seconds 150 --protocol sv2 --node 2 --workdir $O/node2 \
  > $O/soak_node2_sv2.jsonl 2>&1 && echo "node soak ok"
