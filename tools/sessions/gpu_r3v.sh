#!/bin/bash
# Round 3: production rehearsal with exact rate windows (device-timeline completion times), twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3v}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
for i in 1 2; do
  timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 20 --out-dir $O/node_rehearsal_$i > $O/node_rehearsal_$i.json 2> $O/node_rehearsal_$i.err || exit 1
done && echo "rehearsals ok"
