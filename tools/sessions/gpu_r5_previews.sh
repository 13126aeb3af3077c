#!/bin/bash
# Round 5: share previews on the one GPU. `otedama node` with 2 and 4 gloo ranks sharing GPU 0, SHA-256d and scrypt,
# with and without previews (OTEDAMA_NODE_SHARE_PREVIEWS=0: R2 only): remote device hit -> pool accept.
set -o pipefail
out=gpurun_out/${1:-r5l}
mkdir -p "$out"
for pv in 1 0; do
  OTEDAMA_NODE_SHARE_PREVIEWS=$pv OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python tools/node_switch_rehearsal.py \
    --worlds 2,4 --algorithms sha256d --switches 4 > "$out/node_pv$pv.jsonl" 2> "$out/node_pv$pv.err" || exit $?
  OTEDAMA_NODE_SHARE_PREVIEWS=$pv OTEDAMA_DIST_BACKEND=gloo timeout -k 10 200 python tools/node_switch_rehearsal.py \
    --worlds 2 --algorithms scrypt --switches 4 >> "$out/node_pv$pv.jsonl" 2>> "$out/node_pv$pv.err" || exit $?
done
