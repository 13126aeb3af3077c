#!/bin/bash
# Round 5: a 10-minute node soak (4 gloo ranks sharing the one GPU, share previews, a job every 5 s, a block every
# 20 s, a share per 0.05 s on the leader's connection): rejects, RSS and rate over a long window.
set -o pipefail
out=gpurun_out/${1:-r5s}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 720 python tools/soak.py --node 4 --seconds 600 --every 20 --warmup 30 \
  --difficulty 0.1 --share-seconds 0.05 --job-interval 5 --block-interval 20 --workdir "$out/soak_sha4" \
  > "$out/soak_node4_sha256d_600s.jsonl" 2> "$out/soak_node4_sha256d_600s.err"
