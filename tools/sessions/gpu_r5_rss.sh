#!/bin/bash
# Round 5: where the long node soak's ~20 MB of RSS growth went: per-process RSS growth over 600 s soaks at 20
# shares/s, the 4-rank node (gloo ranks sharing the GPU) and the standalone engine (one device process).
set -o pipefail
out=gpurun_out/${1:-r5x}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 720 python tools/soak.py --node 4 --seconds 600 --every 30 --warmup 40 \
  --difficulty 0.1 --share-seconds 0.05 --job-interval 5 --block-interval 20 --max-rss-growth-mb 1000 \
  --workdir "$out/node4" > "$out/soak_node4.jsonl" 2> "$out/soak_node4.err"
