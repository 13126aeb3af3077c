#!/bin/bash
# Round 5: where the long node soak's ~20 MB of RSS growth went: per-process RSS growth over 300 s soaks at 20
# shares/s, the 4-rank node (gloo ranks sharing the GPU) and the standalone engine (one device process).
set -o pipefail
out=gpurun_out/${1:-r5t}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 420 python tools/soak.py --node 4 --seconds 300 --every 20 --warmup 40 \
  --difficulty 0.1 --share-seconds 0.05 --job-interval 5 --block-interval 20 --max-rss-growth-mb 1000 \
  --workdir "$out/node4" > "$out/soak_node4.jsonl" 2> "$out/soak_node4.err"
timeout -k 10 420 python tools/soak.py --seconds 300 --every 20 --warmup 40 \
  --difficulty 0.1 --share-seconds 0.05 --job-interval 5 --block-interval 20 --max-rss-growth-mb 1000 \
  --workdir "$out/run1" > "$out/soak_run1.jsonl" 2> "$out/soak_run1.err"
