#!/bin/bash
# Round 5: node soaks with share previews, scrypt (2 ranks) and X11 (4 ranks) sharing the one GPU.
set -o pipefail
out=gpurun_out/${1:-r5o}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 220 python tools/soak.py --node 2 --seconds 90 --every 10 --warmup 30 \
  --algorithm scrypt --difficulty 16 --share-seconds 0.05 --job-interval 5 --block-interval 20 \
  --workdir "$out/soak_scrypt2" > "$out/soak_node2_scrypt.jsonl" 2> "$out/soak_node2_scrypt.err" || exit $?
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 220 python tools/soak.py --node 4 --seconds 90 --every 10 --warmup 30 \
  --algorithm x11 --difficulty 0.01 --share-seconds 0.05 --job-interval 5 --block-interval 20 \
  --workdir "$out/soak_x11_4" > "$out/soak_node4_x11.jsonl" 2> "$out/soak_node4_x11.err"
