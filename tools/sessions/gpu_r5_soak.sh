#!/bin/bash
# Round 5: node soaks with share previews under job and block churn (gloo ranks sharing the one GPU): every share
# re-hashed by the pool, no duplicate or stale reject, no RSS growth.
set -o pipefail
out=gpurun_out/${1:-r5n}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python tools/soak.py --node 4 --seconds 150 --every 10 --warmup 30 \
  --difficulty 0.1 --share-seconds 0.05 --job-interval 5 --block-interval 20 --workdir "$out/soak_sha4" > "$out/soak_node4_sha256d.jsonl" \
  2> "$out/soak_node4_sha256d.err" || exit $?
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 220 python tools/soak.py --node 2 --seconds 90 --every 10 --warmup 30 \
  --algorithm scrypt --difficulty 16 --share-seconds 0.05 --job-interval 5 --block-interval 20 --workdir "$out/soak_scrypt2" \
  > "$out/soak_node2_scrypt.jsonl" 2> "$out/soak_node2_scrypt.err"
