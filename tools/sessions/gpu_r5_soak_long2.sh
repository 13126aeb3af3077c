#!/bin/bash
# Round 5: 600 s node soaks of scrypt (2 ranks) and X11 (4 ranks) on the one GPU after the memory fixes: rejects,
# rate, and RSS per process.
set -o pipefail
out=gpurun_out/${1:-r5z}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 720 python tools/soak.py --node 2 --seconds 600 --every 30 --warmup 40 \
  --algorithm scrypt --difficulty 16 --share-seconds 0.05 --job-interval 5 --block-interval 20 \
  --max-rss-growth-mb 1000 --workdir "$out/scrypt2" > "$out/soak_node2_scrypt_600s.jsonl" \
  2> "$out/soak_node2_scrypt_600s.err"
rc=$?
# soak.py exits 1 when its strict "ok" fails (e.g. one stale share at a block change): not a GPU problem, go on;
# a time limit, a crash or a signal ends the script here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 720 python tools/soak.py --node 4 --seconds 600 --every 30 --warmup 40 \
  --algorithm x11 --difficulty 0.01 --share-seconds 0.05 --job-interval 5 --block-interval 20 \
  --max-rss-growth-mb 1000 --workdir "$out/x11_4" > "$out/soak_node4_x11_600s.jsonl" 2> "$out/soak_node4_x11_600s.err"
