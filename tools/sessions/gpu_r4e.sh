#!/bin/bash
# Round 4, GPU pass e: the miner without any null-stream use (one hardware queue less), and why scrypt ran slower
# through the production miner inside bench.py than in a torch-free process (tools/miner_ctx_ab.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4e
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 120 python tools/rss_breakdown.py --only default > $D/rss.jsonl 2> $D/rss.err && echo "rss ok" &&
timeout -k 10 400 python tools/miner_ctx_ab.py --algo scrypt > $D/ctx_scrypt.jsonl 2> $D/ctx_scrypt.err && cat $D/ctx_scrypt.jsonl &&
timeout -k 10 300 python tools/miner_ctx_ab.py --algo x11 > $D/ctx_x11.jsonl 2> $D/ctx_x11.err && cat $D/ctx_x11.jsonl
