#!/bin/bash
# Round 4, GPU pass d: can the device process run on one normal-priority hardware queue (GPU_MAX_HW_QUEUES=1: both
# search streams share it; the abort word needs no control queue any more) without losing rate or job-switch time?
# Then the 2-rank gloo node with host-memory collective buffers and ops carried on the doorbell.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4d
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
HW1=GPU_MAX_HW_QUEUES=1
timeout -k 10 60 tools/bin/queue_rss > $D/queue_rss_default.json && GPU_MAX_HW_QUEUES=1 timeout -k 10 60 tools/bin/queue_rss > $D/queue_rss_hw1.json && cat $D/queue_rss_*.json &&
timeout -k 10 300 python tools/ab_miner.py --a . --b . --algo sha256d --rounds 6 --seconds 6 --env-b $HW1 > $D/ab_sha256d_hw1.json 2> $D/ab_sha256d_hw1.err && cat $D/ab_sha256d_hw1.json &&
timeout -k 10 400 python tools/ab_miner.py --a . --b . --algo scrypt --rounds 4 --seconds 8 --env-b $HW1 > $D/ab_scrypt_hw1.json 2> $D/ab_scrypt_hw1.err && cat $D/ab_scrypt_hw1.json &&
timeout -k 10 300 python tools/ab_miner.py --a . --b . --algo x11 --rounds 4 --seconds 6 --env-b $HW1 > $D/ab_x11_hw1.json 2> $D/ab_x11_hw1.err && cat $D/ab_x11_hw1.json &&
for a in sha256d scrypt x11; do
  timeout -k 10 360 python tools/switch_ab.py --algo $a --env-b $HW1 > $D/switch_${a}_hw1.jsonl 2> $D/switch_${a}_hw1.err || exit 1
  cut -c1-300 $D/switch_${a}_hw1.jsonl
done &&
timeout -k 10 200 python tools/rss_breakdown.py --only default,hw_queues_1,hw_queues_1+no_fragments > $D/rss.jsonl 2> $D/rss.err && echo "rss ok" &&
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python -c "
import json
from otedama_amd.parallel.node_probe import measure_node
print(json.dumps(measure_node(2, seconds=10, expected_per_gpu=9.7e9, shares_per_gpu=25.0)))
" > $D/node2_gloo.json 2> $D/node2_gloo.err && echo "node2 ok" &&
timeout -k 10 200 python -u -m pytest tests/test_miner_probe.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_miner_probe.log 2>&1 && tail -3 $D/pytest_miner_probe.log &&
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > $D/bench.json 2> $D/bench.err && echo "bench ok" && cut -c1-600 $D/bench.json
