#!/bin/bash
# Round 3: share-latency probe alone, three times in one session (12-17 shares per probe: its p50 is noisy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3au}
mkdir -p $O
timeout -k 10 200 python -u -c "
import json
from otedama_amd.engine.latency_probe import measure_share_latency
for i in range(3):
    r = measure_share_latency(device_index=0, seconds=10.0)
    print(json.dumps({k: r[k] for k in ('p50_ms', 'device_hit_to_accept_p50_ms', 'device_hit_to_accept_p95_ms', 'hit_to_accept_p50_ms', 'accepted', 'engine_hashrate')}), flush=True)
" > $O/latency.jsonl 2> $O/latency.err && echo "latency ok"
