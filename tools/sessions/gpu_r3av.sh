#!/bin/bash
# Round 3: latency probe with its 3 s warm-up (cold first shares not recorded): three probes in one session, then the
# GPU test that holds it under 2 ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3av}
mkdir -p $O
timeout -k 10 200 python -u -c "
import json
from otedama_amd.engine.latency_probe import measure_share_latency
for i in range(3):
    r = measure_share_latency(device_index=0, seconds=6.0)
    print(json.dumps({k: r[k] for k in ('p50_ms', 'device_hit_to_accept_p50_ms', 'device_hit_to_accept_p95_ms', 'hit_to_accept_p50_ms', 'accepted', 'engine_hashrate', 'engine_hashrate_trace_ghs')}), flush=True)
" > $O/latency.jsonl 2> $O/latency.err && echo "latency ok" &&
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_devproc.py -k share_latency > $O/pytest_latency.txt 2>&1 && echo "test ok"
