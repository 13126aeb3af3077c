#!/bin/bash
# BASELINE config 5 over a long window: the pool probe (one MI355X, SHA-256d + scrypt streams over SV2, 0.1 s target
# share interval) recording 300 s of steady state instead of the bench's 25 s, to see whether vardiff stays put and
# how the validation quantiles look over thousands of samples.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5pool}
mkdir -p "$out"
timeout -k 10 600 python -u -c "
import json, threading, time
from otedama_amd.pool.pool_probe import measure_pool
def tick():  # progress line while the window records
    while True:
        time.sleep(50); print('pool probe running', flush=True)
threading.Thread(target=tick, daemon=True).start()
r = measure_pool(1, seconds=300.0)
json.dump(r, open('$out/pool_long.json', 'w'), indent=1)
print(json.dumps({a: {'acc': v['accepted'], 'rej': v['rejected'], 'p': v['validate_ms'],
                      'w': [(w['retargets'], w['converged_after_s'], w['settled_after_s'], w['window_opened_after_s'],
                             w['interval_vs_target']) for w in v['workers']]}
                  for a, v in r['algorithms'].items()}))
" > "$out/pool_long.log" 2>&1
