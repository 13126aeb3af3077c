#!/bin/bash
# X11 job switch with every stage polling the abort word: the switch probe (engine -> device process -> new batch)
# for X11 and scrypt, then an interleaved same-session A/B of the production miner's X11 rate with the middle-stage
# polls on (A) and off (B, OTEDAMA_X11_MIDPOLL=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/x11_switch
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 200 python -c "
import json
from otedama_amd.engine.latency_probe import measure_job_switch
for algo in ('x11', 'scrypt', 'sha256d'):
    print(json.dumps({algo: measure_job_switch(0, algo)}), flush=True)
" > gpurun_out/x11_switch/switch.jsonl 2> gpurun_out/x11_switch/switch.err && cat gpurun_out/x11_switch/switch.jsonl &&
timeout -k 10 300 python tools/ab_miner.py --a . --b . --algo x11 --rounds 4 --seconds 6 --env-b OTEDAMA_X11_MIDPOLL=0 \
  > gpurun_out/x11_switch/ab_x11.json 2> gpurun_out/x11_switch/ab_x11.err && cat gpurun_out/x11_switch/ab_x11.json
