#!/bin/bash
# Round 3: one vs two search streams in the production miner, exact windows, same tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3ab}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 400 python tools/ab_miner.py --a . --b . --env-a OTEDAMA_SEARCH_STREAMS=1 --rounds 4 --seconds 10 > $O/streams_1_vs_2.json 2> $O/streams.err && echo "streams ab ok"
