#!/bin/bash
# Round 4, GPU pass g: the production miner's scrypt rate after a bench-like 128 GiB torch pad (freed / held) and
# after a minute of scrypt load (tools/miner_ctx_ab.py --pad).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4g
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 600 python tools/miner_ctx_ab.py --algo scrypt --pad > $D/ctx_pad.jsonl 2> $D/ctx_pad.err; rc=$?; cat $D/ctx_pad.jsonl; exit $rc
