#!/bin/bash
# Round 4, GPU pass i: bisect bench.py's preamble for the in-bench miner scrypt rate (tools/miner_bench_bisect.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4i
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 600 python tools/miner_bench_bisect.py > $D/bisect.jsonl 2> $D/bisect.err; rc=$?; cat $D/bisect.jsonl; exit $rc
