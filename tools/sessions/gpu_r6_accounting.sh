#!/bin/bash
# Round 6: the miner's hash counter against the Poisson count of its hits (tools/experiments/hash_accounting.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r6_acct}
mkdir -p "$out"
timeout -k 10 150 python tools/experiments/hash_accounting.py 20 scrypt,sha256d,x11 > "$out/halves.jsonl" 2> "$out/err.log" &&
OTEDAMA_SCRYPT_HALVES=0 timeout -k 10 100 python tools/experiments/hash_accounting.py 20 scrypt > "$out/single.jsonl" 2>> "$out/err.log"
