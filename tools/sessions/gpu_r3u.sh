#!/bin/bash
# Round 3: exact-window production-miner A/B (split abort poll vs previous commit vs pre-abort tree) and the
# SHA-256d launch paths in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3u}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 300 python tools/sha_paths.py > $O/sha_paths.json 2> $O/sha_paths.err && echo "sha paths ok" &&
timeout -k 10 300 python tools/ab_miner.py --a . --b ab_prev --rounds 3 --seconds 10 > $O/ab_miner_prev.json 2> $O/ab_miner_prev.err && echo "ab prev ok" &&
timeout -k 10 300 python tools/ab_miner.py --a . --b ab_old --rounds 3 --seconds 10 > $O/ab_miner_old.json 2> $O/ab_miner_old.err && echo "ab old ok"
