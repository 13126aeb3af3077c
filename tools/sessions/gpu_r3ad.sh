#!/bin/bash
# Round 3: single-midstate SHA-256d (BASELINE config 2) under its abort-poll forms, same process; grid sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3ad}
mkdir -p $O
true &&
timeout -k 10 90 tools/bin/sha_single_ab 5 1536 > $O/single_1536.json 2> $O/single.err && echo "1536 ok" &&
timeout -k 10 90 tools/bin/sha_single_ab 3 3072 > $O/single_3072.json 2>> $O/single.err && echo "3072 ok" &&
timeout -k 10 90 tools/bin/sha_single_ab 3 1024 > $O/single_1024.json 2>> $O/single.err && echo "1024 ok" &&
timeout -k 10 90 tools/bin/sha_single_ab 5 1536 > $O/single_1536_b.json 2>> $O/single.err && echo "1536 again ok"
