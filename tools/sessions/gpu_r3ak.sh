#!/bin/bash
# Round 3: production-path soaks on the latest tree (device processes, hit ring, abort word): SV2 and V1 SHA-256d
# and SV2 scrypt against the local validating pool with fast job/block churn; engine + device-process RSS tracked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3ak}
mkdir -p $O
true &&
timeout -k 10 300 python -u tools/soak.py --seconds 150 --protocol sv2 --workdir $O/sv2 > $O/soak_sv2.jsonl 2>&1 && echo "sv2 ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol v1 --workdir $O/v1 > $O/soak_v1.jsonl 2>&1 && echo "v1 ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol sv2 --algorithm scrypt \
  --workdir $O/scrypt > $O/soak_scrypt.jsonl 2>&1 && echo "scrypt ok"
