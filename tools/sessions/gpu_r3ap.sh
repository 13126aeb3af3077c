#!/bin/bash
# Round 3: pool restart mid-run on the MI355X: the engine loses the session, pauses its device process, reconnects
# with backoff and resumes (SV2 SHA-256d, V1 scrypt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3ap}
mkdir -p $O
true &&
timeout -k 10 300 python -u tools/soak.py --seconds 120 --protocol sv2 --bounce-at 50 --workdir $O/sv2_bounce \
  > $O/soak_sv2_bounce.jsonl 2>&1 && echo "sv2 bounce ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 100 --protocol v1 --algorithm scrypt --bounce-at 45 \
  --workdir $O/v1_scrypt_bounce > $O/soak_v1_scrypt_bounce.jsonl 2>&1 && echo "v1 scrypt bounce ok"
