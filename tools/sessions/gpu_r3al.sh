#!/bin/bash
# Round 3: scrypt soak again after the engine drops shares below a raised share target (r3ak: 3 low-difficulty
# rejects in the vardiff ramp right after connect), and the SV2 SHA-256d soak once more.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3al}
mkdir -p $O
true &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol sv2 --algorithm scrypt --workdir $O/scrypt \
  > $O/soak_scrypt.jsonl 2>&1 && echo "scrypt ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol sv2 --algorithm x11 --workdir $O/x11 \
  > $O/soak_x11.jsonl 2>&1 && echo "x11 ok"
