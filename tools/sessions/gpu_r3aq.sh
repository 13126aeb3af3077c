#!/bin/bash
# Round 3: long production soak (SV2 SHA-256d, 8 minutes): engine + device-process RSS over time, 0 rejects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3aq}
mkdir -p $O
true &&
timeout -k 10 600 python -u tools/soak.py --seconds 480 --every 15 --protocol sv2 --workdir $O/sv2_long \
  > $O/soak_sv2_480s.jsonl 2>&1 && echo "long soak ok"
