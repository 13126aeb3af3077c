#!/bin/bash
# Round 3: Stratum V1 soaks with a high share rate (scrypt: vardiff ramps through mining.set_difficulty) and the
# SV2 extended-channel path is not covered here (CPU tests); checks the raised-target filter on V1 too.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3am}
mkdir -p $O
true &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol v1 --algorithm scrypt --workdir $O/v1_scrypt \
  > $O/soak_v1_scrypt.jsonl 2>&1 && echo "v1 scrypt ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol v1 --algorithm sha256d --difficulty 0.05 \
  --workdir $O/v1_sha_lowdiff > $O/soak_v1_sha_lowdiff.jsonl 2>&1 && echo "v1 sha low-diff ok"
