#!/bin/bash
# Round 3: production-path soaks through SV2 extended channels (miner-side extranonce rolling) over Noise NX with the
# EllSwift suite (SHA-256d), and through the legacy 32-byte suite on a standard channel (scrypt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3ao}
mkdir -p $O
true &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol sv2 --extended --noise ellswift --workdir $O/ext_noise \
  > $O/soak_sv2_extended_ellswift.jsonl 2>&1 && echo "extended+ellswift ok" &&
timeout -k 10 240 python -u tools/soak.py --seconds 90 --protocol sv2 --algorithm scrypt --noise legacy \
  --workdir $O/scrypt_legacy > $O/soak_sv2_scrypt_legacy_noise.jsonl 2>&1 && echo "scrypt legacy noise ok"
