#!/bin/bash
# Round 4, GPU pass o: production scrypt soak with the batched AVX-512 host verifier (16 candidates per pass) at an
# easy share difficulty, then a short SHA-256d SV2 soak on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 python -u tools/soak.py --seconds 180 --protocol v1 --algorithm scrypt --workdir $O/scrypt_v1 > $O/soak_scrypt_v1.jsonl 2>&1 && echo "scrypt soak ok" && tail -1 $O/soak_scrypt_v1.jsonl | cut -c1-500 &&
timeout -k 10 240 python -u tools/soak.py --seconds 120 --protocol sv2 --workdir $O/sha_sv2 > $O/soak_sha256d_sv2.jsonl 2>&1 && echo "sha256d soak ok" && tail -1 $O/soak_sha256d_sv2.jsonl | cut -c1-500
