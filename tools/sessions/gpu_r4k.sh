#!/bin/bash
# Round 4, GPU pass k: production-path soaks on the round-4 runtime (host-stored abort word, per-launch clock
# probes, scrypt write-loop polls and staggered halves, X11 digest planes, the node's inline ops and host buffers):
# the local pool with a job every 5 s and a block every 45 s, 0 rejects and no RSS growth required.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 420 python -u tools/soak.py --seconds 300 --protocol sv2 --workdir $O/sha_sv2 > $O/soak_sha256d_sv2.jsonl 2>&1 && echo "sha256d soak ok" && tail -1 $O/soak_sha256d_sv2.jsonl | cut -c1-400 &&
timeout -k 10 300 python -u tools/soak.py --seconds 180 --protocol v1 --algorithm scrypt --workdir $O/scrypt_v1 > $O/soak_scrypt_v1.jsonl 2>&1 && echo "scrypt soak ok" && tail -1 $O/soak_scrypt_v1.jsonl | cut -c1-400 &&
timeout -k 10 240 python -u tools/soak.py --seconds 120 --protocol sv2 --algorithm x11 --workdir $O/x11_sv2 > $O/soak_x11_sv2.jsonl 2>&1 && echo "x11 soak ok" && tail -1 $O/soak_x11_sv2.jsonl | cut -c1-400 &&
timeout -k 10 300 python -u tools/soak.py --seconds 120 --protocol sv2 --node 2 --workdir $O/node2 > $O/soak_node2_sv2.jsonl 2>&1 && echo "node soak ok" && tail -1 $O/soak_node2_sv2.jsonl | cut -c1-400
