#!/bin/bash
# Round 3: two-chain V kernel under its abort-poll forms (same process), bench hit counts over several synthetic
# seeds (each seed is one Poisson draw), and the whole GPU suite with the 256-blocks-per-CU single-midstate grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3ag}
mkdir -p $O
seeds() {
  for s in 2 3 4 5 6 7; do
    timeout -k 10 120 python -u bench.py --steps 4 --warmup 1 --seed $s --single-midstate-headers 0 --scrypt-steps 0 \
      --x11-steps 0 --no-latency > $O/seed_$s.json 2>> $O/seeds.err || return 1
    echo "seed $s ok"
  done
}
true &&
timeout -k 10 120 tools/bin/sha_v_ab 3 64 128 256 > $O/v_forms.json 2> $O/v_forms.err && echo "v forms ok" &&
seeds &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 && echo "gpu tests ok"
