#!/bin/bash
# Round 5 GPU check: smoke (oracle comparisons), the GPU test suite, and the bench's pool section alone.
set -o pipefail
out=gpurun_out/${1:-r5b}
mkdir -p "$out"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --single-midstate-headers 0 --scrypt-steps 0 --x11-steps 0 \
  --miner-seconds 0 --no-latency --cpu-seconds 0 --node-seconds 0 > "$out/pool.json" 2> "$out/pool.err"
