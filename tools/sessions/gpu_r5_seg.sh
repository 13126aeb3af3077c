#!/bin/bash
# Round 5: the segmented scrypt ROMix (OTEDAMA_SCRYPT_SEGMENTS) -- numerics, then the comm-under-load A/B against the
# one-launch kernel (rate and op latency per segment count), and X11's loaded numbers.
set -o pipefail
out=gpurun_out/${1:-r5h}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k scrypt -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_scrypt.log" 2>&1 || exit $?
timeout -k 10 500 python -m otedama_amd.parallel.comm_probe --algorithms scrypt --seconds 4 --windows 2 \
  --variants "OTEDAMA_SCRYPT_SEGMENTS=4;OTEDAMA_SCRYPT_SEGMENTS=8;OTEDAMA_SCRYPT_SEGMENTS=16;OTEDAMA_SCRYPT_SEGMENTS=32" \
  > "$out/comm_scrypt.json" 2> "$out/comm_scrypt.err" || exit $?
timeout -k 10 300 python -m otedama_amd.parallel.comm_probe --algorithms x11 --seconds 4 --windows 2 \
  > "$out/comm_x11.json" 2> "$out/comm_x11.err" || exit $?
timeout -k 10 200 python -c "
import json
from otedama_amd.pool.pool_probe import measure_pool
print(json.dumps(measure_pool(1)))" > "$out/pool.json" 2> "$out/pool.err"
