#!/bin/bash
# Round 5: where the segmented scrypt ROMix loses its ~3% (S=1 = the segmented kernel's code in one launch).
set -o pipefail
out=gpurun_out/${1:-r5i}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k segmented -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_seg.log" 2>&1 || exit $?
timeout -k 10 400 python -m otedama_amd.parallel.comm_probe --algorithms scrypt --seconds 4 --windows 2 \
  --variants "OTEDAMA_SCRYPT_SEGMENTS=1;OTEDAMA_SCRYPT_SEGMENTS=2;OTEDAMA_SCRYPT_HALVES=0;OTEDAMA_SCRYPT_HALVES=0&OTEDAMA_SCRYPT_SEGMENTS=32" \
  > "$out/comm_scrypt.json" 2> "$out/comm_scrypt.err"
