#!/bin/bash
# Round 5: the segmented scrypt ROMix with a resident-size launch grid (no second round of blocks per segment).
set -o pipefail
out=gpurun_out/${1:-r5j}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k segmented -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_seg.log" 2>&1 || exit $?
timeout -k 10 500 python -m otedama_amd.parallel.comm_probe --algorithms scrypt --seconds 4 --windows 2 \
  --variants "OTEDAMA_SCRYPT_HALVES=0&OTEDAMA_SCRYPT_SEGMENTS=32;OTEDAMA_SCRYPT_HALVES=0&OTEDAMA_SCRYPT_SEGMENTS=32&OTEDAMA_SCRYPT_SEG_GRID=resident;OTEDAMA_SCRYPT_HALVES=0&OTEDAMA_SCRYPT_SEGMENTS=16&OTEDAMA_SCRYPT_SEG_GRID=resident;OTEDAMA_SCRYPT_HALVES=0&OTEDAMA_SCRYPT_SEGMENTS=64&OTEDAMA_SCRYPT_SEG_GRID=resident" \
  > "$out/comm_scrypt.json" 2> "$out/comm_scrypt.err"
