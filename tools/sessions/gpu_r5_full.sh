#!/bin/bash
# Round 5: reserved-CU comm A/B, then the bench as the driver runs it (N=1).
set -o pipefail
out=gpurun_out/${1:-r5f}
mkdir -p "$out"
timeout -k 10 600 python -m otedama_amd.parallel.comm_probe --seconds 4 --windows 2 \
  --reserves "0;0,1,2,3,4,5,6,7;0,32,64,96,128,160,192,224" > "$out/comm.json" 2> "$out/comm.err" || exit $?
timeout -k 10 620 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
