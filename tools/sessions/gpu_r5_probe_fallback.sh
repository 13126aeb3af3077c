#!/bin/bash
# Round 5: the bench's data-plane probe meeting a real RCCL failure. Two ranks share the one GPU through the driver's
# torchrun line; their probe children try an RCCL group on the same device, which RCCL refuses ("Duplicate GPU
# detected"), so both ranks fall back to gloo together and the headline is still measured.
set -o pipefail
out=gpurun_out/${1:-r5ac}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo OTEDAMA_BENCH_PROBE=1 OTEDAMA_PROBE_TIMEOUT=60 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 \
  bench.py --gpus 2 --steps 3 --warmup 1 --miner-seconds 0 --node-seconds 0 --pool-seconds 0 --cpu-seconds 0 \
  --no-latency --scrypt-steps 2 --x11-steps 2 > "$out/bench.json" 2> "$out/bench.err"
