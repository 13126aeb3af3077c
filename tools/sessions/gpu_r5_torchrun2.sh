#!/bin/bash
# Round 5: the driver's torchrun line at N=2 on the one GPU (gloo ranks sharing it), with the latency and node
# sections that run under torchrun's environment on rank 0 (the pool section needs a second GPU; the miner section's
# two 128 GiB scrypt pads do not fit one GPU next to each other).
set -o pipefail
out=gpurun_out/${1:-r5r}
mkdir -p "$out"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 4 --warmup 1 --miner-seconds 0 \
  --node-algorithms sha256d,x11 --pool-seconds 0 > "$out/bench.json" 2> "$out/bench.err"
