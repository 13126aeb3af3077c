#!/bin/bash
# Rehearse bench.py's N=2 control flow on ONE GPU: two torchrun ranks share cuda:0 over gloo
# (R1/R2/R3 collectives, barriers, MAX-over-ranks timing, rank-0-only output). RCCL is not exercised
# (it refuses two ranks per GPU); the real N=2/4/8 runs are the driver's 8-GPU scaling bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --scrypt-steps 0 \
  > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err && echo "rehearse n2 ok"
