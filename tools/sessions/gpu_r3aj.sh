#!/bin/bash
# Round 3: bench.py's multi-rank paths on the one-GPU box with gloo (ranks share the MI355X; RCCL refuses two ranks
# on one GPU): --gpus 2 through bench.py's own launcher, --gpus 4 through the driver's torchrun command line.
# scrypt is skipped: two 128 GiB pads on one GPU would leave too little HBM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${R3_TAG:-r3aj}
mkdir -p $O
export OTEDAMA_DIST_BACKEND=gloo
true &&
timeout -k 10 240 python -u bench.py --gpus 2 --steps 4 --warmup 1 --scrypt-steps 0 --no-latency \
  > $O/bench_n2_launcher.json 2> $O/bench_n2_launcher.err && echo "n2 launcher ok" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 4 --steps 4 --warmup 1 --scrypt-steps 0 --no-latency \
  > $O/bench_n4_torchrun.json 2> $O/bench_n4_torchrun.err && echo "n4 torchrun ok"
