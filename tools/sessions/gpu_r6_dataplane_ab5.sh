#!/bin/bash
# Round 6: native (R2 through the one-rank RCCL group) / native with R2 as a local copy (OTEDAMA_RCCL_LOCAL_R2=1) /
# torch, interleaved on one box: is the -0.25% the per-step RCCL op or the communicator's existence?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r6_ab5}
mkdir -p "$out"
args="--steps 20 --warmup 5 --single-midstate-headers 0 --scrypt-steps 0 --x11-steps 0 --miner-seconds 0 --comm-ops 0
      --cpu-seconds 0 --no-latency --node-seconds 0 --pool-seconds 0"
for i in 1 2; do
  for mode in native local torch; do  # native: GPU_MAX_HW_QUEUES raised to 8 in-process
    if [[ $mode == local ]]; then
      OTEDAMA_RCCL_LOCAL_R2=1 OTEDAMA_BENCH_DETAIL="$out/detail_${mode}_$i.json" timeout -k 10 200 python bench.py $args \
        > "$out/${mode}_$i.json" 2>> "$out/err.log" || exit $?
    else
      OTEDAMA_BENCH_COMM=$mode OTEDAMA_BENCH_DETAIL="$out/detail_${mode}_$i.json" timeout -k 10 200 python bench.py \
        $args > "$out/${mode}_$i.json" 2>> "$out/err.log" || exit $?
    fi
  done
done
