#!/bin/bash
# Round 6: does the native data plane (R2 as an RCCL all_gather on the comm stream, one-rank group at N=1) cost the
# headline anything against torch (a plain device copy at world 1)? Alternating runs of the headline section only,
# driver step counts, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r6_ab}
mkdir -p "$out"
args="--steps 20 --warmup 5 --single-midstate-headers 0 --scrypt-steps 0 --x11-steps 0 --miner-seconds 0 --comm-ops 0
      --cpu-seconds 0 --no-latency --node-seconds 0 --pool-seconds 0"
for i in 1 2 3; do
  for mode in native torch; do
    OTEDAMA_BENCH_COMM=$mode OTEDAMA_BENCH_DETAIL="$out/detail_${mode}_$i.json" timeout -k 10 200 python bench.py $args \
      > "$out/${mode}_$i.json" 2>> "$out/err.log" || exit $?
  done
done
