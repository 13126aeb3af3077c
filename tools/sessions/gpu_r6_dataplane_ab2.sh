#!/bin/bash
# Round 6: where does the native data plane's -0.25% at N=1 come from? native / torch / native with 8 hardware
# queues per process (GPU_MAX_HW_QUEUES: RCCL's own streams may push the search streams onto shared queues).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r6_ab2}
mkdir -p "$out"
args="--steps 20 --warmup 5 --single-midstate-headers 0 --scrypt-steps 0 --x11-steps 0 --miner-seconds 0 --comm-ops 0
      --cpu-seconds 0 --no-latency --node-seconds 0 --pool-seconds 0"
for i in 1 2; do
  for mode in native torch q8; do
    if [[ $mode == q8 ]]; then
      GPU_MAX_HW_QUEUES=8 OTEDAMA_BENCH_DETAIL="$out/detail_${mode}_$i.json" timeout -k 10 200 python bench.py $args \
        > "$out/${mode}_$i.json" 2>> "$out/err.log" || exit $?
    else
      OTEDAMA_BENCH_COMM=$mode OTEDAMA_BENCH_DETAIL="$out/detail_${mode}_$i.json" timeout -k 10 200 python bench.py \
        $args > "$out/${mode}_$i.json" 2>> "$out/err.log" || exit $?
    fi
  done
done
