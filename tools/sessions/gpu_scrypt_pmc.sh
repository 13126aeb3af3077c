#!/bin/bash
# scrypt ROMix memory-path counters (one small counter group per pass, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
run() {  # run <tag> <gap> <counters...>
  local tag=$1 gap=$2; shift 2
  timeout -k 10 200 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 tools/prof_kernels.py scrypt $gap > gpurun_out/pmc_$tag.log 2>&1 && echo "pmc $tag ok"
}
for gap in 1 2 8; do
  run ta_g$gap $gap TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE &&
  run tlb_g$gap $gap TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE &&
  run tcp_g$gap $gap TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE || exit 1
done
