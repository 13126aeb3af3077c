#!/bin/bash
# Round 3: which runtime knob owns the ~190 MB of host memory per hardware queue (tools/stream_rss.hip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3w
mkdir -p $O
true &&
for kv in NONE=1 HIP_FORCE_DEV_KERNARG=1 GPU_STAGING_BUFFER_SIZE=1 GPU_PINNED_XFER_SIZE=1 HSA_ENABLE_SDMA=0 \
          ROC_SIGNAL_POOL_SIZE=64 HIP_MEM_POOL_SUPPORT=0 GPU_MAX_REMOTE_MEM_SIZE=1 HSA_SCRATCH_SINGLE_LIMIT=1048576 \
          DEBUG_HIP_BLOCK_SYNC=0 GPU_IMAGE_DMA=0 ROC_USE_FGS_KERNARG=0 HSA_NO_SCRATCH_RECLAIM=1; do
  env $kv timeout -k 10 60 tools/bin/stream_rss > $O/$kv.json 2>&1 || exit 1
done && echo "knobs ok"
