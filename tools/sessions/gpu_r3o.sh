#!/bin/bash
# Round 3: host resident set per HIP stream / hardware queue, with runtime knobs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3o}
mkdir -p $O
true &&
timeout -k 10 60 tools/bin/stream_rss > $O/default.json 2>&1 && echo "default ok" &&
ROC_AQL_QUEUE_SIZE=1024 timeout -k 10 60 tools/bin/stream_rss > $O/aql1024.json 2>&1 && echo "aql ok" &&
GPU_MAX_HW_QUEUES=1 timeout -k 10 60 tools/bin/stream_rss > $O/hwq1.json 2>&1 && echo "hwq1 ok" &&
HIP_HOST_COHERENT=0 timeout -k 10 60 tools/bin/stream_rss > $O/noncoherent.json 2>&1 && echo "noncoh ok"
