#!/bin/bash
# Round 3: kernel A/B against the pre-abort tree (ab_old), then the production entry points rehearsal
# (otedama run with device processes; otedama node --gpus 2 over gloo sharing the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3e}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 500 python tools/ab_kernels.py --rounds 3 > $O/ab_kernels.jsonl 2> $O/ab_kernels.err && echo "ab ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 20 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok"
