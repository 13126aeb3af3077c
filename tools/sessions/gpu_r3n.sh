#!/bin/bash
# Round 3: device-process resident set, phase by phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3n}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 120 python tools/rss_probe.py > $O/rss_default.json 2> $O/rss_default.err && echo "rss default ok" &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 90 --timeout-method thread -k startup > $O/pytest_startup.txt 2>&1 && echo "startup test ok" &&
HIP_HOST_COHERENT=0 timeout -k 10 120 python tools/rss_probe.py > $O/rss_noncoherent.json 2> $O/rss_noncoherent.err && echo "rss knob ok"
