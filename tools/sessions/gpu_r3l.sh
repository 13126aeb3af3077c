#!/bin/bash
# Round 3: SHAvite / JH variants against the round-2 kernels (time + SQ VALU counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3l}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 120 tools/bin/x11_variants 5 > $O/x11_variants.json 2> $O/x11_variants.err && echo "x11 variants ok" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --stats -d $O/pmc -o run --output-format csv -- tools/bin/x11_variants 1 > $O/pmc.log 2>&1 && echo "pmc ok"
