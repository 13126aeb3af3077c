#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" &&
{ timeout -k 10 120 python -m otedama_amd doctor --json > gpurun_out/doctor.json 2>&1; rc=$?; echo "doctor rc=$rc"; [ $rc -le 2 ]; }
