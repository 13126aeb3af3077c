#!/bin/bash
# One GPU-box session, parameterised (replaces the per-round tools/gpu_r5_*.sh one-offs; those live on under
# tools/sessions/ for the record). Usage, from the repo root on the box (gpurun):
#
#   bash tools/gpu_session.sh <out-name> <step> [<step> ...]
#
# steps (each under its own time limit; the session stops at the first step that fails, since a GPU fault, abort or
# time-out must not be followed by more GPU work in the same call):
#   smoke                 __graft_entry__.smoke()
#   tests[=<-k expr>]     pytest -m gpu (optionally -k <expr>)
#   bench[=<args>]        bench.py with the driver's defaults (or the given args, ',' for ' ')
#   trace                 rocprofv3 --kernel-trace --stats over the production miner (tools/trace_native_miner.py)
#   pmc=<c1,c2,...>       rocprofv3 --pmc <counters> over the production miner (one pass; mind the per-block limits)
#   comm                  parallel/comm_probe.py (single-GPU comm under load)
#   scrypt-split          tools/prof_scrypt_split.py: per-kernel VALU / busy of the scrypt chain
# Results go to gpurun_out/<out-name>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
name=${1:?out name}
shift
out=gpurun_out/$name
mkdir -p "$out"
for step in "$@"; do
  key=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  echo "[gpu_session] $(date +%T) $step" >&2
  case "$key" in
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 ;;
    tests)
      if [[ -n "$arg" ]]; then
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$arg" \
          > "$out/pytest.log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
          > "$out/pytest.log" 2>&1
      fi ;;
    bench)
      # shellcheck disable=SC2086
      OTEDAMA_BENCH_DETAIL="$out/bench_detail.json" timeout -k 10 700 python bench.py ${arg//,/ } \
        > "$out/bench.json" 2> "$out/bench.err" ;;
    trace)
      timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv \
        -- python3 tools/trace_native_miner.py 3 > "$out/prof.log" 2>&1 ;;
    pmc)
      timeout -s KILL 120 rocprofv3 --pmc ${arg//,/ } -d "$out/pmc" -o run --output-format csv \
        -- python3 tools/trace_native_miner.py 3 > "$out/pmc.log" 2>&1 ;;
    comm)
      timeout -k 10 300 python -m otedama_amd.parallel.comm_probe > "$out/comm.json" 2> "$out/comm.err" ;;
    scrypt-split)
      timeout -k 10 300 python tools/prof_scrypt_split.py ${arg//,/ } > "$out/scrypt_split.json" 2> "$out/scrypt_split.err" ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  if [[ $rc -ne 0 ]]; then
    echo "[gpu_session] step $step failed with exit code $rc" >&2
    exit $rc
  fi
done
echo "[gpu_session] $(date +%T) done" >&2
