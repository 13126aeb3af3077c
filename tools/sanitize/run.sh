#!/usr/bin/env bash
# Host-only sanitizer builds of the native runtime + the job-epoch race stress.
# Usage: tools/sanitize/run.sh [seconds-per-run]   (also: make sanitize)
# GPU sanitizers are not used (no GPU ASan/XNACK on this pool): this covers the C++ host code only.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${OTEDAMA_SANITIZE_OUT:-$ROOT/build/sanitize}"
SECS="${1:-4}"
mkdir -p "$OUT"
SRCS=("$ROOT/csrc/cpu/sha256_cpu.cpp" "$ROOT/csrc/cpu/job_prepare.cpp" "$ROOT/csrc/cpu/aead.cpp" "$ROOT/csrc/cpu/x11_cpu.cpp"
      "$ROOT/csrc/runtime/miner_common.cpp" "$ROOT/tools/sanitize/stress_runtime.cpp")
# ROCm clang: its compiler-rt TSan intercepts pthread_cond_clockwait (libstdc++ wait_for);
# GCC 11's libtsan does not and reports a false "double lock" on the pause path.
CXX="${CXX:-/opt/rocm/lib/llvm/bin/clang++}"
FLAGS=(-std=c++17 -O1 -g -fno-omit-frame-pointer -march=x86-64-v2 "-I$ROOT/csrc/include" -pthread
       -DOTEDAMA_STRESS_HOOKS)

declare -A SAN=([tsan]="-fsanitize=thread" [asan]="-fsanitize=address,undefined -fno-sanitize-recover=undefined")
rc=0
for name in tsan asan; do
  bin="$OUT/stress_runtime_$name"
  # shellcheck disable=SC2086
  "$CXX" "${FLAGS[@]}" ${SAN[$name]} "${SRCS[@]}" -o "$bin" -lcrypto
  echo "== $name: $bin $SECS"
  if [ "$name" = tsan ]; then
    TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$bin" "$SECS" || rc=$?
  else
    ASAN_OPTIONS="detect_leaks=1 abort_on_error=0" UBSAN_OPTIONS="print_stacktrace=1" "$bin" "$SECS" || rc=$?
  fi
  [ "$rc" -eq 0 ] || { echo "$name run failed (rc=$rc)"; exit "$rc"; }
done
# libFuzzer (ASan + UBSan) over the SV2 frame scanner and the CPU hash paths.
fz="$OUT/fuzz_native"
"$CXX" -std=c++17 -O1 -g -march=x86-64-v2 "-I$ROOT/csrc/include" -fsanitize=fuzzer,address,undefined \
  -fno-sanitize-recover=undefined -mllvm -asan-globals=0 "$ROOT/tools/sanitize/fuzz_native.cpp" \
  "$ROOT/csrc/cpu/sv2_frame.cpp" "$ROOT/csrc/cpu/sha256_cpu.cpp" "$ROOT/csrc/cpu/x11_cpu.cpp" -o "$fz" -lcrypto
echo "== fuzz: $fz ${SECS}s"
(cd "$OUT" && "$fz" -max_total_time="$SECS" -max_len=2048 -print_final_stats=1) || { echo "fuzz failed"; exit 1; }
echo "sanitize: tsan + asan/ubsan + fuzz clean"
