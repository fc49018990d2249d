#!/usr/bin/env bash
# Builds the host runtime (csrc/runtime/*.cc) together with its concurrency stress test
# (csrc/runtime/tests/ps_stress.cc) under ThreadSanitizer and under AddressSanitizer+UBSan,
# and runs both. Host code only: GPU sanitizers are not available on MI355X boxes here.
#   tools/sanitize_runtime.sh [outdir]
set -euo pipefail
root="$(cd "$(dirname "$0")/.." && pwd)"
rt="$root/tensorflow_train_distributed_amd/csrc/runtime"
out="${1:-$(mktemp -d /tmp/ttd_san.XXXXXX)}"
mkdir -p "$out"
cxx="${CXX:-g++}"
common=(-std=c++17 -O1 -g -pthread -fno-omit-frame-pointer)
"$cxx" "${common[@]}" -fsanitize=thread "$rt"/*.cc "$rt/tests/ps_stress.cc" -o "$out/ps_stress_tsan" &
p1=$!
"$cxx" "${common[@]}" -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  "$rt"/*.cc "$rt/tests/ps_stress.cc" -o "$out/ps_stress_asan" &
p2=$!
wait $p1
wait $p2
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"
export ASAN_OPTIONS="detect_leaks=1 halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1 halt_on_error=1"
timeout -k 5 300 "$out/ps_stress_tsan" "$out" > "$out/tsan.log" 2>&1 || { cat "$out/tsan.log"; echo "TSAN FAILED"; exit 1; }
timeout -k 5 300 "$out/ps_stress_asan" "$out" > "$out/asan.log" 2>&1 || { cat "$out/asan.log"; echo "ASAN FAILED"; exit 1; }
grep -q PASS "$out/tsan.log" && grep -q PASS "$out/asan.log"
echo "runtime sanitizers: TSan + ASan/UBSan clean ($out)"
