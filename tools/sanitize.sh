#!/bin/bash
# Runs the CPU-side sanitizer builds (make -C k8s-1m_amd sanitize builds them
# first): the ksgather concurrency driver under ThreadSanitizer and under
# AddressSanitizer + UBSan, then the relay tests (gRPC CollectScore over the
# ASan libksgather) and the oracle tests (ASan liboracle, ASan libksynth) in a
# Python whose first preloaded library is the ASan runtime; libksched's
# host-thread protocols (ksched_sync.hpp: rendezvous, run queue, thread pool)
# through tools/sync_stress.cpp under both.  Log:
# profiles/r6/sanitize/sanitize.log; exits non-zero on any report.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${SANITIZE_OUT:-$R/profiles/r6/sanitize}
mkdir -p "$OUT"
LOG=$OUT/sanitize.log
: > "$LOG"
B=$R/k8s-1m_amd/build/san
say() { echo "$*" | tee -a "$LOG"; }
say "sanitize run $(date -u +%Y-%m-%dT%H:%M:%SZ) on $(uname -m), $(g++ --version | head -1)"
make -s -C "$R/oracle" sanitize >> "$LOG" 2>&1 || { say "oracle sanitizer build FAILED"; exit 1; }

say "== ksg_stress under ThreadSanitizer"
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$B/ksg_stress_tsan" >> "$LOG" 2>&1 || { say "TSAN FAILED"; exit 1; }
say "== ksg_stress under AddressSanitizer + UBSan"
ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" \
  "$B/ksg_stress_asan" >> "$LOG" 2>&1 || { say "ASAN FAILED"; exit 1; }
say "== sync_stress (libksched host threads) under ThreadSanitizer"
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$B/sync_stress_tsan" >> "$LOG" 2>&1 || { say "TSAN FAILED"; exit 1; }
say "== sync_stress under AddressSanitizer + UBSan"
ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" \
  "$B/sync_stress_asan" >> "$LOG" 2>&1 || { say "ASAN FAILED"; exit 1; }

# Python itself is not instrumented: the ASan runtime goes first in the
# preload list (whatever is preloaded already stays after it), leaks are not
# reported (the interpreter's own allocations), every other report aborts.
ASAN_RT=$(g++ -print-file-name=libasan.so)
UBSAN_RT=$(g++ -print-file-name=libubsan.so)
export LD_PRELOAD="$ASAN_RT $UBSAN_RT${LD_PRELOAD:+ $LD_PRELOAD}"
export ASAN_OPTIONS="detect_leaks=0 halt_on_error=1 verify_asan_link_order=0"
export UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1"
export KSCHED_HOST_LIB_DIR=$R/k8s-1m_amd/ksched/lib/asan
export ORACLE_LIB=$R/oracle/_build/asan/liboracle.so
cd "$R"
say "== relay tests (libksgather: ASan + UBSan)"
python -m pytest -q -p no:cacheprovider tests/test_relay.py >> "$LOG" 2>&1 || { say "RELAY TESTS FAILED"; exit 1; }
say "== oracle tests (liboracle, libksynth: ASan + UBSan)"
python -m pytest -q -p no:cacheprovider tests/test_oracle_kat.py tests/test_oracle_semantics.py \
  tests/test_oracle_spread.py tests/test_golden.py tests/test_stream_oracle.py -m "not gpu" >> "$LOG" 2>&1 \
  || { say "ORACLE TESTS FAILED"; exit 1; }
if grep -q "ERROR: AddressSanitizer\|runtime error:\|WARNING: ThreadSanitizer" "$LOG"; then
  say "SANITIZER REPORTS FOUND"; exit 1
fi
say "sanitize: clean"
