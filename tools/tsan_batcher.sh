#!/bin/bash
# ThreadSanitizer build of the host micro-batcher (weaviate_amd/csrc/batcher.hip)
# against a CPU mock of the batch search, driven by many threads.  CPU only.
# clang's TSan runtime (ROCm's clang++): GCC 11's libtsan does not intercept
# pthread_cond_clockwait (std::condition_variable::wait_for) and then reports
# a false "double lock" on the next wait.
set -e
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/wv_tsan"
mkdir -p "$OUT"
CXX=/opt/rocm/lib/llvm/bin/clang++
[ -x "$CXX" ] || CXX=clang++
"$CXX" -std=c++17 -O1 -g -fsanitize=thread -fno-omit-frame-pointer -pthread -x c++ "$REPO/tools/tsan_batcher.cpp" \
    -o "$OUT/tsan_batcher"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/tsan_batcher" "${1:-48}" "${2:-60}"
