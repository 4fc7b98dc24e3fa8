#!/bin/bash
# Build and run the host runtime under ASan+UBSan and under TSan (CPU only:
# GPU sanitizers are not used on this pool).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/fm_sanitize}
mkdir -p "$OUT"
SRC="$ROOT/csrc/runtime/tests/promparse_fuzz.cpp"
g++ -std=c++17 -g -O1 -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -pthread "$SRC" -o "$OUT/promparse_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/promparse_asan"
g++ -std=c++17 -g -O1 -fsanitize=thread -pthread "$SRC" -o "$OUT/promparse_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/promparse_tsan"
