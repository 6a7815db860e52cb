#!/bin/bash
# Host sanitizers over the CPU code the tests run: the oracle restatements rebuilt with
# -fsanitize=address,undefined and the CPU test suite (-m "not gpu") run against them.
# GPU code is not sanitized (not available on this pool).
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle sanitize || exit 1
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
GB_ORACLE_SO=$PWD/oracle/_build/liboracle_san.so \
LD_PRELOAD="$ASAN $UBSAN" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout -k 10 1200 python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
