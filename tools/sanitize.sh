#!/bin/bash
# The CPU suite's host-code tests under AddressSanitizer + UBSan: the
# oracle and libfks.so's host code built with -fsanitize=address,undefined
# (make -C oracle asan; make -C fate-llm_amd asan), loaded through FKS_ORACLE_LIB /
# FKS_LIB_OVERRIDE with g++'s ASan runtime preloaded (python itself is not instrumented).
# No GPU: device code is not sanitized (not available on this pool).
#   bash tools/sanitize.sh [extra pytest args]
set -e
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -C fate-llm_amd asan
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
export LD_PRELOAD="$ASAN_LIB $UBSAN_LIB"
# leaks of the (uninstrumented) interpreter are not ours; stop at the first real error
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export FKS_ORACLE_LIB=$PWD/oracle/liboracle_asan.so
export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_asan.so
python -m pytest -q -x -m "not gpu" -p no:cacheprovider \
  tests/test_capi_host.py tests/test_oracle_golden.py tests/test_bitslice_host.py tests/test_libm_serial.py \
  tests/test_shard_gloo.py tests/test_temper_fold.py tests/test_seed_shard_gloo.py "$@"
