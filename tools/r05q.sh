#!/bin/bash
# fp32 radius sqrt with the integer correction (FKS_SQRT_INTFIX=1, ab/libfks_sqint.so): the
# correct-rounding check and the fp32 parity tests on that build, then the 19-seed fp32
# kernel alternated with the in-tree build.
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
LIB=$PWD/fate-llm_amd/ab/libfks_sqint.so
FKS_LIB_OVERRIDE=$LIB timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_selfcheck.py tests/test_gpu_parity.py tests/test_gpu_c4.py > $OUT/pytest_sqint.log 2>&1 || { tail -5 $OUT/pytest_sqint.log; exit 1; }
tail -1 $OUT/pytest_sqint.log
AB_DT=f32 AB_SEEDS=19 timeout -k 10 600 python -u tools/ab_apply.py intree $LIB intree $LIB > $OUT/ab_sqint.log 2>&1
