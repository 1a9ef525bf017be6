#!/bin/bash
# A/B of the eight-item torch_rocm kernel: wave-uniform tensor lookups (1: global, 2: LDS copy)
# or the per-lane search (in tree), one-seed calls and 32-seed launches on the
# 7B layout, builds alternated.
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
for round in 1 2; do
  for lib in intree fate-llm_amd/ab/libfks_u1.so fate-llm_amd/ab/libfks_u2.so; do
    echo "== $lib" >> $OUT/ab_u.log
    if [ $lib = intree ]; then
      FKS_STREAM_MODE=torch_rocm timeout -k 10 200 python -u tools/perf_smallk.py --ks 1,32 --calls perturb,zo_step >> $OUT/ab_u.log 2>&1 || exit $?
    else
      FKS_LIB_OVERRIDE=$PWD/$lib FKS_STREAM_MODE=torch_rocm timeout -k 10 200 python -u tools/perf_smallk.py --ks 1,32 --calls perturb,zo_step >> $OUT/ab_u.log 2>&1 || exit $?
    fi
  done
done
