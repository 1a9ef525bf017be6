#!/bin/bash
# A/B of the eight-item torch_rocm kernel: with the next group's runs prefetched
# (FKS_PHX_VEC_PREFETCH=1) or not (in tree), one-seed calls and 32-seed launches on the
# 7B layout, builds alternated.
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
for round in 1 2; do
  for lib in intree fate-llm_amd/ab/libfks_pf.so; do
    echo "== $lib" >> $OUT/ab_pf.log
    if [ $lib = intree ]; then
      FKS_STREAM_MODE=torch_rocm timeout -k 10 200 python -u tools/perf_smallk.py --ks 1,32 --calls perturb,zo_step >> $OUT/ab_pf.log 2>&1 || exit $?
    else
      FKS_LIB_OVERRIDE=$PWD/$lib FKS_STREAM_MODE=torch_rocm timeout -k 10 200 python -u tools/perf_smallk.py --ks 1,32 --calls perturb,zo_step >> $OUT/ab_pf.log 2>&1 || exit $?
    fi
  done
done
