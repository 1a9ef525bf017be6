#!/bin/bash
# time the apply kernel in full / diagnostic builds: VARIANTS="full diag1 diag2 ..."
for v in ${VARIANTS:-full diag1 diag2 diag3 diag4}; do
  if [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  rm -rf gpurun_out/diag_$v
  rocprofv3 --kernel-trace --stats -d gpurun_out/diag_$v -o run --output-format csv -- python3 tools/perf_one.py ${1:-bf16} ${2:-30} ${3:-19} > gpurun_out/diag_$v.log 2>&1 || exit 1
done
