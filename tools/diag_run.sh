#!/bin/bash
# time the apply kernel in full / twist-only / pair-only builds
for v in "" diag1 diag2; do
  if [ -n "$v" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  rocprofv3 --kernel-trace --stats -d gpurun_out/diag_$v -o run --output-format csv -- python3 tools/perf_one.py ${1:-bf16} > gpurun_out/diag_$v.log 2>&1 || exit 1
done
