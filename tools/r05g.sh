#!/bin/bash
# torch_rocm single-seed calls (the local ZO step on a GPU client's default stream)
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
FKS_STREAM_MODE=torch_rocm timeout -k 10 300 python -u tools/perf_smallk.py --ks 1,4,32 --calls perturb,perturb_step,zo_step > $OUT/smallk_rocm.log 2>&1
