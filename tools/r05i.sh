#!/bin/bash
# fks_philox_vec_kernel for the 32-seed reconstruct passes too? the 7B bf16 wd-0 torch_rocm
# reconstruct with FKS_PHX_VEC_MAXK 32 (vec for every launch) and 4 (default), alternated.
set -o pipefail
OUT=gpurun_out/r05i
mkdir -p $OUT
for maxk in 32 4 32 4; do
  FKS_PHX_VEC_MAXK=$maxk timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 >> $OUT/rocm_rate_ab.log 2>&1 || exit $?
  echo "maxk $maxk done" >> $OUT/rocm_rate_ab.log
done
