#!/bin/bash
# The few-seed torch_rocm kernel (fks_philox_vec_kernel): parity, then single-seed call
# times against the item-loop kernel (FKS_PHX_VEC_MAXK=0) and K=32 in both forms, then one
# client's warm 7B round on the default stream.
set -o pipefail
bash tools/gpu.sh r05h pytest:test_gpu_torch_rocm.py,test_gpu_torch_rocm_fullsize.py,test_gpu_fuzz.py,test_gpu_optimizer_kseed.py || exit $?
OUT=gpurun_out/r05h
for maxk in 4 0 32; do
  FKS_PHX_VEC_MAXK=$maxk FKS_STREAM_MODE=torch_rocm timeout -k 10 300 python -u tools/perf_smallk.py --ks 1,4,32 \
    --calls perturb,perturb_step,zo_step > $OUT/smallk_rocm_maxk$maxk.log 2>&1 || exit $?
done
FKS_STREAM_MODE=auto timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned > $OUT/c5_auto.json 2> $OUT/c5_auto.err
