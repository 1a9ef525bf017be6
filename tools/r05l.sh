#!/bin/bash
# The LDS tensor table in the eight-item torch_rocm kernel: parity, one-seed call times,
# one client's warm 7B round on the default stream.
set -o pipefail
bash tools/gpu.sh r05l pytest:test_gpu_torch_rocm.py,test_gpu_torch_rocm_fullsize.py,test_gpu_fuzz.py,test_gpu_optimizer_kseed.py || exit $?
OUT=gpurun_out/r05l
FKS_STREAM_MODE=torch_rocm timeout -k 10 300 python -u tools/perf_smallk.py --ks 1,4,32 \
  --calls perturb,perturb_step,zo_step > $OUT/smallk_rocm.log 2>&1 || exit $?
FKS_STREAM_MODE=auto timeout -k 10 600 python -u harness/c5_round.py --rounds 3 --warm --placement pinned > $OUT/c5_auto.json 2> $OUT/c5_auto.err
