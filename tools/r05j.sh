#!/bin/bash
# fks_philox_vec_kernel for every torch_rocm launch: the whole GPU suite, then the
# single-seed call times and the 7B torch_rocm reconstruct on this build.
set -o pipefail
bash tools/gpu.sh r05j pytestall || exit $?
OUT=gpurun_out/r05j
FKS_STREAM_MODE=torch_rocm timeout -k 10 300 python -u tools/perf_smallk.py --ks 1,4,32 \
  --calls perturb,perturb_step,zo_step > $OUT/smallk_rocm.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 > $OUT/rocm_rate.log 2>&1
