#!/bin/bash
# Default bench (the driver's command) + the f32 19-seed kernel's per-launch time, on the
# GPU box from the repo root:  bash tools/gpu_bench_f32.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r01c}
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || exit 99
cat gpurun_out/bench_$tag.log
AB_DT=f32 AB_N=$((1 << 28)) AB_K=38 AB_SEEDS=19 timeout -k 10 200 python3 -u tools/ab_apply.py "" \
  > gpurun_out/ab_f32_$tag.log 2>&1 || exit 98
cat gpurun_out/ab_f32_$tag.log
timeout -k 10 300 python3 -u tools/c4_70b.py --scale 0.01 --ks 19 > gpurun_out/c4_smoke_$tag.log 2>&1 || exit 97
cat gpurun_out/c4_smoke_$tag.log
