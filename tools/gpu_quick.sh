#!/bin/bash
# GPU parity tests + a short bench probe (268M bf16 params, K=4096: the jump kernel at
# the 7B chunk count, the apply kernel on a 1/25 slice).  Run from the repo root on the box.
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh 600 gpurun_out/t_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 99
tail -2 gpurun_out/t_gpu.log
grep -q " passed" gpurun_out/t_gpu.log && ! grep -q "failed" gpurun_out/t_gpu.log || exit 1
tools/gpu_step.sh 300 gpurun_out/b_small.log python -u bench.py --params 268435456 --k 4096 --steps 1 --warmup 1 --no-cpu-baseline || exit 99
cat gpurun_out/b_small.log
