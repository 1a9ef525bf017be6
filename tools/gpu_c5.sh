#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh 300 gpurun_out/c5_small.log python -u harness/c5_round.py --params 16777216 --k 64 --steps 5 --rounds 2 || exit 99
cat gpurun_out/c5_small.log
grep -q '"harness"' gpurun_out/c5_small.log || exit 1
tools/gpu_step.sh 400 gpurun_out/c5_7b_warm.log python -u harness/c5_round.py --warm --rounds 1 || exit 99
cat gpurun_out/c5_7b_warm.log
tools/gpu_step.sh 400 gpurun_out/c5_7b_warm_resident.log python -u harness/c5_round.py --warm --rounds 1 --resident || exit 99
cat gpurun_out/c5_7b_warm_resident.log
