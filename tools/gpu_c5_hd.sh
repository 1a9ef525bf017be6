#!/bin/bash
# Refresh the C5 round and the PCIe-inclusive / K-sweep numbers (GPU box, repo root).
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh 300 gpurun_out/hd_rate.log python -u tools/hd_rate.py || exit 99
tail -1 gpurun_out/hd_rate.log
tools/gpu_step.sh 400 gpurun_out/c5_7b_warm.log python -u harness/c5_round.py --warm --rounds 1 || exit 99
tail -2 gpurun_out/c5_7b_warm.log
tools/gpu_step.sh 400 gpurun_out/c5_7b_warm_resident.log python -u harness/c5_round.py --warm --rounds 1 --resident || exit 99
tail -2 gpurun_out/c5_7b_warm_resident.log
