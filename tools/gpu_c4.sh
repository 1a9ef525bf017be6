#!/bin/bash
# C4 on the GPU box from the repo root: a 1 % smoke of the 70B fp32 layout, then the
# full 275.9 GB buffer with two K samples (tools/c4_70b.py).
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python3 -u tools/c4_70b.py --scale 0.01 --ks 19 > gpurun_out/c4_smoke.log 2>&1 || exit 99
tail -2 gpurun_out/c4_smoke.log
timeout -k 10 400 python3 -u tools/c4_70b.py --ks 19,38 > gpurun_out/c4_full.log 2>&1 || exit 98
tail -3 gpurun_out/c4_full.log
