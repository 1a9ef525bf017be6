#!/bin/bash
# C4 measured end to end (no extrapolation): the 70B fp32 buffer reconstructed from all
# 4055 non-zero seeds of K=4096, 8 chunks, one progress line per chunk (~70 s each).
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python3 -u tools/c4_70b.py --ks 4096 --progress > gpurun_out/c4_full_k4096.log 2>&1 || exit 99
tail -2 gpurun_out/c4_full_k4096.log
