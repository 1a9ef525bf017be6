#!/bin/bash
# Where the twist wave's cost is (wd 0.0 chain): in-tree vs no twist (bsd1), twist without
# its row stores (bsd6), twist without its row loads after round 0 (bsd7); wrong values.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
AB_WD=0.0 AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "" \
  fate-llm_amd/build/libfks_bsd1.so fate-llm_amd/build/libfks_bsd6.so fate-llm_amd/build/libfks_bsd7.so \
  > gpurun_out/r02l_ab_twdiag.log 2>&1 || { cat gpurun_out/r02l_ab_twdiag.log; exit 99; }
cat gpurun_out/r02l_ab_twdiag.log
