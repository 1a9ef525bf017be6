#!/bin/bash
# Round 2g: slice-kernel A/B at weight decay 0.0 (in-tree vs variants), then the round's
# measurement set (tools/profile_round.sh: PMC of the wd0 chain, bench line, kernel trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
libs=("")
for v in $VARIANTS; do libs+=("fate-llm_amd/build/libfks_$v.so"); done
AB_WD=0.0 AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 400 python3 -u tools/ab_apply.py "${libs[@]}" \
  > gpurun_out/r02g_ab_wd0.log 2>&1 || { cat gpurun_out/r02g_ab_wd0.log; exit 99; }
cat gpurun_out/r02g_ab_wd0.log
TAG=r02g timeout -k 10 900 bash tools/profile_round.sh || exit $?
