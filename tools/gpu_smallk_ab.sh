#!/bin/bash
# Small-K (ZO-step) call costs on the 7B bf16 layout for several builds (GPU box, repo
# root):  bash tools/gpu_smallk_ab.sh [variants...]   (default: full swg5 swg6 swg8)
cd "$GRAFT_REPO_ROOT" || exit 1
for v in ${@:-full swg5 swg6 swg8}; do
  if [ "$v" = full ]; then unset FKS_LIB_OVERRIDE; else export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python3 -u tools/perf_smallk.py --ks 1,2,4 --reps 5 > gpurun_out/smallk_$v.log 2>&1 || exit 99
  grep '^{' gpurun_out/smallk_$v.log
done
