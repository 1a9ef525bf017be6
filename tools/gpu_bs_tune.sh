#!/bin/bash
# Slice-kernel schedule knobs with the packed (C,S) table at wd 0.0 (timing only; every
# variant computes the same values): lookahead 2 / 4 seeds, compiler fence every 4 / 16 seeds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
AB_WD=0.0 AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 400 python3 -u tools/ab_apply.py "" \
  fate-llm_amd/build/libfks_la2.so fate-llm_amd/build/libfks_la4.so fate-llm_amd/build/libfks_fe4.so \
  fate-llm_amd/build/libfks_fe16.so > gpurun_out/r02t_ab_tune.log 2>&1 || { cat gpurun_out/r02t_ab_tune.log; exit 99; }
cat gpurun_out/r02t_ab_tune.log
