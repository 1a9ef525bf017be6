#!/bin/bash
# fp32 19-seed kernel at wd 0.0: the fma form (in tree) vs the kModeUpdateWd launch (f32m0), twice
# each, and at wd 0.01 for reference.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_f32m0.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "zero_weight_decay or golden" > gpurun_out/r02n_pytest.log 2>&1 || { tail -30 gpurun_out/r02n_pytest.log; exit 97; }
tail -1 gpurun_out/r02n_pytest.log
for rep in 1 2; do
  for wd in 0.0 0.01; do
    AB_WD=$wd AB_DT=f32 AB_N=$((1 << 26)) AB_K=95 AB_SEEDS=19 timeout -k 10 200 python3 -u tools/ab_apply.py "" \
      fate-llm_amd/build/libfks_f32m0.so >> gpurun_out/r02n_ab_f32wd0.log 2>&1 || { cat gpurun_out/r02n_ab_f32wd0.log; exit 99; }
  done
done
cat gpurun_out/r02n_ab_f32wd0.log
