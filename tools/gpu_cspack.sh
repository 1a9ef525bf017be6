#!/bin/bash
# Packed (C,S) table per mode: parity of the in-tree build, then per-launch time of the
# slice kernel at wd 0.0 / 0.01 / None for the in-tree build (FKS_BS_CSPACK=2) and cs0 / cs1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_slice.py tests/test_gpu_c3.py tests/test_gpu_seed_shard.py > gpurun_out/r02h_pytest.log 2>&1 || { tail -40 gpurun_out/r02h_pytest.log; exit 97; }
tail -2 gpurun_out/r02h_pytest.log
for wd in 0.0 0.01 none; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "" \
    fate-llm_amd/build/libfks_cs0.so fate-llm_amd/build/libfks_cs1.so >> gpurun_out/r02h_ab.log 2>&1 || { cat gpurun_out/r02h_ab.log; exit 99; }
done
cat gpurun_out/r02h_ab.log
