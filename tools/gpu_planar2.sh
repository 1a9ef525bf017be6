#!/bin/bash
# Planar C|S tables read by two ds_read_b32: parity of the pl2 variant (slice tests through FKS_LIB_OVERRIDE), then
# per-launch time at wd 0.0 and 0.01, in-tree vs rm1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_pl2.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_slice.py > gpurun_out/r02u_pytest.log 2>&1 || { tail -30 gpurun_out/r02u_pytest.log; exit 97; }
tail -1 gpurun_out/r02u_pytest.log
for wd in 0.0 0.01 none; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "" \
    fate-llm_amd/build/libfks_pl2.so >> gpurun_out/r02u_ab.log 2>&1 || { cat gpurun_out/r02u_ab.log; exit 99; }
done
cat gpurun_out/r02u_ab.log
