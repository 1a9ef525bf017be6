#!/bin/bash
# Zero-weight-decay chain (kModeUpdateWd0): parity of the changed kernels, then the
# per-launch time of the slice kernel and the fp32 kernel at wd = 0.01 / 0.0 / None.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_slice.py tests/test_gpu_smallk.py > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 97; }
tail -2 gpurun_out/${tag}_pytest.log
for wd in 0.01 0.0 none; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 200 python3 -u tools/ab_apply.py >> gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
done
for wd in 0.01 0.0; do
  AB_WD=$wd AB_DT=f32 AB_N=$((1 << 26)) AB_K=95 AB_SEEDS=19 timeout -k 10 200 python3 -u tools/ab_apply.py >> gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
done
cat gpurun_out/${tag}_ab.log
