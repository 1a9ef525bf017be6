#!/bin/bash
# Round-3 variant check on the GPU box (repo root): the slice + parity tests against a
# VARIANT build (FKS_LIB_OVERRIDE), then the per-launch A/B of the in-tree build and the
# variants on 2^28 bf16 params x AB_K seeds at AB_WD (default 0.0, the bench's).
#   TESTS="..." bash tools/r03/gpu_var.sh <tag> <variant> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread ${TESTS:-tests/test_gpu_slice.py tests/test_gpu_parity.py} \
    > gpurun_out/${tag}_${v}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_${v}_pytest.log; exit 97; }
  tail -2 gpurun_out/${tag}_${v}_pytest.log
done
libs=("")
for v in "$@"; do libs+=("fate-llm_amd/build/libfks_$v.so"); done
for wd in ${AB_WD:-0.0}; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=${AB_K:-128} AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "${libs[@]}" \
    >> gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
done
cat gpurun_out/${tag}_ab.log
