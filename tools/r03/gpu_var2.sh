#!/bin/bash
# Round-3 variant check: parity tests (slice + parity files) of the variants in $CHECK,
# then the per-launch A/B of the in-tree build and every variant given.
#   CHECK="a b" bash tools/r03/gpu_var2.sh <tag> <variant> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
for v in $CHECK; do
  FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread ${TESTS:-tests/test_gpu_slice.py tests/test_gpu_parity.py} \
    > gpurun_out/${tag}_${v}_pytest.log 2>&1
  rc=$?
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_pytest.log)"
  # a wrong-result variant is reported and timed; a crash, hang or timeout ends the call
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 97
done
libs=("")
for v in "$@"; do libs+=("fate-llm_amd/build/libfks_$v.so"); done
for wd in ${AB_WD:-0.0}; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=${AB_K:-128} AB_SEEDS=${AB_SEEDS:-64} timeout -k 10 400 python3 -u tools/ab_apply.py "${libs[@]}" \
    >> gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
done
cat gpurun_out/${tag}_ab.log
