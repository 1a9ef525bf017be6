#!/bin/bash
# Round-3 slice-kernel A/B on the GPU box (repo root): parity tests of the in-tree build
# (TESTS, default the slice + parity files), then per-launch time of each build on 2^28
# bf16 params x AB_K seeds at weight decay AB_WD (default 0.0, the bench's).
#   TESTS="..." bash tools/r03/gpu_ab.sh <tag> [variant ...]   (variant -> fate-llm_amd/build/libfks_<variant>.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
if [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_slice.py tests/test_gpu_parity.py} \
    > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 97; }
  tail -2 gpurun_out/${tag}_pytest.log
fi
libs=("")
for v in "$@"; do libs+=("fate-llm_amd/build/libfks_$v.so"); done
for wd in ${AB_WD:-0.0}; do
  AB_WD=$wd AB_N=$((1 << 28)) AB_K=${AB_K:-128} AB_SEEDS=${AB_SEEDS:-64} timeout -k 10 300 python3 -u tools/ab_apply.py "${libs[@]}" \
    >> gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
done
cat gpurun_out/${tag}_ab.log
