#!/bin/bash
# Round-2 slice-kernel A/B on the GPU box (repo root): parity of the in-tree build, then
# per-launch time of each build on 2^28 bf16 params x 128 seeds (4 full 32-seed slices).
#   bash tools/gpu_ab2.sh <tag> [variant ...]     (variant NAME -> fate-llm_amd/build/libfks_NAME.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_slice.py \
  tests/test_gpu_parity.py > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 97; }
tail -2 gpurun_out/${tag}_pytest.log
libs=("")
for v in "$@"; do libs+=("fate-llm_amd/build/libfks_$v.so"); done
AB_N=$((1 << 28)) AB_K=${AB_K:-128} AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "${libs[@]}" \
  > gpurun_out/${tag}_ab.log 2>&1 || { cat gpurun_out/${tag}_ab.log; exit 99; }
cat gpurun_out/${tag}_ab.log
