#!/bin/bash
# Round-3 one-slice / two-slice check: slice parity both ways, per-launch A/B of the
# prefetch-depth variants (K=128: full passes; K=23: one split pass, a probe of the serial
# twist chain), the default bench line.   bash tools/r03/gpu_slices.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
for sl in 1 2; do
  FKS_BS_SLICES=$sl timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_slice.py \
    > gpurun_out/${tag}_slices${sl}_pytest.log 2>&1 || { tail -20 gpurun_out/${tag}_slices${sl}_pytest.log; exit 97; }
  echo "slices=$sl: $(tail -1 gpurun_out/${tag}_slices${sl}_pytest.log)"
done
TESTS=none AB_K=128 bash tools/r03/gpu_ab.sh ${tag} "$@" > /dev/null || exit 98
FKS_BS_SLICES=1 TESTS=none AB_K=128 bash tools/r03/gpu_ab.sh ${tag}_s1 "$@" > /dev/null || exit 98
TESTS=none AB_K=23 bash tools/r03/gpu_ab.sh ${tag}_k23 "$@" > /dev/null || exit 98
cat gpurun_out/${tag}_ab.log gpurun_out/${tag}_s1_ab.log gpurun_out/${tag}_k23_ab.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit 99
tail -1 gpurun_out/${tag}_bench.log | cut -c1-330
