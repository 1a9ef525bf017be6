#!/bin/bash
# Round-3 full GPU check (repo root on the box): pytest -m gpu, the smoke, and (optional)
# an A/B of the in-tree slice kernel against build variants:  bash tools/r03/gpu_suite.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 91; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail gpurun_out/${tag}_smoke.log; exit 92; }
tail -1 gpurun_out/${tag}_smoke.log
if [ $# -gt 0 ]; then TESTS=none AB_WD="${AB_WD:-0.0}" bash tools/r03/gpu_ab.sh ${tag} "$@" || exit 93; fi
