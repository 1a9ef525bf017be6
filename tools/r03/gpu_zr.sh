#!/bin/bash
# z-index replay A/B (repo root on the box): replay + ZO-step timing of the in-tree build
# and variants on the 7B bf16 layout (tools/perf_smallk.py); the replay parity tests of
# every variant first.   bash tools/r03/gpu_zr.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_wincache.py tests/test_gpu_optimizer_kseed.py > gpurun_out/${tag}_${v}_pytest.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_${v}_pytest.log; exit 97; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_pytest.log)"
done
for v in "" "$@"; do
  if [ -n "$v" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  timeout -k 10 300 python3 -u tools/perf_smallk.py --calls replay,zo_step --ks 1 > gpurun_out/${tag}_${v:-intree}.log 2>&1 || exit 98
  echo "${v:-intree}: $(grep '^{' gpurun_out/${tag}_${v:-intree}.log | python3 -c 'import sys,json; print([(json.loads(l)["call"], json.loads(l)["apply_ms"]) for l in sys.stdin])')"
done
