#!/bin/bash
# Small-K A/B with the jumped-window cache (repo root on the GPU box): parity of the
# in-tree build, then tools/perf_smallk.py per build, and the in-tree build with the
# cache off (FKS_NO_WIN_CACHE).  bash tools/gpu_smallk_ab3.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_smallk.py tests/test_gpu_optimizer_kseed.py tests/test_gpu_seed_shard.py > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 97; }
tail -2 gpurun_out/${tag}_pytest.log
for v in full nocache "$@"; do
  unset FKS_LIB_OVERRIDE FKS_NO_WIN_CACHE
  if [ "$v" = "nocache" ]; then export FKS_NO_WIN_CACHE=1; elif [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python3 -u tools/perf_smallk.py --reps 5 --ks 1,2,4 2>&1 | grep '^{' || exit 98
done
