#!/bin/bash
# Small-K kernel A/B (repo root on the GPU box): parity of the in-tree build, then the
# ZO step's calls on the 7B bf16 layout for each build.  bash tools/gpu_smallk_ab2.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_smallk.py tests/test_gpu_optimizer_kseed.py tests/test_gpu_seed_shard.py > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 97; }
tail -2 gpurun_out/${tag}_pytest.log
for v in full "$@"; do
  if [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  echo "== $v"
  timeout -k 10 200 python3 -u tools/perf_smallk.py --reps 5 --ks 1,2,4 2>&1 | grep '^{' || exit 98
done
