#!/bin/bash
# Jump-kernel A/B (repo root on the box): the GPU suite on variant $1's library, then the
# per-rank shard timing (jump and apply seconds, N = 1 and 8) of the in-tree build and
# the variant, alternating.   bash tools/r03/gpu_jr.sh <tag> <variant>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; v=$2
mkdir -p gpurun_out
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 200 \
  --timeout-method thread tests > gpurun_out/${tag}_${v}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_${v}_pytest.log; exit 97; }
echo "$v: $(tail -1 gpurun_out/${tag}_${v}_pytest.log)"
for lib in "" "$v" "" "$v"; do
  if [ -n "$lib" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$lib.so; else unset FKS_LIB_OVERRIDE; fi
  echo "== ${lib:-intree}" >> gpurun_out/${tag}_shard.log
  timeout -k 10 300 python3 -u tools/shard_rank_time.py --ns 1,8 >> gpurun_out/${tag}_shard.log 2>&1 || { tail -20 gpurun_out/${tag}_shard.log; exit 98; }
done
cat gpurun_out/${tag}_shard.log
