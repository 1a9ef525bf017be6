#!/bin/bash
# Same-box A/B of one- and two-slice passes on the 7B bench (FKS_BS_SLICES), in-tree and
# variant builds; slice parity of the variants in two-slice mode first.
#   bash tools/r03/gpu_slices_bench.sh <tag> [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so FKS_BS_SLICES=2 timeout -k 10 400 python3 -u -m pytest -x -q \
    --timeout 200 --timeout-method thread tests/test_gpu_slice.py tests/test_gpu_seed_shard.py > gpurun_out/${tag}_${v}_pytest.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_${v}_pytest.log; exit 97; }
  echo "$v: $(tail -1 gpurun_out/${tag}_${v}_pytest.log)"
done
run() {  # name slices [lib]
  local name=$1 sl=$2 lib=$3
  if [ -n "$lib" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$lib.so; else unset FKS_LIB_OVERRIDE; fi
  FKS_BS_SLICES=$sl timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --alt-wd 0.0 > gpurun_out/${tag}_$name.log 2>&1 || exit 98
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_$name.log') if l.startswith('{')][-1]); print('$name', d['ms_per_step'], d['jump_kernel_ms_per_step'])"
}
run intree_s1 1
run intree_s2 2
for v in "$@"; do run ${v}_s2 2 $v; done
run intree_s1b 1
