#!/bin/bash
# Jump kernel with 63 lanes x 10 words (jw10): parity through FKS_LIB_OVERRIDE on the jump-heavy
# tests, then rank-0 shard times (apply + jump) at N = 1 and 8, in-tree vs jw10.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_jw10.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slice.py tests/test_gpu_c4.py tests/test_gpu_fullsize.py \
  > gpurun_out/r02r_pytest.log 2>&1 || { tail -30 gpurun_out/r02r_pytest.log; exit 97; }
tail -1 gpurun_out/r02r_pytest.log
timeout -k 10 200 python3 -u tools/shard_rank_time.py --ns 1,8 > gpurun_out/r02r_shard_intree.log 2>&1 || exit 98
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_jw10.so timeout -k 10 200 python3 -u tools/shard_rank_time.py --ns 1,8 \
  > gpurun_out/r02r_shard_jw10.log 2>&1 || exit 99
grep nshards gpurun_out/r02r_shard_intree.log gpurun_out/r02r_shard_jw10.log
