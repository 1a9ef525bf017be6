#!/bin/bash
# Per-rank shard work on the final build: the bench's torch_cpu reconstruct cold and warm,
# and the default stream (torch_rocm, no jumps) cold.
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
timeout -k 10 400 python -u tools/shard_rank_time.py > $OUT/shard_cold.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/shard_rank_time.py --warm > $OUT/shard_warm.log 2>&1 || exit $?
FKS_STREAM_MODE=torch_rocm timeout -k 10 400 python -u tools/shard_rank_time.py > $OUT/shard_rocm.log 2>&1
