#!/bin/bash
# Default bench (the driver's command) + the rocprofv3 trace/PMC passes, for profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r01b}
tools/gpu_step.sh 900 gpurun_out/bench_default_$tag.log python -u bench.py || exit 99
cat gpurun_out/bench_default_$tag.log
bash tools/profile_bench.sh $tag || exit 99
