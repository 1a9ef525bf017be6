#!/bin/bash
# GPU parity tests, smoke, the small-K probe and the default bench line, each step under
# its own limit; stops at the first crash-class exit.  Run from the repo root on the box.
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-v}
tools/gpu_step.sh 600 gpurun_out/t_gpu_$tag.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 99
tail -2 gpurun_out/t_gpu_$tag.log
grep -q " passed" gpurun_out/t_gpu_$tag.log && ! grep -q "failed" gpurun_out/t_gpu_$tag.log || exit 1
tools/gpu_step.sh 300 gpurun_out/smoke_$tag.log python -u -c "import __graft_entry__ as g; g._paths(); g.smoke()" || exit 99
tools/gpu_step.sh 300 gpurun_out/smallk_$tag.log python -u tools/perf_smallk.py || exit 99
cat gpurun_out/smallk_$tag.log
if [ "${BENCH:-1}" = 1 ]; then
  tools/gpu_step.sh 400 gpurun_out/bench_$tag.log python -u bench.py || exit 99
  cat gpurun_out/bench_$tag.log
fi
