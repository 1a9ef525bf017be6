#!/bin/bash
# What the driver runs at round end, then the C5 / PCIe refresh (GPU box, repo root):
#   bash tools/gpu_round.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-r01d}
tools/gpu_step.sh 600 gpurun_out/t_gpu_$tag.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 99
tail -2 gpurun_out/t_gpu_$tag.log
grep -q " passed" gpurun_out/t_gpu_$tag.log && ! grep -q "failed\|error" gpurun_out/t_gpu_$tag.log || exit 1
tools/gpu_step.sh 300 gpurun_out/smoke_$tag.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 99
tail -1 gpurun_out/smoke_$tag.log
tools/gpu_step.sh 400 gpurun_out/bench_$tag.log python -u bench.py || exit 99
grep '^{' gpurun_out/bench_$tag.log
bash tools/gpu_c5_hd.sh || exit 99
