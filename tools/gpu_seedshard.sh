cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 600 gpurun_out/t_gpu.log python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread || exit 99
grep -E "passed|failed|seed-sharded fp32" gpurun_out/t_gpu.log
grep -q " passed" gpurun_out/t_gpu.log && ! grep -q "failed" gpurun_out/t_gpu.log || exit 1
tools/gpu_step.sh 300 gpurun_out/b_ss.log python -u bench.py --mode seed-shard --steps 1 --warmup 1 --no-cpu-baseline || exit 99
cat gpurun_out/b_ss.log
