cd $GRAFT_REPO_ROOT
[ -n "$SKIP_TESTS" ] || tools/gpu_step.sh 600 gpurun_out/t_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 99
tail -1 gpurun_out/t_gpu.log
[ -n "$SKIP_TESTS" ] || grep -q " passed" gpurun_out/t_gpu.log && ! grep -q "failed" gpurun_out/t_gpu.log || exit 1
tools/gpu_step.sh 600 gpurun_out/ab.log python -u tools/ab_apply.py "" fate-llm_amd/build/libfks_diag3.so fate-llm_amd/build/libfks_staged.so || exit 99
cat gpurun_out/ab.log
