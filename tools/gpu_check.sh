cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 600 gpurun_out/t_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 99
tools/gpu_step.sh 300 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g._paths(); g.smoke()" || exit 99
tail -3 gpurun_out/t_gpu.log; tail -2 gpurun_out/smoke.log
