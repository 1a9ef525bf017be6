set -o pipefail
mkdir -p gpurun_out/r05d
bash tools/gpu.sh r05d3 pytest:test_gpu_torch_rocm.py,test_gpu_fuzz.py || exit $?
timeout -k 10 300 python -u tools/diag_phx_edge2.py -0.0 > gpurun_out/r05d/diag_phx_edge2.log 2>&1; tail -3 gpurun_out/r05d/diag_phx_edge2.log
