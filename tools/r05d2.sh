set -o pipefail
mkdir -p gpurun_out/r05d
bash tools/gpu.sh r05d2 pytest:test_gpu_selfcheck.py || exit $?
timeout -k 10 300 python -u tools/diag_phx_edge.py > gpurun_out/r05d/diag_phx_edge.log 2>&1
tail -50 gpurun_out/r05d/diag_phx_edge.log | grep -v '"differ": 0'
FKS_PHX_KEEP_WD_FMA=1 timeout -k 10 300 python -u tools/diag_phx_edge.py > gpurun_out/r05d/diag_phx_edge_fma.log 2>&1
grep -v '"differ": 0' gpurun_out/r05d/diag_phx_edge_fma.log | head -20
