set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/diag_phx_edge2.py -0.0 > gpurun_out/r05d/diag_phx_edge2.log 2>&1; tail -20 gpurun_out/r05d/diag_phx_edge2.log
timeout -k 10 300 python -u tools/diag_phx_edge2.py 0.01 > gpurun_out/r05d/diag_phx_edge2_wd.log 2>&1; tail -5 gpurun_out/r05d/diag_phx_edge2_wd.log
