set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/diag_phx_f16.py > gpurun_out/r05d/diag_phx_f16.log 2>&1; tail -30 gpurun_out/r05d/diag_phx_f16.log
