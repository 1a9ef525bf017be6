set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/diag_f16_tail.py > gpurun_out/r05d/diag_f16_tail.log 2>&1; tail -25 gpurun_out/r05d/diag_f16_tail.log
