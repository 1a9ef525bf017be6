set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u tools/diag_f16_mul.py > gpurun_out/r05d/diag_f16_mul.log 2>&1; tail -12 gpurun_out/r05d/diag_f16_mul.log
