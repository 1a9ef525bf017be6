#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#  1) kernel trace + stats of the full bench command (7B, K=4096, one step)
#  2) PMC passes (separate, no tracing domains) on a 268M-param slice: HBM bytes and VALU instructions
# Output under gpurun_out/prof_<tag>/ ; copy the summaries to profiles/.
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace -o bench --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/bench_trace.log 2>&1 || exit 99
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o bench --output-format csv -- \
    python3 bench.py --params 268435456 --k 512 --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_fetch.log 2>&1 || exit 99
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o bench --output-format csv -- \
    python3 bench.py --params 268435456 --k 512 --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_write.log 2>&1 || exit 99
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $out/pmc_sq -o bench --output-format csv -- \
    python3 bench.py --params 268435456 --k 512 --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_sq.log 2>&1 || exit 99
echo profile done
