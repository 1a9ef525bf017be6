#!/bin/bash
# One GPU call for a round's measurement set (repo root on the GPU box):
#   TAG=r04 bash tools/profile_round.sh
# 1) PMC passes of the slice kernel (tools/gpu_pmc2.sh) -> pmc_apply_${TAG}_{wd0,full}.json
#    (wd0: the bench's weight decay 0.0; full: wd 0.01), of the torch_rocm stream's kernel
#    -> pmc_apply_${TAG}_phx_wd0.json, and of the fp32 19-seed kernel (tools/gpu_pmc_f32.sh)
#    -> pmc_apply_${TAG}_f32.json, each carrying the build id of the libfks.so it profiled
#    (bench.py uses a summary only for the same build); copied to gpurun_out/
# 2) the default bench line (N=1, with cpu_baseline)      -> gpurun_out/${TAG}_bench_default.log
# 3) rocprofv3 --kernel-trace --stats of one bench step   -> gpurun_out/${TAG}_trace/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r05}
PMCV=${PMCV:-wd0 full}
TAG=$TAG VARIANTS="$PMCV" timeout -k 10 600 bash tools/gpu_pmc2.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { tail gpurun_out/${TAG}_pmc.log; exit 91; }
for v in $PMCV; do cp profiles/pmc_apply_${TAG}_$v.json gpurun_out/ 2>/dev/null; done
if [ -z "$NO_PHX" ]; then
  PERF_STREAM=torch_rocm PERF_ARGS="bf16 28 64" PMC_SEEDS=32 PMC_KERNEL=fks_philox_vec_kernel TAG=${TAG}_phx VARIANTS=wd0 \
    timeout -k 10 600 bash tools/gpu_pmc2.sh > gpurun_out/${TAG}_pmc_phx.log 2>&1 || { tail gpurun_out/${TAG}_pmc_phx.log; exit 94; }
  cp profiles/pmc_apply_${TAG}_phx_wd0.json gpurun_out/
fi
if [ -z "$NO_F32" ]; then
  TAG=$TAG timeout -k 10 600 bash tools/gpu_pmc_f32.sh > gpurun_out/${TAG}_pmc_f32.log 2>&1 || { tail gpurun_out/${TAG}_pmc_f32.log; exit 95; }
  cp profiles/pmc_apply_${TAG}_f32.json gpurun_out/
fi
timeout -k 10 400 python3 -u bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || { tail gpurun_out/${TAG}_bench_default.log; exit 92; }
tail -1 gpurun_out/${TAG}_bench_default.log
rm -rf gpurun_out/${TAG}_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- \
  python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --alt-wd 0.0 --alt-stream-steps 1 --no-hd \
  > gpurun_out/${TAG}_bench_trace_run.log 2>&1 || exit 93
tail -1 gpurun_out/${TAG}_bench_trace_run.log
