#!/bin/bash
# PMC passes of the small-K (double-buffered) apply kernel on the 7B bf16 layout: the ZO
# step's perturb (K=1), one rocprofv3 pass per counter group, plus a kernel trace
# (repo root on the GPU box):  TAG=r02 bash tools/gpu_pmc_smallk.sh [variant ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02}
GROUPS_=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE"
         "FETCH_SIZE GRBM_GUI_ACTIVE"
         "WRITE_SIZE GRBM_GUI_ACTIVE")
for v in ${@:-full}; do
  if [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/ab/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  i=0
  for g in "${GROUPS_[@]}"; do
    rm -rf gpurun_out/pmcsk_${v}_$i
    timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/pmcsk_${v}_$i -o run --output-format csv -- \
      python3 tools/perf_smallk.py --reps 3 --ks 1 > gpurun_out/pmcsk_${v}_$i.log 2>&1 || exit 99
    i=$((i+1))
  done
  rm -rf gpurun_out/trsk_$v
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/trsk_$v -o run --output-format csv -- \
    python3 tools/perf_smallk.py --reps 5 --ks 1 > gpurun_out/trsk_$v.log 2>&1 || exit 98
  cat gpurun_out/trsk_$v.log | grep '^{'
  python3 tools/summarize_pmc_smallk.py ${TAG}_$v $v
done
