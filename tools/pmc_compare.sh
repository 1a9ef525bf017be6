#!/bin/bash
# PMC counters of the apply kernel for several library variants (run on the GPU box
# from the repo root):  VARIANTS="full diag6" bash tools/pmc_compare.sh [bf16|f32]
# Each counter group is its own rocprofv3 pass (no tracing domains).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
GROUPS_=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_IFETCH SQ_WAIT_INST_LDS"
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC")
for v in ${VARIANTS:-full}; do
  if [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/build/libfks_$v.so; else unset FKS_LIB_OVERRIDE; fi
  i=0
  for g in "${GROUPS_[@]}"; do
    rm -rf gpurun_out/pmc_${v}_$i
    timeout -k 10 240 rocprofv3 --pmc $g -d gpurun_out/pmc_${v}_$i -o run --output-format csv -- \
      python3 tools/perf_one.py ${1:-bf16} > gpurun_out/pmc_${v}_$i.log 2>&1 || exit 99
    i=$((i+1))
  done
done
python3 tools/pmc_show.py ${VARIANTS:-full}
