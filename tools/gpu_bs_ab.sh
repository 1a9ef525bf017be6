#!/bin/bash
# Slice kernel (fks_apply_bs_kernel) A/B + PMC on the GPU box, from the repo root:
#   bash tools/gpu_bs_ab.sh [variants...]   (default: full bsd1 bsd2 bsd3)
# 1) per-launch time of each build on 2^28 bf16 params x 128 seeds (4 full slices);
# 2) PMC passes of the in-tree build (one counter group per rocprofv3 run).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
libs=()
for v in ${@:-full bsd1 bsd2 bsd3}; do
  if [ "$v" = full ]; then libs+=(""); else libs+=("fate-llm_amd/build/libfks_$v.so"); fi
done
AB_N=$((1 << 28)) AB_K=128 AB_SEEDS=32 timeout -k 10 300 python3 -u tools/ab_apply.py "${libs[@]}" \
  > gpurun_out/bs_ab.log 2>&1 || exit 99
cat gpurun_out/bs_ab.log
GROUPS_=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_IFETCH SQ_WAIT_INST_LDS"
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC")
i=0
for g in "${GROUPS_[@]}"; do
  rm -rf gpurun_out/pmc_bs_$i
  timeout -k 10 120 rocprofv3 --pmc $g -d gpurun_out/pmc_bs_$i -o run --output-format csv -- \
    python3 tools/perf_one.py bf16 28 64 > gpurun_out/pmc_bs_$i.log 2>&1 || exit 98
  i=$((i+1))
done
KERNEL=fks_apply_bs_kernel python3 tools/pmc_show.py bs
