#!/bin/bash
# PMC passes of the full 19-seed fp32 kernel (C4's kernel: fks_apply_kernel<F32, MODE,
# FULL>) on a 2^28-param fp32 buffer, K = 38 (two full passes per reconstruct, two
# reconstructs), plus a kernel trace (repo root on the GPU box):  TAG=r02 bash tools/gpu_pmc_f32.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r02}
GROUPS_=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE"
         "FETCH_SIZE GRBM_GUI_ACTIVE"
         "WRITE_SIZE GRBM_GUI_ACTIVE")
python3 -c 'import sys; sys.path.insert(0, "fate-llm_amd/python"); from fate_llm.algo.fedkseed import _native; print(_native.build_id())' \
  > gpurun_out/pmc2_f32_buildid || exit 97
i=0
for g in "${GROUPS_[@]}"; do
  rm -rf gpurun_out/pmc2_f32_$i
  timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/pmc2_f32_$i -o run --output-format csv -- \
    python3 tools/perf_one.py f32 28 38 > gpurun_out/pmc2_f32_$i.log 2>&1 || exit 99
  i=$((i+1))
done
rm -rf gpurun_out/trf32
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/trf32 -o run --output-format csv -- \
  python3 tools/perf_one.py f32 28 38 > gpurun_out/trf32.log 2>&1 || exit 98
python3 tools/summarize_pmc2.py ${TAG}_f32 f32 $((1 << 28)) 19 "fks_apply_kernel<0, 3, true, false>" 4
