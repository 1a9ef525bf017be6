#!/bin/bash
# Round-2 PMC passes of the slice kernel for library variants, plus the issue2 ubench for
# calibration (repo root on the GPU box):  VARIANTS="full cs0" bash tools/gpu_pmc2.sh
# One rocprofv3 pass per counter group; results under gpurun_out/pmc2_<variant>_<group>/.
# PERF_ARGS (tools/perf_one.py arguments), PERF_STREAM, PMC_SEEDS (seeds per launch) and
# PMC_KERNEL (kernel-name substring for the summary) select another kernel, e.g. the
# torch_rocm stream: PERF_STREAM=torch_rocm PMC_SEEDS=32 PMC_KERNEL=fks_philox_vec_kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
GROUPS_=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE"
         "FETCH_SIZE GRBM_GUI_ACTIVE"
         "WRITE_SIZE GRBM_GUI_ACTIVE")
for v in ${VARIANTS:-full}; do
  # full: the in-tree library at wd 0.01; wd0: the in-tree library at wd 0.0 (kModeUpdateWd0)
  if [ "$v" = "wd0" ]; then unset FKS_LIB_OVERRIDE; export PERF_WD=0.0
  elif [ "$v" != "full" ]; then export FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/ab/libfks_$v.so; unset PERF_WD
  else unset FKS_LIB_OVERRIDE; unset PERF_WD; fi
  # the device-code identity of the library these passes profile (summarize_pmc2.py records it)
  python3 -c 'import sys; sys.path.insert(0, "fate-llm_amd/python"); from fate_llm.algo.fedkseed import _native; print(_native.build_id())' \
    > gpurun_out/pmc2_${v}_buildid || exit 97
  i=0
  for g in "${GROUPS_[@]}"; do
    rm -rf gpurun_out/pmc2_${v}_$i
    timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/pmc2_${v}_$i -o run --output-format csv -- \
      python3 tools/perf_one.py ${PERF_ARGS:-bf16 28 64} > gpurun_out/pmc2_${v}_$i.log 2>&1 || exit 99
    i=$((i+1))
  done
done
if [ -n "$UBENCH" ]; then
  GROUPS_=("${GROUPS_[@]:0:1}")
  i=0
  for g in "${GROUPS_[@]}"; do
    rm -rf gpurun_out/pmc2_ub_$i
    timeout -s KILL 120 rocprofv3 --pmc $g -d gpurun_out/pmc2_ub_$i -o run --output-format csv -- \
      ./tools/ubench/issue2 > gpurun_out/pmc2_ub_$i.log 2>&1 || exit 98
    i=$((i+1))
  done
fi
python3 tools/pmc2_show.py ${VARIANTS:-full}
for v in ${VARIANTS:-full}; do python3 tools/summarize_pmc2.py "${TAG:-r02}_$v" $v $((1 << 28)) ${PMC_SEEDS:-64} $PMC_KERNEL > /dev/null; done
