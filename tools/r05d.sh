# round 5: slice-kernel lag bound (wd 0.01 traffic) and the fp32 integer-mask log, A/B + PMC
set -o pipefail
bash tools/gpu.sh r05d pytest:test_gpu_selfcheck.py,test_gpu_torch_rocm.py,test_gpu_fuzz.py,test_gpu_slice.py,test_gpu_parity.py,test_gpu_fullsize.py,test_gpu_jwin.py,test_gpu_c4.py || exit $?
AB_WD=0.01 AB_K=256 AB_SEEDS=64 timeout -k 10 300 python -u tools/ab_apply.py intree fate-llm_amd/ab/libfks_lag0.so intree fate-llm_amd/ab/libfks_lag0.so > gpurun_out/r05d/ab_lag_wd001.log 2>&1 || exit 11
AB_WD=0.0 AB_K=256 AB_SEEDS=64 timeout -k 10 300 python -u tools/ab_apply.py intree fate-llm_amd/ab/libfks_lag0.so intree fate-llm_amd/ab/libfks_lag0.so > gpurun_out/r05d/ab_lag_wd0.log 2>&1 || exit 12
AB_DT=f32 AB_WD=0.01 AB_K=95 timeout -k 10 300 python -u tools/ab_apply.py intree fate-llm_amd/ab/libfks_f32q0.so intree fate-llm_amd/ab/libfks_f32q0.so > gpurun_out/r05d/ab_f32_intmask.log 2>&1 || exit 13
timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 > gpurun_out/r05d/rocm_wdpos0.log 2>&1 || exit 15
FKS_PHX_KEEP_WD_FMA=1 timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 > gpurun_out/r05d/rocm_keepfma.log 2>&1 || exit 16
FKS_LIB_OVERRIDE=$PWD/fate-llm_amd/ab/libfks_phxslow.so timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 > gpurun_out/r05d/rocm_slowlog.log 2>&1 || exit 18
timeout -k 10 300 python -u tools/rocm_rate.py --ref-seeds 0 --modes torch_rocm --k 64 > gpurun_out/r05d/rocm_wdpos0_b.log 2>&1 || exit 17
TAG=r05d VARIANTS="full lag0" timeout -k 10 600 bash tools/gpu_pmc2.sh > gpurun_out/r05d/pmc.log 2>&1 || exit 14
cp profiles/pmc_apply_r05d_*.json gpurun_out/r05d/
