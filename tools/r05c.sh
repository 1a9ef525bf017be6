export AB_DT=f32 AB_WD=0.01 AB_SEEDS=19 AB_K=95
bash tools/gpu.sh r05c pytest:test_gpu_parity.py,test_gpu_c4.py,test_gpu_c1.py,test_gpu_fuzz.py,test_gpu_jwin.py,test_gpu_torch_rocm.py ab:fate-llm_amd/ab/libfks_f32q0.so,intree,fate-llm_amd/ab/libfks_f32q1.so,fate-llm_amd/ab/libfks_f32q3.so,fate-llm_amd/ab/libfks_f32q0.so,intree
