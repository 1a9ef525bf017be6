import ctypes, os, sys, torch
sys.path.insert(0, "fate-llm_amd/python")
from fate_llm.algo.fedkseed import _native as N
L = N.load()
dev = torch.device("cuda", 0)
ws = torch.empty(1 << 18, dtype=torch.uint8, device=dev)
bad = ctypes.c_uint64(123)
N.check(L.fks_device_selfcheck(N.CHECK_SQRT_DOMAIN, ctypes.byref(bad), ws.data_ptr(), ws.numel(), torch.cuda.current_stream(dev).cuda_stream))
print(os.environ.get("FKS_LIB_OVERRIDE"), "sqrt domain violations:", bad.value)
