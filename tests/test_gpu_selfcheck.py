"""Device properties the kernels rely on, checked on the GPU through the C ABI
(fks_device_selfcheck): the fp32 Box-Muller's radius square root is correctly rounded --
as the reference's _mm256_sqrt_ps -- on every one of the 2^24 inputs -2 log(u1) the
reference can produce (exact midpoint criterion, no square root in the check).  The
bare v_sqrt_f32 is not: it misses on some of them, which the fp32 stream parity tests
catch as well."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sqrt_domain_is_correctly_rounded():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from fate_llm.algo.fedkseed import _native as N
    L = N.load()
    dev = torch.device("cuda", 0)
    ws = torch.empty(1 << 18, dtype=torch.uint8, device=dev)
    bad = ctypes.c_uint64(123)
    with torch.cuda.device(dev):
        N.check(L.fks_device_selfcheck(N.CHECK_SQRT_DOMAIN, ctypes.byref(bad), ws.data_ptr(), ws.numel(),
                                       torch.cuda.current_stream(dev).cuda_stream))
    assert bad.value == 0


def test_philox_radius_equals_ocml_on_all_words():
    """The torch_rocm kernel's trimmed radius (phx_radius2) equals ocml's general
    sqrtf(-2 logf(u)) -- what torch.normal runs on the device -- on all 2^32 words."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from fate_llm.algo.fedkseed import _native as N
    L = N.load()
    dev = torch.device("cuda", 0)
    ws = torch.empty(1 << 18, dtype=torch.uint8, device=dev)
    bad = ctypes.c_uint64(123)
    with torch.cuda.device(dev):
        N.check(L.fks_device_selfcheck(N.CHECK_PHILOX_RADIUS, ctypes.byref(bad), ws.data_ptr(), ws.numel(),
                                       torch.cuda.current_stream(dev).cuda_stream))
    assert bad.value == 0


def test_philox_bf16_fast_radius_within_two_ulps():
    """The bf16 fast path's radius (one-rounding -2 ln(u), raw v_sqrt_f32) stays within 2
    f32 ulps of ocml's sqrtf(-2 logf(u)) on all 2^32 words -- the bound phx_z_bf16's
    midpoint window (W = 2 k + 2 = 6 ulps) is built on."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from fate_llm.algo.fedkseed import _native as N
    L = N.load()
    dev = torch.device("cuda", 0)
    ws = torch.empty(1 << 18, dtype=torch.uint8, device=dev)
    worst = ctypes.c_uint64(123)
    with torch.cuda.device(dev):
        N.check(L.fks_device_selfcheck(N.CHECK_PHILOX_BF16_RADIUS, ctypes.byref(worst), ws.data_ptr(), ws.numel(),
                                       torch.cuda.current_stream(dev).cuda_stream))
    print(f"largest radius distance: {worst.value} ulps")
    assert worst.value <= 2


def test_selfcheck_rejects_bad_arguments():
    from fate_llm.algo.fedkseed import _native as N
    L = N.load()
    bad = ctypes.c_uint64(0)
    assert L.fks_device_selfcheck(99, ctypes.byref(bad), None, 0, None) != 0
    assert L.fks_device_selfcheck(N.CHECK_SQRT_DOMAIN, ctypes.byref(bad), None, 0, None) != 0
