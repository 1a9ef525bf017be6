"""How the drop-in directional_derivative_step reads g (zo_utils.py:49 semantics, host
logic only): a python number, a 0-dim tensor (cast to the parameter dtype), or a
1-element tensor of shape (1,) -- the same update when torch's promotion keeps the
parameter's dtype and shape, refused when the reference would rebind param.data to
another dtype or shape."""
import pytest
import torch

from fate_llm.algo.fedkseed.codec import ParamSpec
from fate_llm.algo.fedkseed.zo_utils import _value_kind


def test_number_and_0dim():
    assert _value_kind(1.5) == (1.5, False)
    assert _value_kind(torch.tensor(2.25)) == (2.25, True)


@pytest.mark.parametrize("gdt,pdt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                     (torch.bfloat16, torch.float32), (torch.float16, torch.float16)])
def test_one_element_same_update(gdt, pdt):
    g = torch.tensor([0.75], dtype=gdt)
    specs = [ParamSpec(torch.zeros(4, 3, dtype=pdt)), ParamSpec(torch.zeros(5, dtype=pdt))]
    assert _value_kind(g, specs) == (0.75, True)


@pytest.mark.parametrize("g,p", [(torch.tensor([0.5]), torch.zeros(8, dtype=torch.bfloat16)),
                                 (torch.tensor([0.5]), torch.tensor(1.0)),
                                 (torch.tensor([0.5], dtype=torch.float16), torch.zeros(8, dtype=torch.bfloat16))])
def test_one_element_that_would_rebind_is_refused(g, p):
    with pytest.raises(NotImplementedError):
        _value_kind(g, [ParamSpec(p)])


def test_more_than_one_element_is_an_error():
    with pytest.raises(ValueError):
        _value_kind(torch.tensor([0.5, 0.5]), [])


def test_cpu_scalar_g_with_z_on_the_gpu_is_not_cast(monkeypatch):
    """torch_rocm (z on the GPU): a 0-dim CPU g is a CPU scalar, its f32 value enters the
    multiply unrounded (a python number's kind); a 0-dim GPU g is cast to the parameter
    dtype; a dimensioned CPU g is torch's device-mismatch error.  (Specs stand in for GPU
    tensors: only .device and .dtype are read.)"""
    from fate_llm.algo.fedkseed import codec

    class FakeCuda:
        device = torch.device("cuda", 0)
        dtype = torch.bfloat16

        def dim(self):
            return 1

    specs = [ParamSpec(FakeCuda())]
    g = torch.tensor(0.1234567)
    assert _value_kind(g, specs, stream_mode="torch_rocm") == (float(g), False)
    assert _value_kind(g, specs, stream_mode="torch_cpu") == (float(g), True)
    monkeypatch.setattr(codec, "_stream_mode", "auto")  # the default resolves to torch_rocm on cuda
    assert _value_kind(g, specs) == (float(g), False)
    with pytest.raises(RuntimeError, match="same device"):
        _value_kind(torch.tensor([0.5]), specs, stream_mode="torch_rocm")
