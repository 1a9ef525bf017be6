"""Diagnostic for tests/test_gpu_torch_rocm.py::test_f16_unaligned_view_later_calls_read_a_fresh_tensor:
mismatch counts against the reference after every stage, with and without the rebind record."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fate_llm.algo.fedkseed import codec, zo_utils  # noqa: E402
from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer  # noqa: E402
from oracle import torch_replica as R  # noqa: E402

dev = torch.device("cuda", 0)
n, off = 3_000_001, int(sys.argv[1]) if len(sys.argv) > 1 else 1
gen = torch.Generator(dev).manual_seed(21)
buf = (torch.randn(n + off + 64, device=dev, generator=gen) * 0.05).to(torch.float16)
frozen0 = (torch.randn(777, device=dev, generator=gen) * 0.05).to(torch.float16)
orig = codec.is_rebound
for record in (True, False):
    codec.is_rebound = orig if record else (lambda p: False)
    ref_buf, got_buf = buf.clone(), buf.clone()
    ref = [torch.nn.Parameter(ref_buf[off:off + n]), torch.nn.Parameter(frozen0.clone(), requires_grad=False)]
    got = [torch.nn.Parameter(got_buf[off:off + n]), torch.nn.Parameter(frozen0.clone(), requires_grad=False)]
    rg = [{"params": ref, "lr": 0.1, "weight_decay": 0.01, "eps": 1e-3}]
    gg = [{"params": got, "lr": 0.1, "weight_decay": 0.01, "eps": 1e-3}]
    codec.set_stream_mode("torch_rocm")

    def cmp(stage):
        torch.cuda.synchronize()
        a, b = got[0].detach().view(torch.int16), ref[0].detach().view(torch.int16)
        bad = (a != b).nonzero()
        print(f"record={record} off={off} {stage}: {bad.shape[0]} differ" +
              (f", first {bad[0].item()}: {got[0][bad[0].item()].item()} vs {ref[0][bad[0].item()].item()}" if bad.numel() else ""),
              flush=True)

    for seed, v in [(5, 2e-3), (6, -1.5e-3), (7, 1e-3)]:
        R.directional_derivative_step(rg, seed, v)
        zo_utils.directional_derivative_step(gg, seed, v)
        cmp(f"directional step seed {seed}")
    opt = ZerothOrderOptimizer(gg, lr=0.1, eps=1e-3, weight_decay=0.01, grad_clip=0.0)
    R.random_perturb_parameters(rg, 99, 1.0)
    opt.random_perturb_parameters(99, 1.0)
    cmp("perturb +1")
    R.random_perturb_parameters(rg, 99, -2.0)
    opt.random_perturb_parameters(99, -2.0)
    cmp("perturb -2")
    R.random_perturb_parameters(rg, 99, 1.0)
    opt.random_perturb_parameters(99, 1.0)
    cmp("perturb +1")
    g = torch.tensor(0.0123456)
    R.directional_derivative_step(rg, 99, g)
    opt.directional_derivative_step(99, g)
    cmp("update with a tensor g")
    codec.set_stream_mode("torch_cpu")
