"""KSeedZerothOrderOptimizer (optimizer.py:176-235) and the grad_clip branch of
RandomWalkOptimizer.directional_derivative_step (optimizer.py:89-91) on the GPU codec,
against the reference's own run (tests/golden/optimizer_kseed.npz, cases.json
["optimizer"]["kseed"], written by tests/golden/make_golden.py) and the oracle.

* the KSeed run: four kseed_zeroth_order_step calls with a pre-set loss sequence whose
  third step sees a NaN loss -- the unseeded sampler generator's draws, the returned
  losses (NaN on the skipped step), the recorded history and the final parameters;
* grad_clip > 0 that fires: NaN is returned, nothing is updated, the parameters are the
  restored x of the three perturbations bit for bit; and one that does not fire;
* both with the losses on the device, where g, the NaN checks and the clip decision stay
  on the device (ZerothOrderOptimizer.device_step, fks_perturb_step_dev) and the history
  is recorded lazily -- the same returns, history and parameters as the host path, and
  no host synchronisation inside the step (torch.cuda sync debug mode "error").
"""
import math

import numpy as np
import pytest
import torch

from conftest import assert_bitwise
from oracle import fks_oracle as O
from test_gpu_parity import DTC, _dev, from_np, rand_params, to_np

pytestmark = pytest.mark.gpu


def test_kseed_optimizer_golden(golden, cases):
    from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer
    dev = _dev()
    case = cases["optimizer"]["kseed"]
    z = golden("optimizer_kseed.npz")
    order = [n for grp in case["groups"] for n in grp]
    params = {n: torch.nn.Parameter(from_np(z[f"init/{n}"].reshape(-1), "float32", dev)) for n in order}
    groups = [{"params": [params[n] for n in grp], "weight_decay": wd}
              for grp, wd in zip(case["groups"], (0.0, case["wd"]))]
    cand = torch.tensor(case["candidates"], dtype=torch.long)
    probs = torch.ones(len(cand)) / len(cand)
    opt = KSeedZerothOrderOptimizer(groups, cand, probs, lr=case["lr"], eps=case["eps"], weight_decay=case["wd"],
                                    grad_clip=-100.0)
    # CPU losses, as in the reference's run: g = (loss_right - loss_left) / (2 eps) is a CPU
    # true division (a device tensor would divide by multiplying with the reciprocal)
    it = iter([torch.tensor(x) for x in case["losses"]])
    rets = [float(opt.kseed_zeroth_order_step(lambda: next(it))) for _ in range(4)]
    assert not opt._last_step_on_device
    torch.cuda.synchronize()
    for got, want in zip(rets, case["returns"]):
        assert (math.isnan(got) and math.isnan(want)) or got == want, (rets, case["returns"])
    hist = {str(k): v for k, v in opt.directional_derivative_history.items() if v}
    assert hist == case["history"]
    assert set(opt.directional_derivative_history) == set(case["candidates"])
    for n in order:
        assert_bitwise(to_np(params[n].data), z[f"final/{n}"].reshape(-1), "float32", f"final/{n}")


def test_kseed_step_without_closure_is_a_nan_noop():
    from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer
    dev = _dev()
    p = torch.nn.Parameter(torch.ones(64, device=dev))
    opt = KSeedZerothOrderOptimizer([{"params": [p], "weight_decay": 0.0}], torch.arange(4) + 1, torch.ones(4) / 4,
                                    lr=1e-3, eps=5e-4, weight_decay=0.0, grad_clip=-100.0)
    assert math.isnan(float(opt.step()))
    assert torch.equal(p.data, torch.ones(64, device=dev))
    with pytest.raises(ValueError):
        opt.kseed_zeroth_order_step(None)


@pytest.mark.parametrize("device_step", [True, False])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("fires", [True, False])
def test_grad_clip(dtype, fires, device_step):
    """g = (2.5 - 2.375) / (2 * 5e-4) = 125: a clip of 100 fires (NaN, no update, the
    parameters are x after +1, -2, +1 perturbations), a clip of 200 does not."""
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    shapes = [4800, 48, 7, 185]
    arrays = rand_params(shapes, dtype, seed=51)
    params = [torch.nn.Parameter(from_np(a, dtype, dev)) for a in arrays]
    groups = [{"params": params[:2], "weight_decay": 0.0}, {"params": params[2:], "weight_decay": 0.01}]
    clip = 100.0 if fires else 200.0
    opt = ZerothOrderOptimizer(groups, lr=1e-3, eps=5e-4, weight_decay=0.01, grad_clip=clip)
    opt.device_step = device_step
    losses = iter([torch.tensor(2.5, device=dev), torch.tensor(2.375, device=dev)])
    g, lr_, ll_ = opt.zeroth_order_step(4242, lambda: next(losses))
    assert opt._last_step_on_device == device_step
    torch.cuda.synchronize()
    for sf in (1.0, -2.0, 1.0):
        O.perturb_params(arrays, [DTC[dtype]] * len(arrays), 4242, sf * 5e-4)
    if fires:
        assert math.isnan(float(g))
    else:
        gv = float(g)
        assert gv == float(np.float32((2.5 - 2.375)) / np.float32(1e-3)) or abs(gv - 125.0) < 1e-3
        if dtype == "bfloat16":
            gv = float(torch.tensor(gv, dtype=torch.float32).to(torch.bfloat16).float())
        O.reconstruct(arrays, [DTC[dtype]] * len(arrays), [1e-3] * 4, [0.0] * 4, [4242], [gv])
    for i, (p, a) in enumerate(zip(params, arrays)):
        assert_bitwise(to_np(p.data), a, dtype, f"tensor {i}")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("nan_at", [None, 1])
def test_device_step_has_no_host_sync(nan_at, dtype):
    """Four KSeed steps with device losses under torch.cuda's sync debug mode "error":
    nothing in the step synchronises with the host; the history (read afterwards) and
    the parameters equal the host path's (device_step = False) on the same draws."""
    from fate_llm.algo.fedkseed.optimizer import KSeedZerothOrderOptimizer
    dev = _dev()
    shapes = [4096, 33, 1000]
    arrays = rand_params(shapes, dtype, seed=61)
    loss_vals = [2.5, 2.25, 2.375, 2.5, 2.0, 2.125, 3.0, 2.875]
    if nan_at is not None:
        loss_vals[2 * nan_at] = math.nan
    runs = {}
    for device_step in (False, True):
        params = [torch.nn.Parameter(from_np(a, dtype, dev)) for a in arrays]
        groups = [{"params": params[:2], "weight_decay": 0.0}, {"params": params[2:], "weight_decay": 0.01}]
        opt = KSeedZerothOrderOptimizer(groups, torch.arange(8) + 100, torch.ones(8) / 8, lr=1e-3, eps=5e-4,
                                        weight_decay=0.01, grad_clip=-100.0)
        opt.device_step = device_step
        opt.sample_random_generator.manual_seed(7)
        losses = [torch.tensor(x, device=dev) for x in loss_vals]
        it = iter(losses)
        rets = []
        torch.cuda.synchronize()
        if device_step:
            torch.cuda.set_sync_debug_mode("error")
        try:
            for _ in range(4):
                rets.append(opt.kseed_zeroth_order_step(lambda: next(it)))
        finally:
            torch.cuda.set_sync_debug_mode("default")
        hist = {k: list(v) for k, v in opt.directional_derivative_history.items()}
        runs[device_step] = ([float(r) for r in rets], hist, [to_np(p.data) for p in params])
    (r0, h0, p0), (r1, h1, p1) = runs[False], runs[True]
    assert [math.isnan(x) for x in r0] == [math.isnan(x) for x in r1]
    assert [x for x in r0 if not math.isnan(x)] == [x for x in r1 if not math.isnan(x)]
    assert h0 == h1 and sum(len(v) for v in h1.values()) == (4 if nan_at is None else 3)
    for i, (a, b) in enumerate(zip(p0, p1)):
        assert_bitwise(b, a, dtype, f"tensor {i}")
