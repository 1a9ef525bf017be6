"""torch's global generators after a drop-in call stand where the reference leaves them.

The reference calls torch.manual_seed(seed) and then draws z from the generator of the
parameters' device (zo_utils.py:42,47; optimizer.py:165,170-172), so whatever runs next
-- the zeroth-order closure's dropout between the perturbations, a sampler's next
permutation -- draws from the state those draws left.  The drop-in draws nothing from
torch; codec._leave re-seeds and moves the generator of the call's stream to that state:
the device generator's Philox offset (torch_rocm), the CPU generator's mt19937 state and
cached normal (torch_cpu).

Checked against the reference's own calls (oracle/torch_replica.py: zo_utils.py:42-54 and
optimizer.py:127-173 re-typed), run on the device (torch_rocm: the stream an unmodified
reference client on this GPU draws) or on CPU copies (torch_cpu: a reference client on the
CPU): torch.get_rng_state() and torch.cuda.get_rng_state() after reconstruct_,
random_perturb_parameters and zeroth_order_step -- whose closure draws noise from the
generator between the perturbations, so its losses, g and the update depend on the state
-- plus the parameters, bit for bit."""
import pytest
import torch

from oracle import torch_replica as R
from test_gpu_parity import _dev

pytestmark = pytest.mark.gpu

SHAPES = [(4096,), (48,), (5,), (1000, 17), (3,), (700_001,), (0,), (9,)]


def _bits(t):
    return t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)


def _same(a, b, what):
    assert torch.equal(_bits(a.detach().cpu()), _bits(b.detach().cpu())), what


def _states(dev):
    return torch.get_rng_state(), torch.cuda.get_rng_state(dev)


def _assert_states(got, want, what):
    assert torch.equal(got[0], want[0]), f"{what}: CPU generator state differs"
    assert torch.equal(got[1], want[1]), f"{what}: device generator state differs"


def _init(dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(s, generator=g) * 0.02).to(dtype) for s in SHAPES]


def _groups(params, wd=0.0, eps=1e-3):
    return [{"params": params[:3], "weight_decay": 0.0, "lr": 1e-4, "eps": eps},
            {"params": params[3:], "weight_decay": wd, "lr": 1e-4, "eps": eps}]


@pytest.mark.parametrize("stream", ["torch_rocm", "torch_cpu"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_reconstruct_leaves_the_generators(stream, dtype):
    from fate_llm.algo.fedkseed import codec, zo_utils
    dev = _dev()
    ref_dev = dev if stream == "torch_rocm" else torch.device("cpu")
    init = _init(dtype)
    ref = [torch.nn.Parameter(t.to(ref_dev)) for t in init]
    got = [torch.nn.Parameter(t.to(dev)) for t in init]
    g = torch.Generator().manual_seed(5)
    seeds = torch.randint(0, 2**32, (41,), generator=g).tolist()
    vals = (torch.randn(41, generator=g, dtype=torch.float64) * 20).tolist()
    vals[-1] = 0.0  # the last applied seed is the one before (train_once skips zeros)
    torch.manual_seed(999)
    R.reconstruct(ref, seeds, vals, 1e-4, 0.0)
    want = _states(dev)
    torch.manual_seed(999)
    codec.set_stream_mode(stream)
    try:
        zo_utils.reconstruct_([{"params": got, "weight_decay": 0.0, "lr": 0.0}], seeds, vals, lr=1e-4,
                              weight_decay=0.0)
    finally:
        codec.set_stream_mode("torch_cpu")
    torch.cuda.synchronize()
    _assert_states(_states(dev), want, f"{stream} reconstruct_")
    for i, (a, b) in enumerate(zip(got, ref)):
        _same(a, b, f"tensor {i}")


@pytest.mark.parametrize("stream", ["torch_rocm", "torch_cpu"])
def test_zeroth_order_steps_see_the_reference_generator(stream):
    """Three KSeed-style zeroth-order steps, frozen tensor included (the unfused path) and
    not (the fused device path): the closure draws noise from the stream's generator
    between the perturbations, so every loss, g and update follows the state the previous
    call left."""
    from fate_llm.algo.fedkseed import codec
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    ref_dev = dev if stream == "torch_rocm" else torch.device("cpu")
    for frozen in (False, True):
        init = _init(torch.bfloat16, seed=3)
        ref = [torch.nn.Parameter(t.to(ref_dev)) for t in init]
        got = [torch.nn.Parameter(t.to(dev)) for t in init]
        if frozen:
            ref[1].requires_grad_(False)
            got[1].requires_grad_(False)
        w = torch.linspace(-1, 1, 4096)

        def closure_on(params, where):
            # noise from the generator the previous call left (the reference client's device);
            # the loss is computed there too, from the same bits on both sides
            def closure():
                noise = torch.rand(4096, device=where)
                x = params[0].detach().to(where).float()
                return (x * noise * w.to(where)).sum() * 100.0
            return closure

        rgroups = _groups(ref, wd=0.01)
        opt = ZerothOrderOptimizer(_groups(got, wd=0.01), lr=1e-4, eps=1e-3, weight_decay=0.01, grad_clip=0.0)
        codec.set_stream_mode(stream)
        try:
            for step, seed in enumerate([17, 2**33 + 5, 17]):
                noise_dev = ref_dev  # the closure draws where the reference client's model lives
                torch.manual_seed(1000 + step)
                g_ref, lr_ref, ll_ref = R.zeroth_order_step(rgroups, seed, closure_on(ref, noise_dev), 1e-3)
                want = _states(dev)
                torch.manual_seed(1000 + step)
                g_got, lr_got, ll_got = opt.zeroth_order_step(seed, closure_on(got, noise_dev))
                torch.cuda.synchronize()
                _assert_states(_states(dev), want, f"{stream} frozen={frozen} step {step}")
                assert float(lr_got) == float(lr_ref) and float(ll_got) == float(ll_ref), (step, frozen)
                assert float(g_got) == float(g_ref), (step, frozen)
        finally:
            codec.set_stream_mode("torch_cpu")
        for i, (a, b) in enumerate(zip(got, ref)):
            _same(a, b, f"frozen={frozen} tensor {i}")


@pytest.mark.parametrize("stream", ["torch_rocm", "torch_cpu"])
def test_perturb_leaves_the_generators(stream):
    from fate_llm.algo.fedkseed import codec
    from fate_llm.algo.fedkseed.optimizer import ZerothOrderOptimizer
    dev = _dev()
    ref_dev = dev if stream == "torch_rocm" else torch.device("cpu")
    init = _init(torch.float32, seed=4)
    ref = [torch.nn.Parameter(t.to(ref_dev)) for t in init]
    got = [torch.nn.Parameter(t.to(dev)) for t in init]
    ref[4].requires_grad_(False)  # draws nothing in the reference's perturb
    got[4].requires_grad_(False)
    opt = ZerothOrderOptimizer(_groups(got), lr=1e-4, eps=1e-3, weight_decay=0.0, grad_clip=0.0)
    codec.set_stream_mode(stream)
    try:
        for seed, sf in [(8, 1.0), (8, -2.0), (2**40 + 1, 1.0)]:
            R.random_perturb_parameters(_groups(ref), seed, sf)
            want = _states(dev)
            torch.manual_seed(1)
            opt.random_perturb_parameters(seed, sf)
            torch.cuda.synchronize()
            _assert_states(_states(dev), want, f"{stream} perturb seed {seed}")
    finally:
        codec.set_stream_mode("torch_cpu")
    for i, (a, b) in enumerate(zip(got, ref)):
        _same(a, b, f"tensor {i}")


def test_seed_sharded_reconstruct_leaves_the_generators():
    """The C3 variant draws only its rank's seeds, but leaves the generators where the
    reference's whole loop leaves them (the last seed's draws)."""
    from fate_llm.algo.fedkseed import codec, zo_utils
    dev = _dev()
    init = _init(torch.float32, seed=6)
    ref = [t.to(dev) for t in init]
    got = [torch.nn.Parameter(t.to(dev)) for t in init]
    seeds, vals = [3, 9, 27, 81], [1.5, -2.0, 0.5, 4.0]
    R.reconstruct(ref, seeds, vals, 1e-4, None)
    want = _states(dev)
    torch.manual_seed(5)
    codec.set_stream_mode("auto")  # torch_rocm for tensors on the GPU: the drop-in default
    try:
        zo_utils.reconstruct_seed_sharded_([{"params": got, "weight_decay": None, "lr": 0.0}], seeds, vals,
                                           lr=1e-4, weight_decay=None)
    finally:
        codec.set_stream_mode("torch_cpu")
    _assert_states(_states(dev), want, "seed-sharded reconstruct")


def test_grid_cap_is_torchs():
    """The grid cap the library draws with (fks_capi.cpp phx_geometry) and carries on the
    wire is the one torch's calc_execution_policy derives (DistributionTemplates.h:55-57)
    from the device properties; and a tensor of exactly 256 x cap x 4 + 1 elements -- one
    past a single loop iteration of the full grid -- draws torch's values."""
    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    props = torch.cuda.get_device_properties(dev)
    cap = props.multi_processor_count * (props.max_threads_per_multi_processor // 256)
    assert codec.rocm_grid_cap(dev) == cap
    n = 256 * cap * 4 + 1
    torch.manual_seed(77)
    want = torch.normal(mean=0, std=1, size=(n,), device=dev)
    got = torch.empty(n, device=dev)
    codec.normal_([got], 77, stream_mode="torch_rocm")
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


@pytest.mark.parametrize("case", range(12))
def test_generator_state_fuzz(case):
    """Random tensor lists (the serial path's < 16 elements with its cached normal, ragged
    sizes, whole blocks, mixed dtypes), random K and stream: the generator state after
    codec.directional_step equals the one after the reference's loop, and so do the
    parameters."""
    import numpy as np

    from fate_llm.algo.fedkseed import codec
    dev = _dev()
    rng = np.random.default_rng(700 + case)
    nt = int(rng.integers(1, 7))
    sizes = [int(rng.choice([rng.integers(1, 16), rng.integers(16, 3000), 16 * rng.integers(1, 2000)])) for _ in range(nt)]
    dts = [[torch.float32, torch.bfloat16, torch.float16][int(rng.integers(0, 3))] for _ in range(nt)]
    stream = ["torch_cpu", "torch_rocm"][case % 2]
    k = int(rng.integers(1, 40))
    seeds = [int(s) for s in rng.integers(0, 2**40, k)]
    vals = [float(v) for v in rng.normal(0, 5, k)]
    wd = [None, 0.0, 0.01][int(rng.integers(0, 3))]
    ref_dev = dev if stream == "torch_rocm" else torch.device("cpu")
    g = torch.Generator().manual_seed(case)
    init = [(torch.randn(n, generator=g) * 0.05).to(dt) for n, dt in zip(sizes, dts)]
    ref = [t.to(ref_dev) for t in init]
    got = [t.to(dev) for t in init]
    R.reconstruct(ref, seeds, vals, 1e-3, wd)
    want = _states(dev)
    torch.manual_seed(12345)
    codec.directional_step([codec.ParamSpec(t, lr=1e-3, weight_decay=wd) for t in got], seeds, vals,
                           stream_mode=stream)
    torch.cuda.synchronize()
    _assert_states(_states(dev), want, f"case {case} {stream} sizes {sizes}")
    for i, (a, b) in enumerate(zip(got, ref)):
        _same(a, b, f"case {case} tensor {i}")
