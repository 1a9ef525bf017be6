"""The z stream as an explicit, checked part of a FedKSeed round (CPU, no device).

The reference draws z where the parameters live (zo_utils.py:47, optimizer.py:170-172:
``device=param.data.device``, after ``model.to(training_args.device)`` at fedkseed.py:133),
so a reference client on an MI355X draws torch's HIP-generator (Philox) stream and one on
the CPU draws mt19937.  What these tests pin:

* ``FKS_STREAM_MODE`` unset means "auto": the stream the reference draws on the tensors'
  device -- torch_rocm for a client whose ``training_args.device`` is cuda, so the drop-in
  and an unmodified reference client on the same GPU give the same bits;
* the wire records carry the sender's stream (two flag bits) and, for torch_rocm, its
  device's grid cap (a u32), and decode to objects equal to the originals;
* two clients on different streams -- or on torch_rocm devices of different grid caps, e.g.
  an MI355X in SPX mode (256 CUs: 2,048) and one in a CPX partition (32 CUs: 256) -- make
  the drop-in arbiter fail loudly, and a client refuses an arbiter that declared another
  stream; an arbiter that learnt the stream from the first tagged history declares it into
  its own later records.
"""
import os
import queue
import subprocess
import sys
import threading

import pytest
import torch

from fate_llm.algo.fedkseed import codec
from fate_llm.algo.fedkseed import fedkseed as F
from fate_llm.algo.fedkseed import payload as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def setting():
    old = codec.get_stream_mode()
    yield codec.set_stream_mode
    codec.set_stream_mode(old)


def test_unset_env_means_auto_which_follows_the_device():
    env = {k: v for k, v in os.environ.items() if k != "FKS_STREAM_MODE"}
    code = ("import sys; sys.path.insert(0, 'fate-llm_amd/python'); import torch\n"
            "from fate_llm.algo.fedkseed import codec\n"
            "print(codec.get_stream_mode(), codec.resolve_stream_mode(torch.device('cuda', 0)), "
            "codec.resolve_stream_mode('cpu'), codec.resolve_stream_mode(None))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["auto", "torch_rocm", "torch_cpu", "torch_cpu"]


def test_resolve_stream_mode(setting):
    setting("auto")
    assert codec.resolve_stream_mode("cuda:1") == "torch_rocm"
    assert codec.resolve_stream_mode(torch.device("cpu")) == "torch_cpu"
    assert codec.resolve_stream_mode("cuda", stream_mode="torch_cpu") == "torch_cpu"
    setting("torch_cpu")
    assert codec.resolve_stream_mode("cuda") == "torch_cpu"
    assert codec.resolve_stream_mode("cuda", stream_mode="auto") == "torch_rocm"
    with pytest.raises(ValueError):
        codec.resolve_stream_mode("cuda", stream_mode="philox")
    with pytest.raises(ValueError):
        setting("mt19937")


class _Args:
    learning_rate, weight_decay = 1e-5, 0.0

    def __init__(self, device):
        self.device = device


def test_client_stream_follows_training_device(setting):
    setting("auto")
    gpu = F.ClientTrainer(None, torch.nn.Linear(2, 2), F.FedKSeedTrainingArguments(), _Args("cuda:0"),
                          None, None, None, None)
    cpu = F.ClientTrainer(None, torch.nn.Linear(2, 2), F.FedKSeedTrainingArguments(), _Args(torch.device("cpu")),
                          None, None, None, None)
    assert (gpu.stream_mode, cpu.stream_mode) == ("torch_rocm", "torch_cpu")
    setting("torch_cpu")  # an explicit setting wins on any device
    assert gpu.stream_mode == "torch_cpu"


def test_wire_records_carry_the_stream():
    cands = [3, 1 << 31, 7]
    hist = {3: [0.25, -1.5], 1 << 31: [], 7: [2.0]}
    for stream in ("torch_cpu", "torch_rocm"):
        for c in (cands, None):  # sparse and explicit-key forms
            back = W.decode_history(W.encode_history(hist, c, stream), c)
            assert isinstance(back, W.History) and back == hist and back.stream_mode == stream
            assert list(back) == list(hist)
    plain = W.decode_history(W.encode_history(hist, cands), cands)
    assert type(plain) is dict and plain == hist and getattr(plain, "stream_mode", None) is None
    # the tag costs no bytes
    assert len(W.encode_history(hist, cands, "torch_rocm")) == len(W.encode_history(hist, cands))
    msg = (False, {"seed_candidates": torch.tensor(cands), "seed_probabilities": torch.ones(3) / 3,
                   "direction_derivative_sum": {3: 1.0, 1 << 31: 0.0, 7: -2.0}})
    ex, kw = W.decode_train_once(W.encode_train_once(msg, "torch_rocm"))
    assert kw["stream_mode"] == "torch_rocm" and kw["direction_derivative_sum"] == msg[1]["direction_derivative_sum"]
    ex, kw = W.decode_train_once(W.encode_train_once(msg))
    assert "stream_mode" not in kw
    with pytest.raises(W.WireFormatError):
        W.encode_history(hist, cands, "mt")


def test_wire_records_carry_the_grid_cap():
    cands = [3, 1 << 31, 7]
    hist = {3: [0.25, -1.5], 1 << 31: [], 7: [2.0]}
    for c in (cands, None):
        back = W.decode_history(W.encode_history(hist, c, "torch_rocm", 2048), c)
        assert back == hist and (back.stream_mode, back.stream_grid) == ("torch_rocm", 2048)
        back = W.decode_history(W.encode_history(hist, c, "torch_rocm"), c)
        assert back == hist and (back.stream_mode, back.stream_grid) == ("torch_rocm", None)
    assert len(W.encode_history(hist, cands, "torch_rocm", 256)) == len(W.encode_history(hist, cands)) + 4
    msg = (False, {"seed_candidates": torch.tensor(cands), "seed_probabilities": torch.ones(3) / 3,
                   "direction_derivative_sum": {3: 1.0, 1 << 31: 0.0, 7: -2.0}})
    ex, kw = W.decode_train_once(W.encode_train_once(msg, "torch_rocm", 2432))
    assert (kw["stream_mode"], kw["stream_grid"]) == ("torch_rocm", 2432)
    assert kw["seed_candidates"].tolist() == cands and kw["direction_derivative_sum"] == msg[1]["direction_derivative_sum"]
    with pytest.raises(W.WireFormatError):  # the cap belongs to the counter-mode stream only
        W.encode_history(hist, cands, "torch_cpu", 2048)
    with pytest.raises(W.WireFormatError):
        W.encode_train_once(msg, "torch_rocm", 0)
    # the check: another cap on torch_rocm is another stream; an unknown cap passes
    W.check_stream("torch_rocm", "torch_rocm", "x", 2048, 2048)
    W.check_stream("torch_rocm", "torch_rocm", "x", 2048, None)
    with pytest.raises(W.StreamMismatchError, match="grid cap 256"):
        W.check_stream("torch_rocm", "torch_rocm", "x", 2048, 256)


# --------------------------------------------------------------- a loopback federation
class _Party:
    def __init__(self, out_q, in_q):
        self.out_q, self.in_q = out_q, in_q

    def put(self, key, value):
        self.out_q.put((key, value))

    def get(self, key):
        k, v = self.in_q.get(timeout=5)
        assert k == key, (k, key)
        return v


class _ArbiterCtx:
    def __init__(self, links):
        self.guest = _Party(links[0][0], links[0][1])
        self.hosts = [_Party(a, b) for a, b in links[1:]]

    def ctxs_range(self, n):
        for i in range(n):
            yield i, self


class _ClientCtx:
    def __init__(self, link):
        self.arbiter = _Party(link[1], link[0])

    def ctxs_range(self, n):
        for i in range(n):
            yield i, self


class _ScalarClient(F.ClientTrainer):
    """The drop-in ClientTrainer's round loop with a host-only local phase: one g for the
    first sampled candidate (the codec is not needed to exercise the protocol).  ``grid``
    stands for the device's grid cap (codec.rocm_grid_cap reads it from the device)."""

    grid = 2048

    def _device_grid_cap(self):
        return self.grid

    def train_once(self, seed_candidates, seed_probabilities, direction_derivative_sum):
        first = int(seed_candidates[0])
        return {int(s): ([0.5] if int(s) == first else []) for s in seed_candidates}


def _federation(devices, arbiter_stream=None, rounds=1, grids=None, arbiter_grid=None):
    links = [(queue.Queue(), queue.Queue()) for _ in devices]
    errors, threads = {}, []

    def run(name, fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- reported to the test
            errors[name] = e

    arb = F.Trainer(W.WireContext(_ArbiterCtx(links), stream_mode=arbiter_stream, stream_grid=arbiter_grid),
                    torch.tensor([11, 22, 33]), None, F.FedKSeedTrainingArguments(num_aggregations=rounds, k=3))
    threads.append(threading.Thread(target=run, args=("arbiter", arb.train), daemon=True))
    for i, (dev, link) in enumerate(zip(devices, links)):
        cl = _ScalarClient(W.WireContext(_ClientCtx(link)), torch.nn.Linear(2, 2),
                           F.FedKSeedTrainingArguments(num_aggregations=rounds), _Args(dev), None, None, None, None)
        if grids is not None:
            cl.grid = grids[i]
        threads.append(threading.Thread(target=run, args=(f"client{i}", cl.train), daemon=True))
    for t in threads:
        t.start()
    threads[0].join(timeout=30)
    assert not threads[0].is_alive()
    for t in threads[1:]:
        t.join(timeout=5)
    return arb, errors


def test_same_stream_federation_runs(setting):
    setting("auto")
    arb, errors = _federation(["cuda:0", "cuda:0", "cuda:1"], rounds=2)
    assert not errors
    assert arb.stream_mode == "torch_rocm"


def test_clients_on_different_streams_fail_loudly(setting):
    setting("auto")  # guest and host 1 on a GPU (torch_rocm), host 2 on the CPU (torch_cpu)
    arb, errors = _federation(["cuda:0", "cuda:0", "cpu"])
    assert isinstance(errors.get("arbiter"), W.StreamMismatchError)
    assert "client 2" in str(errors["arbiter"]) and "torch_cpu" in str(errors["arbiter"])


def test_client_refuses_an_arbiter_on_another_stream(setting):
    setting("torch_rocm")
    arb, errors = _federation(["cuda:0"], arbiter_stream="torch_cpu")
    assert isinstance(errors.get("client0"), W.StreamMismatchError)
    assert "the arbiter" in str(errors["client0"])


def test_same_stream_federation_learns_and_declares_the_grid(setting):
    setting("auto")
    arb, errors = _federation(["cuda:0", "cuda:1"], rounds=3)
    assert not errors
    assert (arb.stream_mode, arb.stream_grid) == ("torch_rocm", 2048)
    assert (arb.ctx.stream_mode, arb.ctx.stream_grid) == ("torch_rocm", 2048)  # its later records carry it


def test_clients_on_different_grid_caps_fail_loudly(setting):
    setting("auto")  # three torch_rocm clients: two MI355X in SPX mode, one in a CPX partition
    arb, errors = _federation(["cuda:0", "cuda:1", "cuda:2"], grids=[2048, 2048, 256])
    assert isinstance(errors.get("arbiter"), W.StreamMismatchError)
    assert "client 2" in str(errors["arbiter"]) and "grid cap 256" in str(errors["arbiter"])


def test_client_refuses_an_arbiter_of_another_grid_cap(setting):
    setting("auto")
    arb, errors = _federation(["cuda:0"], arbiter_stream="torch_rocm", arbiter_grid=2432)  # an MI300X's cap
    assert isinstance(errors.get("client0"), W.StreamMismatchError)
    assert "grid cap 2432" in str(errors["client0"])


def test_arbiter_declares_the_learnt_stream_to_later_rounds(setting):
    # the arbiter declares nothing; round 1 teaches it torch_rocm / 2048 from the clients'
    # histories; from round 2 on its train_once records carry that, and a client drawing
    # another cap refuses them
    setting("auto")
    arb, errors = _federation(["cuda:0"], rounds=2)
    assert not errors and arb.ctx.stream_grid == 2048


def test_grid_field_edge_cases():
    """A torch_rocm record whose grid field is cut off, and a grid flag on a record that is
    not torch_rocm, are malformed; an untagged reference record still decodes unchanged."""
    import struct
    cands = [3, 7]
    hist = {3: [0.5], 7: []}
    rec = W.encode_history(hist, cands, "torch_rocm", 2048)
    with pytest.raises(W.WireFormatError):
        W.decode_history(rec[:W._HEADER.size + 2], cands)  # the u32 cap cut in half
    magic, version, kind, flags, count = W._HEADER.unpack_from(rec, 0)
    bad = W._HEADER.pack(magic, version, kind, (flags & ~W._F_STREAM_ROCM), count) + rec[W._HEADER.size:]
    with pytest.raises(W.WireFormatError):
        W.decode_history(bad, cands)  # grid flag on a torch_cpu record
    plain = W.encode_history(hist, cands)
    assert W.decode_history(plain, cands) == hist
    assert struct.unpack_from("<I", rec, W._HEADER.size)[0] == 2048
