"""Wire format of the FedKSeed round payloads (payload.py):
round trips on the reference's own arbiter payloads (tests/golden/cases.json "server",
written by importing the reference), the WireContext end to end around the drop-in
arbiter, malformed buffers, and the byte counts at K = 4096 against the pickled
objects the reference hands its transport (fedkseed.py:57-68, :128)."""
import math
import pickle

import numpy as np
import pytest
import torch

from fate_llm.algo.fedkseed import payload as W
from fate_llm.algo.fedkseed.fedkseed import FedKSeedTrainingArguments, Trainer


def _train_once_obj(sent):
    sums = sent["direction_derivative_sum"]
    return (sent["should_exit"], {
        "seed_candidates": torch.tensor(sent["seed_candidates"], dtype=torch.long),
        "seed_probabilities": torch.tensor(sent["seed_probabilities"], dtype=torch.float32),
        "direction_derivative_sum": None if sums is None else {int(k): v for k, v in sums.items()}})


def _same_train_once(a, b):
    (ea, ka), (eb, kb) = a, b
    assert ea == eb
    assert ka["seed_candidates"].dtype == kb["seed_candidates"].dtype == torch.long
    assert torch.equal(ka["seed_candidates"], kb["seed_candidates"])
    if ka["seed_probabilities"] is None:
        assert kb["seed_probabilities"] is None
    else:
        assert kb["seed_probabilities"].dtype == torch.float32
        assert torch.equal(ka["seed_probabilities"].view(torch.int32), kb["seed_probabilities"].view(torch.int32))
    sa, sb = ka["direction_derivative_sum"], kb["direction_derivative_sum"]
    if sa is None:
        assert sb is None
    else:
        assert list(sa.keys()) == list(sb.keys())
        assert np.array_equal(np.array(list(sa.values())).view(np.uint64), np.array(list(sb.values())).view(np.uint64))


def test_train_once_roundtrip_golden(cases):
    t = cases["server"]["trainer"]
    for sent in t["guest_sent"] + t["host_sent"]:
        obj = _train_once_obj(sent)
        buf = W.encode_train_once(obj)
        _same_train_once(obj, W.decode_train_once(buf))
        # the sums' keys are the candidates in order: values only on the wire
        k = len(sent["seed_candidates"])
        has_sums = sent["direction_derivative_sum"] is not None
        assert len(buf) == 16 + 4 * k + 4 * k + (8 * k if has_sums else 0)


def test_history_roundtrip_golden(cases):
    t = cases["server"]["trainer"]
    for rep in t["guest_replies"] + t["host_replies"]:
        h = {int(k): list(v) for k, v in rep.items()}
        back = W.decode_history(W.encode_history(h))
        assert list(back) == list(h)
        for k in h:
            assert np.array_equal(np.array(back[k], np.float64).view(np.uint64), np.array(h[k], np.float64).view(np.uint64))


def test_history_f32_values_travel_as_f32():
    """g.item() of a 0-dim f32 tensor is f32-exact: 4 bytes per value; NaN/inf kept."""
    vals = [float(np.float32(x)) for x in (1.5, -2.25, 3.0e-8, 125.0)] + [math.inf, -0.0]
    h = {7: vals[:3], 9: [], 2**31: vals[3:]}
    buf = W.encode_history(h)
    assert len(buf) == 16 + 4 * 3 + 4 * 3 + 4 * len(vals)
    back = W.decode_history(buf)
    assert back == h and math.copysign(1.0, back[2**31][-1]) < 0
    hn = {1: [float("nan")]}
    assert math.isnan(W.decode_history(W.encode_history(hn))[1][0])


def test_wide_seeds_and_reordered_sums():
    seeds = torch.tensor([5, 2**40, -3], dtype=torch.long)
    obj = (True, {"seed_candidates": seeds, "seed_probabilities": torch.ones(3) / 3,
                  "direction_derivative_sum": {2**40: 1.0, 5: -2.5, -3: 0.0}})
    back = W.decode_train_once(W.encode_train_once(obj))
    _same_train_once(obj, back)
    h = {2**40: [1.0], -3: [2.0]}
    assert W.decode_history(W.encode_history(h)) == h


@pytest.mark.parametrize("cut", [0, 5, 15, 17, 30])
def test_truncated_and_malformed_buffers_raise(cut):
    obj = _train_once_obj({"should_exit": False, "seed_candidates": [1, 2, 3, 4],
                           "seed_probabilities": [0.25] * 4, "direction_derivative_sum": {1: 1.0, 2: 0.0, 3: 0.0, 4: 2.0}})
    buf = W.encode_train_once(obj)
    with pytest.raises(W.WireFormatError):
        W.decode_train_once(buf[:cut])
    with pytest.raises(W.WireFormatError):
        W.decode_train_once(buf + b"\0")
    with pytest.raises(W.WireFormatError):
        W.decode_history(buf)  # wrong record kind
    with pytest.raises(W.WireFormatError):
        W.decode_train_once(b"XXXX" + buf[4:])


class _Loop:
    """A loopback link that only carries bytes (what a real transport would move)."""

    def __init__(self, replies):
        self.replies = replies
        self.sent = []
        self.wire_bytes = 0

    def put(self, key, value):
        if key in ("train_once", "direction_derivative_history"):
            assert isinstance(value, bytes), f"{key} travelled as {type(value)}"
            self.wire_bytes += len(value)
        if key == "train_once":
            self.last_candidates = W.decode_train_once(value)[1]["seed_candidates"].tolist()
        self.sent.append((key, value))

    def get(self, key):
        value = self.replies.pop(0)
        if key == "direction_derivative_history":  # what a wrapped client sends: sparse
            cand = [int(s) for s in self.last_candidates]
            value = W.encode_history(value, cand if list(value) == cand else None)
            self.wire_bytes += len(value)
        return value


class _Ctx:
    def __init__(self, guest, hosts):
        self.guest, self.hosts = guest, hosts

    def ctxs_range(self, n):
        for i in range(n):
            yield i, self


def test_wire_context_around_the_arbiter(cases):
    """The drop-in arbiter run through WireContext: the client-side decode of every
    put equals the object the arbiter passed at that moment (the plain run's payloads,
    snapshot at put time), and the replies decode back into the same bookkeeping."""
    t = cases["server"]["trainer"]
    reps = lambda rr: [{int(k): list(v) for k, v in r.items()} for r in rr]  # noqa: E731
    seeds = torch.tensor(t["seeds"], dtype=torch.long)
    args = FedKSeedTrainingArguments(num_aggregations=t["rounds"], k=len(t["seeds"]))

    class Snap:
        def __init__(self, replies):
            self.replies, self.sent = replies, []

        def put(self, key, value):
            self.sent.append(pickle.loads(pickle.dumps(value)))  # as a transport serialises at put

        def get(self, key):
            return self.replies.pop(0)

    pg, ph = Snap(reps(t["guest_replies"])), Snap(reps(t["host_replies"]))
    Trainer(_Ctx(pg, [ph]), seeds, None, args).train()
    wg, wh = _Loop(reps(t["guest_replies"])), _Loop(reps(t["host_replies"]))
    Trainer(W.WireContext(_Ctx(wg, [wh])), seeds, None, args).train()
    for plain, wired in ((pg, wg), (ph, wh)):
        assert len(plain.sent) == len(wired.sent) == t["rounds"]
        for obj, (key, buf) in zip(plain.sent, wired.sent):
            assert key == "train_once"
            _same_train_once(obj, W.decode_train_once(buf))


def test_sparse_history_needs_and_restores_candidates():
    cand = [11, 22, 33, 44]
    h = {11: [], 22: [1.5, 2.5], 33: [], 44: [float(np.float32(0.1))]}
    buf = W.encode_history(h, cand)
    assert len(buf) == 16 + 8 * 2 + 4 * 3
    back = W.decode_history(buf, cand)
    assert back == h and list(back) == cand
    with pytest.raises(W.WireFormatError):
        W.decode_history(buf)
    # keys not equal to the candidates in order: dense form
    h2 = {22: [1.0], 11: []}
    assert W.decode_history(W.encode_history(h2, cand)) == h2


def test_wire_bytes_k4096():
    """Per round at K = 4096: the arbiter's payload is 16 + 16 K bytes (u32 seed, f32
    probability, f64 sum per seed) and a client's history of 151 local steps 16 + 8 K +
    4 per step in the dense form, 16 + 8 per sampled seed + 4 per step in the sparse form
    (WireContext), against the pickled objects the reference moves."""
    k, steps = 4096, 151
    g = torch.Generator().manual_seed(0)
    seeds = torch.randint(0, 2**32, (k,), generator=g)
    probs = torch.softmax(torch.randn(k, generator=g), 0)
    sums = {int(s): float(v) for s, v in zip(seeds, torch.randn(k, generator=g, dtype=torch.float64))}
    obj = (False, {"seed_candidates": seeds, "seed_probabilities": probs, "direction_derivative_sum": sums})
    buf = W.encode_train_once(obj)
    assert len(buf) == 16 + 16 * k
    hist = {int(s): [] for s in seeds}
    idx = torch.randint(0, k, (steps,), generator=g)
    for i in idx.tolist():
        hist[int(seeds[i])].append(float(torch.randn(1, generator=g).float()))
    hb = W.encode_history(hist)
    assert len(hb) == 16 + 8 * k + 4 * steps
    sb = W.encode_history(hist, seeds.tolist())
    distinct = sum(1 for v in hist.values() if v)
    assert len(sb) == 16 + 8 * distinct + 4 * steps
    assert W.decode_history(sb, seeds.tolist()) == hist
    pk_obj, pk_hist = len(pickle.dumps(obj)), len(pickle.dumps(hist))
    print(f"K=4096 wire: train_once {len(buf)} B (pickle {pk_obj} B), history {len(sb)} B sparse / {len(hb)} B "
          f"dense (pickle {pk_hist} B)")
    assert len(buf) < pk_obj and len(hb) < pk_hist and len(sb) < 2048
