"""C5 round harness (harness/c5_round.py) on one GPU: client processes and the
aggregator process exchange the drop-in Trainer / ClientTrainer payloads over gloo.

* one client, two rounds: round 1 has nothing to reconstruct, round 2 replays exactly
  the seeds the first round's local steps touched (non-zero cumulative sums), as the
  reference's train_once does;
* eight clients sharing the GPU, the full ClientTrainer.train loop with the local steps
  through KSeedZOExtendedTrainer.training_step in the transformers loop, payloads in the
  compact wire format: what every client received each round equals what the drop-in
  arbiter computes offline from the same client histories (fedkseed.py:41-85), and the
  histories travel as a few hundred bytes;
* the same run replayed, client by client and round by round, through the oracle: the
  reconstruct from model_0 of the cumulative (seed, sum) list (fedkseed.py:130-141), then
  every local step -- perturb +eps, -2 eps, +eps, the update with g (optimizer.py:108-150,
  :210-235) -- must give the client's first 4096 parameters bit for bit after the
  reconstruct and after the local steps; each g must be the loss difference of the
  oracle's perturbed parameters (the synthetic closure recomputed in float64), and each
  client's history must be its steps' g in order."""
import math

import numpy as np
import pytest
import torch

from oracle import fks_oracle as O

pytestmark = pytest.mark.gpu


def test_two_rounds_small():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from harness import c5_round
    out = c5_round.main(["--params", "1048576", "--k", "32", "--steps", "6", "--rounds", "2"])
    r0, r1 = out["rounds"]
    assert r0["seeds_reconstructed"] == 0
    assert 1 <= r1["seeds_reconstructed"] <= 6  # distinct seeds sampled in round 1 with g != 0
    assert r1["reconstruct_s"] > 0 and r1["local_steps_s"] > 0


def test_eight_clients_trainer_loop_wire():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from harness import c5_round
    rounds, k, steps = 3, 64, 5
    out = c5_round.main(["--params", "262144", "--k", str(k), "--steps", str(steps), "--rounds", str(rounds),
                         "--clients", "8", "--driver", "trainer", "--wire", "--placement", "pinned", "--record"])
    assert len(out["rounds"]) == rounds
    got = out["client_received_sums"]
    assert len(got) == 8
    # every client received the same cumulative sums each round: None, then non-empty
    per_round = list(zip(*[got[c] for c in sorted(got)]))
    for r, recv in enumerate(per_round):
        assert all(x == recv[0] for x in recv)
        if r == 0:
            assert recv[0] is None
        else:
            nz = sum(1 for v in recv[0].values() if v != 0.0)
            assert 1 <= nz <= 8 * steps * r
    # the drop-in arbiter offline, fed the clients' own histories: the sums it puts each
    # round are exactly what the clients received over the wire
    from fate_llm.algo.fedkseed.fedkseed import FedKSeedTrainingArguments, Trainer
    hists = out["client_histories"]

    class Client:
        def __init__(self, replies):
            self.replies, self.sent = list(replies), []

        def put(self, key, value):
            sums = value[1]["direction_derivative_sum"]
            self.sent.append(None if sums is None else dict(sums))

        def get(self, key):
            return self.replies.pop(0)

    class Ctx:
        def __init__(self, cl):
            self.guest, self.hosts = cl[0], cl[1:]

        def ctxs_range(self, n):
            for i in range(n):
                yield i, self

    cl = [Client([{int(s): v for s, v in h.items()} for h in hists[c]]) for c in sorted(hists)]
    Trainer(Ctx(cl), torch.tensor(out["seeds"], dtype=torch.long), None,
            FedKSeedTrainingArguments(num_aggregations=rounds, k=k)).train()
    for c, client in zip(sorted(got), cl):
        assert client.sent == [None if x is None else {int(s): v for s, v in x.items()} for x in got[c]]
    # the wire moved sparse histories: 16 + 8 per sampled seed + 4 per step per client-round
    b = out["bytes_per_round_per_client"]
    assert b["direction_derivative_history.recv"] < 400
    assert out["rounds"][1]["seeds_reconstructed"] >= 1

    # ---- the offline arbiter's probabilities too: what each client received, bit for bit,
    # shaped as the reference's payload (tests/golden/cases.json "server": K candidates, K
    # float32 probabilities, the sums keyed by the candidates in order, None in round 0)
    recs = out["client_records"]
    seeds = [int(x) for x in out["seeds"]]
    for c, client in zip(sorted(got), cl):
        for r, rnd in enumerate(recs[c]["rounds"]):
            assert rnd["candidates"] == seeds
            assert len(rnd["probabilities"]) == k
            assert np.float32(sum(rnd["probabilities"])) == pytest.approx(1.0, abs=1e-5)
            assert (rnd["sums"] is None) == (r == 0)
            if rnd["sums"] is not None:
                assert [int(x) for x in rnd["sums"]] == seeds
    probs_sent = _offline_probabilities(hists, out["seeds"], rounds, k)
    for c in sorted(got):
        assert [rnd["probabilities"] for rnd in recs[c]["rounds"]] == probs_sent

    # ---- every client's rounds through the oracle
    checked = 0
    for c in sorted(recs):
        checked += _replay_client(recs[c], steps)
    assert checked == 8 * rounds * steps


def test_default_stream_clients_replayed_by_torch_on_the_device(monkeypatch):
    """FKS_STREAM_MODE unset ("auto"): clients whose model sits on the GPU draw the
    torch_rocm stream, the z an unmodified reference client on that GPU draws.  Two clients,
    three rounds, the optimizer loop with the wire format (the records carry the stream
    tag); each client's whole tensor replayed through the reference's own torch ops on the
    device -- the reconstruct (fedkseed.py:130-141 into zo_utils.py:42-52), then every
    local step (optimizer.py:108-173: perturb +eps, -2 eps, +eps with torch.normal on the
    device, g from the synthetic closure, the update with the 0-dim g) -- bit for bit,
    every g equal to the reference's, every history its steps'."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from harness import c5_round
    from oracle import torch_replica as R
    monkeypatch.setenv("FKS_STREAM_MODE", "auto")  # the spawned clients see it at import
    rounds, k, steps, n = 3, 32, 4, 65536
    out = c5_round.main(["--params", str(n), "--k", str(k), "--steps", str(steps), "--rounds", str(rounds),
                         "--clients", "2", "--wire", "--placement", "pinned", "--record", "--record-prefix", "0"])
    recs = out["client_records"]
    dev = torch.device("cuda", 0)

    def tensor(bits):
        return torch.from_numpy(np.array(bits, dtype=np.uint16).view(np.int16)).view(torch.bfloat16).to(dev)

    def perturb(p, seed, sf, eps=5e-4):  # optimizer.py:165-173
        torch.manual_seed(seed)
        z = torch.normal(mean=0, std=1, size=p.size(), device=p.device, dtype=p.dtype)
        return p + sf * eps * z

    def loss(p):  # harness SyntheticModel.forward
        return p.view(-1)[:4096].float().square().mean() * 1e3

    checked = 0
    for c in sorted(recs):
        model_0 = tensor(recs[c]["model_0"])
        assert model_0.numel() == n
        for r, rnd in enumerate(recs[c]["rounds"]):
            p = [model_0.clone()]
            if rnd["sums"]:
                keep = [(int(s), v) for s, v in rnd["sums"].items() if v != 0.0]
                R.reconstruct(p, [s for s, _ in keep], [v for _, v in keep], 1e-5, 0.0)
            assert torch.equal(p[0].view(torch.int16), tensor(rnd["after_reconstruct"]).view(torch.int16)), (c, r)
            hist = {}
            for seed, g, lr in rnd["steps"]:
                x = perturb(p[0], seed, 1.0)
                right = loss(x)
                x = perturb(x, seed, -2.0)
                left = loss(x)
                x = perturb(x, seed, 1.0)
                g_ref = (right - left) / (2 * 5e-4)
                assert float(g_ref) == g, (c, r, seed, float(g_ref), g)
                torch.manual_seed(seed)  # zo_utils.py:42-52, group 0's lr and weight decay 0.0
                z = torch.normal(mean=0, std=1, size=x.size(), device=x.device, dtype=x.dtype)
                p[0] = x - lr * (g_ref * z + 0.0 * x)
                hist.setdefault(seed, []).append(g)
                checked += 1
            assert torch.equal(p[0].view(torch.int16), tensor(rnd["after_steps"]).view(torch.int16)), (c, r)
            h = {int(s): v for s, v in rnd["history"].items()}
            assert {s: v for s, v in h.items() if v} == hist
    assert checked == 2 * rounds * steps


def _offline_probabilities(hists, seeds, rounds, k):
    from fate_llm.algo.fedkseed.fedkseed import FedKSeedTrainingArguments, Trainer

    class Client:
        def __init__(self, replies):
            self.replies, self.probs = list(replies), []

        def put(self, key, value):
            self.probs.append(value[1]["seed_probabilities"].tolist())

        def get(self, key):
            return self.replies.pop(0)

    class Ctx:
        def __init__(self, cl):
            self.guest, self.hosts = cl[0], cl[1:]

        def ctxs_range(self, n):
            for i in range(n):
                yield i, self

    cl = [Client([{int(s): v for s, v in h.items()} for h in hists[c]]) for c in sorted(hists)]
    Trainer(Ctx(cl), torch.tensor(seeds, dtype=torch.long), None, FedKSeedTrainingArguments(num_aggregations=rounds, k=k)).train()
    assert all(x.probs == cl[0].probs for x in cl)
    return cl[0].probs


def _bf16_value(x: float) -> float:
    """A 0-dim f32 g as the reference's bf16 update sees it: cast to the parameter dtype
    (zo_utils._value_kind), RNE."""
    return float(torch.tensor(x, dtype=torch.float32).to(torch.bfloat16).float())


def _loss64(bits: np.ndarray) -> float:
    """harness SyntheticModel.forward on the prefix: mean(p^2) * 1e3, in float64."""
    v = (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return float(np.mean(v * v) * 1e3)


def _replay_client(rec, steps_per_round, eps=5e-4, lr_reconstruct=1e-5):
    """Replay one client's rounds through the oracle (bf16, the prefix of its one flat
    tensor: a 262,144-element tensor's first 4096 z are a 4096-element tensor's); returns
    the number of local steps checked."""
    model_0 = np.array(rec["model_0"], dtype=np.uint16)
    n = 0
    for r, rnd in enumerate(rec["rounds"]):
        p = model_0.copy()  # every round restarts from model_0 (fedkseed.py:132)
        sums = rnd["sums"]
        if sums:
            keep = [(int(s), v) for s, v in sums.items() if v != 0.0]
            # ClientTrainer passes training_args' lr and weight decay (0.0) explicitly (:138-141)
            O.reconstruct([p], [O.BF16], [lr_reconstruct], [0.0], [s for s, _ in keep], [v for _, v in keep])
        got = np.array(rnd["after_reconstruct"], dtype=np.uint16)
        assert np.array_equal(got, p), f"round {r}: reconstruct differs from the oracle at {int(np.argmax(got != p))}"
        hist = {}
        assert len(rnd["steps"]) == steps_per_round
        for seed, g, lr in rnd["steps"]:
            O.perturb_params([p], [O.BF16], seed, 1.0 * eps)
            loss_right = _loss64(p)
            O.perturb_params([p], [O.BF16], seed, -2.0 * eps)
            loss_left = _loss64(p)
            O.perturb_params([p], [O.BF16], seed, 1.0 * eps)
            assert not math.isnan(g)  # the synthetic closure's losses are finite
            g64 = (loss_right - loss_left) / (2 * eps)
            # g = (L+ - L-) / (2 eps) of the very parameters the oracle holds: the GPU
            # evaluates the closure in f32, so compare within its rounding of the losses
            assert abs(g - g64) <= 2e-3 * abs(g64) + 2e-3, (r, seed, g, g64)
            # local update: the sticky group-0 lr and weight decay 0.0 (zo_utils.py:44-45);
            # the 0-dim f32 g is cast to bf16 by the reference's g * z
            O.reconstruct([p], [O.BF16], [lr], [0.0], [seed], [_bf16_value(g)])
            hist.setdefault(seed, []).append(g)
            n += 1
        got = np.array(rnd["after_steps"], dtype=np.uint16)
        assert np.array_equal(got, p), f"round {r}: local steps differ from the oracle at {int(np.argmax(got != p))}"
        h = {int(s): v for s, v in rnd["history"].items()}
        assert {s: v for s, v in h.items() if v} == hist
        assert list(h) == rnd["candidates"]
    return n
