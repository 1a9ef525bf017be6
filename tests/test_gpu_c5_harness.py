"""C5 round harness (harness/c5_round.py) on one GPU: client processes and the
aggregator process exchange the drop-in Trainer / ClientTrainer payloads over gloo.

* one client, two rounds: round 1 has nothing to reconstruct, round 2 replays exactly
  the seeds the first round's local steps touched (non-zero cumulative sums), as the
  reference's train_once does;
* eight clients sharing the GPU, the full ClientTrainer.train loop with the local steps
  through KSeedZOExtendedTrainer.training_step in the transformers loop, payloads in the
  compact wire format: what every client received each round equals what the drop-in
  arbiter computes offline from the same client histories (fedkseed.py:41-85), and the
  histories travel as a few hundred bytes."""
import pytest
import torch

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
                         "--clients", "8", "--driver", "trainer", "--wire", "--placement", "pinned"])
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
