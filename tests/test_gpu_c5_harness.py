"""C5 round harness (harness/c5_round.py) on one GPU: one client process and the
aggregator process exchange the drop-in Trainer / ClientTrainer payloads over gloo;
round 1 has nothing to reconstruct, round 2 replays exactly the seeds the first round's
local steps touched (non-zero cumulative sums), as the reference's train_once does."""
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
