"""C4 at its real size (BASELINE.json configs[3]): the 70B fp32 K=4096 reconstruct that
tools/c4_70b.py --verify ran on an MI355X (723 tensors, 275.9 GB resident, 8 chunks)
recorded the first 4096 elements of embed_tokens before and after the whole run; this
CPU test replays those elements through the oracle over all 4055 non-zero seeds
(zo_utils.py:47-49 with the explicit lr / weight decay of fedkseed.py:138-141) and
requires the device's result bit for bit.  The same run's chunk-boundary check (one
call against the two calls of the timed run) is in the log beside the record
(profiles/r05_c4_70b_fp32_k4096.log)."""
import glob
import os

import numpy as np
import pytest

from oracle import fks_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _records():
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*_c4_verify.npz")))


@pytest.mark.parametrize("path", _records() or [None])
def test_c4_fullsize_embed_prefix_matches_oracle(path):
    if path is None:
        pytest.skip("no C4 full-size record under profiles/")
    with np.load(path, allow_pickle=False) as z:
        rec = {k: z[k] for k in z.files}
    assert rec["params"] == 68_976_648_192 and rec["seeds"].size == 4055
    p = rec["embed_before"].astype(np.float32).copy()
    O.reconstruct([p], [O.F32], [float(rec["lr"])], [float(rec["weight_decay"])],
                  rec["seeds"].tolist(), rec["scalars"].tolist())
    assert np.array_equal(p.view(np.uint32), rec["embed_after"].view(np.uint32))
    assert not np.array_equal(rec["embed_before"], rec["embed_after"])
