"""Diagnostic (GPU): which torch_rocm reconstruct configurations differ from the reference's
torch ops on the device -- one dtype per call, weight decay +0 / -0 / 0.01 / None, scalars
with and without +-1e-45, with and without edge parameters.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fate-llm_amd", "python"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import torch_replica as R  # noqa: E402
from fate_llm.algo.fedkseed import codec  # noqa: E402

DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
dev = torch.device("cuda", 0)
edge = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 1e-40, -1e-42, 3e38, -3e38,
                     1e-3, -2.5e-2, 65000.0, 1.0, -1.0, 1e-8, 7e-39], dtype=torch.float32)
for dt in ("float16", "bfloat16", "float32"):
    for wd in (0.0, -0.0, 0.01, None):
        for tiny in (False, True):
            for with_edge in (False, True):
                g = torch.Generator().manual_seed(14)
                x = torch.randn(5647, generator=g) * 0.02
                if with_edge:
                    x[:16] = edge
                    x[1000:1016] = edge
                base = x.to(DT[dt]).to(dev)
                g = torch.Generator().manual_seed(3)
                seeds = torch.randint(0, 2**32, (35,), generator=g).tolist()
                vals = (torch.randn(35, generator=g, dtype=torch.float64) * 20.0).tolist()
                vals[4] = -vals[4]
                if tiny:
                    vals[9], vals[10] = 1e-45, -1e-45
                ref = [base.clone()]
                R.reconstruct(ref, seeds, vals, 1e-5, wd)
                got = base.clone()
                codec.directional_step([codec.ParamSpec(got, lr=1e-5, weight_decay=wd)], seeds, vals, stream_mode="torch_rocm")
                torch.cuda.synchronize()
                a, b = got.float(), ref[0].float()
                an, bn = torch.isnan(a), torch.isnan(b)
                bits = (lambda t: t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32))
                diff = (bits(got) != bits(ref[0])) & ~(an & bn)
                idx = diff.nonzero().flatten().tolist()[:5]
                print(json.dumps({"dtype": dt, "wd": None if wd is None else repr(wd), "tiny": tiny, "edge": with_edge,
                                  "differ": int(diff.sum()), "first": idx,
                                  "got": [got[i].item() for i in idx], "want": [ref[0][i].item() for i in idx],
                                  "init": [base[i].item() for i in idx]}), flush=True)
