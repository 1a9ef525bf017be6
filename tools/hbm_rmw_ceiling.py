"""In-place read-modify-write ceiling of HBM on the 7B bf16 buffer (13.48 GB): torch's own
vectorized elementwise kernel, x.mul_(s), timed with HIP events -- the bandwidth a one-seed
pass (read p, write p) could reach if its compute were free.
python tools/hbm_rmw_ceiling.py"""
import json

import torch


def main():
    n = 6_738_415_616
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_(0, 0.02)
    for _ in range(2):
        x.mul_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        x.mul_(1.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"op": "bf16 x.mul_(1.0), in place", "elements": n, "ms": round(ms, 3),
                      "TBps_read_plus_write": round(2 * 2 * n / ms / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
