import torch, time, json
dev = torch.device("cuda", 0)
n = 6738415616
x = torch.empty(n, dtype=torch.bfloat16, device=dev).normal_()
y = torch.empty(n, dtype=torch.uint8, device=dev).random_(0, 255)
def t(f, reps=5):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3
ms = t(lambda: x.mul_(1.0001))
print(json.dumps({"op": "bf16 x.mul_ (read+write 2 B each)", "ms": round(ms, 3), "TBps": round(4 * n / ms / 1e9, 3)}))
xv = x.view(torch.int16)
ms = t(lambda: torch.add(xv, y, out=xv))
print(json.dumps({"op": "int16 x += uint8 y (2+1 read, 2 write)", "ms": round(ms, 3), "TBps": round(5 * n / ms / 1e9, 3)}))
