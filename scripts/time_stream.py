"""Streaming reference rates on one MI355X: torch copy (read + write), fill (write),
sum (read) and a 3-stream axpby-like op on 16M fp64 (the C2 fine vector, 134 MB), each
the median of 5 rounds of 20 launches -- the bandwidth a 2- or 3-stream SpMV epilogue
can hope for."""
import json

import torch

n = 256 ** 3
x = torch.rand(n, dtype=torch.float64, device="cuda")
y = torch.rand(n, dtype=torch.float64, device="cuda")
z = torch.empty_like(x)


def t(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    r = []
    for _ in range(5):
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        e1.synchronize()
        r.append(e0.elapsed_time(e1) / it)
    r.sort()
    return r[2]


res = {}
for name, fn, byts in (("copy", lambda: z.copy_(x), 16 * n), ("fill", lambda: z.fill_(1.0), 8 * n),
                       ("sum", lambda: x.sum(), 8 * n), ("add3", lambda: torch.add(x, y, out=z), 24 * n)):
    ms = t(fn)
    res[name] = {"us": round(ms * 1e3, 2), "TBs": round(byts / (ms * 1e-3) / 1e12, 3)}
print(json.dumps(res))
