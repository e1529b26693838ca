"""A/B of the x-staged SELL kernels (xsell.hip) on roofline.general's operator
(random 7-pt 256^3, rows shuffled within windows of 4096): per epilogue the
median of 5 alternating rounds of 20 launches each for xs_pipe = 0 / 1 / 2, the
results of the two kernels compared bitwise.
  python scripts/time_xs.py [WINDOW]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import faer_amg_amd as fa  # noqa: E402
from bench import time_kernel, spmv_bytes  # noqa: E402

window = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
stream = torch.cuda.Stream()  # a real stream (Context treats the null stream as 'make your own')
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)  # the library launches on the stream the events time
M = fa.SparseMatOp.random7(ctx, 256, 256, 256, seed=42, window=window)
n = M.nrows
info = M.spmv_info()
g = torch.Generator(device="cuda").manual_seed(3)
x = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
b = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
d = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
y = torch.empty_like(x)
moved = info["stream_bytes"] + 16 * n
csr_b = spmv_bytes(n, n, M.nnz)
res = {"kernel": info["kernel"], "window": window, "moved_bytes": moved, "csr_bytes": csr_b}
for mode in ("set", "resid", "jacobi"):
    t = {0: [], 1: [], 2: []}
    outs = {}
    for _ in range(5):
        for pipe in (0, 1, 2):
            fa.set_flag("xs_pipe", pipe)
            fn = lambda: M.spmv_epilogue(mode, x, y, b, d)  # noqa: E731
            for _ in range(3):
                fn()
            t[pipe].append(time_kernel(fn, 20, stream))
            outs[pipe] = y.clone()
    same = bool(torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]))
    mb = moved + (8 * n if mode == "resid" else 24 * n if mode == "jacobi" else 0)
    res[mode] = {f"pipe{p}": {"ms": round(float(np.median(t[p])), 5),
                              "frac_moved": round(mb / (np.median(t[p]) * 1e-3) / 8e12, 4)} for p in (0, 1, 2)}
    res[mode]["bitwise_equal"] = same
fa.set_flag("xs_pipe", 2)
print(json.dumps(res), flush=True)
