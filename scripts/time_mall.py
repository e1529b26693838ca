"""Does the 256 MB MALL (Infinity Cache) carry the fine SpMV's vectors across
back-to-back launches?  The C2 fine operator's SET (DIA, constant stencil: x read,
y written, 268 MB) timed on one (x, y) pair -- what bench.py's roofline does --
against alternating between two pairs (536 MB: nothing left in the MALL from the
previous launch); the same for a 134 MB device copy."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import faer_amg_amd as fa  # noqa: E402
from bench import time_kernel  # noqa: E402

stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)
A = fa.SparseMatOp.laplace3d_7pt(ctx, 256, 256, 256)
mg = fa.sa_build_box(A, (256, 256, 256), (2, 2, 2), coarsest_dim=1000)  # the cycle's storage: constant-stencil DIA
n = A.nrows
assert A.spmv_info()["stream_bytes"] == 56, A.spmv_info()
xs = [torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(4)]
ys = [torch.empty_like(xs[0]) for _ in range(4)]
res = {}
for name, pairs in (("same_pair", [(0, 0)]), ("two_pairs", [(0, 0), (1, 1)]), ("four_pairs", [(i, i) for i in range(4)])):
    k = [0]

    def f():
        i, j = pairs[k[0] % len(pairs)]
        A.apply(ys[j], xs[i])
        k[0] += 1
    for _ in range(4):
        f()
    t = [time_kernel(f, 20, stream) for _ in range(5)]
    res["spmv_set_" + name] = round(1000 * sorted(t)[2], 2)
for name, pairs in (("same_pair", [(0, 0)]), ("two_pairs", [(0, 0), (1, 1)])):
    k = [0]

    def h():
        i, j = pairs[k[0] % len(pairs)]
        A.spmv_epilogue("resid", xs[i], ys[j], xs[(i + 2) % 4])
        k[0] += 1
    for _ in range(4):
        h()
    t = [time_kernel(h, 20, stream) for _ in range(5)]
    res["spmv_resid_" + name] = round(1000 * sorted(t)[2], 2)
for name, m in (("same_pair", 1), ("two_pairs", 2)):
    k = [0]

    def g():
        i = k[0] % m
        ys[i].copy_(xs[i])
        k[0] += 1
    for _ in range(4):
        g()
    t = [time_kernel(g, 20, stream) for _ in range(5)]
    res["copy_134MB_" + name] = round(1000 * sorted(t)[2], 2)
print(json.dumps({"us_per_launch": res}))
