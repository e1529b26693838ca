"""Does the placement of a matrix in HBM change SpMV speed?  The same 256^3
7-pt operator is built several times with unrelated allocations in between and
all copies are timed in interleaved rounds (one process, one device), once per
device allocation policy (plain hipMalloc vs physically contiguous)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)
N = 256
n = N ** 3
ops, pads = [], []
for k in range(8):
    fa.set_alloc_policy(k % 2 == 1)
    ops.append(fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N))
    pads.append(torch.empty((k + 1) * 37 * 1024 * 1024 + 12345, dtype=torch.uint8, device="cuda:0"))
fa.set_alloc_policy(True)
xs = [torch.rand(n, dtype=torch.float64, device="cuda:0") for _ in range(2)]
y = torch.empty(n, dtype=torch.float64, device="cuda:0")


def t(op, x, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    op.apply(y, x)
    e0.record(stream)
    for _ in range(it):
        op.apply(y, x)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


res = {}
for r in range(5):
    for i, op in enumerate(ops):
        for j, x in enumerate(xs):
            res.setdefault((i, j), []).append(t(op, x))
for k, v in sorted(res.items()):
    pol = "contiguous" if k[0] % 2 else "hipMalloc "
    print(f"matrix copy {k[0]} ({pol}) x{k[1]}: min {min(v):7.1f} us  median {sorted(v)[2]:7.1f} us")
