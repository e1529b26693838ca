"""Does the placement of a matrix in HBM change SpMV speed?  The same 256^3
7-pt operator is built several times with unrelated allocations in between, and
every (matrix copy, output vector) pair is timed in interleaved rounds (one
process, one device).  Plain streaming reads of same-sized buffers do not vary
(scripts/placement_stream.py), so a per-pair pattern points at conflicts
between the matrix stream and the y writes."""
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
ops, pads, ys = [], [], []
for k in range(4):
    ops.append(fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N))
    pads.append(torch.empty((k + 1) * 37 * 1024 * 1024 + 12345, dtype=torch.uint8, device="cuda:0"))
    ys.append(torch.empty(n, dtype=torch.float64, device="cuda:0"))
x = torch.rand(n, dtype=torch.float64, device="cuda:0")


def t(op, y, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    op.apply(y, x)
    e0.record(stream)
    for _ in range(it):
        op.apply(y, x)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


res = {}
for r in range(3):
    for i, op in enumerate(ops):
        for j, y in enumerate(ys):
            res.setdefault((i, j), []).append(t(op, y))
print("median us: rows = matrix copy, columns = y buffer " + " ".join(f"{y.data_ptr():#x}" for y in ys))
for i in range(len(ops)):
    print(f"A{i}: " + "  ".join(f"{sorted(res[(i, j)])[1]:7.1f}" for j in range(len(ys))))
