"""A/B of the SpMV kernels on every operator of the 256^3 SA hierarchy (and the
storage the cycle runs, "cycle").

For each level l >= 1 (and the fine P/R), the operator is re-uploaded under each
storage policy (csr-stream / vector / sell) and y = M x is timed with HIP
events in interleaved rounds in one process.  Prints GB/s (algorithmic bytes,
32-bit index formula) per operator and policy.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

EDGE = int(os.environ.get("AB_EDGE", "256"))
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = fa.Context(0, stream=stream.cuda_stream)
dims = (EDGE,) * 3
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)


def timeit(op, x, y, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    op.apply(y, x)
    e0.record(stream)
    for _ in range(iters):
        op.apply(y, x)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for l in range(mg.levels() - 1):
    Al, _, Rl, Pl = mg.level(l)
    for name, M in (("A", Al), ("R", Rl), ("P", Pl)):
        if l == 0 and name == "A":
            continue
        m, n = M.dims()
        arrs = M.arrays()
        nnz = M.nnz
        ops = {}
        for fmt in ("csr", "vector", "sell"):
            fa.set_spmv_format(fmt)
            ops[fmt] = fa.SparseMatOp.from_arrays(ctx, m, n, *arrs)
        fa.set_spmv_format("auto")
        ops["auto"] = fa.SparseMatOp.from_arrays(ctx, m, n, *arrs)
        ops["cycle"] = M  # the storage the cycle runs (grid classes / transfer classes)
        x = torch.rand(n, dtype=torch.float64, device="cuda:0")
        y = torch.empty(m, dtype=torch.float64, device="cuda:0")
        res = {k: [] for k in ops}
        for _ in range(5):
            for k, op in ops.items():
                res[k].append(timeit(op, x, y))
        byts = 12 * nnz + 4 * (m + 1) + 8 * n + 8 * m
        line = f"L{l} {name} {m}x{n} nnz/row {nnz / max(m, 1):7.1f} [{M.spmv_info()['kernel']}]: "
        line += "  ".join(f"{k} {min(v) * 1e3:8.1f}us {byts / (min(v) * 1e-3) / 1e9:6.0f}GB/s"
                          for k, v in res.items())
        print(line, flush=True)
        del ops
