"""Workload for an SQ-counter rocprofv3 pass: the fine transfer operators and
A_1 of the 256^3 hierarchy in SET mode (10 launches each, in this order: P_0,
R_0, A_1, the fine DIA operator)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

ctx = fa.Context(0)
dims = (256,) * 3
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
_, _, R0, P0 = mg.level(0)
A1 = mg.level(1)[0]
for name, M in (("P0", P0), ("R0", R0), ("A1", A1), ("A0", A)):
    m, n = M.dims()
    x = torch.rand(n, dtype=torch.float64, device="cuda:0")
    y = torch.empty(m, dtype=torch.float64, device="cuda:0")
    for _ in range(10):
        M.apply(y, x)
    ctx.synchronize()
    print(name, M.spmv_info()["kernel"], flush=True)
