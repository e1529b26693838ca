"""Workload for the stencil-class PMC passes (scripts/pmc_xscs.sh): A_1, A_2
and A_3 of the 256^3 7-point box hierarchy (x-staged stencil classes) in SET
mode, 10 launches each, in this order; their storage info to stdout."""
import json
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
for l in (1, 2, 3):
    M = mg.level(l)[0]
    m, n = M.dims()
    x = torch.rand(n, dtype=torch.float64, device="cuda:0")
    y = torch.empty(m, dtype=torch.float64, device="cuda:0")
    for _ in range(10):
        M.apply(y, x)
    ctx.synchronize()
    info = M.spmv_info()
    print(json.dumps({"level": l, "rows": m, "nnz": M.nnz, "info": info}, default=str), flush=True)
