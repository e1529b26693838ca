"""Diagnostic: BlockSmoother apply vs its into_sparse_mat SpMV."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import faer_amg_amd as fa  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import _box_partition  # noqa: E402

ctx = fa.Context(0)
OA = O.laplace3d_7pt(12, 10, 8)
A = fa.SparseMatOp.from_arrays(ctx, *OA.dims()[:2], *OA.arrays())
part = _box_partition((12, 10, 8), (2, 2, 2))
B = fa.BlockSmoother(A, part)
S = B.to_sparse()
print("spmv_info", S.spmv_info())
r = np.random.default_rng(41).standard_normal(OA.nrows)
rd = torch.as_tensor(r, device="cuda:0")
z1, z2 = torch.empty_like(rd), torch.empty_like(rd)
B.apply(z1, rd)
S.apply(z2, rd)
ctx.synchronize()
a, b = z1.cpu().numpy(), z2.cpu().numpy()
d = np.flatnonzero(a != b)
print("differ", len(d), "max", np.abs(a - b).max(), "rows", d[:20])
rp, ci, va = S.arrays()
i = d[0] if len(d) else 0
print("row", i, "cols", ci[rp[i]:rp[i + 1]], "vals", va[rp[i]:rp[i + 1]])
acc = 0.0
for c, v in zip(ci[rp[i]:rp[i + 1]], va[rp[i]:rp[i + 1]]):
    acc = float(np.fma(v, r[c], acc)) if hasattr(np, "fma") else acc + v * r[c]
print("host seq", acc, "block", a[i], "spmv", b[i])
