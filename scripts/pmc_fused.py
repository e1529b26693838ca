"""Workload for counter passes over the fused fine-level kernels (fine.hip):
the C2 hierarchy (7-pt 256^3), then 10 launches of k_fine_resid_restrict and
10 of k_fine_interp_jacobi exactly as the cycle makes them
(amg_multigrid_fine_launch), between k_trace_mark<<<1>>> and <<<2>>>."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

ctx = fa.Context(0)
N = 256
A = fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N)
mg = fa.sa_build_box(A, (N, N, N), (2, 2, 2), coarsest_dim=1000)
b = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, N ** 3), device="cuda:0")
z = torch.empty_like(b)
mg.apply(z, b)
ctx.synchronize()
ctx.trace_mark(1)
for which in (0, 1):
    for _ in range(10):
        assert mg.fine_launch(which, z, b)
ctx.synchronize()
ctx.trace_mark(2)
print("done", flush=True)
