"""Workload for rocprofv3 PMC passes on the C5 stand-in's fine-level SpMV (3x3
block storage, spmv_bsr3_kernel).

  CAL: y = B x with B block-diagonal (one dense 3x3 block per node, n = 3 * 80^3
       * ... rows matching the stand-in): through the same 3x3-block kernel, its
       traffic is exactly the format bytes + 8 n read + 8 n written -- calibrates
       FETCH_SIZE for this kernel's access widths;
  FINE: y = A x, the Q1 elasticity stand-in (80^3 elements, node numbering
       shuffled within windows of 4096 nodes: bench.py --problem elast).
CAL runs ITERS launches first, then FINE ITERS; the summariser splits by order
(scripts/pmc_summary.py ... --kernel spmv_bsr3_kernel).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

ITERS = 10
ctx = fa.Context(0)
A = fa.elasticity_q1((80, 80, 80), contrast=1.0, nu=0.3, seed=42, permute=4096).upload(ctx)
n = A.nrows
nodes = n // 3
rp = np.arange(0, 9 * nodes + 1, 3, dtype=np.int64)
ci = np.repeat(np.arange(n, dtype=np.int64).reshape(nodes, 3), 3, axis=0).reshape(-1)
va = np.random.default_rng(1).uniform(0.5, 1.5, 9 * nodes)  # > 65536 distinct values: no value codes
B = fa.SparseMatOp.from_arrays(ctx, n, n, rp, ci, va)
assert B.spmv_info()["kernel"] == "bsr" and A.spmv_info()["kernel"] == "bsr", (B.spmv_info(), A.spmv_info())
x = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, n), device="cuda:0")
y = torch.empty_like(x)
for _ in range(ITERS):
    B.apply(y, x)
ctx.synchronize()
for _ in range(ITERS):
    A.apply(y, x)
ctx.synchronize()
info = {"cal": B.spmv_info(), "fine": A.spmv_info(), "n": n, "kernel": "spmv_bsr3_kernel",
        "workload": "Q1 elasticity 80^3 elements, block size 3 (C5 stand-in), y = A x"}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(info, open(os.path.join(ROOT, "gpurun_out", "pmc_known_bsr.json"), "w"), indent=1)
print(f"done: n={n} nnz(A)={A.nnz} storage={info}")
