"""Workload for rocprofv3 PMC passes on the fine-level SpMV.

Runs, on one GPU:
  * CAL: y = D x with D a diagonal 16.7M x 16.7M matrix through the same SELL-64
    kernel (one implicit-column step per slice): exactly known traffic per
    launch (the matrix bytes the format streams + 8n x read, 8n y written) --
    calibrates FETCH_SIZE/WRITE_SIZE for this kernel's access widths (the
    guide: only 16-B/lane streams are calibrated, FETCH_SIZE = half the bytes).
  * FINE: y = A_0 x, the 256^3 7-point operator (SELL-64).
The two are told apart in the trace by grid size (CAL 65536 blocks of 256
threads for 262144 slices; FINE the same slice count -- so CAL runs first,
ITERS launches, then FINE, ITERS launches; the summariser splits by order).
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
N = 256
ctx = fa.Context(0)
n = N ** 3
rp = np.arange(n + 1, dtype=np.int64)
D = fa.SparseMatOp.from_arrays(ctx, n, n, rp, np.arange(n, dtype=np.int64),
                               np.full(n, 2.0))
A = fa.SparseMatOp.laplace3d_7pt(ctx, N, N, N)
x = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, n), device="cuda:0")
y = torch.empty_like(x)
torch.cuda.synchronize()
for _ in range(ITERS):
    D.apply(y, x)
ctx.synchronize()
assert torch.equal(y, 2.0 * x)
for _ in range(ITERS):
    A.apply(y, x)
ctx.synchronize()
info = {"cal": D.spmv_info(), "fine": A.spmv_info(), "n": n}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(info, open(os.path.join(ROOT, "gpurun_out", "pmc_known.json"), "w"), indent=1)
print(f"done: n={n} nnz(A)={A.nnz} storage={info}")
