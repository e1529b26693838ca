"""Workload for rocprofv3 PMC passes on roofline.general (scripts/pmc_general_summary.py).

  python scripts/pmc_general.py xsell|sell

Runs, on one GPU, ITERS launches each of
  * CAL: y = D x, D = a permutation matrix that shuffles rows within windows of
    4096 (the general operator's numbering) with random values in [1, 2) (fp64
    values, as the general operator's): one entry per row with a
    gathered column, so the storage (x-staged SELL / SELL-64 with u16 columns)
    is the one the general operator gets, and the traffic is known exactly
    (its stream bytes + 8n of x read once + 8n of y written) -- calibrates
    FETCH_SIZE for this kernel's access widths;
  * GEN: y = A x, A = the roofline.general operator (random 7-pt 256^3, window 4096).
'xsell' builds both in the auto policy (x-staged SELL), 'sell' under the SELL
policy (SELL-64).  CAL runs first; the summariser splits the dispatches by order.
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
which = sys.argv[1] if len(sys.argv) > 1 else "xsell"
ctx = fa.Context(0)
n = N ** 3
rng = np.random.default_rng(0)
perm = (rng.permuted(np.tile(np.arange(4096, dtype=np.int64), (n // 4096, 1)), axis=1)
        + (np.arange(n // 4096, dtype=np.int64) * 4096)[:, None]).ravel()
if which == "sell":
    fa.set_spmv_format("sell")
try:
    dv = rng.uniform(1.0, 2.0, n)
    D = fa.SparseMatOp.from_arrays(ctx, n, n, np.arange(n + 1, dtype=np.int64), perm, dv)
    A = fa.SparseMatOp.random7(ctx, N, N, N, seed=42, window=4096)
finally:
    fa.set_spmv_format("auto")
x = torch.as_tensor(rng.uniform(-1, 1, n), device="cuda:0")
y = torch.empty_like(x)
torch.cuda.synchronize()
for _ in range(ITERS):
    D.apply(y, x)
ctx.synchronize()
assert torch.equal(y, torch.as_tensor(dv, device="cuda:0") * x[torch.as_tensor(perm, device="cuda:0")])
for _ in range(ITERS):
    A.apply(y, x)
ctx.synchronize()
info = {"cal": D.spmv_info(), "gen": A.spmv_info(), "n": n, "nnz": A.nnz, "which": which}
assert info["cal"]["kernel"] == info["gen"]["kernel"], info
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(info, open(os.path.join(ROOT, "gpurun_out", f"pmc_general_known_{which}.json"), "w"), indent=1)
print(f"done: {info}")
