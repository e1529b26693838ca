"""PMC workload: HBM traffic of the C5 stand-in's fine 3x3-block SpMV as the cycle
runs it (the locality-renumbered copy, amg_multigrid_get_run_level).  The SA
hierarchy is built first (its setup SpMVs precede everything counted), then
CAL: y = B x with B block-diagonal (one 3x3 block per node: its traffic is the
format bytes + 8 n read + 8 n written, the FETCH_SIZE calibration for this
kernel's access widths), ITERS launches; then FINE: y = A_0' x, ITERS launches.
Writes the known byte counts to gpurun_out/pmc_bsr_renum_known.json."""
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
A = fa.elasticity_q1((80, 80, 80), seed=42, permute=4096).upload(ctx)
n = A.nrows
nn = fa.constant_candidates(n, 3)
mg = fa.smoothed_aggregation(A, nn, block_size=3, candidate_dimension=3, coarsest_dim=1000, smoother="l1")
assert mg.reordered(0)
Ar = mg.run_level(0)[0]
nodes = n // 3
rp = np.arange(0, 9 * nodes + 1, 3, dtype=np.int64)
ci = np.repeat(np.arange(n, dtype=np.int64).reshape(nodes, 3), 3, axis=0).reshape(-1)
va = np.random.default_rng(1).uniform(0.5, 1.5, 9 * nodes)
B = fa.SparseMatOp.from_arrays(ctx, n, n, rp, ci, va)
assert B.spmv_info()["kernel"] == "bsr" and Ar.spmv_info()["kernel"] == "bsr"
x = torch.as_tensor(np.random.default_rng(0).uniform(-1, 1, n), device="cuda:0")
y = torch.empty_like(x)
ctx.synchronize()
for _ in range(ITERS):
    B.apply(y, x)
ctx.synchronize()
for _ in range(ITERS):
    Ar.apply(y, x)
ctx.synchronize()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"n": n, "iters": ITERS, "cal_alg": B.spmv_info()["stream_bytes"] + 16 * n,
           "fine_alg": Ar.spmv_info()["stream_bytes"] + 16 * n},
          open(os.path.join(ROOT, "gpurun_out", "pmc_bsr_renum_known.json"), "w"))
print("ok", n)
