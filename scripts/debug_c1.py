"""Diagnostic: C1 two-grid V-cycle under each SpMV storage policy vs the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "faer-amg_amd"), os.path.join(ROOT, "oracle")]
import faer_amg_amd as fa  # noqa: E402
import oracle as O  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "g2_gmg2d_c1.npz"))
ctx = fa.Context(0)
for fmt in ("csr", "sell", "auto"):
    fa.set_spmv_format(fmt)
    ops = {}
    for key in ("A0", "R0", "P0", "A1"):
        m, n = g[f"{key}_shape"]
        ops[key] = fa.SparseMatOp.from_arrays(ctx, m, n, g[f"{key}_rowptr"], g[f"{key}_col"], g[f"{key}_val"])
        om = O.Csr.from_arrays(m, n, g[f"{key}_rowptr"], g[f"{key}_col"], g[f"{key}_val"])
        x = np.random.default_rng(0).standard_normal(n)
        y = np.zeros(m)
        ops[key].apply(y, x)
        print(fmt, key, "spmv max abs err", np.max(np.abs(y - om.spmv(x))))
    for graph in (False, True):
        mg = fa.Multigrid(ops["A0"], fa.new_jacobi(ops["A0"], 0.66))
        mg.add_level(ops["A1"], fa.CoarseCholesky(ops["A1"]), ops["R0"], ops["P0"])
        mg.set_graph(graph)
        b = torch.ones(ops["A0"].nrows, dtype=torch.float64, device="cuda:0")
        z = torch.empty_like(b)
        mg.apply(z, b)
        ctx.synchronize()
        zz = z.cpu().numpy()
        print(fmt, "graph", graph, "vcycle rel err", np.linalg.norm(zz - g["z"]) / np.linalg.norm(g["z"]))
    fa.set_spmv_format("auto")
