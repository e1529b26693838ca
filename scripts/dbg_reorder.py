"""Debug aid for the locality reordering: per level sizes, storage, whether it
is renumbered, and the cycle plans with reordering off / forced / auto."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import torch  # noqa: E402

import faer_amg_amd as fa  # noqa: E402

e = int(sys.argv[1]) if len(sys.argv) > 1 else 30
ctx = fa.Context(0)
H = fa.elasticity_q1((e, e, e), seed=3, permute=True if len(sys.argv) < 3 else int(sys.argv[2]))
A = H.upload(ctx)
n = A.nrows
nn = fa.constant_candidates(n, 3)
S = H.to_scipy()
w = [1.0 / float(nn[:, c] @ (S @ nn[:, c])) for c in range(nn.shape[1])]
mg = fa.smoothed_aggregation(A, nn, weights=w, block_size=3, candidate_dimension=3, coarsest_dim=150, smoother="l1")
b = torch.as_tensor(np.random.default_rng(31).uniform(-1, 1, n), device="cuda:0")
out = {}
for mode in (0, 2, 1):
    mg.set_reorder(mode)
    z = torch.empty_like(b)
    mg.apply(z, b)
    ctx.synchronize()
    out[mode] = {"z": z.cpu().numpy(), "reordered": [mg.reordered(l) for l in range(mg.levels())],
                 "plan": [f"{p['level']}:{p['role']}:{p['name']}:{p['mode']}" for p in mg.cycle_plan()]}
info = {"levels": [(mg.level(l)[0].nrows,) + tuple(o.spmv_info()["kernel"] if o is not None else None
                                                  for o in (mg.level(l)[0], mg.level(l)[2], mg.level(l)[3]))
                   for l in range(mg.levels())]}
for mode in (0, 2, 1):
    info[f"mode{mode}"] = {"reordered": out[mode]["reordered"], "plan": out[mode]["plan"],
                           "z_equal_to_mode0": bool(np.array_equal(out[mode]["z"], out[0]["z"])),
                           "z_maxrel": float(np.max(np.abs(out[mode]["z"] - out[0]["z"])) / np.max(np.abs(out[0]["z"])))}
print(json.dumps(info, indent=1))
