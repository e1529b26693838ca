"""A/B of the x-staged stencil-class tiles on the coarse operators of the C2
(7-pt 256^3) and C3 (27-pt 256^3) box hierarchies: microseconds per RESID and
JACOBI epilogue launch for each tile (FAMG_XSCS_TILE) against the
cache-gathering stencil-class / previous storage (grid hint cleared)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

ctx = fa.Context(0)
prob = os.environ.get("PROB", "7pt")
dims = (256, 256, 256)
A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims) if prob == "7pt" else fa.SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)


def time_level(M, reps=100):
    n = M.nrows
    rng = np.random.default_rng(0)
    x = torch.as_tensor(rng.standard_normal(n), device="cuda:0")
    b = torch.as_tensor(rng.standard_normal(n), device="cuda:0")
    d = torch.as_tensor(rng.uniform(0.1, 1, n), device="cuda:0")
    y = torch.empty_like(x)
    res = {}
    for mode in ("resid", "jacobi"):
        for _ in range(3):
            M.spmv_epilogue(mode, x, y, b, d)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            M.spmv_epilogue(mode, x, y, b, d)
        ctx.synchronize()
        res[mode] = (time.perf_counter() - t0) * 1e6 / reps  # back-to-back launches: kernel-bound
    return res


for l in range(1, mg.levels() - 1):
    M = mg.level(l)[0]
    g = tuple(-(-v // 2 ** l) for v in dims)
    info = M.spmv_info()
    print(f"level {l} grid {g} rows {M.nrows} storage {info['kernel']} xstaged {info['xstaged']} "
          f"tile {info.get('tile')}", flush=True)
    if not info["xstaged"]:
        continue
    t = time_level(M)
    print(f"   auto tile {info.get('tile')}: resid {t['resid']:.1f} us, jacobi {t['jacobi']:.1f} us", flush=True)
    for tile in ("4,4,4", "8,4,4", "8,8,2", "8,8,4", "16,8,2", "16,4,4", "16,16,1", "32,8,1", "8,8,8", "16,8,4"):
        os.environ["FAMG_XSCS_TILE"] = tile
        M.set_grid(*g)
        i2 = M.spmv_info()
        if not i2["xstaged"]:
            continue
        t = time_level(M)
        print(f"   tile {i2['tile']}: resid {t['resid']:.1f} us, jacobi {t['jacobi']:.1f} us", flush=True)
    os.environ.pop("FAMG_XSCS_TILE")
    M.set_grid(0, 0, 0)
    t = time_level(M)
    print(f"   no grid ({M.spmv_info()['kernel']}): resid {t['resid']:.1f} us, jacobi {t['jacobi']:.1f} us",
          flush=True)
