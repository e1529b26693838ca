"""Distributed stationary solve residual history vs the single-GPU one (loopback
ranks on one GPU): rho_0 must be exactly 1 and the histories agree to 1e-8."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

fa.set_flag("dense_tail", 0)


def run(dims, nranks, agglo, overlap=True):
    ctx = fa.Context(0)
    A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
    n = A.nrows
    b = torch.as_tensor(np.random.default_rng(1).uniform(-1, 1, n), device="cuda:0")
    z = torch.empty_like(b)
    mg.apply(z, b)
    x = torch.zeros_like(b)
    _, hs = fa.stationary_solve(A, mg, b, x, max_iter=4, rel_tol=1e-300)
    nl = mg.levels()
    splits = fa.slab_splits(fa.box_level_dims(dims, (2, 2, 2), nl), nranks)
    hub = fa.LoopbackHub(nranks)
    out = [None] * nranks

    def body(r):
        comm = fa.Comm(ctx, hub=hub, rank=r)
        dm = fa.DistMultigrid(comm, mg, splits, agglomerate_rows=agglo).set_overlap(overlap)
        r0, r1 = dm.local_rows()
        bl = b[r0:r1]
        xl = torch.zeros_like(bl)
        _, h = dm.stationary_solve(bl, xl, max_iter=4, rel_tol=1e-300)
        out[r] = (h, dm.level_matrix(0, "A").spmv_info()["kernel"] if dm.level_info(0)["redundant"] == 0 else "-")
    th = [threading.Thread(target=body, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    hd, kern = out[0]
    print(f"{dims} ranks {nranks} agglo {agglo} overlap {overlap} fine {kern}: rho0 dist {hd[0]!r} "
          f"max rel diff {np.max(np.abs(hd - hs) / hs):.3e}", flush=True)


for dims, nr, ag in (((16, 12, 24), 2, 1000), ((64, 64, 64), 2, 16384 * 2), ((128, 128, 128), 4, 16384 * 4),
                     ((256, 256, 256), 8, 16384 * 8)):
    run(dims, nr, ag)
    run(dims, nr, ag, overlap=False)
