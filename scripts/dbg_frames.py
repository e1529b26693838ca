"""Per-matrix check of the rank-local slab-frame storages (debug aid): for 2
loopback ranks on a small 7-pt hierarchy, apply every local A_l / R_l / P_l to
x = [owned | ghost planes] of a global vector and compare with the global
operator's rows."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "faer-amg_amd"))
import faer_amg_amd as fa  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32, 32, 64)))
nr = 2
hub = fa.LoopbackHub(nr)
out = [None] * nr


def rank(r):
    ctx = fa.Context(0)
    A = fa.SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa.sa_build_box(A, dims, (2, 2, 2), coarsest_dim=60)
    nl = mg.levels()
    ldims = fa.box_level_dims(dims, (2, 2, 2), nl)
    splits = fa.slab_splits(ldims, nr)
    comm = fa.Comm(ctx, hub=hub, rank=r)
    dm = fa.DistMultigrid(comm, mg, splits, agglomerate_rows=200)
    infos = [dm.level_info(l) for l in range(nl)]
    La = sum(1 for i in infos if i["redundant"] == 0)
    rep = []
    rng = np.random.default_rng(1)
    xs = [rng.standard_normal(mg.level(l)[0].nrows) for l in range(nl)]

    def local_vec(l):
        nx, ny, nz = ldims[l]
        pl = nx * ny
        s0, s1 = splits[l][r], splits[l][r + 1]
        ng = infos[l]["n_ghost"]
        gl = (ng // pl) if r == 1 else 0
        gh = (ng // pl) - gl
        v = np.concatenate([xs[l][s0:s1], xs[l][s0 - gl * pl:s0], xs[l][s1:s1 + gh * pl]])
        return v, s0, s1

    for l in range(La):
        Ag, _, Rg, Pg = mg.level(l)
        for w, G in (("A", Ag), ("R", Rg), ("P", Pg)):
            M = dm.level_matrix(l, w)
            info = M.spmv_info()
            m, n = M.dims()
            if w == "A":
                xl, s0, s1 = local_vec(l)
                rows = (s0, s1)
                xg = xs[l]
            elif w == "R":
                xl, _, _ = local_vec(l)
                if l + 1 < La:
                    rows = (splits[l + 1][r], splits[l + 1][r + 1])
                else:
                    rows = (splits[l + 1][r], splits[l + 1][r + 1])
                xg = xs[l]
            else:
                if l + 1 < La:
                    xl, _, _ = local_vec(l + 1)
                else:
                    xl = xs[l + 1]
                rows = (splits[l][r], splits[l][r + 1])
                xg = xs[l + 1]
            if len(xl) != n:
                rep.append((l, w, "len mismatch", len(xl), n, info["kernel"], info["gtc"]))
                continue
            yl = torch.empty(m, dtype=torch.float64, device="cuda:0")
            M.apply(yl, torch.as_tensor(xl, device="cuda:0"))
            yg = torch.empty(G.nrows, dtype=torch.float64, device="cuda:0")
            G.apply(yg, torch.as_tensor(xg, device="cuda:0"))
            ctx.synchronize()
            d = np.abs(yl.cpu().numpy() - yg.cpu().numpy()[rows[0]:rows[1]])
            bad = np.nonzero(d > 1e-12 * (1 + np.abs(yg.cpu().numpy()).max()))[0]
            rep.append((l, w, info["kernel"], info["xstaged"], info["gtc"], len(bad),
                        int(bad[0]) if len(bad) else -1, float(d.max()) if len(d) else 0.0, m))
    out[r] = rep


th = [threading.Thread(target=rank, args=(r,)) for r in range(nr)]
for t in th:
    t.start()
for t in th:
    t.join()
for r in range(nr):
    for x in out[r]:
        print(r, x)
