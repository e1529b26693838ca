"""CPU coverage of the N > 1 path (world_size 2, gloo): a numpy restatement of the
distributed V-cycle design of csrc/dist.hip -- per-level [owned | ghost] spaces
whose ghost set is the union of the columns referenced by the rank's rows of
A_l, R_l and P_{l-1}; halo requests exchanged once; one exchange per vector
refresh; levels below `agglomerate` gathered and cycled redundantly -- run over
torch.distributed (gloo) on the oracle hierarchy, compared with the global
oracle V-cycle.  Also checks the bench's weak-scaling decomposition helpers.
"""
import os
import socket
import sys

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Space:
    def __init__(self, splits, rank, ncols, mats, dist):
        self.r0, self.r1 = splits[rank], splits[rank + 1]
        self.n_own = self.r1 - self.r0
        cols = np.unique(np.concatenate([m.indices for m in mats] + [np.zeros(0, np.int64)]))
        self.ghost = cols[(cols < self.r0) | (cols >= self.r1)]
        owner = np.searchsorted(splits, self.ghost, side="right") - 1
        world = len(splits) - 1
        reqs = [self.ghost[owner == q] for q in range(world)]
        allreq = [None] * world
        dist.all_gather_object(allreq, reqs)
        # what the others want from me (global ids in my range)
        self.send = {q: allreq[q][rank] - self.r0 for q in range(world)
                     if q != rank and len(allreq[q][rank])}
        self.recv = {}
        off = 0
        for q in range(world):
            if len(reqs[q]):
                self.recv[q] = (off, len(reqs[q]))
            off += len(reqs[q])
        self.local_of = {g: self.n_own + k for k, g in enumerate(self.ghost)}

    def remap(self, M):
        M = M.tocsr().copy()
        c = M.indices.astype(np.int64)
        own = (c >= self.r0) & (c < self.r1)
        out = np.empty_like(c)
        out[own] = c[own] - self.r0
        out[~own] = [self.local_of[g] for g in c[~own]]
        return sp.csr_matrix((M.data, out, M.indptr), shape=(M.shape[0], self.n_own + len(self.ghost)))

    def halo(self, x, dist):
        import torch
        reqs = []
        for q, idx in self.send.items():
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(x[idx])), q))
        bufs = {}
        for q, (off, cnt) in self.recv.items():
            bufs[q] = torch.empty(cnt, dtype=torch.float64)
            reqs.append(dist.irecv(bufs[q], q))
        for r in reqs:
            r.wait()
        for q, (off, cnt) in self.recv.items():
            x[self.n_own + off:self.n_own + off + cnt] = bufs[q].numpy()


def worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "oracle"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import np_oracle as N
        import oracle as O

        dims = (8, 6, 16)
        A = O.laplace3d_7pt(*dims)
        levels = O.sa_hierarchy_box(A, dims, (2, 2, 2), coarsest_dim=20)
        S = [{k: lev[k].to_scipy() for k in ("A", "R", "P") if k in lev} for lev in levels]
        nl = len(levels)
        # z-slab splits of the box-coarsened grids (same helper as the bench)
        ldims = [dims]
        for _ in range(nl - 1):
            ldims.append(tuple(-(-a // 2) for a in ldims[-1]))
        splits = []
        for (nx, ny, nz) in ldims:
            splits.append(np.array([(p * nz) // world * nx * ny for p in range(world + 1)], np.int64))
        agglo = 60
        La = nl - 1
        for l in range(nl - 1):
            if S[l]["A"].shape[0] < agglo:
                La = l
                break
        loc = []
        for l in range(La):
            s0, s1 = splits[l][rank], splits[l][rank + 1]
            c0, c1 = splits[l + 1][rank], splits[l + 1][rank + 1]
            loc.append({"A": S[l]["A"][s0:s1], "P": S[l]["P"][s0:s1], "R": S[l]["R"][c0:c1],
                        "d": 0.66 / S[l]["A"].diagonal()[s0:s1]})
        spaces = []
        for l in range(La):
            mats = [loc[l]["A"], loc[l]["R"]] + ([loc[l - 1]["P"]] if l > 0 else [])
            spaces.append(Space(splits[l], rank, S[l]["A"].shape[0], mats, dist))
        for l in range(La):
            loc[l]["Al"] = spaces[l].remap(loc[l]["A"])
            loc[l]["Rl"] = spaces[l].remap(loc[l]["R"])
            if l + 1 < La:
                loc[l]["Pl"] = spaces[l + 1].remap(loc[l]["P"])
            else:
                loc[l]["Pl"] = loc[l]["P"]  # global coarse ids into the replicated vector
        tail_levels = [dict(S[l]) for l in range(La, nl)]
        for l, lev in enumerate(tail_levels):
            lev["smoother"] = "chol" if La + l == nl - 1 else "jacobi"
        tail = N.Multigrid(tail_levels)
        ts = splits[La]

        def ext(l, v):
            x = np.zeros(spaces[l].n_own + len(spaces[l].ghost))
            x[:spaces[l].n_own] = v
            spaces[l].halo(x, dist)
            return x

        def cycle(l, v, f, zero):
            L = loc[l]
            v = L["d"] * f if zero else v + L["d"] * (f - L["Al"] @ ext(l, v))
            r = f - L["Al"] @ ext(l, v)
            if l + 1 < La:
                fc = L["Rl"] @ ext(l, r)
                vc = cycle(l + 1, None, fc, True)
                v = v + L["Pl"] @ ext(l + 1, vc)
            else:
                fc_own = L["Rl"] @ ext(l, r)
                parts = [None] * world
                dist.all_gather_object(parts, fc_own)
                fc = np.concatenate(parts)
                vc = tail._cycle(np.zeros(len(fc)), fc, 0)
                v = v + L["Pl"] @ vc
            return v + L["d"] * (f - L["Al"] @ ext(l, v))

        b = np.random.default_rng(3).uniform(-1, 1, A.nrows)
        s0, s1 = splits[0][rank], splits[0][rank + 1]
        z_loc = cycle(0, None, b[s0:s1], True)
        parts = [None] * world
        dist.all_gather_object(parts, z_loc)
        z = np.concatenate(parts)
        for l, lev in enumerate(levels):
            lev["smoother"] = "chol" if l == nl - 1 else "jacobi"
        zref = O.Multigrid(levels).apply(b)
        err = np.linalg.norm(z - zref) / np.linalg.norm(zref)
        # bench helpers: weak-scaling dims and slab splits are consistent
        wd = bench.weak_dims(64, world)
        assert np.prod(wd) == world * 64 ** 3
        import torch
        t = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, err, La, [len(s.ghost) for s in spaces], float(t[0])))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None, None))
    finally:
        dist.destroy_process_group()


def test_dist_vcycle_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
    res.sort()
    for rank, err, La, ghosts, tmax in res:
        assert not isinstance(err, str), err
        assert err <= 1e-13, (rank, err)
        assert La >= 1
        assert ghosts[0] == 8 * 6  # one 8x6 plane from the neighbour slab
        assert tmax == 1.0
