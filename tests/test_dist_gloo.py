"""CPU coverage of the N > 1 path (gloo, world sizes 2 and 3) that runs the
PRODUCT's distributed planner: every rank builds its per-level halo plans with
the library's host planner (faer_amg_amd.HaloPlan = amg_halo_plan_*, the code
amg_dist_multigrid_create runs: ghost sets from the rank's rows of A_l, R_l and
P_{l-1}, request/send lists, neighbour table, the [owned | ghost] column
renumbering and the interior row segment, the agglomeration level), exchanges
the requests over torch.distributed (gloo), and

  1. compares every plan with an independent numpy restatement (`Space`);
  2. runs the distributed V-cycle in numpy on the library's plans (halo
     refreshes packed with the library's send lists into the library's receive
     offsets, SpMVs on the library-renumbered local matrices, redundant tail
     below the library's agglomeration level) and compares it with the global
     oracle V-cycle.

Two hierarchies: the 7-pt box SA hierarchy on z-slabs (aggregates never cross
a slab), and a general smoothed-aggregation hierarchy of a Q1 elasticity
problem (block size 3, MIS aggregates, block-Jacobi smoothed P) on equal row
splits aligned to the block size, where aggregates straddle ranks: P's coarse
halo and R's row ownership differ from the z-slab case
(reference SA: /root/reference/src/interpolation/mod.rs:730-836).
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
    """numpy restatement of one level's plan (independent of plan.cpp)."""

    def __init__(self, splits, rank, mats, dist):
        self.r0, self.r1 = splits[rank], splits[rank + 1]
        self.n_own = self.r1 - self.r0
        cols = np.unique(np.concatenate([m.indices.astype(np.int64) for m in mats] + [np.zeros(0, np.int64)]))
        self.ghost = cols[(cols < self.r0) | (cols >= self.r1)]
        owner = np.searchsorted(splits, self.ghost, side="right") - 1
        world = len(splits) - 1
        reqs = [self.ghost[owner == q] for q in range(world)]
        allreq = [None] * world
        dist.all_gather_object(allreq, reqs)
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


def interior(L, n_own):
    """numpy restatement of the interior segment: longest run of rows reading owned columns only."""
    n = L.shape[0]
    flag = np.array([np.any(L.indices[L.indptr[i]:L.indptr[i + 1]] >= n_own) for i in range(n)], bool)
    best, i = (0, 0), 0
    while i < n:
        if flag[i]:
            i += 1
            continue
        j = i
        while j < n and not flag[j]:
            j += 1
        if j - i > best[1] - best[0]:
            best = (i, j)
        i = j
    return (n, n) if best[1] == best[0] else best


class LibSpace:
    """One level's plan from the library's planner, with a gloo halo refresh that
    uses only the library's send lists / neighbour table."""

    def __init__(self, fa, splits, rank, world, mats, dist):
        self.plan = fa.HaloPlan(world, rank, splits)
        for m in mats:
            self.plan.add_columns(m.indices)
        self.ghost, reqs = self.plan.requests()
        allreq = [None] * world
        dist.all_gather_object(allreq, reqs)
        self.plan.set_incoming([allreq[q][rank] if q != rank else np.zeros(0, np.int64) for q in range(world)])
        self.info = self.plan.info()
        self.nb = self.plan.neighbors()
        self.sidx = self.plan.send_indices()
        self.n_own = self.info["n_own"]

    def halo(self, x, dist):
        import torch
        reqs, bufs = [], []
        for k, q in enumerate(self.nb["nbr"]):
            s0, sc = int(self.nb["soff"][k]), int(self.nb["scnt"][k])
            if sc:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(x[self.sidx[s0:s0 + sc]])), int(q)))
            r0, rc = int(self.nb["roff"][k]), int(self.nb["rcnt"][k])
            if rc:
                b = torch.empty(rc, dtype=torch.float64)
                reqs.append(dist.irecv(b, int(q)))
                bufs.append((r0, b))
        for r in reqs:
            r.wait()
        for r0, b in bufs:
            x[self.n_own + r0:self.n_own + r0 + len(b)] = b.numpy()


def box_problem(world):
    import oracle as O
    dims = (8, 6, 16)
    A = O.laplace3d_7pt(*dims)
    levels = O.sa_hierarchy_box(A, dims, (2, 2, 2), coarsest_dim=20)
    S = [{k: lev[k].to_scipy() for k in ("A", "R", "P") if k in lev} for lev in levels]
    ldims = [dims]
    for _ in range(len(levels) - 1):
        ldims.append(tuple(-(-a // 2) for a in ldims[-1]))
    splits = [np.array([(p * nz) // world * nx * ny for p in range(world + 1)], np.int64) for (nx, ny, nz) in ldims]
    return S, splits, 60


def elast_problem(world):
    """General SA hierarchy (numpy restatement of sa.hip's pipeline on a Q1
    elasticity operator): constant candidates, strength graph (depth 1),
    MIS aggregates, tentative P by per-aggregate SVD, block-Jacobi smoothing,
    R = P^T, A_c = R A P; three levels, block size 3 on each."""
    import sa_oracle as SA
    A = SA.elasticity_q1(4, 4, 6, contrast=1.0, nu=0.3, seed=7, permute=True)
    bs = 3
    S = []
    nn = np.tile(np.eye(bs), (A.shape[0] // bs, 1))
    for _ in range(2):
        n = A.shape[0]
        w = [1.0 / float(nn[:, c] @ (A @ nn[:, c])) for c in range(bs)]
        G = SA.strength_graph(A, nn, w, depth=1, block_size=bs)
        agg, na = SA.aggregate_mis(G)
        rows, cols, vals = [], [], []
        cnn = np.zeros((na * bs, bs))
        for a in range(na):
            nodes = np.flatnonzero(agg == a)
            r = (nodes[:, None] * bs + np.arange(bs)).ravel()
            U, s, Vt = np.linalg.svd(nn[r], full_matrices=False)
            for i, ri in enumerate(r):
                for c in range(bs):
                    rows.append(ri)
                    cols.append(a * bs + c)
                    vals.append(U[i, c])
            cnn[a * bs:(a + 1) * bs] = np.diag(s) @ Vt
        Pt = sp.csr_matrix((vals, (rows, cols)), shape=(n, na * bs))
        P = SA.block_jacobi(A, Pt, bs)
        P.sort_indices()
        R = P.T.tocsr()
        R.sort_indices()
        Ac = (R @ (A @ P)).tocsr()
        Ac.sort_indices()
        S.append({"A": A, "R": R, "P": P})
        A, nn = Ac, cnn
    S.append({"A": A})
    splits = []
    for lev in S:
        nb = lev["A"].shape[0] // bs
        splits.append(np.array([((p * nb) // world) * bs for p in range(world)] + [lev["A"].shape[0]], np.int64))
    return S, splits, 30


def worker(rank, world, port, q, case):
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "faer-amg_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import faer_amg_amd as fa
        import np_oracle as N
        import oracle as O

        S, splits, agglo = (box_problem if case == "box" else elast_problem)(world)
        nl = len(S)
        La = fa.first_redundant_level([lev["A"].shape[0] for lev in S], agglo)
        La_np = next((l for l in range(nl - 1) if S[l]["A"].shape[0] < agglo), nl - 1)
        assert La == La_np, (La, La_np)
        assert La >= 1, "the test needs at least one distributed level"
        loc = []
        for l in range(La):
            s0, s1 = splits[l][rank], splits[l][rank + 1]
            c0, c1 = splits[l + 1][rank], splits[l + 1][rank + 1]
            loc.append({"A": S[l]["A"][s0:s1], "P": S[l]["P"][s0:s1], "R": S[l]["R"][c0:c1],
                        "d": 0.66 / S[l]["A"].diagonal()[s0:s1]})
        lib, ref = [], []
        for l in range(La):
            mats = [loc[l]["A"], loc[l]["R"]] + ([loc[l - 1]["P"]] if l > 0 else [])
            lib.append(LibSpace(fa, splits[l], rank, world, mats, dist))
            ref.append(Space(splits[l], rank, mats, dist))
        # 1. the library's plans against the numpy restatement
        stats = []
        for l in range(La):
            L, R_ = lib[l], ref[l]
            assert np.array_equal(L.ghost, R_.ghost), l
            assert L.info["n_own"] == R_.n_own and L.info["n_ghost"] == len(R_.ghost)
            nb = L.nb
            assert sorted(set(R_.send) | set(R_.recv)) == [int(x) for x in nb["nbr"]]
            for k, qq in enumerate(nb["nbr"]):
                qq = int(qq)
                s0, sc = int(nb["soff"][k]), int(nb["scnt"][k])
                assert np.array_equal(L.sidx[s0:s0 + sc], R_.send.get(qq, np.zeros(0, np.int64))), (l, qq)
                off, cnt = R_.recv.get(qq, (None, 0))
                assert int(nb["rcnt"][k]) == cnt and (cnt == 0 or int(nb["roff"][k]) == off), (l, qq)
            mats = {"A": loc[l]["A"], "R": loc[l]["R"]}
            if l > 0:
                mats["Pprev"] = loc[l - 1]["P"]
            for name, M in mats.items():
                Ml, lo, hi = L.plan.remap(M)
                Mr = R_.remap(M)
                assert np.array_equal(Ml.indices, Mr.indices) and np.array_equal(Ml.indptr, Mr.indptr), (l, name)
                if name in ("A", "R"):
                    exp = interior(Mr, R_.n_own) if len(R_.ghost) else (M.shape[0], M.shape[0])
                    assert (lo, hi) == exp, (l, name, lo, hi, exp)
                if name == "A":
                    loc[l]["Al"] = Ml
                if name == "R":
                    loc[l]["Rl"] = Ml
                if name == "Pprev":
                    loc[l - 1]["Pl"] = Ml
            stats.append((L.info["n_ghost"], L.info["neighbors"], L.info["nsend"]))
        loc[La - 1]["Pl"] = loc[La - 1]["P"]  # global coarse ids into the replicated vector
        # 2. distributed V-cycle on the library's plans
        tail_levels = [dict(S[l]) for l in range(La, nl)]
        for l, lev in enumerate(tail_levels):
            lev["smoother"] = "chol" if La + l == nl - 1 else "jacobi"
        tail = N.Multigrid(tail_levels)

        def ext(l, v):
            x = np.zeros(lib[l].info["n_own"] + lib[l].info["n_ghost"])
            x[:lib[l].info["n_own"]] = v
            lib[l].halo(x, dist)
            return x

        def cycle(l, f):
            Lv = loc[l]
            v = Lv["d"] * f
            r = f - Lv["Al"] @ ext(l, v)
            if l + 1 < La:
                vc = cycle(l + 1, Lv["Rl"] @ ext(l, r))
                v = v + Lv["Pl"] @ ext(l + 1, vc)
            else:
                parts = [None] * world
                dist.all_gather_object(parts, Lv["Rl"] @ ext(l, r))
                fc = np.concatenate(parts)
                v = v + Lv["Pl"] @ tail._cycle(np.zeros(len(fc)), fc, 0)
            return v + Lv["d"] * (f - Lv["Al"] @ ext(l, v))

        n0 = S[0]["A"].shape[0]
        b = np.random.default_rng(3).uniform(-1, 1, n0)
        s0, s1 = splits[0][rank], splits[0][rank + 1]
        z_loc = cycle(0, b[s0:s1])
        parts = [None] * world
        dist.all_gather_object(parts, z_loc)
        z = np.concatenate(parts)
        levels = []
        for l in range(nl):
            d = {"A": O.Csr.from_scipy(S[l]["A"]), "smoother": "chol" if l == nl - 1 else "jacobi"}
            if l + 1 < nl:
                d["R"] = O.Csr.from_scipy(S[l]["R"])
                d["P"] = O.Csr.from_scipy(S[l]["P"])
            levels.append(d)
        zref = O.Multigrid(levels).apply(b)
        err = np.linalg.norm(z - zref) / np.linalg.norm(zref)
        q.put((rank, err, La, stats))
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None))
    finally:
        dist.destroy_process_group()


def run_world(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
    res.sort(key=lambda t: t[0])
    for rank, err, La, stats in res:
        assert not isinstance(err, str), err
        assert err <= 1e-13, (rank, err)
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_dist_plans_and_vcycle_box_slabs(world):
    res = run_world(world, "box")
    for l in range(len(res[0][3])):  # every requested entry is sent by exactly one rank
        assert sum(r[3][l][0] for r in res) == sum(r[3][l][2] for r in res)
    if world == 2:
        # slabs aligned with the 2^3 boxes: one 8x6 plane from the neighbouring slab
        for rank, err, La, stats in res:
            assert stats[0] == (8 * 6, 1, 8 * 6), stats


@pytest.mark.parametrize("world", [2, 3])
def test_dist_plans_and_vcycle_general_sa(world):
    """MIS aggregates straddle the equal row splits: some rank's P_0 rows read
    coarse columns another rank owns, and its R_0 rows read fine columns it
    does not own."""
    res = run_world(world, "elast")
    for l in range(len(res[0][3])):
        assert sum(r[3][l][0] for r in res) == sum(r[3][l][2] for r in res)
    assert any(s[1][0] > 0 for _, _, _, s in res), "level 1 should need a coarse halo"


def test_bench_weak_dims():
    sys.path.insert(0, ROOT)
    import bench
    for N in (1, 2, 3, 4, 8):
        assert np.prod(bench.weak_dims(64, N)) == N * 64 ** 3
    assert bench.weak_dims(256, 8) == (512, 512, 512)
