"""General smoothed aggregation (config C5 path: unstructured SPD, block size 3,
three candidates) on the GPU against the restatements: oracle/sa_oracle.py for
the setup pieces, oracle/amg_oracle.c for the V-cycle on the same hierarchy.

Tolerances: strength graph and aggregates bitwise (same operation order);
tentative P through basis-independent checks (per-aggregate projector equal to
LAPACK's to 1e-12, orthonormal columns, P * coarse_nn = near-null) because the
SVD of a degenerate block has no unique basis; block_jacobi / RAP to 1e-12 of
the row scale; V-cycle 1e-11; rho_k 1e-8 (+ noise floor).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
import sa_oracle as SO

pytestmark = pytest.mark.gpu
EPS = np.finfo(float).eps


def fa():
    import faer_amg_amd
    return faer_amg_amd


def elasticity(ctx, elements, seed=11):
    H = fa().elasticity_q1(elements, seed=seed)
    return H.upload(ctx), H.to_scipy()


def weights(S, nn):
    return [1.0 / float(nn[:, c] @ (S @ nn[:, c])) for c in range(nn.shape[1])]


def csr_close(G, R, rtol):
    """Same matrix up to rtol of the largest entry (pattern may carry explicit zeros)."""
    D = (G - R).tocsr()
    return abs(D).max() <= rtol * abs(R).max() if D.nnz else True


def test_strength_graph_bitwise(ctx):
    A, S = elasticity(ctx, (4, 3, 3))
    nn = fa().constant_candidates(S.shape[0], 3)
    w = weights(S, nn)
    G = fa().strength_graph(A, nn, w, depth=1, block_size=3)
    R = SO.strength_graph(S, nn, w, depth=1, block_size=3)
    assert np.array_equal(G.indptr, R.indptr) and np.array_equal(G.indices, R.indices)
    assert np.array_equal(G.data, R.data)
    # depth 2 on a scalar problem with two random candidates (extract_local_subgraph BFS)
    L = fa().SparseMatOp.laplace3d_7pt(ctx, 5, 4, 3)
    LS = L.to_scipy()
    rnn = np.random.default_rng(3).standard_normal((LS.shape[0], 2))
    G2 = fa().strength_graph(L, rnn, [1.0, 0.5], depth=2, block_size=1)
    R2 = SO.strength_graph(LS, rnn, [1.0, 0.5], depth=2, block_size=1)
    assert np.array_equal(G2.indptr, R2.indptr) and np.array_equal(G2.indices, R2.indices)
    assert np.array_equal(G2.data, R2.data)


@pytest.mark.parametrize("kind", ["constant", "random"])
def test_tentative_block(ctx, kind):
    A, S = elasticity(ctx, (4, 4, 3))
    n = S.shape[0]
    if kind == "constant":
        nn, cd = fa().constant_candidates(n, 3), 3
    else:
        nn, cd = np.asfortranarray(np.random.default_rng(4).standard_normal((n, 4))), 2
    G = SO.strength_graph(S, fa().constant_candidates(n, 3), [1.0] * 3, 1, 3)
    agg, na = fa().aggregate_mis(G)
    P, cnn = fa().sa_tentative_block(ctx, agg, na, nn, block_size=3, candidate_dimension=cd)
    Ph = P.to_scipy()
    assert Ph.shape == (n, na * cd) and np.all(np.diff(Ph.indptr) == cd)
    node_agg = np.repeat(agg, 3)
    for a, (rows, proj, s) in enumerate(SO.tentative_projectors(agg, na, nn, 3, cd)):
        Pa = Ph[rows][:, a * cd:(a + 1) * cd].toarray()
        assert np.allclose(Pa.T @ Pa, np.eye(cd), atol=1e-13)          # orthonormal columns
        assert np.max(np.abs(Pa @ Pa.T - proj)) <= 1e-12               # same subspace as LAPACK
        assert np.all(node_agg[rows] == a)
        # coarse near-null = S V^T: its first cd rows carry the singular values
        assert np.allclose(np.sort(np.linalg.svd(cnn[a * cd:(a + 1) * cd], compute_uv=False))[::-1],
                           s[:cd], rtol=1e-12)
    if cd == nn.shape[1]:
        assert np.max(np.abs(Ph @ cnn - nn)) <= 1e-13 * np.max(np.abs(nn))  # exact reconstruction
    if kind == "constant":  # orthogonal candidates: U = local / sqrt(|agg|), no rotation
        sizes = np.bincount(agg)
        for i in range(0, n, 37):
            row = Ph[i].toarray().ravel()
            a = agg[i // 3]
            expect = np.zeros(na * 3)
            expect[a * 3 + i % 3] = 1.0 / np.sqrt(sizes[a])
            assert np.allclose(row, expect, rtol=1e-14, atol=0)


def test_block_jacobi_and_rap(ctx):
    A, S = elasticity(ctx, (4, 4, 3))
    n = S.shape[0]
    nn = fa().constant_candidates(n, 3)
    G = SO.strength_graph(S, nn, weights(S, nn), 1, 3)
    agg, na = fa().aggregate_mis(G)
    P, cnn = fa().sa_tentative_block(ctx, agg, na, nn, block_size=3)
    Ps = fa().block_jacobi(A, P, 3)
    ref = SO.block_jacobi(S, P.to_scipy(), 3)
    assert csr_close(Ps.to_scipy(), ref, 1e-12)
    R = fa().transpose(Ps)
    Ac = fa().galerkin_rap(R, A, Ps)
    Psh = Ps.to_scipy()
    assert csr_close(Ac.to_scipy(), (Psh.T @ S @ Psh).tocsr(), 1e-12)
    # block size 1: the scalar Jacobi smoothing (smooth_interpolation)
    P1 = fa().smooth_interpolation(A, P)
    assert csr_close(P1.to_scipy(), SO.smooth_interpolation(S, P.to_scipy()), 1e-12)
    # coarse near-null post-processing (3 L1 steps + thin QR) for 3 columns
    x = fa().nn_postprocess(Ac, cnn, 3)
    xr = SO.nn_postprocess(Ac.to_scipy(), cnn, 3)
    assert np.max(np.abs(x - xr)) <= 1e-10
    assert np.allclose(x.T @ x, np.eye(3), atol=1e-12)


def _build(ctx, elements, smoother="l1", coarsest=150, seed=11):
    A, S = elasticity(ctx, elements, seed)
    nn = fa().constant_candidates(S.shape[0], 3)
    mg = fa().smoothed_aggregation(A, nn, weights=weights(S, nn), block_size=3, candidate_dimension=3,
                                   coarsest_dim=coarsest, smoother=smoother)
    return A, S, nn, mg


def test_sa_build_equals_composition(ctx):
    """amg_sa_build's first level is the pieces composed as Hierarchy::coarsen
    does (strength -> MIS -> tentative -> block_jacobi -> R, RAP): bitwise."""
    A, S, nn, mg = _build(ctx, (5, 4, 4))
    assert mg.levels() >= 2
    G = fa().strength_graph(A, nn, weights(S, nn), depth=1, block_size=3)
    agg, na = fa().aggregate_mis(G)
    P, cnn = fa().sa_tentative_block(ctx, agg, na, nn, block_size=3)
    Ps = fa().block_jacobi(A, P, 3)
    Ac = fa().galerkin_rap(fa().transpose(Ps), A, Ps)
    A1, _, _, _ = mg.level(1)
    _, _, R0, P0 = mg.level(0)
    for X, Y in ((P0, Ps), (A1, Ac)):
        a, b = X.arrays(), Y.arrays()
        assert all(np.array_equal(u, v) for u, v in zip(a, b))
    assert R0.dims() == (na * 3, S.shape[0])


def oracle_levels(mg, smoother):
    levels = []
    nl = mg.levels()
    for l in range(nl):
        Al, Sl, Rl, Pl = mg.level(l)
        d = {"A": O.Csr.from_arrays(*Al.dims(), *Al.arrays()), "smoother": "chol" if l == nl - 1 else smoother}
        if Rl is not None:
            d["R"] = O.Csr.from_arrays(*Rl.dims(), *Rl.arrays())
            d["P"] = O.Csr.from_arrays(*Pl.dims(), *Pl.arrays())
        levels.append(d)
    return levels


@pytest.mark.parametrize("smoother", ["l1", "jacobi"])
def test_sa_elasticity_vcycle_parity(ctx, smoother):
    """C5's path end to end on the stand-in: one V-cycle to 1e-11 of the oracle
    on the same hierarchy, 10 stationary cycles (rho_k) to 1e-8, PCG converges."""
    import torch
    A, S, nn, mg = _build(ctx, (8, 6, 6), smoother=smoother)
    n = S.shape[0]
    levels = oracle_levels(mg, smoother)
    b = np.random.default_rng(12).uniform(-1, 1, n)
    zref = O.Multigrid(levels).apply(b)
    bd = torch.as_tensor(b, device="cuda:0")
    z = torch.empty_like(bd)
    mg.apply(z, bd)
    ctx.synchronize()
    assert np.linalg.norm(z.cpu().numpy() - zref) <= 1e-11 * np.linalg.norm(zref)
    x = torch.zeros_like(bd)
    it, hist = fa().stationary_solve(A, mg, bd, x, max_iter=11, rel_tol=1e-300)
    _, it_o, hist_o = O.stationary_solve(levels[0]["A"], O.Multigrid(levels), b, max_iter=11, rel_tol=1e-300)
    floor = EPS * abs(S).sum(axis=1).max() * float(torch.max(torch.abs(x))) / np.max(np.abs(b))
    assert it == it_o == 11
    assert np.all(np.abs(hist - hist_o) <= 1e-8 * hist_o + floor)
    if smoother == "jacobi":
        return  # point Jacobi (omega 0.66) does not converge on elasticity: parity only
    assert hist[-1] < hist[0]
    x = torch.zeros_like(bd)
    itp, _ = fa().pcg_solve(A, mg, bd, x, max_iter=300, rel_tol=1e-8)
    itc, _ = fa().pcg_solve(A, None, bd, torch.zeros_like(bd), max_iter=3000, rel_tol=1e-8)
    assert itp < itc
    assert np.linalg.norm(b - S @ x.cpu().numpy()) <= 1e-7 * np.linalg.norm(b)


def test_sa_scalar_random_candidates(ctx):
    """Block size 1, two random candidates, one kept (cd < k), depth 2 strength:
    the scalar smooth_interpolation path and the k > 1 QR post-processing."""
    import torch
    dims = (12, 10, 9)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    n = A.nrows
    rng = np.random.default_rng(6)
    nn = np.asfortranarray(np.column_stack([np.ones(n), rng.uniform(0.5, 1.5, n)]))
    mg = fa().smoothed_aggregation(A, nn, block_size=1, candidate_dimension=1, strength_depth=2,
                                   coarsest_dim=60, smoother="jacobi")
    assert mg.levels() >= 2
    levels = oracle_levels(mg, "jacobi")
    b = rng.uniform(-1, 1, n)
    zref = O.Multigrid(levels).apply(b)
    bd = torch.as_tensor(b, device="cuda:0")
    z = torch.empty_like(bd)
    mg.apply(z, bd)
    ctx.synchronize()
    assert np.linalg.norm(z.cpu().numpy() - zref) <= 1e-11 * np.linalg.norm(zref)


@pytest.mark.parametrize("gap", [False, True])
def test_bsr_storage_bitwise(ctx, gap):
    """3x3 block storage: picked for the elasticity operator and its SA levels,
    SpMV bitwise equal to the oracle's CSR row sums (blocks summed in ascending
    column order), V-cycle bitwise equal to the same hierarchy with the block
    storage disabled (FAMG_NO_BSR is read at first use: compared through a
    CSR-only copy instead).  gap: explicit entries removed from blocks (partly
    filled blocks carry zeros)."""
    import torch
    H = fa().elasticity_q1((16, 12, 12), seed=5)
    S = H.to_scipy().tocsr()
    if gap:  # drop the (0,1) / (1,0) entries of one block in five: partly filled blocks
        C = S.tocoo()
        I, J = C.row // 3, C.col // 3
        hole = ((I + J) % 5 == 0) & (I != J) & (((C.row % 3 == 0) & (C.col % 3 == 1)) | ((C.row % 3 == 1) & (C.col % 3 == 0)))
        keep = ~hole
        S = sp.csr_matrix((C.data[keep], (C.row[keep], C.col[keep])), shape=S.shape)
        # each removed symmetric pair a_ij is given back as |a_ij| on both
        # diagonals (a PSD 2x2 update): the operator stays SPD
        S = (S + sp.diags(np.bincount(C.row[hole], weights=np.abs(C.data[hole]), minlength=S.shape[0]))).tocsr()
        S.sort_indices()
    A = fa().SparseMatOp.from_scipy(ctx, S)
    info = A.spmv_info()
    assert info["kernel"] == "bsr", info
    assert info["stream_bytes"] < 12 * S.nnz
    OA = O.Csr.from_scipy(S)
    x = np.random.default_rng(2).standard_normal(S.shape[0])
    xd = torch.as_tensor(x, device="cuda:0")
    yd = torch.empty_like(xd)
    A.apply(yd, xd)
    ctx.synchronize()
    assert np.array_equal(yd.cpu().numpy(), OA.spmv(x))
    # every 3x3-block kernel (flag bsr_kernel: round-2 kernel, columns first
    # with 4-step batches, 2- / 4-step pipelined) and epilogue: bitwise
    ax = OA.spmv(x)
    b0 = np.random.default_rng(8).standard_normal(S.shape[0])
    d0 = np.random.default_rng(9).uniform(0.1, 0.2, S.shape[0])
    bd, dd = torch.as_tensor(b0, device="cuda:0"), torch.as_tensor(d0, device="cuda:0")
    # (bsr_long: the prefetching long-row kernel for slices averaging at least that
    # many block steps -- 0 always, -1 never)
    try:
        for k, split in ((0, -1), (1, -1), (2, -1), (3, -1), (0, 0)):
            fa().set_flag("bsr_kernel", k)
            fa().set_flag("bsr_long", split)
            for mode, ref in (("set", ax), ("add", 0.5 + ax), ("resid", b0 - ax), ("jacobi", x + d0 * (b0 - ax))):
                yk = torch.full_like(xd, 0.5)
                A.spmv_epilogue(mode, xd, yk, bd, dd)
                ctx.synchronize()
                assert np.array_equal(yk.cpu().numpy().view(np.int64), ref.view(np.int64)), (k, split, mode)
    finally:
        fa().set_flag("bsr_kernel", 0)
        fa().set_flag("bsr_long", 48)
    nn = fa().constant_candidates(S.shape[0], 3)
    w = weights(S, nn)
    mg = fa().smoothed_aggregation(A, nn, weights=w, block_size=3, candidate_dimension=3, coarsest_dim=150,
                                   smoother="l1")
    kinds = [mg.level(l)[0].spmv_info()["kernel"] for l in range(mg.levels() - 1)]
    assert kinds[0] == "bsr"
    fa().set_spmv_format("csr")
    try:
        Ac = fa().SparseMatOp.from_scipy(ctx, S)
        mgc = fa().smoothed_aggregation(Ac, nn, weights=w, block_size=3, candidate_dimension=3, coarsest_dim=150,
                                        smoother="l1")
    finally:
        fa().set_spmv_format("auto")
    b = torch.as_tensor(np.random.default_rng(3).uniform(-1, 1, S.shape[0]), device="cuda:0")
    z1, z2 = torch.empty_like(b), torch.empty_like(b)
    mg.apply(z1, b)
    mgc.apply(z2, b)
    ctx.synchronize()
    # CSR-stream splits long rows over lanes: equal to rounding, not bitwise
    assert float(torch.linalg.norm(z1 - z2)) <= 1e-13 * float(torch.linalg.norm(z2))
    levels = oracle_levels(mg, "l1")
    zref = O.Multigrid(levels).apply(b.cpu().numpy())
    assert np.linalg.norm(z1.cpu().numpy() - zref) <= 1e-11 * np.linalg.norm(zref)


def test_strength_depth3_block3_and_vcycle(ctx):
    """The reference's strength setting: BFS depth 3 (PartitionerConfig::build,
    partitioners/mod.rs:290) on a block-3 elasticity problem -- the strength
    graph bitwise against sa_oracle, the aggregates bitwise, and a hierarchy
    built with depth 3 cycled to 1e-11 of the oracle on the same arrays."""
    import torch
    A, S = elasticity(ctx, (4, 3, 3))
    n = S.shape[0]
    nn = fa().constant_candidates(n, 3)
    w = weights(S, nn)
    G = fa().strength_graph(A, nn, w, depth=3, block_size=3)
    R = SO.strength_graph(S, nn, w, depth=3, block_size=3)
    assert np.array_equal(G.indptr, R.indptr) and np.array_equal(G.indices, R.indices)
    assert np.array_equal(G.data, R.data)
    G1 = fa().strength_graph(A, nn, w, depth=1, block_size=3)
    assert G.nnz > G1.nnz  # depth 3 reaches further than the matrix graph
    agg, na = fa().aggregate_mis(G)
    agg_r, na_r = SO.aggregate_mis(R)
    assert na == na_r and np.array_equal(agg, agg_r)
    A2, S2 = elasticity(ctx, (6, 5, 5), seed=3)
    nn2 = fa().constant_candidates(S2.shape[0], 3)
    mg = fa().smoothed_aggregation(A2, nn2, weights=weights(S2, nn2), block_size=3, candidate_dimension=3,
                                   strength_depth=3, coarsest_dim=100, smoother="l1")
    assert mg.levels() >= 2
    b = np.random.default_rng(4).uniform(-1, 1, S2.shape[0])
    zref = O.Multigrid(oracle_levels(mg, "l1")).apply(b)
    bd = torch.as_tensor(b, device="cuda:0")
    z = torch.empty_like(bd)
    mg.apply(z, bd)
    ctx.synchronize()
    assert np.linalg.norm(z.cpu().numpy() - zref) <= 1e-11 * np.linalg.norm(zref)


def _reorder_runs(ctx, e, modes):
    """elasticity stand-in with shuffled nodes, e^3 elements: z = M b and an
    11-cycle stationary history per reorder mode"""
    import torch
    H = fa().elasticity_q1((e, e, e), seed=3, permute=True)
    A, S = H.upload(ctx), H.to_scipy()
    nn = fa().constant_candidates(S.shape[0], 3)
    mg = fa().smoothed_aggregation(A, nn, weights=weights(S, nn), block_size=3, candidate_dimension=3,
                                   coarsest_dim=150, smoother="l1")
    b = torch.as_tensor(np.random.default_rng(31).uniform(-1, 1, S.shape[0]), device="cuda:0")
    out = {}
    for mode in modes:
        mg.set_reorder(mode)
        z = torch.empty_like(b)
        mg.apply(z, b)
        x = torch.zeros_like(b)
        _, hist = fa().stationary_solve(A, mg, b, x, max_iter=11, rel_tol=1e-300)
        ctx.synchronize()
        out[mode] = {"z": z.cpu().numpy(), "hist": np.asarray(hist), "plan": mg.cycle_plan(),
                     "reordered": [mg.reordered(l) for l in range(mg.levels())]}
    return mg, b, out


def _renumbered_plan_ok(plan, n, mg):
    names = [p["name"] for p in plan]
    # (perm_gather_df: the gather writes the fine level's first Jacobi step from zero too)
    assert names[0] in ("perm_gather", "perm_gather_df") and names[-1] == "perm_scatter", names
    assert any(p["name"] == "bsr3" and p["level"] == 0 for p in plan), names
    assert mg.level(0)[0].nrows == n and mg.level(0)[0].spmv_info()["kernel"] == "bsr"
    Ar = mg.run_level(0)[0]  # the renumbered copy the cycle runs
    assert Ar.nrows == n and Ar.nnz == mg.level(0)[0].nnz and Ar.spmv_info()["kernel"] == "bsr"


def test_locality_reordering_bitwise(ctx):
    """Locality reordering (multigrid option 5, reorder.hip): a general operator
    with its nodes shuffled (elasticity stand-in, 3x3 blocks) runs its eligible
    levels in a locality numbering (reverse Cuthill-McKee, or nodes grouped by
    aggregate in the coarse level's order) -- renumbered copies of A_l, the L1
    diagonal, R_l, P_l with every row's entries in their original order and the
    original's kind of storage, one gather of rhs and one scatter of z per apply.
    56^3 elements (546K rows; A_0, P_0 3x3-block): the auto rule renumbers the
    fine level and the cycle and 10 stationary cycles are bitwise those of the
    unrenumbered cycle.  30^3 (89K rows): P_0 takes CSR-stream, whose lanes per
    row follow the rows of its block, so auto leaves the level alone (bitwise by
    doing nothing), while the forced mode renumbers it and agrees to rounding.
    The operators the multigrid hands back are the caller's (oracle parity).  A
    grid operator's levels (C2-like) are never renumbered."""
    mg, b, out = _reorder_runs(ctx, 56, (0, 1))
    assert not any(out[0]["reordered"]) and out[1]["reordered"][0]
    _renumbered_plan_ok(out[1]["plan"], b.numel(), mg)
    assert np.array_equal(out[1]["z"].view(np.int64), out[0]["z"].view(np.int64))
    assert np.array_equal(out[1]["hist"], out[0]["hist"])
    del mg, out
    mg, b, out = _reorder_runs(ctx, 30, (0, 2, 1))
    assert not any(out[0]["reordered"]) and not any(out[1]["reordered"]) and out[2]["reordered"][0]
    assert [p["name"] for p in out[0]["plan"] if p["level"] == 0 and p["role"] == "interp"] == ["csr-stream"]
    _renumbered_plan_ok(out[2]["plan"], b.numel(), mg)
    assert np.array_equal(out[1]["z"].view(np.int64), out[0]["z"].view(np.int64))
    z0 = out[0]["z"]
    assert np.linalg.norm(out[2]["z"] - z0) <= 1e-14 * np.linalg.norm(z0)
    assert np.allclose(out[2]["hist"], out[0]["hist"], rtol=1e-10, atol=0)
    # the handed-back operators are the caller's: the oracle on them matches
    levels = oracle_levels(mg, "l1")
    zref = O.Multigrid(levels).apply(b.cpu().numpy())
    assert np.linalg.norm(out[2]["z"] - zref) <= 1e-11 * np.linalg.norm(zref)
    # a grid operator: nothing to renumber
    dims = (64, 64, 64)
    G = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mgg = fa().sa_build_box(G, dims, (2, 2, 2), coarsest_dim=500)
    assert not any(mgg.reordered(l) for l in range(mgg.levels()))
