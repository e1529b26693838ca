"""CPU tests: the oracle (C restatement) against the committed golden fixtures,
the independent numpy/scipy restatement and closed-form answers.

Parity is UNPINNED against the reference itself (it cannot be built or run
here and ships no golden data -- SURVEY.md F2-F4); these tests pin the oracle
as far as the available evidence allows.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import np_oracle as N
import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def csr_from(g, prefix):
    m, n = g[prefix + "_shape"]
    return O.Csr.from_arrays(m, n, g[prefix + "_rowptr"], g[prefix + "_col"], g[prefix + "_val"])


def noise_floor(A, x, b):
    anorm = abs(A.to_scipy()).sum(axis=1).max()
    return np.finfo(float).eps * anorm * np.max(np.abs(x)) / np.max(np.abs(b))


# ------------------------------------------------------------- generators

@pytest.mark.parametrize("dims", [(5, 4, 3), (1, 1, 1), (7, 1, 2), (8, 8, 8)])
def test_laplace3d_matches_kron(dims):
    A = O.laplace3d_7pt(*dims).to_scipy()
    B = N.laplace3d_7pt(*dims)
    assert (A != B).nnz == 0
    assert A.nnz == B.nnz


@pytest.mark.parametrize("dims", [(4, 5, 3), (2, 2, 2), (6, 6, 6)])
def test_aniso27_matches_kron_and_is_spd(dims):
    A = O.aniso27(*dims).to_scipy()
    B = N.aniso27(*dims)
    assert abs(A - B).max() <= 1e-15
    assert (A != A.T).nnz == 0
    assert np.linalg.eigvalsh(A.toarray()).min() > 0


def test_aniso27_stencil_sums():
    c = O.aniso27_stencil(1.0, 1.0, 0.01).reshape(3, 3, 3)
    # T sums to 0 along its axis, so the full stencil sums to 0 (constants in the kernel)
    assert abs(c.sum()) < 1e-15
    assert c[1, 1, 1] > 0


def test_fd1d_and_2d():
    A = O.fd1d(40).to_scipy()
    assert abs(A - N.fd1d(40)).max() < 1e-9
    B = O.laplace2d_5pt(16).to_scipy()
    assert abs(B - N.laplace2d_5pt(16)).max() < 1e-9


# ------------------------------------------------------------------ SpMV

def test_spmv_golden_irregular():
    g = load("g5_spmv_irregular.npz")
    m, n = g["shape"]
    A = O.Csr.from_arrays(m, n, g["rowptr"], g["col"], g["val"])
    y = A.spmv(g["x"])
    assert np.array_equal(y, g["y"])  # bitwise: sequential fma order
    ys = sp.csr_matrix((g["val"], g["col"], g["rowptr"]), shape=(m, n)) @ g["x"]
    absx = sp.csr_matrix((np.abs(g["val"]), g["col"], g["rowptr"]), shape=(m, n)) @ np.abs(g["x"])
    nnz_row = np.diff(g["rowptr"])
    assert np.all(np.abs(y - ys) <= 2 * nnz_row * 2.0**-53 * absx + 1e-300)


def test_parspmm_bitwise_equals_csr():
    """ParSpmmOp restatement (8192 CSC tiles) gives the same bits as CSR order."""
    A = O.laplace3d_7pt(40, 30, 20)  # 24000 rows -> 3 block rows
    x = np.random.default_rng(1).standard_normal(A.ncols)
    ps = O.ParSpmm(A)
    assert np.array_equal(ps.apply(x), A.spmv(x))
    # rectangular (P-like) operator: rows past ncols are computed (reference bug a3 not copied)
    g = load("g3_sa7pt16.npz")
    P = csr_from(g, "P0")
    xc = np.random.default_rng(2).standard_normal(P.ncols)
    assert np.array_equal(O.ParSpmm(P).apply(xc), P.spmv(xc))


# --------------------------------------------------------------- smoothers

def test_diag_smoothers():
    A = O.aniso27(5, 5, 5)
    S = A.to_scipy()
    d = S.diagonal()
    assert np.allclose(O.jacobi_diag(A, 0.66), 0.66 / d, rtol=0, atol=0)
    assert np.allclose(O.l1_diag(A), 1.0 / np.asarray(abs(S).sum(axis=1)).ravel(), rtol=1e-15)
    ds = np.sqrt(d)
    l2 = 1.0 / np.asarray((abs(S).multiply(np.outer(ds, 1.0 / ds))).sum(axis=1)).ravel()
    assert np.allclose(O.l2_diag(A), l2, rtol=1e-14)


@pytest.mark.parametrize("gen,ncolors", [(lambda: O.laplace3d_7pt(6, 5, 4), 2),
                                         (lambda: O.aniso27(6, 5, 4), 8)])
def test_greedy_coloring_is_parity_coloring(gen, ncolors):
    A = gen()
    color, nc = O.greedy_coloring(A)
    assert nc == ncolors
    S = A.to_scipy().tocoo()
    off = S.row != S.col
    assert np.all(color[S.row[off]] != color[S.col[off]])
    c2, nc2 = N.greedy_coloring(A.to_scipy())
    assert np.array_equal(color, c2)


def test_sgs_matches_numpy_and_is_symmetric():
    A = O.aniso27(5, 4, 6)
    S = A.to_scipy()
    color, nc = O.greedy_coloring(A)
    rng = np.random.default_rng(3)
    r = rng.standard_normal(A.nrows)
    e = O.sgs_apply(A, color, nc, r)
    en = N.sgs(S, color, nc, 1.0 / S.diagonal(), r)
    assert np.allclose(e, en, rtol=1e-13, atol=1e-15)
    # M = SGS operator must be symmetric: u^T M v == v^T M u
    u, v = rng.standard_normal(A.nrows), rng.standard_normal(A.nrows)
    a, b = u @ O.sgs_apply(A, color, nc, v), v @ O.sgs_apply(A, color, nc, u)
    assert abs(a - b) <= 1e-12 * max(abs(a), 1)


def test_chol_solve():
    A = O.laplace3d_7pt(4, 4, 4)
    D = A.to_scipy().toarray()
    L = np.zeros_like(D)
    assert O.lib().orc_chol_factor(64, np.ascontiguousarray(D), L) == 0
    b = np.random.default_rng(4).standard_normal(64)
    x = b.copy()
    O.lib().orc_chol_solve(64, L, x)
    assert np.allclose(D @ x, b, rtol=1e-12, atol=1e-12)
    bad = -np.eye(3)
    assert O.lib().orc_chol_factor(3, bad, np.zeros((3, 3))) != 0


# ----------------------------------------------------------- setup (SA)

def test_spgemm_transpose_match_scipy():
    A = O.aniso27(6, 5, 4)
    agg, na, _ = O.box_aggregates((6, 5, 4), (2, 2, 2))
    Pt, cnn = O.sa_tentative(agg, na, np.ones(A.nrows))
    AP = O.spgemm(A, Pt).to_scipy()
    ref = A.to_scipy() @ Pt.to_scipy()
    assert abs(AP - ref).max() < 1e-14
    T = O.transpose(Pt).to_scipy()
    assert (T != Pt.to_scipy().T).nnz == 0
    # tentative P columns are orthonormal and reproduce the candidate
    Pts = Pt.to_scipy()
    assert np.allclose((Pts.T @ Pts).toarray(), np.eye(na), atol=1e-14)
    assert np.allclose(Pts @ cnn, np.ones(A.nrows), rtol=1e-14)


def test_box_aggregates_match_numpy():
    for dims, box in [((7, 5, 3), (2, 2, 2)), ((9, 9, 9), (3, 3, 3)), ((4, 1, 1), (2, 2, 2))]:
        a, na, cd = O.box_aggregates(dims, box)
        b, nb, cdn = N.box_aggregates(dims, box)
        assert na == nb and cd == cdn and np.array_equal(a, b)


def test_sa_hierarchy_golden_g3():
    g = load("g3_sa7pt16.npz")
    levels = O.sa_hierarchy_box(O.laplace3d_7pt(16, 16, 16), (16, 16, 16), (2, 2, 2))
    assert len(levels) == int(g["nlevels"][0])
    for l, lev in enumerate(levels):
        for key in ("A", "R", "P"):
            if key not in lev:
                continue
            rp, ci, va = lev[key].arrays()
            assert np.array_equal(rp, g[f"{key}{l}_rowptr"])
            assert np.array_equal(ci, g[f"{key}{l}_col"])
            assert np.array_equal(va, g[f"{key}{l}_val"])
    # Galerkin identity (G6): A_{l+1} == R_l A_l P_l (scipy product, rounding tol)
    for l in range(len(levels) - 1):
        A, R, P = (csr_from(g, f"{k}{l}").to_scipy() for k in "ARP")
        Ac = csr_from(g, f"A{l + 1}").to_scipy()
        assert abs(Ac - R @ (A @ P)).max() <= 1e-12 * abs(Ac).max()
        assert (R != P.T).nnz == 0


def vcycle_case(name, smoother):
    g = load(name)
    nl = int(g["nlevels"][0])
    levels = []
    for l in range(nl):
        d = {"A": csr_from(g, f"A{l}"), "smoother": "chol" if l == nl - 1 else smoother}
        if l < nl - 1:
            d["R"] = csr_from(g, f"R{l}")
            d["P"] = csr_from(g, f"P{l}")
        levels.append(d)
    return g, levels


@pytest.mark.parametrize("name,smoother", [("g3_sa7pt16.npz", "jacobi"),
                                           ("g4_sa27pt12_sgs.npz", "sgs")])
def test_vcycle_golden(name, smoother):
    g, levels = vcycle_case(name, smoother)
    mg = O.Multigrid(levels)
    z = mg.apply(g["b"])
    assert np.array_equal(z, g["z"])
    _, it, hist = O.stationary_solve(levels[0]["A"], mg, g["b"], max_iter=len(g["hist"]),
                                     rel_tol=1e-300)
    assert np.array_equal(hist, g["hist"])
    # independent numpy V-cycle on the same hierarchy
    nlev = []
    for lev in levels:
        d = {"A": lev["A"].to_scipy(), "smoother": lev["smoother"]}
        if "R" in lev:
            d["R"], d["P"] = lev["R"].to_scipy(), lev["P"].to_scipy()
        nlev.append(d)
    zn = N.Multigrid(nlev).apply(g["b"])
    assert np.linalg.norm(z - zn) <= 1e-12 * np.linalg.norm(z)


def test_vcycle_mu_steps_variants():
    """W-cycle (mu=2) and 2 smoothing steps: C oracle == numpy restatement."""
    g, levels = vcycle_case("g3_sa7pt16.npz", "jacobi")
    nlev = []
    for lev in levels:
        d = {"A": lev["A"].to_scipy(), "smoother": lev["smoother"]}
        if "R" in lev:
            d["R"], d["P"] = lev["R"].to_scipy(), lev["P"].to_scipy()
        nlev.append(d)
    for mu, steps in [(2, 1), (1, 2), (3, 2)]:
        z = O.Multigrid(levels, mu=mu, steps=steps).apply(g["b"])
        zn = N.Multigrid(nlev, mu=mu, steps=steps).apply(g["b"])
        assert np.linalg.norm(z - zn) <= 1e-12 * np.linalg.norm(z)


def test_vcycle_is_symmetric():
    """Multigrid with Jacobi/SGS smoothing and Cholesky coarse solve is a symmetric
    operator (the reference's symmetry_test, multigrid.rs:520-580)."""
    for name, sm in [("g3_sa7pt16.npz", "jacobi"), ("g4_sa27pt12_sgs.npz", "sgs")]:
        g, levels = vcycle_case(name, sm)
        mg = O.Multigrid(levels)
        rng = np.random.default_rng(7)
        n = levels[0]["A"].nrows
        U, V = rng.standard_normal((5, n)), rng.standard_normal((5, n))
        MV = np.array([mg.apply(v) for v in V])
        MU = np.array([mg.apply(u) for u in U])
        utav = U @ MV.T
        vtau = V @ MU.T
        assert np.max(np.abs(utav - vtau.T)) <= 1e-11 * np.max(np.abs(utav))


# ------------------------------------------------------------ solve drivers

def test_gmg1d_golden_and_closed_form():
    g = load("g1_gmg1d.npz")
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gmg1d_oracle_levels
    for r in range(2, 7):
        ne = 10 * 2**r
        levels, _ = gmg1d_oracle_levels(ne, r)
        mg = O.Multigrid(levels)
        A = levels[0]["A"]
        b = np.ones(ne - 1)
        x, it, hist = O.stationary_solve(A, mg, b, max_iter=6000, rel_tol=1e-8)
        assert np.array_equal(hist, g[f"r{r}_hist"])
        xs = np.arange(1, ne) / ne
        assert np.max(np.abs(x - xs * (1 - xs) / 2)) < 1e-6 * 0.125
        # mesh independence of the MG iteration counts (simple_geometric.rs:50-51)
        assert it <= 14
        iters = g[f"r{r}_iters"]
        _, pcg_it, _ = O.pcg_solve(A, b, mg=mg, max_iter=6000, rel_tol=1e-8,
                                   abs_tol=np.finfo(float).eps)
        assert pcg_it == iters[1]


def test_c1_gmg2d_golden():
    g = load("g2_gmg2d_c1.npz")
    levels = [{"A": csr_from(g, "A0"), "R": csr_from(g, "R0"), "P": csr_from(g, "P0"),
               "smoother": "jacobi"},
              {"A": csr_from(g, "A1"), "smoother": "chol"}]
    mg = O.Multigrid(levels)
    b = np.ones(levels[0]["A"].nrows)
    assert np.array_equal(mg.apply(b), g["z"])
    x, it, hist = O.stationary_solve(levels[0]["A"], mg, b, max_iter=30, rel_tol=1e-30)
    assert np.array_equal(hist, g["hist"])
    # the two-grid cycle contracts (rho_k decreasing geometrically)
    assert hist[10] < 1e-3 and np.all(np.diff(hist[:15]) < 0)
    _, pcg_it, _ = O.pcg_solve(levels[0]["A"], b, mg=mg, max_iter=6000, rel_tol=1e-8)
    assert pcg_it == int(g["pcg_iters"][0])


def test_pcg_matches_numpy():
    g, levels = vcycle_case("g3_sa7pt16.npz", "jacobi")
    mg = O.Multigrid(levels)
    A = levels[0]["A"]
    x, it, _ = O.pcg_solve(A, g["b"], mg=mg, rel_tol=1e-10)
    nlev = []
    for lev in levels:
        d = {"A": lev["A"].to_scipy(), "smoother": lev["smoother"]}
        if "R" in lev:
            d["R"], d["P"] = lev["R"].to_scipy(), lev["P"].to_scipy()
        nlev.append(d)
    xn, itn = N.pcg(A.to_scipy(), g["b"], N.Multigrid(nlev).apply, 1000, 1e-10)
    assert abs(it - itn) <= 1
    assert np.linalg.norm(A.to_scipy() @ x - g["b"]) <= 1e-10 * np.linalg.norm(g["b"]) * 1.0001


def test_splitmix_stream():
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import splitmix_uniform
    # sequential splitmix64 reference values (state += golden; mix)
    def seq(seed, n):
        M = (1 << 64) - 1
        st, out = seed, []
        for _ in range(n):
            st = (st + 0x9E3779B97F4A7C15) & M
            z = st
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
            z ^= z >> 31
            out.append(2.0 * ((z >> 11) * 2.0**-53) - 1.0)
        return np.array(out)
    assert np.array_equal(splitmix_uniform(50, 42), seq(42, 50))
    u = splitmix_uniform(100000, 42)
    assert -1 <= u.min() < -0.99 and 0.99 < u.max() < 1 and abs(u.mean()) < 0.01


def test_oracle_envelope_cholesky_large():
    """The oracle's coarsest solve above 4096 rows: the envelope (profile)
    Cholesky factor in the natural order (coarse_solvers.rs:164-206 takes any
    size; a dense n^3/3 factor does not scale) -- A x = b to 1e-12 against
    scipy's sparse direct solve, and the dense path below the threshold."""
    import scipy.sparse.linalg as spla
    for dims in ((17, 19, 21), (10, 10, 10)):
        A = O.laplace3d_7pt(*dims)
        S = A.to_scipy().tocsc()
        b = np.random.default_rng(5).standard_normal(A.nrows)
        x = O.Multigrid([{"A": A, "smoother": "chol"}]).apply(b)
        xs = spla.spsolve(S, b)
        assert np.linalg.norm(x - xs) <= 1e-12 * np.linalg.norm(xs), dims
