"""Generate the golden fixtures under tests/golden/ (G1-G6 of SURVEY.md 8(c)).

The reference publishes no golden data and cannot be built here (SURVEY.md F2,
F4), so these vectors come from the C restatement (oracle/amg_oracle.c) and are
accepted only if the independent numpy/scipy restatement (oracle/np_oracle.py)
agrees at generation time.  Closed-form checks pin what can be pinned (the 1-D
FD solution of -u'' = 1 is exactly x(1-x)/2 at the grid points).  Fixtures are
data only (inputs and expected outputs) in .npz files loaded with
allow_pickle=False.

Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import np_oracle as N  # noqa: E402
import oracle as O  # noqa: E402


def splitmix_uniform(n, seed=42):
    """b ~ U(-1,1) from splitmix64 (counter form of the sequential stream):
    z_i = mix(seed + (i+1)*0x9E3779B97F4A7C15), u = (z >> 11) * 2^-53, b = 2u - 1."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def noise_floor(A, x, b):
    """Absolute noise floor of a computed relative residual ||b - A x|| / ||b||:
    eps * ||A||_inf * ||x||_inf / ||b||_inf (residual-history tolerance)."""
    M = A.to_scipy() if hasattr(A, "to_scipy") else A
    anorm = abs(M).sum(axis=1).max()
    return np.finfo(float).eps * anorm * np.max(np.abs(x)) / np.max(np.abs(b))


def csr_arrays(prefix, M, out):
    rp, ci, va = M.arrays()
    m, n, _ = M.dims()
    out[prefix + "_shape"] = np.array([m, n], np.int64)
    out[prefix + "_rowptr"] = rp
    out[prefix + "_col"] = ci
    out[prefix + "_val"] = va


def gmg1d_oracle_levels(n_elements, refinement, base=10):
    nlev = N.gmg1d_levels(n_elements, refinement, base)
    levels = []
    for l, lev in enumerate(nlev):
        d = {"A": O.Csr.from_scipy(lev["A"])}
        if "R" in lev:
            d["R"] = O.Csr.from_scipy(lev["R"])
            d["P"] = O.Csr.from_scipy(lev["P"])
        d["smoother"] = "chol" if l == len(nlev) - 1 else "jacobi"
        levels.append(d)
    return levels, nlev


def g1():
    """simple_geometric (1-D) refinements r = 2..6: rhs = 1, tol 1e-8."""
    out = {}
    for r in range(2, 7):
        ne = 10 * 2**r
        levels, nlev = gmg1d_oracle_levels(ne, r)
        mg = O.Multigrid(levels)
        A = levels[0]["A"]
        b = np.ones(ne - 1)
        x, it, hist = O.stationary_solve(A, mg, b, max_iter=6000, rel_tol=1e-8)
        _, pcg_it, _ = O.pcg_solve(A, b, mg=mg, max_iter=6000, rel_tol=1e-8, abs_tol=np.finfo(float).eps)
        _, jac_it, _ = O.pcg_solve(A, b, diag=O.jacobi_diag(A), max_iter=6000, rel_tol=1e-8,
                                   abs_tol=np.finfo(float).eps)
        # cross-check with numpy restatement
        for lev in nlev[:-1]:
            lev["smoother"] = "jacobi"
        nlev[-1]["smoother"] = "chol"
        nmg = N.Multigrid(nlev)
        _, nhist = N.stationary(nlev[0]["A"], nmg.apply, b, 6000, 1e-8)
        assert len(nhist) == it, (len(nhist), it)
        assert np.allclose(hist, nhist, rtol=1e-8, atol=noise_floor(A, x, b))
        # closed form: u_i = x_i (1 - x_i) / 2
        xs = np.arange(1, ne) / ne
        assert np.max(np.abs(x - xs * (1 - xs) / 2)) < 1e-6 * np.max(xs * (1 - xs) / 2) + 1e-9
        out[f"r{r}_hist"] = hist
        out[f"r{r}_iters"] = np.array([it, pcg_it, jac_it], np.int64)
    np.savez_compressed(os.path.join(HERE, "g1_gmg1d.npz"), **out)


def g2():
    """Config C1: 2-D 5-pt, 128 elements (127^2 unknowns), two levels."""
    nlev = N.gmg2d_levels(128, 64)
    levels = []
    for l, lev in enumerate(nlev):
        d = {"A": O.Csr.from_scipy(lev["A"])}
        if "R" in lev:
            d["R"] = O.Csr.from_scipy(lev["R"])
            d["P"] = O.Csr.from_scipy(lev["P"])
        d["smoother"] = "chol" if l == len(nlev) - 1 else "jacobi"
        levels.append(d)
    mg = O.Multigrid(levels)
    A = levels[0]["A"]
    n = A.nrows
    b = np.ones(n)
    x, it, hist = O.stationary_solve(A, mg, b, max_iter=30, rel_tol=1e-30)
    _, pcg_it, pcg_hist = O.pcg_solve(A, b, mg=mg, max_iter=6000, rel_tol=1e-8)
    for lev in nlev:
        lev["smoother"] = "jacobi"
    nlev[-1]["smoother"] = "chol"
    nmg = N.Multigrid(nlev)
    _, nhist = N.stationary(nlev[0]["A"], nmg.apply, b, 30, 1e-30)
    assert np.allclose(hist, nhist, rtol=1e-8, atol=noise_floor(A, x, b))
    out = {"hist": hist, "pcg_iters": np.array([pcg_it], np.int64), "pcg_hist": pcg_hist,
           "z": mg.apply(b)}
    # the GMG operators themselves (inputs)
    for l, lev in enumerate(levels):
        csr_arrays(f"A{l}", lev["A"], out)
        if "R" in lev:
            csr_arrays(f"R{l}", lev["R"], out)
            csr_arrays(f"P{l}", lev["P"], out)
    np.savez_compressed(os.path.join(HERE, "g2_gmg2d_c1.npz"), **out)


def sa_case(A, An, dims, box, smoother, name, ncycles=20):
    levels = O.sa_hierarchy_box(A, dims, box)
    nlevels = N.sa_hierarchy_box(An, dims, box)
    assert len(levels) == len(nlevels)
    for a, b_ in zip(levels, nlevels):
        d = (a["A"].to_scipy() - b_["A"])
        assert d.nnz == 0 or abs(d).max() <= 1e-12 * abs(b_["A"]).max()
    for l, lev in enumerate(levels):
        lev["smoother"] = "chol" if l == len(levels) - 1 else smoother
        nlevels[l]["smoother"] = lev["smoother"]
    mg = O.Multigrid(levels)
    nmg = N.Multigrid(nlevels)
    b = splitmix_uniform(A.nrows, 42)
    z = mg.apply(b)
    zn = nmg.apply(b)
    assert np.linalg.norm(z - zn) <= 1e-12 * np.linalg.norm(z)
    _, it, hist = O.stationary_solve(A, mg, b, max_iter=ncycles, rel_tol=1e-300)
    out = {"b": b, "z": z, "hist": hist, "nlevels": np.array([len(levels)], np.int64),
           "dims": np.array(dims, np.int64), "box": np.array(box, np.int64)}
    for l, lev in enumerate(levels):
        csr_arrays(f"A{l}", lev["A"], out)
        if "R" in lev:
            csr_arrays(f"R{l}", lev["R"], out)
            csr_arrays(f"P{l}", lev["P"], out)
    np.savez_compressed(os.path.join(HERE, name), **out)


def g3():
    """7-pt 16^3 SA hierarchy (2^3 boxes, one constant candidate), Jacobi 0.66;
    includes the Galerkin products (G6: A_{l+1} = R_l A_l P_l)."""
    sa_case(O.laplace3d_7pt(16, 16, 16), N.laplace3d_7pt(16, 16, 16), (16, 16, 16), (2, 2, 2),
            "jacobi", "g3_sa7pt16.npz")


def g4():
    """27-pt anisotropic 12^3, SA 2^3 boxes, multicolor SGS smoother."""
    sa_case(O.aniso27(12, 12, 12), N.aniso27(12, 12, 12), (12, 12, 12), (2, 2, 2), "sgs",
            "g4_sa27pt12_sgs.npz")


def g5():
    """SpMV on an irregular random CSR: empty rows, 1-nnz rows, a 300-nnz row and
    a 3000-nnz row (longer than one LDS block), rectangular."""
    rng = np.random.default_rng(5)
    m, n = 700, 5000
    rows = []
    for i in range(m):
        if i % 7 == 3:
            k = 0
        elif i % 11 == 5:
            k = 1
        elif i == 100:
            k = 300
        elif i == 200:
            k = 3000
        else:
            k = int(rng.integers(2, 40))
        rows.append(np.sort(rng.choice(n, size=k, replace=False)))
    rp = np.zeros(m + 1, np.int64)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.concatenate(rows).astype(np.int64)
    va = rng.standard_normal(len(ci))
    x = rng.standard_normal(n)
    A = O.Csr.from_arrays(m, n, rp, ci, va)
    y = A.spmv(x)
    import scipy.sparse as sp
    ys = sp.csr_matrix((va, ci, rp), shape=(m, n)) @ x
    assert np.allclose(y, ys, rtol=1e-12, atol=1e-12)
    np.savez_compressed(os.path.join(HERE, "g5_spmv_irregular.npz"), shape=np.array([m, n]),
                        rowptr=rp, col=ci, val=va, x=x, y=y)


if __name__ == "__main__":
    O.build()
    g1()
    g2()
    g3()
    g4()
    g5()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
