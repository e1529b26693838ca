"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on
the same inputs.  Tolerances (DESIGN.md "Parity"):
  SpMV            |y - y_ref|_i <= 2 nnz_i u sum_j |a_ij x_j|   (bitwise for <=128-nnz rows)
  one V-cycle     ||z - z_ref|| / ||z_ref|| <= 1e-11
  residual hist   |rho_k - rho_ref_k| <= 1e-8 rho_ref_k + eps ||A||_inf ||x||_inf / ||b||_inf
  RAP / SpGEMM    identical pattern, values bitwise (ascending-k fma in both)
  PCG iterations  equal or +-1
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import np_oracle as N
import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EPS = np.finfo(float).eps


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def T(x):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x, np.float64), device="cuda:0")


def H(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def fa():
    import faer_amg_amd
    return faer_amg_amd


def gpu_csr(ctx, Ocsr):
    m, n, _ = Ocsr.dims()
    rp, ci, va = Ocsr.arrays()
    return fa().SparseMatOp.from_arrays(ctx, m, n, rp, ci, va)


def spmv_bound(S, x):
    absx = abs(S) @ np.abs(x)
    return 2 * np.diff(S.indptr) * 2.0**-53 * absx + 1e-300


def apply_dev(ctx, op, x, nout):
    xd = T(x)
    yd = T(np.full(nout, np.nan))
    op.apply(yd, xd)
    ctx.synchronize()
    return H(yd)


# ------------------------------------------------------------------ SpMV

def test_generators_bitwise(ctx):
    A = fa().SparseMatOp.laplace3d_7pt(ctx, 9, 7, 5)
    rp, ci, va = A.arrays()
    orp, oci, ova = O.laplace3d_7pt(9, 7, 5).arrays()
    assert np.array_equal(rp, orp) and np.array_equal(ci, oci) and np.array_equal(va, ova)
    B = fa().SparseMatOp.aniso27(ctx, 6, 5, 7, 1.0, 1.0, 0.01)
    rp, ci, va = B.arrays()
    orp, oci, ova = O.aniso27(6, 5, 7).arrays()
    assert np.array_equal(rp, orp) and np.array_equal(ci, oci) and np.array_equal(va, ova)


def test_spmv_7pt_bitwise(ctx):
    A = fa().SparseMatOp.laplace3d_7pt(ctx, 40, 33, 17)
    OA = O.laplace3d_7pt(40, 33, 17)
    x = np.random.default_rng(0).standard_normal(OA.ncols)
    y = apply_dev(ctx, A, x, OA.nrows)
    assert np.array_equal(y, OA.spmv(x))


def test_spmv_27pt(ctx):
    A = fa().SparseMatOp.aniso27(ctx, 20, 17, 11, 1.0, 1.0, 0.01)
    OA = O.aniso27(20, 17, 11)
    x = np.random.default_rng(1).standard_normal(OA.ncols)
    y = apply_dev(ctx, A, x, OA.nrows)
    assert np.all(np.abs(y - OA.spmv(x)) <= spmv_bound(OA.to_scipy(), x))


def test_spmv_irregular_golden(ctx):
    """Empty rows, 1-nnz rows, a 300-nnz row, a 3000-nnz row (whole-workgroup path)."""
    g = load("g5_spmv_irregular.npz")
    m, n = g["shape"]
    A = fa().SparseMatOp.from_arrays(ctx, m, n, g["rowptr"], g["col"], g["val"])
    y = apply_dev(ctx, A, g["x"], m)
    S = sp.csr_matrix((g["val"], g["col"], g["rowptr"]), shape=(m, n))
    assert np.all(np.abs(y - g["y"]) <= spmv_bound(S, g["x"]))
    assert np.all(y[np.diff(g["rowptr"]) == 0] == 0)


@pytest.mark.parametrize("fmt", ["csr", "sell", "vector", "vector-w2", "vector-w4"])
def test_spmv_formats(ctx, fmt):
    """Both storage paths (CSR-stream and SELL-64) on short, long, empty and
    rectangular rows.  SELL sums every row sequentially in one lane (bitwise
    equal to the oracle); CSR-stream does so when a block holds >= 128 rows
    (rows of <= 16 entries) and splits longer rows over lanes (bounded); the
    wave-per-row kernel with 1, 2 or 4 waves per row (bounded; odd row counts
    leave a workgroup's last row slots empty)."""
    if fmt.startswith("vector-w"):
        fa().set_flag("vec_wpr", int(fmt[-1]))
        fmt = "vector"
    fa().set_spmv_format(fmt)
    try:
        OA = O.laplace3d_7pt(33, 17, 9)
        x = np.random.default_rng(10).standard_normal(OA.ncols)
        y = apply_dev(ctx, gpu_csr(ctx, OA), x, OA.nrows)
        if fmt == "vector":
            assert np.all(np.abs(y - OA.spmv(x)) <= spmv_bound(OA.to_scipy(), x))
        else:
            assert np.array_equal(y, OA.spmv(x))
        g = load("g3_sa7pt16.npz")
        for key in ("P0", "R0", "A1"):
            m, n = g[f"{key}_shape"]
            OM = O.Csr.from_arrays(m, n, g[f"{key}_rowptr"], g[f"{key}_col"], g[f"{key}_val"])
            xx = np.random.default_rng(11).standard_normal(n)
            y = apply_dev(ctx, gpu_csr(ctx, OM), xx, m)
            if fmt == "sell" or (key == "P0" and fmt == "csr"):
                assert np.array_equal(y, OM.spmv(xx)), key
            else:
                assert np.all(np.abs(y - OM.spmv(xx)) <= spmv_bound(OM.to_scipy(), xx)), key
        g5 = load("g5_spmv_irregular.npz")
        m, n = g5["shape"]
        A = fa().SparseMatOp.from_arrays(ctx, m, n, g5["rowptr"], g5["col"], g5["val"])
        y = apply_dev(ctx, A, g5["x"], m)
        S = sp.csr_matrix((g5["val"], g5["col"], g5["rowptr"]), shape=(m, n))
        assert np.all(np.abs(y - g5["y"]) <= spmv_bound(S, g5["x"]))
    finally:
        fa().set_spmv_format("auto")
        fa().set_flag("vec_wpr", 0)


def _random_rows(rng, m, n, per_row, spread):
    """CSR with per_row random sorted columns per row within +-spread of the
    diagonal position (clipped), plus some empty rows."""
    rp, ci = [0], []
    for i in range(m):
        k = 0 if i % 17 == 5 else int(rng.integers(1, per_row + 1))
        c0 = i * n // m
        lo, hi = max(0, c0 - spread), min(n, c0 + spread + 1)
        cols = np.sort(rng.choice(np.arange(lo, hi), size=min(k, hi - lo), replace=False))
        ci.extend(cols.tolist())
        rp.append(len(ci))
    rp = np.asarray(rp, np.int64)
    ci = np.asarray(ci, np.int64)
    return O.Csr.from_arrays(m, n, rp, ci, rng.standard_normal(len(ci)))


def test_sell_column_modes(ctx):
    """SELL-64 stores a slice's columns implicitly (stencil offsets, aligned
    steps), as 16-bit deltas or as int32; every mode sums each row in stored
    order in one lane, so results are bitwise equal to the oracle."""
    rng = np.random.default_rng(21)
    fa().set_spmv_format("sell")
    try:
        cases = {
            "7pt": (O.laplace3d_7pt(64, 12, 6), "slices_implicit"),
            "27pt": (O.aniso27(64, 9, 5), "slices_implicit"),
            "band": (_random_rows(rng, 3001, 3001, 12, 2000), "slices_u16"),
            "wide": (_random_rows(rng, 1000, 400000, 9, 200000), "slices_i32"),
        }
        for name, (OM, dominant) in cases.items():
            M = gpu_csr(ctx, OM)
            info = M.spmv_info()
            assert info["kernel"] == "sell", name
            assert info[dominant] * 2 > info["slices"], (name, info)
            x = rng.standard_normal(OM.ncols)
            assert np.array_equal(apply_dev(ctx, M, x, OM.nrows), OM.spmv(x)), name
            if name == "7pt":
                # aligned steps: boundary rows padded, but < 20 % extra entries,
                # and 8 B/entry + metadata instead of 12
                assert info["stored_entries"] < 1.2 * OM.dims()[2]
                assert info["stream_bytes"] < 0.8 * info["csr_bytes"]
    finally:
        fa().set_spmv_format("auto")


def test_vcycle_forced_sell(ctx):
    fa().set_spmv_format("sell")
    try:
        dims = (20, 16, 12)
        A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=200)
        levels = oracle_levels_from_gpu(mg, "jacobi")
        b = np.random.default_rng(12).uniform(-1, 1, A.nrows)
        zref = O.Multigrid(levels).apply(b)
        z = apply_dev(ctx, mg, b, A.nrows)
        assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    finally:
        fa().set_spmv_format("auto")


def test_spmv_host_memory_and_multicolumn(ctx):
    OA = O.laplace3d_7pt(10, 10, 10)
    A = gpu_csr(ctx, OA)
    X = np.asfortranarray(np.random.default_rng(2).standard_normal((1000, 3)))
    Y = np.asfortranarray(np.zeros((1000, 3)))
    A.apply(Y, X)  # AMG_MEM_HOST, k = 3
    for c in range(3):
        assert np.array_equal(Y[:, c], OA.spmv(X[:, c]))


def test_transpose_apply(ctx):
    g = load("g3_sa7pt16.npz")
    m, n = g["P0_shape"]
    P = fa().SparseMatOp.from_arrays(ctx, m, n, g["P0_rowptr"], g["P0_col"], g["P0_val"])
    x = np.random.default_rng(3).standard_normal(m)
    out = np.zeros(n)
    P.transpose_apply(out, x)
    Ps = sp.csr_matrix((g["P0_val"], g["P0_col"], g["P0_rowptr"]), shape=(m, n))
    assert np.allclose(out, Ps.T @ x, rtol=1e-13, atol=1e-13)


def test_large_spmv_property(ctx):
    """Full-size-style property check: A 1 == boundary-row deficits (integer exact)."""
    import torch
    nx = ny = nz = 96
    A = fa().SparseMatOp.laplace3d_7pt(ctx, nx, ny, nz)
    ones = torch.ones(nx * ny * nz, dtype=torch.float64, device="cuda:0")
    y = torch.empty_like(ones)
    A.apply(y, ones)
    ctx.synchronize()
    z, yy, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    expect = ((x == 0).astype(float) + (x == nx - 1) + (yy == 0) + (yy == ny - 1) + (z == 0)
              + (z == nz - 1)).ravel()
    assert np.array_equal(H(y), expect)


# ------------------------------------------------------------- smoothers

def test_diag_smoothers(ctx):
    OA = O.aniso27(7, 6, 5)
    A = gpu_csr(ctx, OA)
    r = np.random.default_rng(4).standard_normal(OA.nrows)
    for mk, ref in [(lambda: fa().new_jacobi(A, 0.66), O.jacobi_diag(OA, 0.66)),
                    (lambda: fa().new_l1(A), O.l1_diag(OA)),
                    (lambda: fa().new_l2(A), O.l2_diag(OA))]:
        S = mk()
        out = apply_dev(ctx, S, r, OA.nrows)
        assert np.allclose(out, ref * r, rtol=2e-16 * 4, atol=0)
        rd = T(r)
        S.apply_in_place(rd)
        assert np.allclose(H(rd), ref * r, rtol=8e-16, atol=0)


def test_sgs_matches_oracle(ctx):
    OA = O.aniso27(9, 8, 7)
    A = gpu_csr(ctx, OA)
    S = fa().SymGaussSeidel(A)
    color, nc = O.greedy_coloring(OA)
    assert S.ncolors == nc == 8
    r = np.random.default_rng(5).standard_normal(OA.nrows)
    e = apply_dev(ctx, S, r, OA.nrows)
    eref = O.sgs_apply(OA, color, nc, r)
    assert np.linalg.norm(e - eref) <= 1e-13 * np.linalg.norm(eref)
    # explicit coloring, 7-pt red-black
    OB = O.laplace3d_7pt(8, 8, 8)
    B = gpu_csr(ctx, OB)
    cb, ncb = O.greedy_coloring(OB)
    SB = fa().SymGaussSeidel(B, colors=cb)
    assert SB.ncolors == 2
    r = np.random.default_rng(6).standard_normal(OB.nrows)
    e = apply_dev(ctx, SB, r, OB.nrows)
    assert np.array_equal(e, O.sgs_apply(OB, cb, ncb, r))  # 7-pt rows: bitwise
    with pytest.raises(fa().AmgError):
        fa().SymGaussSeidel(B, colors=np.zeros(OB.nrows, np.int32))  # invalid coloring


def test_coarse_cholesky(ctx):
    OA = O.laplace3d_7pt(8, 8, 8)
    A = gpu_csr(ctx, OA)
    C = fa().CoarseCholesky(A)
    b = np.random.default_rng(7).standard_normal(OA.nrows)
    x = apply_dev(ctx, C, b, OA.nrows)
    assert np.linalg.norm(OA.to_scipy() @ x - b) <= 1e-12 * np.linalg.norm(b)
    # not SPD -> AMG_ERR_NOT_SPD
    neg = O.Csr.from_scipy(-OA.to_scipy())
    with pytest.raises(fa().AmgError) as ei:
        fa().CoarseCholesky(gpu_csr(ctx, neg))
    assert ei.value.status == 4


@pytest.mark.parametrize("dims", [(42, 42, 42), (21, 23, 25)])
def test_coarse_cholesky_any_size(ctx, dims):
    """The coarsest solve above 8192 rows (SparseCholeskySolve takes any size,
    coarse_solvers.rs:164-206): the envelope Cholesky factor of the RCM-ordered
    matrix in 64-row blocks (chol.hip).  42^3: a 2-level hierarchy whose
    coarsest level has 9261 rows -- the V-cycle within 1e-11 of the oracle
    (whose envelope factor keeps the natural order), the plan's coarse launch
    the block solve.  21 x 23 x 25: the solve on the 7-point operator itself
    (12075 rows, a ragged last block), A x = b to 1e-11."""
    import torch
    n = int(np.prod(dims))
    if dims == (42, 42, 42):
        A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=20000)
        assert mg.levels() == 2 and mg.level(1)[0].nrows > 8192
        b = np.random.default_rng(3).uniform(-1, 1, n)
        z = torch.empty(n, dtype=torch.float64, device="cuda:0")
        mg.apply(z, T(b))
        ctx.synchronize()
        zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
        assert np.linalg.norm(H(z) - zref) <= 1e-11 * np.linalg.norm(zref)
        assert [p["name"] for p in mg.cycle_plan() if p["role"] == "coarse"] == ["chol-env"]
        return
    OA = O.laplace3d_7pt(*dims)
    C = fa().CoarseCholesky(gpu_csr(ctx, OA))
    b = np.random.default_rng(8).standard_normal(n)
    x = apply_dev(ctx, C, b, n)
    assert np.linalg.norm(OA.to_scipy() @ x - b) <= 1e-11 * np.linalg.norm(b)


# ------------------------------------------------------------------- setup

def csr_equal(G, Oc, exact=True, rtol=0.0):
    rp, ci, va = G.arrays()
    orp, oci, ova = Oc.arrays()
    assert np.array_equal(rp, orp)
    assert np.array_equal(ci, oci)
    if exact:
        assert np.array_equal(va, ova)
    else:
        assert np.max(np.abs(va - ova)) <= rtol * np.max(np.abs(ova))


def test_spgemm_transpose_rap_bitwise(ctx):
    OA = O.aniso27(10, 9, 8)
    A = gpu_csr(ctx, OA)
    agg, na, _ = O.box_aggregates((10, 9, 8), (2, 2, 2))
    nn = 1.0 + 0.1 * np.random.default_rng(8).standard_normal(OA.nrows)
    OPt, ocnn = O.sa_tentative(agg, na, nn)
    Pt, cnn = fa().sa_tentative(ctx, agg, na, nn)
    assert np.array_equal(cnn, ocnn)
    csr_equal(Pt, OPt)
    csr_equal(fa().spgemm(A, Pt), O.spgemm(OA, OPt))
    OP = O.smooth_interpolation(OA, OPt, 0.66)
    P = fa().smooth_interpolation(A, Pt, 0.66)
    csr_equal(P, OP)
    R = fa().transpose(P)
    OR = O.transpose(OP)
    csr_equal(R, OR)
    csr_equal(fa().galerkin_rap(R, A, P), O.rap(OR, OA, OP))


def test_spgemm_wide_rows(ctx):
    """Products with > 512 distinct columns per row (larger LDS hash tables)."""
    rng = np.random.default_rng(9)
    M = sp.random(300, 2000, density=0.02, random_state=rng, format="csr")
    N_ = sp.random(2000, 3000, density=0.03, random_state=rng, format="csr")
    OM, ON = O.Csr.from_scipy(M), O.Csr.from_scipy(N_)
    G = fa().spgemm(gpu_csr(ctx, OM), gpu_csr(ctx, ON))
    csr_equal(G, O.spgemm(OM, ON))


def test_sa_hierarchy_matches_oracle(ctx):
    """sa_build_box (GPU SpGEMM setup) vs the oracle hierarchy driver."""
    dims = (20, 18, 16)
    OA = O.laplace3d_7pt(*dims)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    olev = O.sa_hierarchy_box(OA, dims, (2, 2, 2), coarsest_dim=100)
    assert mg.levels() == len(olev)
    for l in range(mg.levels()):
        Al, Sl, Rl, Pl = mg.level(l)
        # level 0/1 exact; deeper levels see the near-null post-processing, which
        # uses a tree-reduced norm on the GPU (rounding-level differences)
        csr_equal(Al, olev[l]["A"], exact=False, rtol=1e-12)
        if Rl is not None:
            csr_equal(Pl, olev[l]["P"], exact=False, rtol=1e-12)
            csr_equal(Rl, olev[l]["R"], exact=False, rtol=1e-12)


# --------------------------------------------------------------- V-cycle

def oracle_levels_from_gpu(mg, smoother):
    """The GPU hierarchy's arrays as oracle levels, with the smoother each level
    actually got (sa_build_box(smoother='sgs') puts L1 on levels whose greedy
    coloring needs more than 32 colors)."""
    levels = []
    nl = mg.levels()
    for l in range(nl):
        Al, Sl, Rl, Pl = mg.level(l)
        m, n = Al.dims()
        if l == nl - 1:
            sm = "chol"
        elif smoother == "sgs":
            sm = "sgs" if Sl.kind == "sgs" else "l1"
        else:
            sm = smoother
        d = {"A": O.Csr.from_arrays(m, n, *Al.arrays()), "smoother": sm}
        if Rl is not None:
            d["R"] = O.Csr.from_arrays(*Rl.dims(), *Rl.arrays())
            d["P"] = O.Csr.from_arrays(*Pl.dims(), *Pl.arrays())
        levels.append(d)
    return levels


@pytest.mark.parametrize("gen,dims,smoother", [
    ("7pt", (24, 20, 18), "jacobi"),
    ("27pt", (14, 12, 16), "sgs"),
    ("27pt", (12, 12, 12), "l1"),
])
def test_vcycle_parity(ctx, gen, dims, smoother):
    if gen == "7pt":
        A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    else:
        A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=200, smoother=smoother)
    levels = oracle_levels_from_gpu(mg, smoother)
    if smoother == "sgs":
        assert levels[0]["smoother"] == "sgs"  # 8-color fine level
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import splitmix_uniform
    b = splitmix_uniform(A.nrows, 42)
    for mu, steps in [(1, 1), (2, 2)]:
        mg.with_cycle_type(mu).with_smoothing_steps(steps)
        zref = O.Multigrid(levels, mu=mu, steps=steps).apply(b)
        for graph in (True, False):
            mg.set_graph(graph)
            for resid_form in ((False, True) if smoother == "sgs" else (False,)):
                mg.set_sgs_residual_form(resid_form)
                z = apply_dev(ctx, mg, b, A.nrows)
                assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref), \
                    (mu, steps, graph, resid_form)
    mg.with_cycle_type(1).with_smoothing_steps(1)
    mg.set_graph(True)
    mg.set_sgs_residual_form(False)


@pytest.mark.parametrize("layout", ["pair", "step"])
def test_vcycle_fold_and_sell_layout_bitwise(ctx, layout):
    """Two bitwise-neutral rewrites of the Jacobi V-cycle: folding the first
    smoothing step from v = 0 (v = d f) into the residual (RESID0) and the
    correction (ADD0), and the SELL step-pair element order (16-B value loads)
    vs one 512-B row per step.  Each produces the same rounded values as the
    plain sequence, so the outputs are identical, and within 1e-11 of the
    restatement."""
    old = os.environ.get("FAMG_SELL_LAYOUT")
    os.environ["FAMG_SELL_LAYOUT"] = layout
    fa().set_spmv_format("sell")
    fa().set_value_codes(False)  # the fold applies to fp64-valued storage
    try:
        dims = (70, 20, 12)  # > 1 slice per x-line, tail slices
        A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=200)
        levels = oracle_levels_from_gpu(mg, "jacobi")
        b = np.random.default_rng(14).uniform(-1, 1, A.nrows)
        zref = O.Multigrid(levels).apply(b)
        outs = {}
        for fold in (True, False):
            mg.set_fold_zero_guess(fold)
            outs[fold] = apply_dev(ctx, mg, b, A.nrows)
        mg.set_fold_zero_guess(True)
        assert np.array_equal(outs[True].view(np.int64), outs[False].view(np.int64))
        assert np.linalg.norm(outs[True] - zref) <= 1e-11 * np.linalg.norm(zref)
        x = np.random.default_rng(15).standard_normal(A.nrows)
        OA = O.Csr.from_arrays(*A.dims(), *A.arrays())
        assert np.array_equal(apply_dev(ctx, A, x, A.nrows), OA.spmv(x))
    finally:
        fa().set_spmv_format("auto")
        fa().set_value_codes(True)
        if old is None:
            os.environ.pop("FAMG_SELL_LAYOUT", None)
        else:
            os.environ["FAMG_SELL_LAYOUT"] = old


def test_vcycle_golden_fixtures(ctx):
    """G3/G4 hierarchies uploaded as-is (Multigrid::new + add_level by hand)."""
    for name, sm in [("g3_sa7pt16.npz", "jacobi"), ("g4_sa27pt12_sgs.npz", "sgs")]:
        g = load(name)
        nl = int(g["nlevels"][0])
        ops = []
        for l in range(nl):
            m, n = g[f"A{l}_shape"]
            ops.append(fa().SparseMatOp.from_arrays(ctx, m, n, g[f"A{l}_rowptr"], g[f"A{l}_col"], g[f"A{l}_val"]))
        def smoother(A, l):
            if l == nl - 1:
                return fa().CoarseCholesky(A)
            return fa().new_jacobi(A, 0.66) if sm == "jacobi" else fa().SymGaussSeidel(A)
        mg = fa().Multigrid(ops[0], smoother(ops[0], 0))
        for l in range(1, nl):
            Rs, Ps = g[f"R{l - 1}_shape"], g[f"P{l - 1}_shape"]
            R = fa().SparseMatOp.from_arrays(ctx, *Rs, g[f"R{l-1}_rowptr"], g[f"R{l-1}_col"], g[f"R{l-1}_val"])
            P = fa().SparseMatOp.from_arrays(ctx, *Ps, g[f"P{l-1}_rowptr"], g[f"P{l-1}_col"], g[f"P{l-1}_val"])
            mg.add_level(ops[l], smoother(ops[l], l), R, P)
        z = apply_dev(ctx, mg, g["b"], len(g["b"]))
        assert np.linalg.norm(z - g["z"]) <= 1e-11 * np.linalg.norm(g["z"])
        import torch
        x = torch.zeros(len(g["b"]), dtype=torch.float64, device="cuda:0")
        it, hist = fa().stationary_solve(ops[0], mg, T(g["b"]), x, max_iter=len(g["hist"]), rel_tol=1e-300)
        assert it == len(g["hist"])
        OA = O.Csr.from_arrays(*g["A0_shape"], g["A0_rowptr"], g["A0_col"], g["A0_val"])
        floor = EPS * abs(OA.to_scipy()).sum(axis=1).max() * np.max(np.abs(H(x))) / np.max(np.abs(g["b"]))
        assert np.all(np.abs(hist - g["hist"]) <= 1e-8 * g["hist"] + floor)


def test_add_level_dimension_errors(ctx):
    A = fa().SparseMatOp.laplace3d_7pt(ctx, 4, 4, 4)
    mg = fa().Multigrid(A, fa().new_jacobi(A))
    B = fa().SparseMatOp.laplace3d_7pt(ctx, 2, 2, 2)
    with pytest.raises(fa().AmgError) as ei:
        mg.add_level(B, fa().new_jacobi(B), A, A)  # R/P with wrong shapes
    assert ei.value.status == 2


# ------------------------------------------------------------ solve drivers

def test_c1_gmg2d_stationary_and_pcg(ctx):
    """Config C1 (2-D 5-pt 127^2, 2-level, Jacobi 0.66, Cholesky coarsest)."""
    import torch
    g = load("g2_gmg2d_c1.npz")
    ops = {}
    for key in ("A0", "R0", "P0", "A1"):
        m, n = g[f"{key}_shape"]
        ops[key] = fa().SparseMatOp.from_arrays(ctx, m, n, g[f"{key}_rowptr"], g[f"{key}_col"], g[f"{key}_val"])
    mg = fa().Multigrid(ops["A0"], fa().new_jacobi(ops["A0"], 0.66))
    mg.add_level(ops["A1"], fa().CoarseCholesky(ops["A1"]), ops["R0"], ops["P0"])
    n = ops["A0"].nrows
    b = torch.ones(n, dtype=torch.float64, device="cuda:0")
    z = torch.empty_like(b)
    mg.apply(z, b)
    ctx.synchronize()
    assert np.linalg.norm(H(z) - g["z"]) <= 1e-11 * np.linalg.norm(g["z"])
    x = torch.zeros_like(b)
    it, hist = fa().stationary_solve(ops["A0"], mg, b, x, max_iter=30, rel_tol=1e-30)
    OA = O.Csr.from_arrays(*g["A0_shape"], g["A0_rowptr"], g["A0_col"], g["A0_val"])
    floor = EPS * abs(OA.to_scipy()).sum(axis=1).max() * np.max(np.abs(H(x)))
    assert it == 30
    assert np.all(np.abs(hist - g["hist"]) <= 1e-8 * g["hist"] + floor)
    x.zero_()
    it, _ = fa().pcg_solve(ops["A0"], mg, b, x, max_iter=6000, rel_tol=1e-8)
    assert abs(it - int(g["pcg_iters"][0])) <= 1


# ------------------------------------------------------------------ Composite

def test_composite_diag_components_bitwise(ctx):
    """Composite(A, [Jacobi, L1]) = L1, Jacobi, L1 steps of out += c(r);
    r = rhs - A out: every piece is bitwise (one-lane SpMV rows, diag scaling,
    elementwise add), so the whole apply is bitwise equal to the restatement."""
    OA = O.laplace3d_7pt(18, 14, 10)
    A = gpu_csr(ctx, OA)
    J, L = fa().new_jacobi(A, 0.66), fa().new_l1(A)
    Cp = fa().Composite(A, [J, L])
    assert Cp.ncomponents() == 2
    dj, dl = O.jacobi_diag(OA, 0.66), O.l1_diag(OA)
    b = np.random.default_rng(31).uniform(-1, 1, OA.nrows)
    z = apply_dev(ctx, Cp, b, OA.nrows)
    zref = O.composite_apply(OA, [lambda r: dj * r, lambda r: dl * r], b)
    assert np.array_equal(z, zref)
    Cp.push(J)  # Composite::push -> J, L, J, L, J
    z3 = apply_dev(ctx, Cp, b, OA.nrows)
    zref3 = O.composite_apply(OA, [lambda r: dj * r, lambda r: dl * r, lambda r: dj * r], b)
    assert np.array_equal(z3, zref3)


def test_composite_multigrid_and_pcg(ctx):
    """Composite(A, [V-cycle, Jacobi]) against the restatement (1e-11, the
    V-cycle tolerance), then as the PCG preconditioner: iteration count equal
    or +-1 to the restatement's PCG with the same preconditioner."""
    import torch
    dims = (16, 14, 12)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    J = fa().new_jacobi(A, 0.66)
    Cp = fa().Composite(A, [mg, J])
    OA = O.Csr.from_arrays(*A.dims(), *A.arrays())
    omg = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi"))
    dj = O.jacobi_diag(OA, 0.66)
    comps = [omg.apply, lambda r: dj * r]
    b = np.random.default_rng(32).uniform(-1, 1, OA.nrows)
    z = apply_dev(ctx, Cp, b, OA.nrows)
    zref = O.composite_apply(OA, comps, b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    bd = T(b)
    x = torch.zeros_like(bd)
    it, hist = fa().pcg_solve(A, Cp, bd, x, max_iter=200, rel_tol=1e-10)
    _, it_ref = N.pcg(OA.to_scipy(), b, lambda r: O.composite_apply(OA, comps, r), 200, 1e-10)
    assert abs(it - it_ref) <= 1, (it, it_ref)
    xr = H(x)
    assert np.linalg.norm(b - OA.spmv(xr)) <= 1e-9 * np.linalg.norm(b)


# ------------------------------------------------------------- BlockSmoother

def _box_partition(dims, box):
    nx, ny, nz = dims
    bx, by, bz = box
    cx, cy = -(-nx // bx), -(-ny // by)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return (x // bx + cx * (y // by + cy * (z // bz))).ravel().astype(np.int64)


def test_block_smoother_scalar(ctx):
    """Box partition (2^3) on the 7-pt operator and an irregular partition
    (sizes 1 .. 300: a block larger than one 256-row chunk, singletons) on the
    27-pt operator: the GPU block solve (explicit inverses) equals the
    restatement (per-block Cholesky solves) to 1e-13 relative."""
    rng = np.random.default_rng(41)
    for OA, part in (
        (O.laplace3d_7pt(12, 10, 8), _box_partition((12, 10, 8), (2, 2, 2))),
        (O.aniso27(14, 12, 10), None),
    ):
        m = OA.nrows
        if part is None:
            sizes = [300, 1, 1, 57, 128, 256, 3]
            while sum(sizes) < m:
                sizes.append(int(rng.integers(1, 90)))
            ids = np.repeat(np.arange(len(sizes)), sizes)[:m]
            part = rng.permutation(ids)  # scattered, unsorted membership
        A = gpu_csr(ctx, OA)
        B = fa().BlockSmoother(A, part)
        assert B.kind == "block"
        ref = N.block_smoother(OA.to_scipy(), part)
        r = rng.standard_normal(m)
        z = apply_dev(ctx, B, r, m)
        zr = ref(r)
        assert np.linalg.norm(z - zr) <= 1e-13 * np.linalg.norm(zr)
        # in place (Precond::apply_in_place)
        rd = T(r)
        B.apply_in_place(rd)
        assert np.array_equal(H(rd), z)
        # into_sparse_mat: same sums in the same order -> bitwise while every
        # row is summed by one lane (blocks <= 16 rows); long rows within the
        # SpMV bound
        S = B.to_sparse()
        zs = apply_dev(ctx, S, r, m)
        if np.bincount(part).max() <= 16:
            assert np.array_equal(zs, z)
        else:
            assert np.all(np.abs(zs - z) <= spmv_bound(S.to_scipy(), r))


def test_block_smoother_vector():
    """block_size 3 (diagonally_compensate_vector): node couplings -K with K
    symmetric indefinite, so the compensation 0.5 U S U^T = 0.5 |K| differs from
    -0.5 A_IJ; against the restatement's SVD-based blocks."""
    import scipy.sparse as sps
    import faer_amg_amd
    ctx = faer_amg_amd.Context(0)
    rng = np.random.default_rng(42)
    L = O.laplace3d_7pt(6, 5, 4).to_scipy()
    Loff = L - sps.diags(L.diagonal())
    K = rng.standard_normal((3, 3))
    K = K + K.T
    D = np.diag([20.0, 25.0, 30.0])
    A = (sps.kron(-Loff, -K) + sps.kron(sps.identity(L.shape[0]), D)).tocsr()
    A.sort_indices()
    nn = L.shape[0]
    part = _box_partition((6, 5, 4), (3, 2, 2))
    Ad = fa().SparseMatOp.from_scipy(ctx, A)
    B = fa().BlockSmoother(Ad, part, block_size=3)
    ref = N.block_smoother(A, part, block_size=3)
    r = rng.standard_normal(3 * nn)
    z = apply_dev(ctx, B, r, 3 * nn)
    zr = ref(r)
    assert np.linalg.norm(z - zr) <= 1e-12 * np.linalg.norm(zr)


def test_vcycle_block_smoother(ctx):
    """sa_build_box(smoother='block'): BlockSmoother over each level's box
    aggregates inside the V-cycle (generic smoothing path) against the
    restatement's V-cycle with the same block smoothers (1e-11)."""
    dims = (16, 12, 10)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100, smoother="block")
    levels = []
    nl = mg.levels()
    cdims = dims
    for l in range(nl):
        Al, Sl, Rl, Pl = mg.level(l)
        S = Al.to_scipy()
        d = {"A": S}
        if l == nl - 1:
            d["smoother"] = "chol"
        else:
            assert Sl.kind == "block"
            d["smoother"] = N.block_smoother(S, _box_partition(cdims, (2, 2, 2)))
            d["R"], d["P"] = Rl.to_scipy(), Pl.to_scipy()
            cdims = tuple(-(-c // 2) for c in cdims)
        levels.append(d)
    b = np.random.default_rng(43).uniform(-1, 1, A.nrows)
    z = apply_dev(ctx, mg, b, A.nrows)
    zref = N.Multigrid(levels).apply(b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


# ------------------------------------------------------------ multi-RHS SpMM

def _colmajor(rng, n, k, pad):
    """(n x k) column-major device matrix with leading dimension n + pad."""
    import torch
    base = torch.as_tensor(rng.standard_normal((k, n + pad)), device="cuda:0")
    return base.T[:n]


@pytest.mark.parametrize("fmt", ["auto", "sell"])
def test_spmm_multi_rhs(ctx, fmt):
    """k-column apply of a CSR operator (the SpMV generalised to k
    columns, matrix streamed once per 8 columns): every column bitwise equal
    to the single-column oracle SpMV for one-lane rows, within the SpMV bound
    otherwise; leading dimensions > n; k = 1, 3, 8, 13 (column groups 8 + 5)."""
    rng = np.random.default_rng(51)
    fa().set_spmv_format(fmt)
    try:
        for OA in (O.laplace3d_7pt(40, 20, 10), O.aniso27(16, 14, 9)):
            A = gpu_csr(ctx, OA)
            one_lane = A.spmv_info()["kernel"] == "sell"
            m, n, _ = OA.dims()
            for k in (1, 3, 8, 13):
                X = _colmajor(rng, n, k, 5)
                Y = _colmajor(rng, m, k, 3)
                A.apply(Y, X)
                Xh, Yh = H(X), H(Y)
                for c in range(k):
                    ref = OA.spmv(np.ascontiguousarray(Xh[:, c]))
                    if one_lane:
                        assert np.array_equal(Yh[:, c], ref), (k, c)
                    else:
                        assert np.all(np.abs(Yh[:, c] - ref) <= spmv_bound(OA.to_scipy(), Xh[:, c]))
    finally:
        fa().set_spmv_format("auto")


# ------------------------------------------------------------- value codes

def _with_values(rng, OM, pool):
    rp, ci, va = OM.arrays()
    m, n, _ = OM.dims()
    return O.Csr.from_arrays(m, n, rp, ci, rng.choice(np.asarray(pool, np.float64), size=len(va)))


def test_sell_value_codes(ctx):
    """SELL matrices with <= 16 / 256 / 65536 distinct values store 4 / 8 /
    16-bit codes into a per-matrix table: the decoded value is the stored
    value bit for bit, so y = A x is bitwise equal with codes on and off and to
    the oracle, for implicit, u16 and i32 column blocks; -0.0 and 0.0 keep
    separate codes; more than 65536 distinct values keep fp64."""
    rng = np.random.default_rng(61)
    fa().set_spmv_format("sell")
    try:
        cases = [
            ("7pt", O.laplace3d_7pt(64, 12, 6), (4,)),
            ("27pt", O.aniso27(64, 9, 5), (4, 8)),
            ("band-u16", _with_values(rng, _random_rows(rng, 3001, 3001, 12, 2000), rng.standard_normal(200)), (8,)),
            ("wide-i32", _random_rows(rng, 1000, 400000, 9, 200000), (16,)),
            ("signed-zeros", _with_values(rng, O.laplace3d_7pt(40, 9, 3), [0.0, -0.0, 1.5, -2.25]), (4,)),
            ("tail-groups", _with_values(rng, _random_rows(rng, 777, 900, 21, 300), rng.standard_normal(3000)),
             (16,)),
            ("fp64", _random_rows(rng, 14000, 14000, 15, 300), (0,)),  # > 65536 distinct values
        ]
        for name, OM, bits in cases:
            fa().set_value_codes(True)
            M = gpu_csr(ctx, OM)
            info = M.spmv_info()
            assert info["kernel"] == "sell" and info["value_bits"] in bits, (name, info)
            fa().set_value_codes(False)
            M0 = gpu_csr(ctx, OM)
            info0 = M0.spmv_info()
            assert info0["value_bits"] == 0
            if info["value_bits"]:
                assert info["stream_bytes"] < info0["stream_bytes"], name
            x = rng.standard_normal(OM.ncols)
            y = apply_dev(ctx, M, x, OM.nrows)
            y0 = apply_dev(ctx, M0, x, OM.nrows)
            assert np.array_equal(y.view(np.int64), y0.view(np.int64)), name
            assert np.array_equal(y, OM.spmv(x)), name
    finally:
        fa().set_value_codes(True)
        fa().set_spmv_format("auto")


@pytest.mark.parametrize("gen,smoother", [("7pt", "jacobi"), ("27pt", "sgs")])
def test_vcycle_value_codes_bitwise(ctx, gen, smoother):
    """The whole V-cycle (every SELL operator of the hierarchy, SGS color
    sweeps included) is bitwise identical with value codes on and off."""
    dims = (40, 24, 18) if gen == "7pt" else (20, 16, 14)
    b = np.random.default_rng(62).uniform(-1, 1, int(np.prod(dims)))
    outs, bits = [], []
    fa().set_spmv_format("sell")  # every level in SELL storage (the small 27-pt levels too)
    try:
        for codes in (True, False):
            fa().set_value_codes(codes)
            A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if gen == "7pt"
                 else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
            mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=200, smoother=smoother)
            bits.append([mg.level(l)[0].spmv_info()["value_bits"] for l in range(mg.levels())])
            outs.append(apply_dev(ctx, mg, b, A.nrows))
    finally:
        fa().set_value_codes(True)
        fa().set_spmv_format("auto")
    assert any(bits[0]) and not any(bits[1]), bits
    assert np.array_equal(outs[0].view(np.int64), outs[1].view(np.int64))


@pytest.mark.parametrize("gen", ["7pt", "27pt"])
def test_dia_codes(ctx, gen):
    """Constant-stencil operators (<= 32 diagonals, >= 80 % filled, <= 256
    distinct values) get DIA-codes storage in the auto policy: every mode's
    row sums bitwise equal to the oracle / to fp64-valued SELL storage, odd
    row counts (a lane's second row dead) and boundary rows (clamped x)
    included; the V-cycle on a DIA fine level within 1e-11 of the restatement
    and of the same hierarchy without value codes."""
    import torch
    dims = (64, 37, 29) if gen == "7pt" else (48, 41, 35)  # odd row count, > 65536 rows
    mk = (lambda: fa().SparseMatOp.laplace3d_7pt(ctx, *dims)) if gen == "7pt" else \
        (lambda: fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
    A = mk()
    info = A.spmv_info()
    assert info["kernel"] == "dia" and info["value_bits"] in (4, 8), info
    OA = O.Csr.from_arrays(*A.dims(), *A.arrays())
    rng = np.random.default_rng(71)
    x = rng.standard_normal(OA.ncols)
    assert np.array_equal(apply_dev(ctx, A, x, OA.nrows), OA.spmv(x))
    # fused modes through the V-cycle: codes on (DIA) vs off (SELL fp64), bitwise
    b = rng.uniform(-1, 1, OA.nrows)
    outs = []
    try:
        for codes in (True, False):
            fa().set_value_codes(codes)
            Ak = mk()
            mg = fa().sa_build_box(Ak, dims, (2, 2, 2), coarsest_dim=500)
            assert (mg.level(0)[0].spmv_info()["kernel"] == "dia") == codes
            for fold in (True, False):
                mg.set_fold_zero_guess(fold)
                outs.append(apply_dev(ctx, mg, b, OA.nrows))
            if codes:
                zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    finally:
        fa().set_value_codes(True)
    # fold on / off bitwise for each storage; codes on / off differ only where a dense
    # coarse level without codes takes the pattern SELL (lanes per row: another sum order)
    assert np.array_equal(outs[1].view(np.int64), outs[0].view(np.int64))
    assert np.array_equal(outs[3].view(np.int64), outs[2].view(np.int64))
    assert np.linalg.norm(outs[2] - outs[0]) <= 1e-14 * np.linalg.norm(outs[0])
    assert np.linalg.norm(outs[0] - zref) <= 1e-11 * np.linalg.norm(zref)
    # residual / Jacobi-step / add modes against the restatement (one-lane rows: bitwise)
    bd, xd = T(b), T(x)
    r = torch.empty_like(bd)
    it, hist = fa().stationary_solve(A, fa().new_jacobi(A, 0.66), bd, torch.zeros_like(bd), max_iter=3,
                                     rel_tol=1e-300)
    assert it == 3 and hist[2] < hist[0]


def test_dia_pattern33(ctx):
    """A_1 of smoothed aggregation on 2^3 boxes of the 7-pt operator has 33
    diagonals in runs (z-2 | 3 x runs | y-2 | x run | x run of five | x run |
    y+2 | 3 x runs | z+2) and takes DIA codes through the run-pattern kernel
    (9 code words per row, not a power of two): SpMV bitwise equal to the
    oracle (odd row count: a lane's second row dead; boundary rows: clamped x
    runs), and the V-cycle whose level 1 smooths and forms residuals on it
    within 1e-11 of the restatement, fold on and off."""
    dims = (97, 85, 73)  # level 1: 49 x 43 x 37 = 77959 rows (odd, > 65536)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    # keep the DIA pattern (setup would otherwise time it against x-staged classes)
    os.environ["FAMG_XSCS_VS_DIA"] = "0"
    try:
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
    finally:
        del os.environ["FAMG_XSCS_VS_DIA"]
    A1 = mg.level(1)[0]
    info = A1.spmv_info()
    assert info["kernel"] == "dia" and info["dia_diagonals"] == 33 and info["value_bits"] in (4, 8), info
    OA1 = O.Csr.from_arrays(*A1.dims(), *A1.arrays())
    rng = np.random.default_rng(33)
    x = rng.standard_normal(OA1.ncols)
    assert np.array_equal(apply_dev(ctx, A1, x, OA1.nrows).view(np.int64), OA1.spmv(x).view(np.int64))
    b = rng.uniform(-1, 1, A.nrows)
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    for fold in (True, False):
        mg.set_fold_zero_guess(fold)
        z = apply_dev(ctx, mg, b, A.nrows)
        assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


@pytest.mark.timeout(400)
def test_vcycle_256_storage_mix(ctx):
    """The benchmark configuration itself (C2: 7-pt 256^3, SA 2^3 boxes, Jacobi,
    6 levels) against the oracle on the same hierarchy, so the exact storage mix
    the bench times is what is checked: DIA codes on A_0, grid-transfer classes
    on R_0 and P_0 (one 8-bit class per row; the folded d*f + P v_c epilogue),
    x-staged stencil classes on A_1 (by rule, not timed against the 33-diagonal
    DIA run pattern; tiles from the frozen table), x-staged stencil classes on A_2
    (2197 classes) and A_3, 16-bit codes on R_1/P_1, the
    wave-per-row kernel on A_4.  One
    V-cycle to 1e-11 and 10 stationary cycles (rho_k) to 1e-8 (+ noise floor).
    The oracle runs its ParSpmmOp restatement on 16 threads (same per-row order
    as the sequential CSR)."""
    import torch
    dims = (256, 256, 256)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000)
    assert mg.levels() == 6
    info = [(mg.level(l)[0].spmv_info(), mg.level(l)[2].spmv_info() if l < 5 else None,
             mg.level(l)[3].spmv_info() if l < 5 else None) for l in range(6)]
    a0, r0, p0 = info[0]
    assert a0["kernel"] == "dia" and a0["value_bits"] == 4
    assert r0["kernel"] == "gtc" and p0["kernel"] == "gtc"
    # A_1: x-staged stencil classes by rule (the 33-diagonal DIA run pattern is no
    # longer timed against them), every x-staged tile from the frozen per-shape
    # table (tuning.cpp): the plan is the same on every box and under counters
    assert info[1][0]["kernel"] == "classes" and info[1][0]["xstaged"], info[1][0]
    for l in (1, 2, 3):
        assert info[l][0]["tile_source"] == "table", (l, info[l][0])
    assert info[2][0]["kernel"] == "classes" and info[2][0]["classes"] == 2197 and info[2][0]["xstaged"]
    assert info[1][1]["value_bits"] == 16 and info[1][2]["value_bits"] == 16
    assert info[3][0]["kernel"] == "classes" and info[3][0]["xstaged"] and info[4][0]["kernel"] == "vector"
    levels = oracle_levels_from_gpu(mg, "jacobi")
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import splitmix_uniform
    b = splitmix_uniform(A.nrows, 42)
    omg = O.Multigrid(levels)
    omg.set_parallel(16)
    zref = omg.apply(b)
    z = apply_dev(ctx, mg, b, A.nrows)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    x = torch.zeros(A.nrows, dtype=torch.float64, device="cuda:0")
    it, hist = fa().stationary_solve(A, mg, T(b), x, max_iter=11, rel_tol=1e-300)
    OA = levels[0]["A"]
    _, it_o, hist_o = O.stationary_solve(OA, omg, b, max_iter=11, rel_tol=1e-300)
    assert it == it_o == 11
    floor = EPS * 12.0 * np.max(np.abs(H(x))) / np.max(np.abs(b))  # ||A||_inf = 12
    assert np.all(np.abs(hist - hist_o) <= 1e-8 * hist_o + floor), (hist, hist_o)


@pytest.mark.timeout(900)
def test_vcycle_256_27pt_sgs(ctx):
    """Config C3 itself (27-pt anisotropic 256^3, SA 2^3 boxes, multicolour SGS
    on the fine level -- the fused plane-parity phases of sgs27.hip -- L1 on the
    Galerkin levels, Cholesky coarsest) against the oracle on the same
    hierarchy (verdict r03 item 2): one V-cycle to 1e-11 and 10 stationary
    cycles (rho_k) to 1e-8 (+ the fp64 noise floor of a computed residual)."""
    import sys
    import torch
    dims = (256, 256, 256)
    A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=1000, smoother="sgs")
    S0 = mg.level(0)[1]
    assert S0.kind == "sgs" and fa().sgs_fused(S0)  # the fused phases are what runs
    assert sum(1 for p in mg.cycle_plan() if p["name"] == "sgs27_phase") in (6, 8)
    levels = oracle_levels_from_gpu(mg, "sgs")
    assert levels[0]["smoother"] == "sgs"
    sys.path.insert(0, GOLD)
    from make_golden import splitmix_uniform
    b = splitmix_uniform(A.nrows, 42)
    omg = O.Multigrid(levels)
    omg.set_parallel(16)
    zref = omg.apply(b)
    z = apply_dev(ctx, mg, b, A.nrows)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    x = torch.zeros(A.nrows, dtype=torch.float64, device="cuda:0")
    it, hist = fa().stationary_solve(A, mg, T(b), x, max_iter=11, rel_tol=1e-300)
    OA = levels[0]["A"]
    _, it_o, hist_o = O.stationary_solve(OA, omg, b, max_iter=11, rel_tol=1e-300)
    assert it == it_o == 11
    rp, _, val = A.arrays()
    a_inf = float(np.max(np.add.reduceat(np.abs(val), rp[:-1])))
    floor = EPS * a_inf * np.max(np.abs(H(x))) / np.max(np.abs(b))
    assert np.all(np.abs(hist - hist_o) <= 1e-8 * hist_o + floor), (hist, hist_o)


@pytest.mark.parametrize("window", [-1, 0, 64])
def test_random_7pt_generator_and_spmv(ctx, window):
    """The general operator of roofline.general (random coefficients, symmetric
    permutation) against its restatement, and its SpMV bitwise in both the
    SELL (i32 / u16 columns, fp64 values) and the CSR-stream storage."""
    import sa_oracle as SO
    dims = (11, 9, 7)
    A = fa().SparseMatOp.random7(ctx, *dims, seed=5, window=window)
    R = SO.random_7pt(*dims, seed=5, window=window)
    rp, ci, va = A.arrays()
    assert np.array_equal(rp, R.indptr) and np.array_equal(ci, R.indices) and np.array_equal(va, R.data)
    assert abs(R - R.T).max() == 0
    if window != -1:
        assert len(np.unique(R.tocoo().col - R.tocoo().row)) > 50  # no stencil structure
    x = np.random.default_rng(3).standard_normal(R.shape[0])
    OA = O.Csr.from_scipy(R)
    for fmt in ("sell", "csr"):
        fa().set_spmv_format(fmt)
        try:
            M = fa().SparseMatOp.random7(ctx, *dims, seed=5, window=window)
        finally:
            fa().set_spmv_format("auto")
        assert np.array_equal(apply_dev(ctx, M, x, R.shape[0]), OA.spmv(x)), fmt


def test_xsell_general_operator(ctx):
    """x-staged SELL (xsell.hip): the random-coefficient 7-pt operator with rows
    shuffled within windows of 4096 stages each 4096-row group's x chunks in LDS
    (auto policy, >= 512 groups); SpMV bitwise equal to the oracle and to
    SELL-64 (ragged last group: 2^21 - 3096 rows), and a V-cycle on it
    (residual and Jacobi epilogues on xsell; with the zero-guess fold the
    staged d*x residual) within 1e-11 of the restatement, fold on and off
    bitwise equal.  The fully shuffled operator escapes the LDS budget and keeps
    SELL-64."""
    import scipy.sparse as sp
    dims = (128, 128, 128)
    A = fa().SparseMatOp.random7(ctx, *dims, seed=9, window=4096)
    info = A.spmv_info()
    assert info["kernel"] == "xsell" and info["slices_u16"] > 0, info
    # the generator itself is checked against its restatement at small size
    # (test_random_7pt_generator_and_spmv); here its arrays feed the oracle
    n = A.nrows
    rp, ci, va = A.arrays()
    R = sp.csr_matrix((va, ci, rp), shape=(n, n))
    OA = O.Csr.from_arrays(n, n, rp, ci, va)
    x = np.random.default_rng(4).standard_normal(R.shape[0])
    y = apply_dev(ctx, A, x, R.shape[0])
    assert np.array_equal(y.view(np.int64), OA.spmv(x).view(np.int64))
    fa().set_spmv_format("sell")
    try:
        S = fa().SparseMatOp.random7(ctx, *dims, seed=9, window=4096)
    finally:
        fa().set_spmv_format("auto")
    assert S.spmv_info()["kernel"] == "sell"
    assert np.array_equal(apply_dev(ctx, S, x, R.shape[0]).view(np.int64), y.view(np.int64))
    # ragged: rows not a multiple of the group (and of the slice)
    Rr = R[:R.shape[0] - 3096, :R.shape[0] - 3096].tocsr()
    Ar = fa().SparseMatOp.from_scipy(ctx, Rr)
    assert Ar.spmv_info()["kernel"] == "xsell"
    xr = x[:Rr.shape[0]]
    assert np.array_equal(apply_dev(ctx, Ar, xr, Rr.shape[0]).view(np.int64),
                          O.Csr.from_scipy(Rr).spmv(xr).view(np.int64))
    # V-cycle: two levels, piecewise-constant interpolation over blocks of 4096
    # rows (box aggregates of the index grid blow up on a permuted operator)
    nc = n // 4096
    Pm = sp.csr_matrix((np.ones(n), np.arange(n) // 4096, np.arange(n + 1)), shape=(n, nc))
    P = fa().SparseMatOp.from_scipy(ctx, Pm)
    Rt = fa().transpose(P)
    Ac = fa().galerkin_rap(Rt, A, P)
    mg = fa().Multigrid(A, fa().new_jacobi(A, 0.66))
    mg.add_level(Ac, fa().CoarseCholesky(Ac), Rt, P)
    assert mg.level(0)[0].spmv_info()["kernel"] == "xsell"
    b = np.random.default_rng(5).uniform(-1, 1, R.shape[0])
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    zs = []
    for fold in (True, False):
        mg.set_fold_zero_guess(fold)
        zs.append(apply_dev(ctx, mg, b, R.shape[0]))
        assert np.linalg.norm(zs[-1] - zref) <= 1e-11 * np.linalg.norm(zref)
    assert np.array_equal(zs[0].view(np.int64), zs[1].view(np.int64))
    Rw = fa().SparseMatOp.random7(ctx, *dims, seed=9, window=0)
    assert Rw.spmv_info()["kernel"] == "sell"


def test_xsell_pipelined_kernel_bitwise(ctx):
    """The burst x-staged SELL kernel (flag xs_pipe = 2, the default: LDS-DMA
    staging) and the pipelined one (1) against the round-4 kernel (0) and the
    oracle: every epilogue bitwise, on
    an operator with escape slices (a few rows given one far column each: their
    slices keep 32-bit global columns) and an all-empty slice (64 empty rows:
    one padding step)."""
    import scipy.sparse as sp
    dims = (128, 128, 128)
    A0 = fa().SparseMatOp.random7(ctx, *dims, seed=11, window=4096)
    n = A0.nrows
    rp, ci, va = A0.arrays()
    R = sp.csr_matrix((va, ci, rp), shape=(n, n)).tolil()
    rng = np.random.default_rng(12)
    # 40 slices in 40 groups escape (< 1/16 of 32768): 32 far columns each, in 32
    # distinct x chunks, push the group past the 320 staged chunks (its own
    # footprint is ~300) and the least referenced (these) stay out
    far = rng.choice(n // 4096, size=40, replace=False) * 4096 + 64 * rng.integers(0, 64, 40)
    for r in far:
        for j in range(32):
            R[r + j, (r + n // 2 + 64 * j) % n] = 0.25
    R = R.tocsr()
    e0 = 64 * 1000  # slice 1000: 64 empty rows
    Rl = R.tolil()
    for r in range(e0, e0 + 64):
        Rl.rows[r] = []
        Rl.data[r] = []
    R = Rl.tocsr()
    A = fa().SparseMatOp.from_scipy(ctx, R)
    info = A.spmv_info()
    assert info["kernel"] == "xsell" and info["slices_i32"] > 0, info
    x = rng.standard_normal(n)
    b = rng.standard_normal(n)
    d = rng.uniform(0.1, 0.2, n)
    OA = O.Csr.from_scipy(R)
    xd, bd, dd = T(x), T(b), T(d)
    outs = {}
    try:
        for pipe in (0, 1, 2):
            fa().set_flag("xs_pipe", pipe)
            for mode in ("set", "add", "resid", "jacobi"):
                y = T(np.linspace(-1, 1, n))
                A.spmv_epilogue(mode, xd, y, bd, dd)
                ctx.synchronize()
                outs[(pipe, mode)] = H(y)
    finally:
        fa().set_flag("xs_pipe", 2)
    for mode in ("set", "add", "resid", "jacobi"):
        for pipe in (1, 2):
            assert np.array_equal(outs[(0, mode)].view(np.int64), outs[(pipe, mode)].view(np.int64)), (mode, pipe)
    ax = OA.spmv(x)
    assert np.array_equal(outs[(2, "set")].view(np.int64), ax.view(np.int64))
    assert np.all(outs[(2, "set")][e0:e0 + 64] == 0.0)
    assert np.array_equal(outs[(2, "resid")], b - ax)
    assert np.array_equal(outs[(2, "add")], np.linspace(-1, 1, n) + ax)
    assert np.array_equal(outs[(2, "jacobi")], x + d * (b - ax))


def test_sgs_dia_sweeps(ctx):
    """Color sweeps of a constant-stencil operator run on DIA codes of the
    color-permuted copy (diagonals taken against the original row): the same
    row sums in the same order as the SELL sweeps (bitwise equal to them) and
    within 1e-13 of the oracle's SGS; the 27-pt V-cycle within 1e-11."""
    dims = (48, 48, 32)  # >= 64K rows: DIA storage applies
    OA = O.aniso27(*dims)
    A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    S = fa().SymGaussSeidel(A)
    st = fa().sgs_info(S)
    assert st["colors"] == 8 and st["kernel"] == "dia" and st["diagonals"] == 27, st
    fa().set_value_codes(False)  # no value table: the SELL sweeps
    try:
        S2 = fa().SymGaussSeidel(A)
    finally:
        fa().set_value_codes(True)
    assert fa().sgs_info(S2)["kernel"] != "dia"
    r = np.random.default_rng(8).standard_normal(OA.nrows)
    e = apply_dev(ctx, S, r, OA.nrows)
    e2 = apply_dev(ctx, S2, r, OA.nrows)
    assert np.array_equal(e, e2)
    color, nc = O.greedy_coloring(OA)
    eref = O.sgs_apply(OA, color, nc, r)
    assert np.linalg.norm(e - eref) <= 1e-13 * np.linalg.norm(eref)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
    assert fa().sgs_info(mg.level(0)[1])["kernel"] == "dia"
    levels = oracle_levels_from_gpu(mg, "sgs")
    b = np.random.default_rng(9).uniform(-1, 1, OA.nrows)
    zref = O.Multigrid(levels).apply(b)
    for resid_form in (False, True):
        mg.set_sgs_residual_form(resid_form)
        z = apply_dev(ctx, mg, b, OA.nrows)
        assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref), resid_form
    mg.set_sgs_residual_form(False)



def test_sellp_dense_coarse_levels(ctx):
    """Pattern SELL with L lanes per row on a dense fp64 Galerkin level (level 2
    of a 64^3 SA hierarchy, value codes off): SpMV within the summation-order
    bound of the oracle, the V-cycle within 1e-11 of the oracle."""
    dims = (64, 64, 64)
    fa().set_value_codes(False)
    try:
        A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    finally:
        fa().set_value_codes(True)
    A2 = mg.level(2)[0]
    info = A2.spmv_info()
    assert info["kernel"] == "sellp" and info["value_bits"] == 0, info
    OA2 = O.Csr.from_arrays(*A2.dims(), *A2.arrays())
    x = np.random.default_rng(32).standard_normal(A2.ncols)
    y = apply_dev(ctx, A2, x, A2.nrows)
    assert np.all(np.abs(y - OA2.spmv(x)) <= spmv_bound(OA2.to_scipy(), x))
    b = np.random.default_rng(31).uniform(-1, 1, A.nrows)
    z = apply_dev(ctx, mg, b, A.nrows)
    levels = oracle_levels_from_gpu(mg, "jacobi")
    zref = O.Multigrid(levels).apply(b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


def test_sellp_coded_transfer_operators(ctx):
    """Pattern SELL with 4-bit codes and per-row column bases (rectangular,
    implicit columns) on a synthetic structured interpolation P (20 entries per
    row around row // 16, four distinct values) and R = P^T: storage picked
    automatically, P and R (two and more lanes per row) within the
    summation-order bound of the oracle's row sums, and a two-level V-cycle on a DIA fine
    level within 1e-11 of the oracle with and without the zero-guess fold (P in
    ADD0, else ADD; R in SET)."""
    import scipy.sparse as sp
    dims = (50, 49, 31)  # 75950 rows: DIA fine level, not a multiple of 3 (no 3x3 blocks)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    nf = A.nrows
    nc = (nf + 15) // 16
    rows, cols, data = [], [], []
    for k in range(20):  # 1.0 on the row's own coarse column, small couplings around it
        i = np.arange(nf)
        c = i // 16 + k - 9
        ok = (c >= 0) & (c < nc)
        rows.append(i[ok]); cols.append(c[ok])
        data.append(np.full(ok.sum(), 1.0) if k == 9 else 0.125 * (1 + (i[ok] + k) % 3))
    Ps = sp.csr_matrix((np.concatenate(data), (np.concatenate(rows), np.concatenate(cols))), shape=(nf, nc))
    Ps.sort_indices()
    Rs = Ps.T.tocsr()
    Rs.sort_indices()
    P = fa().SparseMatOp.from_scipy(ctx, Ps)
    R = fa().SparseMatOp.from_scipy(ctx, Rs)
    for M in (P, R):
        info = M.spmv_info()
        assert info["kernel"] == "sellp" and info["value_bits"] == 4, info
    rng = np.random.default_rng(77)
    OP, OR = O.Csr.from_scipy(Ps), O.Csr.from_scipy(Rs)
    xc = rng.standard_normal(nc)
    yp = apply_dev(ctx, P, xc, nf)
    assert np.all(np.abs(yp - OP.spmv(xc)) <= spmv_bound(Ps, xc))
    xf = rng.standard_normal(nf)
    yr = apply_dev(ctx, R, xf, nc)
    assert np.all(np.abs(yr - OR.spmv(xf)) <= spmv_bound(Rs, xf))
    assert A.spmv_info()["kernel"] == "dia"
    As = A.to_scipy()
    Acs = (Rs @ As @ Ps).tocsr()
    Acs.sort_indices()
    Ac = fa().SparseMatOp.from_scipy(ctx, Acs)
    mg = fa().Multigrid(A, fa().new_jacobi(A, 0.66))
    mg.add_level(Ac, fa().CoarseCholesky(Ac), R, P)
    levels = [{"A": O.Csr.from_scipy(As), "smoother": "jacobi", "R": OR, "P": OP},
              {"A": O.Csr.from_scipy(Acs), "smoother": "chol"}]
    b = rng.uniform(-1, 1, nf)
    zref = O.Multigrid(levels).apply(b)
    for fold in (True, False):
        mg.set_fold_zero_guess(fold)
        z = apply_dev(ctx, mg, b, nf)
        assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref), fold


def test_stencil_classes(ctx):
    """Stencil-class storage (one class id per row, a dictionary of the distinct
    rows up to a shift) on A_2 of a 128^3 SA hierarchy (32^3 rows, 13^3 boundary
    classes): SpMV bitwise equal to the oracle's row sums (ascending offsets with
    exact zero terms), every row's class reproduces its CSR row, and the V-cycle
    through it (RESID / JACOBI epilogues) within 1e-11 of the oracle."""
    dims = (128, 128, 128)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    A2 = mg.level(2)[0]
    info = A2.spmv_info()
    assert info["kernel"] == "classes" and info["classes"] == 2197, info
    assert info["class_offsets"] >= 179 and info["class_id_bits"] == 16
    assert info["stream_bytes"] < 0.5 * 12 * A2.nnz
    OA2 = O.Csr.from_arrays(*A2.dims(), *A2.arrays())
    x = np.random.default_rng(41).standard_normal(A2.ncols)
    assert np.array_equal(apply_dev(ctx, A2, x, A2.nrows), OA2.spmv(x))
    b = np.random.default_rng(42).uniform(-1, 1, A.nrows)
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    z = apply_dev(ctx, mg, b, A.nrows)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


def _epilogues_bitwise(ctx, M, seed):
    """The four SpMV epilogues of M (amg_csr_spmv_epilogue) against the oracle's
    row sums: y = A x, y += A x, y = b - A x, y = x + d (b - A x), bitwise."""
    OM = O.Csr.from_arrays(*M.dims(), *M.arrays())
    rng = np.random.default_rng(seed)
    m, n = M.dims()
    x, y0, b, d = rng.standard_normal(n), rng.standard_normal(m), rng.standard_normal(m), rng.uniform(0.1, 1, m)
    ax = OM.spmv(x)
    want = {"set": ax, "add": y0 + ax, "resid": b - ax, "jacobi": x + d * (b - ax)}
    for mode, ref in want.items():
        yd = T(y0)
        M.spmv_epilogue(mode, T(x), yd, T(b), T(d))
        assert np.array_equal(H(yd), ref), (mode, M.spmv_info())


@pytest.mark.parametrize("gen", ["27pt", "7pt"])
@pytest.mark.parametrize("dims", [(66, 40, 33), (48, 45, 41)])
def test_dia27_constant_stencil_bitwise(ctx, dims, gen):
    """Constant stencils truncated at the grid faces (aniso27, the 7-point
    Laplacian) on DIA storage run without codes (spmv_dia_pat_kernel /
    spmv_dia_kernel CST: the interior coefficients, x operands outside the grid
    taken as 0.0): all four epilogues bitwise equal to the oracle's row sums, odd
    y/z extents included; the folded and constant-diagonal epilogues of the 7-point
    kernel inside a V-cycle are covered by test_constant_diagonal_epilogues_bitwise."""
    A = (fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01) if gen == "27pt"
         else fa().SparseMatOp.laplace3d_7pt(ctx, *dims))
    if A.spmv_info()["kernel"] != "dia":
        pytest.skip("operator not stored as DIA codes")
    _epilogues_bitwise(ctx, A, 77)


def test_xstaged_stencil_classes(ctx):
    """x-staged stencil classes (scs.hip spmv_xscs_kernel): the coarse operators
    of box hierarchies on a grid (7-pt 128^3: A_2 = 32^3 with 13^3 classes and
    A_3; 27-pt 64^3: A_1 = 32^3 with 125 offsets and 8-bit values) carry the
    grid hint and run one workgroup per grid tile with the tile's x window in
    LDS.  All four SpMV epilogues bitwise equal to the oracle's row sums; a
    wrong grid hint (nonzeros that would leave the grid) is refused and the
    storage falls back; the V-cycle within 1e-11 of the oracle."""
    seen = 0
    for gen, dims, smoother in (("laplace3d_7pt", (128, 128, 128), "jacobi"), ("aniso27", (64, 64, 64), "jacobi")):
        A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if gen == "laplace3d_7pt"
             else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
        for l in range(1, mg.levels() - 1):
            Al = mg.level(l)[0]
            info = Al.spmv_info()
            g = tuple(-(-d // 2 ** l) for d in dims)
            assert info["grid"] == g, (l, info)
            if info["xstaged"]:
                seen += 1
                _epilogues_bitwise(ctx, Al, 100 + l)
                keep = (Al, g)
        b = np.random.default_rng(42).uniform(-1, 1, A.nrows)
        zref = O.Multigrid(oracle_levels_from_gpu(mg, smoother)).apply(b)
        z = apply_dev(ctx, mg, b, A.nrows)
        assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    assert seen >= 2, seen
    # a grid hint the operator does not fit (nonzeros leave the grid): refused
    A1, g = keep
    assert A1.spmv_info()["xstaged"]
    A1.set_grid(g[0] // 2, g[1] * 2, g[2])
    assert not A1.spmv_info()["xstaged"]
    x = np.random.default_rng(7).standard_normal(A1.ncols)
    ref = O.Csr.from_arrays(*A1.dims(), *A1.arrays()).spmv(x)
    y = apply_dev(ctx, A1, x, A1.nrows)  # the fallback storage (its kernel may split rows over lanes)
    assert np.max(np.abs(y - ref)) <= 1e-12 * np.max(np.abs(ref))
    A1.set_grid(0, 0, 0)
    assert A1.spmv_info()["grid"] == (0, 0, 0) and not A1.spmv_info()["xstaged"]


def test_xstaged_classes_fold_zero_guess(ctx, no_tail):
    """The zero-guess smoothing step folded on x-staged stencil-class levels
    (RESID0 stages d*f with the x window, ADD0 writes d*f + P v_c): the plan
    shows RESID0/ADD0 and no d*f pass on those levels, the V-cycle is bitwise
    the unfolded one (the staged products are vec_mul's) and within 1e-11 of
    the oracle.  (Off by default -- measured slower on the C2 cycle -- so the
    test switches it on with amg_set_flag, read whenever the library lays out
    a cycle.)"""
    dims = (128, 128, 128)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    fa().set_flag("fold_xscs", 1)  # off by default (measured slower)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    xs = [l for l in range(1, mg.levels() - 1) if mg.level(l)[0].spmv_info()["xstaged"]]
    assert xs, "no x-staged level"
    plan = mg.cycle_plan()
    for l in xs:
        modes = [p["mode"] for p in plan if p["level"] == l]
        assert modes[0] == "RESID0" and "ADD0" in modes and "-" not in modes, (l, modes)
    b = np.random.default_rng(21).uniform(-1, 1, A.nrows)
    outs = {}
    for fold in (True, False):
        mg.set_fold_zero_guess(fold)
        outs[fold] = apply_dev(ctx, mg, b, A.nrows)
    mg.set_fold_zero_guess(True)
    fa().set_flag("fold_xscs", 0)
    assert np.array_equal(outs[True].view(np.int64), outs[False].view(np.int64))
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    assert np.linalg.norm(outs[True] - zref) <= 1e-11 * np.linalg.norm(zref)


def _smoother_diag(ctx, S, n):
    """d of a Diag smoother (S applied to ones)."""
    import torch
    out = torch.empty(n, dtype=torch.float64, device="cuda:0")
    S.apply(out, T(np.ones(n)))
    return H(out)


@pytest.mark.parametrize("gen,dims", [("7pt", (64, 48, 40)), ("7pt", (67, 45, 39)), ("27pt", (48, 40, 36))])
def test_grid_transfer_classes(ctx, gen, dims):
    """gtc.hip: R and P of a 2x2x2-box hierarchy stored as grid-transfer classes
    (one 8-bit class per row, the coarse / fine window of a grid tile in LDS):
    y = P v_c, y += P v_c and f_c = R r bitwise equal to the oracle's row sums on
    every level that takes the storage, odd extents included; the V-cycle (which
    folds the zero-guess step into P's d*f + P v_c epilogue on the fine level)
    within 1e-11 of the oracle."""
    A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if gen == "7pt"
         else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    seen = 0
    rng = np.random.default_rng(3)
    for l in range(mg.levels() - 1):
        _, _, R, P = mg.level(l)
        for M in (R, P):
            if M.spmv_info()["kernel"] != "gtc":
                continue
            seen += 1
            OM = O.Csr.from_arrays(*M.dims(), *M.arrays())
            m, n = M.dims()
            x, y0 = rng.standard_normal(n), rng.standard_normal(m)
            assert np.array_equal(apply_dev(ctx, M, x, m), OM.spmv(x)), (l, M.dims())
            if m > n:  # P: the interpolate-add epilogue
                yd = T(y0)
                M.spmv_epilogue("add", T(x), yd)
                assert np.array_equal(H(yd), y0 + OM.spmv(x))
    assert seen >= 2, seen
    assert mg.level(0)[3].spmv_info()["kernel"] == "gtc"
    b = np.random.default_rng(42).uniform(-1, 1, A.nrows)
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    z = apply_dev(ctx, mg, b, A.nrows)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


@pytest.mark.parametrize("gen,dims", [("7pt", (64, 48, 40)), ("27pt", (40, 36, 33)), ("7pt", (45, 37, 29))])
def test_wide_grid_transfer_classes(ctx, gen, dims, no_tail):
    """gtx.hip: R and P of the box levels the 8-bit classes cannot take (levels
    >= 1: thousands of classes, steps up to {-5,..,6}^3) as 16-bit classes over a
    global dictionary of (window offset, value) entries: y = P v_c, y += P v_c
    and f_c = R r bitwise equal to the oracle's row sums on every such level,
    odd extents included.  The restriction's SETDF epilogue (f_c and the next
    level's first Jacobi step d f_c in one launch) leaves the V-cycle bitwise
    the one with the separate d*f pass, and within 1e-11 of the oracle."""
    A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if gen == "7pt"
         else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
    fa().set_flag("gtx_time", 0)  # take the classes wherever they build (these levels are small)
    try:
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=60)
    finally:
        fa().set_flag("gtx_time", 2)
    seen = set()
    rng = np.random.default_rng(4)
    for l in range(mg.levels() - 1):
        _, _, R, P = mg.level(l)
        for w, M in (("R", R), ("P", P)):
            if M.spmv_info()["gtc_kind"] != "gtx":
                continue
            seen.add((l, w))
            OM = O.Csr.from_arrays(*M.dims(), *M.arrays())
            m, n = M.dims()
            x, y0 = rng.standard_normal(n), rng.standard_normal(m)
            assert np.array_equal(apply_dev(ctx, M, x, m), OM.spmv(x)), (l, w)
            if w == "P":
                yd = T(y0)
                M.spmv_epilogue("add", T(x), yd)
                assert np.array_equal(H(yd), y0 + OM.spmv(x)), (l, w)
    assert (1, "R") in seen and (1, "P") in seen, seen
    b = np.random.default_rng(43).uniform(-1, 1, A.nrows)
    plan = mg.cycle_plan()
    assert any(p["mode"] == "SETDF" for p in plan), [(p["level"], p["name"], p["mode"]) for p in plan]
    z = apply_dev(ctx, mg, b, A.nrows)
    mg.set_restrict_df(False)
    z0 = apply_dev(ctx, mg, b, A.nrows)
    plan0 = mg.cycle_plan()
    mg.set_restrict_df(True)
    assert not any(p["mode"] == "SETDF" for p in plan0)
    assert len(plan0) > len(plan)  # the d*f passes the SETDF epilogue absorbed
    assert np.array_equal(z.view(np.int64), z0.view(np.int64))
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


@pytest.mark.parametrize("gen,dims,smoother", [("7pt", (64, 48, 40), "jacobi"), ("27pt", (48, 40, 33), "l1"),
                                               ("27pt", (48, 40, 33), "sgs")])
def test_gtc_restrict_setdf(ctx, gen, dims, smoother):
    """The 8-bit grid-transfer restriction (R_0 of a box hierarchy) with the SETDF
    epilogue: f_1 and level 1's first Jacobi-type step from zero d_1 f_1 in one
    launch.  The cycle is bitwise the one with the separate d*f pass (coded,
    constant and fp64 diagonals of the level-1 smoother), one launch shorter per
    such level, and within 1e-11 of the oracle's cycle."""
    # (the 7-point fine level otherwise runs fused with its residual, fine.hip:
    # test_fine_fused_bitwise; here the grid-transfer restriction itself)
    fa().set_flag("fine_fuse", 0)
    try:
        A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if gen == "7pt"
             else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
        mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=60, smoother=smoother)
        assert mg.level(0)[2].spmv_info()["gtc_kind"] == "gtc"
        plan = mg.cycle_plan()
        assert any(p["mode"] == "SETDF" and p["level"] == 0 for p in plan), [(p["level"], p["name"], p["mode"])
                                                                           for p in plan]
        b = np.random.default_rng(44).uniform(-1, 1, A.nrows)
        z = apply_dev(ctx, mg, b, A.nrows)
        mg.set_restrict_df(False)
        try:
            z0 = apply_dev(ctx, mg, b, A.nrows)
            plan0 = mg.cycle_plan()
        finally:
            mg.set_restrict_df(True)
    finally:
        fa().set_flag("fine_fuse", 1)
    assert not any(p["mode"] == "SETDF" for p in plan0)
    assert len(plan0) > len(plan)
    assert np.array_equal(z.view(np.int64), z0.view(np.int64))
    zref = O.Multigrid(oracle_levels_from_gpu(mg, smoother)).apply(b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)


def test_constant_diagonal_epilogues_bitwise(ctx):
    """The 7-point Laplacian's Jacobi diagonal is one value (a_ii = 6): the DIA
    JACOBI / folded RESID0 epilogues and the grid-transfer ADD0 read it as one
    scalar (dt[0]) instead of 1-B codes per row / per gathered column.  The
    V-cycle is bitwise the coded path's (FAMG_DIA_DK=0) and the plan charges
    no code bytes on the fine level (RESID0 16 n + format, JACOBI 24 n +
    format)."""
    import torch
    dims = (64, 64, 64)
    b = T(np.random.default_rng(3).uniform(-1, 1, int(np.prod(dims))))
    outs, plans = {}, {}
    for dk in ("1", "0"):
        fa().set_flag("dia_dk", int(dk))
        try:
            A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
            mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
            mg.set_graph(False)
            z = torch.empty_like(b)
            mg.apply(z, b)
            ctx.synchronize()
            outs[dk] = H(z)
            plans[dk] = [p for p in mg.cycle_plan() if p["level"] == 0]
        finally:
            fa().set_flag("dia_dk", 1)
    assert np.array_equal(outs["1"].view(np.int64), outs["0"].view(np.int64))
    n = int(np.prod(dims))
    if any(p["name"].startswith("fine-") for p in plans["1"]):
        return  # the one-value d runs the fused fine-level kernels (test_fine_fused_bitwise)
    by = {p["mode"]: p["bytes"] for p in plans["1"]}
    by0 = {p["mode"]: p["bytes"] for p in plans["0"]}
    if "RESID0" in by and A.spmv_info()["kernel"] == "dia":
        assert by0["RESID0"] - by["RESID0"] == n and by0["JACOBI"] - by["JACOBI"] == n, (by, by0)


def test_cycle_plan_accounts_for_every_launch(ctx):
    """amg_multigrid_cycle_plan: the launches of one V-cycle as the library makes
    them.  On the 7-pt box hierarchy the fine level folds its zero-guess step
    (RESID0 + ADD0, no separate d*f pass) when the fine operator is DIA and P_0
    runs the short-slice kernel; with the fold off the level issues the d*f pass,
    RESID and ADD instead.  The coarsest level is one GEMV of 8 n^2 + 16 n bytes.
    The plan's launch count equals the dispatches of a replayed cycle (the bench
    checks the same against the rocprofv3 trace)."""
    dims = (64, 64, 64)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    plan = mg.cycle_plan()
    nl = mg.levels()
    # the last level in the plan is the coarsest or the dense tail (the first level
    # l >= 1 of <= 4096 rows above it: one GEMV of 8 n_l^2 + 16 n_l bytes for l..L-1)
    lt = max(p["level"] for p in plan)
    assert lt == nl - 1 or (lt >= 1 and mg.level(lt)[0].nrows <= 4096 < mg.level(lt - 1)[0].nrows), lt
    assert {p["level"] for p in plan} == set(range(lt + 1))
    coarse = [p for p in plan if p["role"] == "coarse"]
    n_c = mg.level(lt)[0].nrows
    assert len(coarse) == 1 and coarse[0]["name"] == "gemv" and coarse[0]["bytes"] == 8 * n_c * n_c + 16 * n_c
    for p in plan:
        assert p["bytes"] > 0 and p["csr_bytes"] >= p["bytes"] or p["kernel"] in (-1, 4, 7)
    f0 = [p for p in plan if p["level"] == 0]
    modes0 = [p["mode"] for p in f0]
    info = A.spmv_info()
    n = A.nrows
    # the restriction is SETDF where it also writes level 1's first step d_1 f_1
    rmode = "SETDF" if any(p["mode"] == "SETDF" for p in f0) else "SET"
    names0 = [p["name"] for p in f0]
    if "fine-pj" in names0:
        # folded, with d f + P v_c and the post-smoothing Jacobi step as one
        # marching launch (fine.hip): f, v_c and z cross HBM once
        assert modes0[-1] == "-" and names0[-1] == "fine-pj", f0
        assert f0[-1]["bytes"] == 17 * n + 8 * mg.level(1)[0].nrows, f0[-1]
        assert modes0[:-1] in (["RESID0", rmode], ["-"]), f0
    elif "RESID0" in modes0:
        # folded: RESID0 (f - A d f), R, ADD0 (d f + P v_c), post-smoothing Jacobi
        assert modes0 == ["RESID0", rmode, "ADD0", "JACOBI"], f0
        if info["kernel"] == "dia":  # 16 n: f read, r written; d = 6/omega everywhere is one scalar
            assert f0[0]["bytes"] == info["stream_bytes"] + 16 * n, f0[0]
    else:
        # d*f pass, residual, restriction, interpolate-add, post-smoothing Jacobi
        assert modes0 == ["-", "RESID", rmode, "ADD", "JACOBI"], f0
        assert f0[1]["bytes"] == info["stream_bytes"] + 24 * n, f0[1]
    mg.set_fold_zero_guess(False)
    plan2 = mg.cycle_plan()
    modes_nf = [p["mode"] for p in plan2 if p["level"] == 0]
    assert "RESID0" not in modes_nf and "ADD0" not in modes_nf
    assert modes_nf[0] == "-" and modes_nf[1] == "RESID"  # d*f pass, then the residual
    # results are unchanged by recording
    import torch
    b = T(np.random.default_rng(0).uniform(-1, 1, A.nrows))
    z1, z2 = torch.empty_like(b), torch.empty_like(b)
    mg.apply(z1, b)
    mg.cycle_plan()
    mg.apply(z2, b)
    ctx.synchronize()
    assert torch.equal(z1, z2)


def test_cycle_plan_sgs_counts_colour_launches(ctx):
    """SGS levels: 1 + (C - 1) + (C - 1) launches for the pre-smoothing from zero
    (first colour pass, forward, backward) and 2 C - 1 for the fused post sweep."""
    dims = (32, 32, 32)
    A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100, smoother="sgs")
    plan = mg.cycle_plan()
    S0 = mg.level(0)[1]
    C = fa().sgs_info(S0)["colors"]
    sweeps = [p for p in plan if p["level"] == 0 and p["mode"] == "SGS"]
    assert len(sweeps) == (C - 1) + (C - 1) + (2 * C - 1), (len(sweeps), C)


@pytest.mark.parametrize("dims", [(48, 48, 32), (50, 45, 37), (64, 40, 33), (49, 48, 32), (65, 40, 33)])
def test_sgs27_fused_phases_bitwise(ctx, dims):
    """The fused plane-parity SGS phases (sgs27.hip: three launches per SGS step
    -- the odd planes' forward and backward colours in one -- or four, in-plane
    colours on shrinking LDS halos) against the colour launches (fifteen per
    step): bitwise equal for the step from e = 0 (the smoother's apply) and
    inside the V-cycle (pre-smoothing from zero, post-smoothing on x), odd and
    even y/z extents; and within 1e-11 of the oracle's V-cycle.  An odd x
    extent (rows not 16-B aligned pairs) takes the colour launches: the test
    asserts that fallback and the same oracle bound."""
    OA = O.aniso27(*dims)
    A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    if A.spmv_info()["kernel"] != "dia":
        pytest.skip("operator not stored as DIA codes")
    S1 = fa().SymGaussSeidel(A)
    if dims[0] % 2:
        assert not fa().sgs_fused(S1)
        mg1 = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
        assert not fa().sgs_fused(mg1.level(0)[1])
        assert sum(1 for p in mg1.cycle_plan() if p["name"] == "sgs27_phase") == 0
        b = np.random.default_rng(9).uniform(-1, 1, OA.nrows)
        z1 = apply_dev(ctx, mg1, b, OA.nrows)
        zref = O.Multigrid(oracle_levels_from_gpu(mg1, "sgs")).apply(b)
        assert np.linalg.norm(z1 - zref) <= 1e-11 * np.linalg.norm(zref)
        return
    fa().set_sgs_fused(False)
    try:
        S0 = fa().SymGaussSeidel(A)
        mg0 = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
        fa().set_sgs_fused(2)
        S2 = fa().SymGaussSeidel(A)
        mg2 = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
        r2 = np.random.default_rng(8).standard_normal(OA.nrows)
        e2 = apply_dev(ctx, S2, r2, OA.nrows)
        b2 = np.random.default_rng(9).uniform(-1, 1, OA.nrows)
        z2 = apply_dev(ctx, mg2, b2, OA.nrows)
        plan2 = mg2.cycle_plan()
    finally:
        fa().set_sgs_fused(True)
    mg1 = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
    assert fa().sgs_fused(S1) and not fa().sgs_fused(S0)
    assert fa().sgs_fused(mg1.level(0)[1]) and not fa().sgs_fused(mg0.level(0)[1])
    r = np.random.default_rng(8).standard_normal(OA.nrows)
    e1 = apply_dev(ctx, S1, r, OA.nrows)
    e0 = apply_dev(ctx, S0, r, OA.nrows)
    assert np.array_equal(e1, e0)
    b = np.random.default_rng(9).uniform(-1, 1, OA.nrows)
    z1 = apply_dev(ctx, mg1, b, OA.nrows)
    z0 = apply_dev(ctx, mg0, b, OA.nrows)
    assert np.array_equal(z1, z0)
    assert np.array_equal(e2, e0) and np.array_equal(z2, z0)
    zref = O.Multigrid(oracle_levels_from_gpu(mg1, "sgs")).apply(b)
    assert np.linalg.norm(z1 - zref) <= 1e-11 * np.linalg.norm(zref)
    plan = mg1.cycle_plan()
    # two SGS steps x three phases (four where the LDS-staged phases take the level)
    assert sum(1 for p in plan if p["name"] == "sgs27_phase") in (6, 8)
    assert sum(1 for p in plan2 if p["name"] == "sgs27_phase") == 8  # two SGS steps x four phases


@pytest.mark.parametrize("dims", [(64, 40, 33), (48, 48, 32), (96, 70, 29)])
def test_sgs27_marching_phases_bitwise(ctx, dims):
    """The marching SGS phases (sgs27.hip k_sgs27_march: a workgroup walks n
    planes of one parity, the other parity's planes rotating through two LDS
    slots, the next plane fetched into registers while the current one runs its
    colours) against the colour launches: bitwise for the step from e = 0 and
    inside the V-cycle, at 1 (no marching), 2, 3 and 5 planes per workgroup and
    the automatic choice -- runs that do not divide the plane count included."""
    A = fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01)
    if A.spmv_info()["kernel"] != "dia":
        pytest.skip("operator not stored as DIA codes")
    n = dims[0] * dims[1] * dims[2]
    r = np.random.default_rng(8).standard_normal(n)
    b = np.random.default_rng(9).uniform(-1, 1, n)
    fa().set_sgs_fused(False)
    try:
        e0 = apply_dev(ctx, fa().SymGaussSeidel(A), r, n)
        z0 = apply_dev(ctx, fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs"), b, n)
    finally:
        fa().set_sgs_fused(True)
    S1 = fa().SymGaussSeidel(A)
    mg1 = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500, smoother="sgs")
    assert fa().sgs_fused(S1)
    try:
        for v in (0, 2, 3, 5, 1):
            fa().set_flag("sgs27_march", v)
            assert np.array_equal(apply_dev(ctx, S1, r, n), e0), v
            assert np.array_equal(apply_dev(ctx, mg1, b, n), z0), v
    finally:
        fa().set_flag("sgs27_march", 1)


def _spmm_vs_spmv(ctx, A, ks=(1, 3, 8, 32), seed=0):
    """Y = A X (k columns, leading dimensions > n) against k single-vector applies: bitwise."""
    import torch
    m, n = A.dims()
    rng = np.random.default_rng(seed)
    for k in ks:
        X = _colmajor(rng, n, k, 3)
        Y = _colmajor(rng, m, k, 5)
        A.apply(Y, X)
        ctx.synchronize()
        for c in range(k):
            y1 = torch.empty(m, dtype=torch.float64, device="cuda:0")
            A.apply(y1, X[:, c].contiguous())
            ctx.synchronize()
            assert torch.equal(Y[:, c], y1), (A.spmv_info()["kernel"], k, c)


def test_spmm_compressed_storages(ctx):
    """f2 (adaptivity.rs:168-244,307-390): k-wide applies on the storages the
    hierarchies use -- DIA codes (7 diagonals; the 33-diagonal run pattern of A_1;
    the 27-point stencil), stencil classes (one row per lane on A_2, one row per
    wave on A_3) and 3x3 blocks (elasticity) -- each column bitwise equal to the
    single-vector kernel, k in {1, 3, 8, 32} (column groups of 8)."""
    seen = set()
    A7 = fa().SparseMatOp.laplace3d_7pt(ctx, 64, 64, 64)
    A27 = fa().SparseMatOp.aniso27(ctx, 48, 48, 32, 1.0, 1.0, 0.01)
    dims = (128, 128, 128)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500)
    mats = [A7, A27] + [mg.level(l)[0] for l in range(1, mg.levels() - 1)]
    H = fa().elasticity_q1((12, 10, 10), seed=3)
    mats.append(H.upload(ctx))
    for M in mats:
        info = M.spmv_info()
        seen.add((info["kernel"], info.get("classes", 0) > 0))
        _spmm_vs_spmv(ctx, M, ks=(1, 3, 8, 32) if M.nrows < 2_000_000 else (3, 8))
    kinds = {k for k, _ in seen}
    assert {"dia", "bsr"} <= kinds, seen


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(64, 64, 64), (70, 62, 50), (256, 128, 8)])
def test_dia7_row_pairs_bitwise(ctx, dims):
    """Constant 7-point DIA kernel with 2 / 4 row pairs per lane (flag dia7_rp,
    spmv_dia7c_kernel): every epilogue and the folded V-cycle (RESID0 / JACOBI
    with the one-value diagonal) bitwise the one-pair kernel's -- a ragged row
    count (70 x 62 x 50) and the 2.5-D band order (256 x 128 planes) included."""
    import torch
    n = int(np.prod(dims))
    rng = np.random.default_rng(5)
    x, b = T(rng.uniform(-1, 1, n)), T(rng.uniform(-1, 1, n))
    d = T(rng.uniform(0.1, 0.2, n))
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    assert A.spmv_info()["kernel"] == "dia"
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    outs = {}
    try:
        for rp in (1, 2, 4, 0):
            fa().set_flag("dia7_rp", rp)
            res = []
            for mode in ("set", "add", "resid", "jacobi"):
                y = torch.full_like(x, 0.5)
                A.spmv_epilogue(mode, x, y, b, d)
                ctx.synchronize()
                res.append(H(y))
            z = torch.empty_like(b)
            mg.apply(z, b)
            ctx.synchronize()
            res.append(H(z))
            outs[rp] = res
    finally:
        fa().set_flag("dia7_rp", 0)
    for rp in (2, 4, 0):
        for u, v in zip(outs[rp], outs[1]):
            assert np.array_equal(u.view(np.int64), v.view(np.int64)), rp


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(64, 64, 64), (66, 62, 50), (32, 48, 96), (256, 128, 8)])
def test_fine_fused_bitwise(ctx, dims):
    """The fine level of the constant 7-point box hierarchy as marching fused
    kernels (fine.hip, flag fine_fuse): the folded residual r = f - A d f with
    f_c = R r, d_c f_c in one launch (r in LDS), v = d f + P v_c with the
    post-smoothing Jacobi step in another (v in LDS).  The V-cycle is bitwise
    the four-launch cycle's (constant 7-point DIA RESID0, k_gtc_restrict_march
    SETDF, k_gtc_interp ADD0, the constant 7-point DIA JACOBI) for
    every run length of planes per workgroup -- ragged x/y tiles (66 x 62), odd
    coarse plane counts (50 -> 25) and chunk ends included -- and within 1e-11
    of the oracle."""
    import torch
    n = int(np.prod(dims))
    b = T(np.random.default_rng(11).uniform(-1, 1, n))
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    outs = {}
    try:
        for ff in (0, 1, 2, 6, 1000):
            fa().set_flag("fine_fuse", ff)
            z = torch.full_like(b, np.nan)
            mg.apply(z, b)
            ctx.synchronize()
            outs[ff] = H(z)
            names = [p["name"] for p in mg.cycle_plan() if p["level"] == 0]
            assert ("fine-pj" in names) == (ff != 0) and ("fine-rr" in names) == (ff != 0), (ff, names)
    finally:
        fa().set_flag("fine_fuse", 1)
    for ff in (1, 2, 6, 1000):
        assert np.array_equal(outs[ff].view(np.int64), outs[0].view(np.int64)), ff
    zref = O.Multigrid(oracle_levels_from_gpu(mg, "jacobi")).apply(H(b))
    assert np.linalg.norm(outs[1] - zref) <= 1e-11 * np.linalg.norm(zref)


def test_fine_timer_in_cycle(ctx):
    """amg_multigrid_set_fine_timer: HIP events around one fused fine-level launch
    inside the cycle (run eagerly while timed) -- a positive time per cycle, and
    the cycle's result bitwise the graph-replayed one."""
    import torch
    dims = (64, 64, 64)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100)
    mg.set_graph(True)
    b = T(np.random.default_rng(5).uniform(-1, 1, A.nrows))
    z0, z1 = torch.empty_like(b), torch.empty_like(b)
    mg.apply(z0, b)
    ctx.synchronize()
    for which in (0, 1):
        mg.set_fine_timer(which)
        try:
            for _ in range(3):
                mg.apply(z1, b)
                ms = mg.fine_timer_ms()
                assert 0.0 < ms < 100.0, ms
        finally:
            mg.set_fine_timer(-1)
        ctx.synchronize()
        assert torch.equal(z0, z1)


@pytest.mark.parametrize("dims,smoother", [((64, 64, 64), "jacobi"), ((48, 40, 36), "sgs")])
def test_dense_tail(ctx, dims, smoother):
    """The dense tail (ops.hip ensure_tail): with mu = 1 the part of the V-cycle
    from the first level of <= 4096 rows down maps that level's f to its v
    linearly, so the cycle takes one GEMV with the matrix of that map (built by
    running that part on the unit vectors) instead of its launches.  The cycle
    agrees with the one that runs every level to rounding (1e-13) and with the
    oracle (1e-11); the plan ends in one GEMV of 8 n^2 + 16 n bytes at that
    level, whose restriction then writes no d f; mu = 2 and the flag at 0 run
    every level."""
    import torch
    A = (fa().SparseMatOp.laplace3d_7pt(ctx, *dims) if smoother == "jacobi"
         else fa().SparseMatOp.aniso27(ctx, *dims, 1.0, 1.0, 0.01))
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=100, smoother=smoother)
    nl = mg.levels()
    ns = [mg.level(l)[0].nrows for l in range(nl)]
    lt = next(l for l in range(1, nl - 1) if ns[l] <= 4096)
    b = np.random.default_rng(61).uniform(-1, 1, A.nrows)
    plan = mg.cycle_plan()
    assert max(p["level"] for p in plan) == lt
    tail = [p for p in plan if p["level"] == lt]
    assert len(tail) == 1 and tail[0]["name"] == "gemv" and tail[0]["bytes"] == 8 * ns[lt] ** 2 + 16 * ns[lt]
    assert all(p["mode"] != "SETDF" for p in plan if p["level"] == lt - 1)
    z = apply_dev(ctx, mg, b, A.nrows)
    fa().set_flag("dense_tail", 0)
    try:
        z0 = apply_dev(ctx, mg, b, A.nrows)
        assert max(p["level"] for p in mg.cycle_plan()) == nl - 1
    finally:
        fa().set_flag("dense_tail", 4096)
    assert np.linalg.norm(z - z0) <= 1e-13 * np.linalg.norm(z0)
    zref = O.Multigrid(oracle_levels_from_gpu(mg, smoother)).apply(b)
    assert np.linalg.norm(z - zref) <= 1e-11 * np.linalg.norm(zref)
    # graph replay equals the eager cycle
    mg.set_graph(True)
    zg = torch.empty(A.nrows, dtype=torch.float64, device="cuda:0")
    for _ in range(2):
        mg.apply(zg, T(b))
    ctx.synchronize()
    assert np.array_equal(H(zg).view(np.int64), z.view(np.int64))
    # a W-cycle enters the tail level twice, the second time from v != 0: no tail
    mg.with_cycle_type(2)
    try:
        assert max(p["level"] for p in mg.cycle_plan()) == nl - 1
    finally:
        mg.with_cycle_type(1)


def test_spmm_xsell_and_pattern_sell(ctx):
    """f2 on the two storages that applied per column before (verdict r05 item
    8): x-staged SELL (the random-coefficient 7-point operator, rows shuffled in
    windows of 4096) and pattern SELL (R / P / A of the box hierarchy's coarse
    levels: fp64 values with 8-64 lanes per row, 4/8-bit codes with one) -- one
    matrix stream per 8 columns, every column bitwise the single-vector kernel
    for k in {1, 3, 8, 32}."""
    seen = set()
    # (x-staged SELL is built from 512 row groups of 4096 up: >= 2.1M rows)
    mats = [fa().SparseMatOp.random7(ctx, 128, 128, 128, seed=3, window=4096),
            fa().SparseMatOp.random7(ctx, 136, 128, 124, seed=4, window=4096)]
    dims = (128, 128, 128)
    A = fa().SparseMatOp.laplace3d_7pt(ctx, *dims)
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=500)
    for l in range(mg.levels()):
        Al, _, Rl, Pl = mg.level(l)
        mats += [M for M in (Al, Rl, Pl) if M is not None and M.spmv_info()["kernel"] in ("xsell", "sellp")]
    for M in mats:
        info = M.spmv_info()
        if info["kernel"] not in ("xsell", "sellp"):
            continue
        seen.add(info["kernel"])
        _spmm_vs_spmv(ctx, M, ks=(1, 3, 8, 32))
    assert {"xsell", "sellp"} <= seen, seen
