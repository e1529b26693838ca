"""Dataset loaders (Matrix Market, MFEM bundle; utils.rs:269-534) through the
C ABI against the pure-Python restatement in oracle/np_oracle.py.  Host-only:
runs without a GPU.  The reference ships no data files and its parser crate
(matrix-market-rs 0.1.3) is absent, so fixtures are generated here: symmetric
and general files with comments, explicit zeros, duplicates and pattern
entries; parity is bitwise on the CSR arrays (duplicates summed in file order
in both)."""
import os

import numpy as np
import pytest

import np_oracle as N


def fa():
    import faer_amg_amd
    return faer_amg_amd


def write_mtx(path, m, n, entries, field="real", sym="general", comments=("% generated",)):
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {field} {sym}\n")
        for c in comments:
            f.write(c + "\n")
        f.write(f"{m} {n} {len(entries)}\n")
        for e in entries:
            if field == "pattern":
                f.write(f"{e[0] + 1} {e[1] + 1}\n")
            else:
                f.write(f"{e[0] + 1} {e[1] + 1} {e[2]!r}\n")


def same_csr(H, S):
    rp, ci, va = H.arrays()
    S = S.tocsr()
    assert H.dims()[:2] == S.shape
    assert np.array_equal(rp, S.indptr) and np.array_equal(ci, S.indices)
    assert np.array_equal(va, S.data)


def random_sym_entries(rng, n, per_row):
    """Lower-triangle entries of an SPD-ish matrix + some explicit zeros and
    duplicated entries."""
    ent = []
    for i in range(n):
        ent.append((i, i, float(per_row + 1 + rng.random())))
        for j in rng.choice(i, size=min(i, per_row), replace=False) if i else []:
            ent.append((i, int(j), float(-rng.random())))
    ent.append((3, 1, 0.0))            # explicit zero: dropped
    ent.append((5, 5, 0.25))           # duplicate diagonal: summed
    ent.append((7, 2, -0.125))         # duplicate (or new) off-diagonal
    rng.shuffle(ent)
    return ent


def test_mtx_symmetric(tmp_path):
    rng = np.random.default_rng(0)
    p = str(tmp_path / "s.mtx")
    write_mtx(p, 40, 40, random_sym_entries(rng, 40, 4), sym="symmetric")
    H = fa().read_mtx(p)
    S = N.load_mtx(p)
    same_csr(H, S)
    assert abs(S - S.T).max() == 0  # mirrored


def test_mtx_general_pattern_integer(tmp_path):
    rng = np.random.default_rng(1)
    ent = [(int(i), int(j), float(rng.standard_normal())) for i, j in
           zip(rng.integers(0, 30, 200), rng.integers(0, 17, 200))]
    p = str(tmp_path / "g.mtx")
    write_mtx(p, 30, 17, ent, comments=("% a", "%", "% b"))
    same_csr(fa().read_mtx(p), N.load_mtx(p))
    p2 = str(tmp_path / "p.mtx")
    write_mtx(p2, 30, 17, ent, field="pattern")
    H = fa().read_mtx(p2)
    same_csr(H, N.load_mtx(p2))
    p3 = str(tmp_path / "i.mtx")
    write_mtx(p3, 30, 17, [(i, j, int(round(v * 10))) for i, j, v in ent], field="integer")
    same_csr(fa().read_mtx(p3), N.load_mtx(p3))


def test_mtx_large_parallel_chunks(tmp_path):
    """> 2 MiB of entries: parsed by several line-aligned chunks."""
    rng = np.random.default_rng(2)
    n = 3000
    ent = random_sym_entries(rng, n, 30)
    p = str(tmp_path / "big.mtx")
    write_mtx(p, n, n, ent, sym="symmetric")
    assert os.path.getsize(p) > (2 << 20)
    same_csr(fa().read_mtx(p), N.load_mtx(p))


def test_mtx_errors(tmp_path):
    with pytest.raises(fa().AmgError):
        fa().read_mtx(str(tmp_path / "missing.mtx"))
    p = str(tmp_path / "arr.mtx")
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    with pytest.raises(fa().AmgError):
        fa().read_mtx(p)
    p = str(tmp_path / "cnt.mtx")
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1.0\n2 2 1.0\n")
    with pytest.raises(fa().AmgError):
        fa().read_mtx(p)
    p = str(tmp_path / "oob.mtx")
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")
    with pytest.raises(fa().AmgError):
        fa().read_mtx(p)


def write_mfem(d, name, n, rng, nb, k=2, dim=2):
    write_mtx(os.path.join(d, name + ".mtx"), n, n, random_sym_entries(rng, n, 5), sym="symmetric")
    b = list(rng.integers(0, n, nb)) + [0]                    # duplicates, unsorted
    with open(os.path.join(d, name + ".bdy"), "w") as f:
        f.write(f"{len(b)}\n")
        for x in b:
            f.write(f"{int(x)}\n\n" if x % 3 == 0 else f"{int(x)}\n")   # blank lines skipped
    with open(os.path.join(d, name + ".coords"), "w") as f:
        for i in range(n):
            f.write(" ".join(repr(float(v)) for v in rng.random(dim)) + "\n")
    with open(os.path.join(d, name + ".rhs"), "w") as f:
        vals = rng.standard_normal(n * k)
        for c in range(0, len(vals), 7):
            f.write(" ".join(repr(float(v)) for v in vals[c:c + 7]) + "\n")


@pytest.mark.parametrize("delete_boundary", [True, False])
def test_mfem_system(tmp_path, delete_boundary):
    rng = np.random.default_rng(3)
    write_mfem(str(tmp_path), "sys", 60, rng, 12)
    S = fa().MfemSystem(str(tmp_path), "sys", delete_boundary)
    A, rhs, coords, bdy, s2m, m2s = N.load_mfem(str(tmp_path), "sys", delete_boundary)
    same_csr(S.matrix, A)
    assert S.n == A.shape[0] and S.original_dim == 60
    assert np.array_equal(S.boundary, bdy)
    assert np.array_equal(S.rhs, rhs) and S.rhs.shape[1] == 2
    assert np.array_equal(S.coords, coords) and S.coords.shape[1] == 2
    assert np.array_equal(S.solution_to_mesh, s2m) and np.array_equal(S.mesh_to_solution, m2s)
    if delete_boundary:
        assert S.n == 60 - len(bdy)


def test_mfem_errors(tmp_path):
    rng = np.random.default_rng(4)
    write_mfem(str(tmp_path), "sys", 20, rng, 3)
    with pytest.raises(fa().AmgError):
        fa().MfemSystem(str(tmp_path), "nope")
    # boundary count mismatch
    with open(os.path.join(str(tmp_path), "sys.bdy"), "w") as f:
        f.write("5\n1\n2\n")
    with pytest.raises(fa().AmgError):
        fa().MfemSystem(str(tmp_path), "sys")
    # rhs length not a multiple of n
    write_mfem(str(tmp_path), "sys2", 20, rng, 3)
    with open(os.path.join(str(tmp_path), "sys2.rhs"), "a") as f:
        f.write("1.0\n")
    with pytest.raises(fa().AmgError):
        fa().MfemSystem(str(tmp_path), "sys2")


@pytest.mark.gpu
def test_mtx_upload_spmv_and_vcycle(tmp_path, ctx):
    """f4 on the GPU: a symmetric .mtx (lower triangle, duplicates split in two,
    explicit zeros) of the 3-D 7-pt Laplacian, read by amg_mtx_read, uploaded by
    amg_host_csr_upload; SpMV bitwise against the oracle and a two-level SA
    V-cycle on the uploaded operator within 1e-11 of the oracle cycle on the
    same hierarchy (utils.rs:508-534 semantics: zeros dropped, mirrored,
    duplicates summed)."""
    import torch
    import oracle as O
    dims = (10, 9, 8)
    OA = O.laplace3d_7pt(*dims)
    S = OA.to_scipy().tocoo()
    ent = []
    for i, j, v in zip(S.row, S.col, S.data):
        if j > i:
            continue
        if i == j:
            ent += [(int(i), int(j), 2.5), (int(i), int(j), float(v) - 2.5)]  # duplicate: summed
        else:
            ent.append((int(i), int(j), float(v)))
    ent += [(4, 0, 0.0), (17, 3, 0.0)]  # explicit zeros outside the pattern: dropped
    np.random.default_rng(0).shuffle(ent)
    p = str(tmp_path / "lap.mtx")
    write_mtx(p, OA.nrows, OA.ncols, ent, sym="symmetric")
    H = fa().read_mtx(p)
    A = H.upload(ctx)
    rp, ci, va = A.arrays()
    orp, oci, ova = OA.arrays()
    assert np.array_equal(rp, orp) and np.array_equal(ci, oci) and np.array_equal(va, ova)
    x = np.random.default_rng(1).standard_normal(OA.ncols)
    xd = torch.as_tensor(x, device="cuda:0")
    yd = torch.empty_like(xd)
    A.apply(yd, xd)
    ctx.synchronize()
    assert np.array_equal(yd.cpu().numpy(), OA.spmv(x))
    mg = fa().sa_build_box(A, dims, (2, 2, 2), coarsest_dim=200)
    assert mg.levels() == 2
    levels = []
    for l in range(2):
        Al, _, Rl, Pl = mg.level(l)
        d = {"A": O.Csr.from_arrays(*Al.dims(), *Al.arrays()), "smoother": "jacobi" if l == 0 else "chol"}
        if Rl is not None:
            d["R"] = O.Csr.from_arrays(*Rl.dims(), *Rl.arrays())
            d["P"] = O.Csr.from_arrays(*Pl.dims(), *Pl.arrays())
        levels.append(d)
    b = np.random.default_rng(2).uniform(-1, 1, OA.nrows)
    bd = torch.as_tensor(b, device="cuda:0")
    z = torch.empty_like(bd)
    mg.apply(z, bd)
    ctx.synchronize()
    zref = O.Multigrid(levels).apply(b)
    assert np.linalg.norm(z.cpu().numpy() - zref) <= 1e-11 * np.linalg.norm(zref)
