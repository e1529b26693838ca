"""CPU tests of the product boundary that need no GPU: the C-ABI library loads,
exports every symbol include/amg.h declares, and rejects bad arguments with a
status code (the reference panics) before touching a device."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "faer-amg_amd", "libfaer_amg_amd.so")
HDR = os.path.join(ROOT, "include", "amg.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "faer-amg_amd")])
    return C.CDLL(LIB)


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(amg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert len(names) >= 50
    for must in ("amg_csr_create", "amg_linop_apply", "amg_precond_apply_in_place",
                 "amg_jacobi_create", "amg_sgs_create", "amg_coarse_chol_create",
                 "amg_multigrid_create", "amg_multigrid_add_level", "amg_multigrid_apply",
                 "amg_galerkin_rap", "amg_last_error", "amg_comm_create"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (amg_\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_python_front_end_binds_every_symbol():
    import faer_amg_amd as fa
    assert set(fa.SIGNATURES) == set(declared_functions())


def test_version_and_null_handles(lib):
    import faer_amg_amd as fa
    L = fa.lib()
    assert "gfx950" in fa.version()
    # null handles are rejected with AMG_ERR_INVALID (1) and a message
    assert L.amg_linop_apply(None, None, 0, None, 0, 1, 1) == 1
    assert b"null" in L.amg_last_error()
    n = C.c_int64()
    assert L.amg_csr_nnz(None, C.byref(n)) == 1
    assert L.amg_multigrid_set(None, 1, 1) == 1
    assert L.amg_linop_destroy(None) == 0
    assert L.amg_comm_unique_id_size() == 128


def test_no_gpu_context_fails_loudly():
    """On a machine without a GPU the product must fail, not fall back to CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import faer_amg_amd as fa
    with pytest.raises(fa.AmgError):
        fa.Context(0)


def _stencil(nx, ny, r, rz=None):
    import itertools
    rz = r if rz is None else rz
    return [dz * nx * ny + dy * nx + dx
            for dz, dy, dx in itertools.product(range(-rz, rz + 1), range(-r, r + 1), range(-r, r + 1))]


@pytest.mark.parametrize("dims,kind", [((256, 256, 256), "7"), ((10, 12, 14), "27"), ((9, 10, 11), "7"),
                                       ((33, 17, 9), "125"), ((128, 128, 128), "a1"), ((30, 30, 1), "5"),
                                       ((100, 1, 1), "3"), ((7, 7, 7), "27")])
def test_grid_inference_from_stencil_offsets(dims, kind):
    """The drop-in path infers the grid hint a generator would have set
    (amg_grid_from_offsets, host only)."""
    import faer_amg_amd as fa
    nx, ny, nz = dims
    n = nx * ny * nz
    pl = nx * ny
    if kind == "7":
        offs = [0, 1, -1, nx, -nx, pl, -pl]
    elif kind == "27":
        offs = _stencil(nx, ny, 1)
    elif kind == "125":
        offs = _stencil(nx, ny, 2)
    elif kind == "a1":  # A_1 of the 7-point box hierarchy (33 diagonals, radius 2)
        offs = ([-2 * pl, 2 * pl, -2 * nx, 2 * nx] + [d for d in range(-2, 3)] +
                [s * pl + dy * nx + dx for s in (-1, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)] +
                [dy * nx + dx for dy in (-1, 1) for dx in (-1, 0, 1)])
    elif kind == "5":
        offs = [0, 1, -1, nx, -nx]
    else:
        offs = [0, 1, -1]
    rng = __import__("random").Random(7)
    rng.shuffle(offs)
    assert fa.grid_from_offsets(offs + offs[:3], n) == dims


def test_grid_inference_rejects_unstructured_offsets():
    import faer_amg_amd as fa
    assert fa.grid_from_offsets([0, 5, 17, -5, -17], 900) is None  # no x coupling
    assert fa.grid_from_offsets([0, 1, -1, 37, -41, 1000], 4096) is None
    assert fa.grid_from_offsets([], 100) is None
