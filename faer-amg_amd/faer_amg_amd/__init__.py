"""Python front end of libfaer_amg_amd.so (the MI355X-native faer-amg V-cycle path).

Mirrors the reference's public surface (aujxn/faer-amg) by name so tests read
like the reference's own usage:

  reference (Rust)                                  here
  SparseMatOp::new (core.rs:56)                     SparseMatOp.from_scipy / from_arrays
  new_jacobi / new_l1 / new_l2 (smoothers.rs:43-86) new_jacobi / new_l1 / new_l2
  SmootherKind::SymGaussSeidel (smoothers.rs:20)    SymGaussSeidel
  CoarseSolverKind::Cholesky (coarse_solvers.rs:29) CoarseCholesky
  Multigrid::new/add_level/with_cycle_type/
      with_smoothing_steps (multigrid.rs:190-239)   Multigrid (same method names)
  LinOp::apply / Precond::apply_in_place            LinOp.apply / LinOp.apply_in_place

Every compute call goes through the C ABI (include/amg.h) into hand-written
HIP kernels; there is no CPU fallback.  If the shared library is missing this
module raises at import time.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FAMG_LIB") or os.path.join(os.path.dirname(_PKG_DIR), "libfaer_amg_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} not found: build the HIP library first "
        "(python -c 'import __graft_entry__ as g; g.build()' or make -C faer-amg_amd)")

_lib = C.CDLL(LIB_PATH)


def source_hash(root=None):
    """sha256[:16] over the library's sources in the Makefile's order (SRCFILES)."""
    import glob
    import hashlib
    root = root or os.path.dirname(_PKG_DIR)
    src = os.path.join(root, "csrc")
    files = []
    for pat in ("*.hip", "*.cpp", "*.hpp", "*.inc"):
        files += sorted(glob.glob(os.path.join(src, pat)))
    files.append(os.path.join(root, "..", "include", "amg.h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_hash():
    f = _lib.amg_source_hash
    f.restype = C.c_char_p
    return f().decode()


# a prebuilt library must match the sources beside it (it travels with the tree
# to the GPU box): a stale one is refused instead of silently running old kernels
if not os.environ.get("FAMG_LIB") and os.path.isdir(os.path.join(os.path.dirname(_PKG_DIR), "csrc")):
    if library_hash() != source_hash():
        raise ImportError(f"{LIB_PATH} was built from other sources (library {library_hash()}, tree "
                          f"{source_hash()}): rebuild with make -C faer-amg_amd")

i32, i64, dbl, vp = C.c_int32, C.c_int64, C.c_double, C.c_void_p
P = C.POINTER

AMG_MEM_HOST, AMG_MEM_DEVICE = 0, 1
KINDS = {0: "csr", 1: "diag", 2: "sgs", 3: "coarse", 4: "multigrid", 5: "dist_csr",
         6: "dist_multigrid", 7: "composite", 8: "block"}

# name -> (restype, argtypes); every exported symbol of include/amg.h
SIGNATURES = {
    "amg_last_error": (C.c_char_p, []),
    "amg_version": (C.c_char_p, []),
    "amg_ctx_create": (i32, [C.c_int, vp, P(vp)]),
    "amg_ctx_destroy": (i32, [vp]),
    "amg_ctx_synchronize": (i32, [vp]),
    "amg_ctx_stream": (i32, [vp, P(vp)]),
    "amg_set_spmv_format": (i32, [i32]),
    "amg_set_value_codes": (i32, [i32]),
    "amg_set_alloc_policy": (i32, [i32]),
    "amg_ctx_join_stream": (i32, [vp, vp, i32]),
    "amg_csr_create": (i32, [vp, i64, i64, vp, vp, vp, P(vp)]),
    "amg_csr_create_device_i32": (i32, [vp, i64, i64, vp, vp, vp, P(vp)]),
    "amg_csr_nnz": (i32, [vp, P(i64)]),
    "amg_csr_spmv_info": (i32, [vp, vp]),
    "amg_csr_value_codes": (i32, [vp, vp]),
    "amg_csr_download": (i32, [vp, vp, vp, vp]),
    "amg_csr_dia_range": (i32, [vp, vp]),
    "amg_csr_class_info": (i32, [vp, vp]),
    "amg_csr_set_grid": (i32, [vp, i64, i64, i64]),
    "amg_csr_spmv_epilogue": (i32, [vp, i32, vp, vp, vp, vp]),
    "amg_csr_grid_info": (i32, [vp, vp]),
    "amg_grid_from_offsets": (i32, [vp, i64, i64, vp, P(i32)]),
    "amg_set_flag": (i32, [i32, i64]),
    "amg_source_hash": (C.c_char_p, []),
    "amg_multigrid_level_reordered": (i32, [vp, i64, P(i32)]),
    "amg_multigrid_get_run_level": (i32, [vp, i64, P(vp), P(vp), P(vp), P(vp)]),
    "amg_get_flag": (i32, [i32, P(i64)]),
    "amg_gen_laplace3d_7pt": (i32, [vp, i64, i64, i64, P(vp)]),
    "amg_gen_aniso27": (i32, [vp, i64, i64, i64, dbl, dbl, dbl, P(vp)]),
    "amg_gen_random_7pt": (i32, [vp, i64, i64, i64, C.c_uint64, i64, P(vp)]),
    "amg_linop_kind_of": (i32, [vp, P(i32)]),
    "amg_linop_dims": (i32, [vp, P(i64), P(i64)]),
    "amg_linop_apply": (i32, [vp, vp, i64, vp, i64, i64, C.c_int]),
    "amg_linop_transpose_apply": (i32, [vp, vp, i64, vp, i64, i64, C.c_int]),
    "amg_precond_apply_in_place": (i32, [vp, vp, i64, i64, C.c_int]),
    "amg_precond_transpose_apply_in_place": (i32, [vp, vp, i64, i64, C.c_int]),
    "amg_linop_destroy": (i32, [vp]),
    "amg_jacobi_create": (i32, [vp, dbl, P(vp)]),
    "amg_l1_create": (i32, [vp, P(vp)]),
    "amg_l2_create": (i32, [vp, P(vp)]),
    "amg_diag_create": (i32, [vp, i64, vp, P(vp)]),
    "amg_sgs_create": (i32, [vp, vp, P(vp)]),
    "amg_sgs_ncolors": (i32, [vp, P(i64)]),
    "amg_sgs_info": (i32, [vp, vp]),
    "amg_coarse_chol_create": (i32, [vp, P(vp)]),
    "amg_multigrid_create": (i32, [vp, vp, P(vp)]),
    "amg_multigrid_add_level": (i32, [vp, vp, vp, vp, vp]),
    "amg_multigrid_set": (i32, [vp, i64, i64]),
    "amg_multigrid_levels": (i32, [vp, P(i64)]),
    "amg_multigrid_set_graph": (i32, [vp, i32]),
    "amg_multigrid_set_option": (i32, [vp, i32, i64]),
    "amg_multigrid_apply": (i32, [vp, vp, i64, vp, i64, i64, C.c_int]),
    "amg_multigrid_get_level": (i32, [vp, i64, P(vp), P(vp), P(vp), P(vp)]),
    "amg_spgemm": (i32, [vp, vp, P(vp)]),
    "amg_transpose": (i32, [vp, P(vp)]),
    "amg_galerkin_rap": (i32, [vp, vp, vp, P(vp)]),
    "amg_smooth_interpolation": (i32, [vp, vp, dbl, P(vp)]),
    "amg_sa_tentative": (i32, [vp, i64, vp, i64, vp, P(vp), vp]),
    "amg_nn_stationary_l1": (i32, [vp, i64, vp]),
    "amg_sa_build_box": (i32, [vp, i64, i64, i64, i64, i64, i64, i64, i64, dbl, i32, P(vp)]),
    "amg_stationary_solve": (i32, [vp, vp, vp, vp, i64, dbl, vp, P(i64)]),
    "amg_pcg_solve": (i32, [vp, vp, vp, vp, i64, dbl, dbl, vp, P(i64)]),
    "amg_composite_create": (i32, [vp, vp, i64, P(vp)]),
    "amg_block_smoother_create": (i32, [vp, vp, i64, i64, P(vp)]),
    "amg_block_smoother_to_csr": (i32, [vp, P(vp)]),
    "amg_composite_push": (i32, [vp, vp]),
    "amg_composite_ncomponents": (i32, [vp, P(i64)]),
    "amg_comm_unique_id_size": (i32, []),
    "amg_rccl_library": (C.c_char_p, []),
    "amg_comm_get_unique_id": (i32, [vp]),
    "amg_comm_create": (i32, [vp, i32, i32, vp, P(vp)]),
    "amg_loopback_hub_create": (i32, [i32, P(vp)]),
    "amg_loopback_hub_destroy": (i32, [vp]),
    "amg_comm_create_loopback": (i32, [vp, vp, i32, P(vp)]),
    "amg_comm_destroy": (i32, [vp]),
    "amg_comm_rank": (i32, [vp, P(i32), P(i32)]),
    "amg_comm_barrier": (i32, [vp]),
    "amg_comm_allreduce_max": (i32, [vp, P(dbl)]),
    "amg_comm_allreduce_sum": (i32, [vp, P(dbl)]),
    "amg_dist_multigrid_create": (i32, [vp, vp, vp, i64, P(vp)]),
    "amg_dist_local_rows": (i32, [vp, P(i64), P(i64)]),
    "amg_dist_level_info": (i32, [vp, i64, vp]),
    "amg_dist_level_operator": (i32, [vp, i64, P(vp)]),
    "amg_dist_level_matrix": (i32, [vp, i64, i32, P(vp)]),
    "amg_dist_set_option": (i32, [vp, i32, i64]),
    "amg_mtx_read": (i32, [C.c_char_p, P(vp)]),
    "amg_host_csr_dims": (i32, [vp, P(i64), P(i64), P(i64)]),
    "amg_host_csr_create": (i32, [i64, i64, vp, vp, vp, P(vp)]),
    "amg_host_csr_arrays": (i32, [vp, vp, vp, vp]),
    "amg_host_csr_upload": (i32, [vp, vp, P(vp)]),
    "amg_host_csr_destroy": (i32, [vp]),
    "amg_mfem_load": (i32, [C.c_char_p, C.c_char_p, i32, P(vp)]),
    "amg_mfem_info": (i32, [vp, vp]),
    "amg_mfem_matrix": (i32, [vp, P(vp)]),
    "amg_mfem_rhs": (i32, [vp, vp, i64]),
    "amg_mfem_coords": (i32, [vp, vp, i64]),
    "amg_mfem_boundary": (i32, [vp, vp]),
    "amg_mfem_index_maps": (i32, [vp, vp, vp]),
    "amg_mfem_destroy": (i32, [vp]),
    "amg_dist_stationary_solve": (i32, [vp, vp, vp, i64, dbl, vp, P(i64)]),
    "amg_sa_config_default": (i32, [vp]),
    "amg_sa_build": (i32, [vp, vp, i64, i64, vp, vp, P(vp)]),
    "amg_strength_graph": (i32, [vp, vp, i64, i64, vp, i64, i64, P(vp)]),
    "amg_aggregate_mis": (i32, [vp, vp, P(i64)]),
    "amg_sa_tentative_block": (i32, [vp, i64, i64, vp, i64, vp, i64, i64, i64, P(vp), vp]),
    "amg_block_jacobi_smooth": (i32, [vp, vp, i64, dbl, P(vp)]),
    "amg_nn_postprocess": (i32, [vp, i64, vp, i64, i64]),
    "amg_gen_elasticity_q1": (i32, [i64, i64, i64, dbl, dbl, C.c_uint64, i32, P(vp)]),
    "amg_dist_pcg_solve": (i32, [vp, i32, vp, vp, i64, dbl, dbl, vp, P(i64)]),
    "amg_multigrid_cycle_plan": (i32, [vp, vp, i64, P(i64)]),
    "amg_multigrid_fine_launch": (i32, [vp, i32, vp, vp]),
    "amg_multigrid_set_fine_timer": (i32, [vp, i32]),
    "amg_multigrid_fine_timer_ms": (i32, [vp, vp]),
    "amg_dist_cycle_plan": (i32, [vp, vp, i64, P(i64)]),
    "amg_set_sgs_fused": (i32, [i32]),
    "amg_sgs_fused": (i32, [vp, P(i32)]),
    "amg_halo_plan_create": (i32, [i32, i32, vp, P(vp)]),
    "amg_halo_plan_destroy": (i32, [vp]),
    "amg_halo_plan_add_columns": (i32, [vp, i64, vp]),
    "amg_halo_plan_requests": (i32, [vp, vp, P(i64)]),
    "amg_halo_plan_ghost_ids": (i32, [vp, vp]),
    "amg_halo_plan_set_incoming": (i32, [vp, vp, vp]),
    "amg_halo_plan_info": (i32, [vp, vp]),
    "amg_halo_plan_neighbors": (i32, [vp, vp, vp, vp, vp, vp]),
    "amg_halo_plan_send_indices": (i32, [vp, vp]),
    "amg_halo_plan_remap": (i32, [vp, i64, vp, vp, vp, P(i64), P(i64)]),
    "amg_dist_first_redundant_level": (i32, [i64, vp, i64, P(i64)]),
    "amg_trace_mark": (i32, [vp, i32]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class LaunchRec(C.Structure):
    """amg_launch_rec (include/amg.h)."""
    _fields_ = [("level", i32), ("role", i32), ("kernel", i32), ("mode", i32), ("rows", i64),
                ("bytes", i64), ("csr_bytes", i64), ("name", C.c_char * 32)]


ROLES = {0: "smooth", 1: "resid", 2: "restrict", 3: "interp", 4: "coarse", 5: "other"}
MODES = {-1: "-", 0: "SET", 1: "ADD", 2: "RESID", 3: "JACOBI", 4: "SGS", 5: "RESID0", 6: "ADD0", 7: "SETDF"}


class AmgError(RuntimeError):
    """Non-OK amg_status (the reference panics in these cases)."""

    def __init__(self, status, msg):
        super().__init__(f"amg status {status}: {msg}")
        self.status = status


def _ck(status):
    if status != 0:
        raise AmgError(status, _lib.amg_last_error().decode())


def lib():
    return _lib


def version():
    return _lib.amg_version().decode()


SPMV_FORMATS = {"auto": 0, "csr": 1, "sell": 2, "vector": 3}


def set_spmv_format(policy):
    """SpMV storage for matrices built afterwards: 'auto', 'csr', 'sell' or 'vector'."""
    _ck(_lib.amg_set_spmv_format(SPMV_FORMATS[policy]))


def set_value_codes(enable):
    """SELL matrices built afterwards store 4/8/16-bit codes into a per-matrix
    table of distinct values when they have <= 65536 of them (default True)."""
    _ck(_lib.amg_set_value_codes(1 if enable else 0))


def set_alloc_policy(contiguous):
    """Physically contiguous device allocations for large buffers: refused (True
    raises) -- they read stale data across kernels on gfx950."""
    _ck(_lib.amg_set_alloc_policy(1 if contiguous else 0))


def _dptr(x):
    """(pointer, mem kind, nrows, ncols, ld) of a torch tensor or numpy array."""
    try:
        import torch
        if isinstance(x, torch.Tensor):
            if x.dtype != torch.float64:
                raise TypeError("vectors must be float64")
            if x.dim() == 1:
                if not x.is_contiguous():
                    raise ValueError("vector must be contiguous")
                n, k, ld = x.shape[0], 1, x.shape[0]
            else:
                # column-major n x k (torch: a (k, n) row-major tensor transposed)
                n, k = x.shape
                if x.stride(0) != 1:
                    raise ValueError("matrix must be column-major (stride(0) == 1)")
                ld = x.stride(1) if k > 1 else n
            return vp(x.data_ptr()), (AMG_MEM_DEVICE if x.is_cuda else AMG_MEM_HOST), n, k, ld
    except ImportError:
        pass
    if not isinstance(x, np.ndarray) or x.dtype != np.float64:
        raise TypeError("vectors must be float64 numpy arrays or torch tensors")
    if x.ndim == 1:
        if not x.flags.c_contiguous:
            raise ValueError("vector must be contiguous")
        return x.ctypes.data_as(vp), AMG_MEM_HOST, x.shape[0], 1, x.shape[0]
    if not x.flags.f_contiguous:
        raise ValueError("matrix must be Fortran (column-major) ordered")
    return x.ctypes.data_as(vp), AMG_MEM_HOST, x.shape[0], x.shape[1], x.shape[0]


class Context:
    """One device per process (amg_ctx).  `stream` may be a raw hipStream_t int.

    Device-memory calls made through this module are ordered against the
    caller's torch.cuda.current_stream() automatically (amg_ctx_join_stream)."""

    def __init__(self, device=0, stream=None):
        h = vp()
        _ck(_lib.amg_ctx_create(device, vp(stream) if stream else None, C.byref(h)))
        self.h = h
        self.device = device
        s = vp()
        _ck(_lib.amg_ctx_stream(self.h, C.byref(s)))
        self._stream = s.value or 0

    def synchronize(self):
        _ck(_lib.amg_ctx_synchronize(self.h))

    def trace_mark(self, tag):
        """Launch k_trace_mark with `tag` blocks (brackets a region of a kernel trace)."""
        _ck(_lib.amg_trace_mark(self.h, tag))

    @property
    def stream(self):
        return self._stream

    def join_torch(self, ctx_waits):
        """Order the library stream with torch's current stream (see amg_ctx_join_stream)."""
        import torch
        cur = torch.cuda.current_stream(self.device).cuda_stream
        if cur != self._stream:
            _ck(_lib.amg_ctx_join_stream(self.h, vp(cur) if cur else None, 1 if ctx_waits else 0))

    def __del__(self, _destroy=_lib.amg_ctx_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None


class _ordered:
    """Context manager: library stream waits for torch's stream before a device
    call, torch's stream waits for the library stream after it."""

    def __init__(self, ctx, mem):
        self.ctx, self.on = ctx, (mem == AMG_MEM_DEVICE and ctx is not None)

    def __enter__(self):
        if self.on:
            self.ctx.join_torch(True)

    def __exit__(self, *exc):
        if self.on:
            self.ctx.join_torch(False)
        return False


class LinOp:
    """Handle on any library operator (faer matrix_free LinOp/Precond/BiPrecond)."""

    def __init__(self, handle, ctx, refs=()):
        self.h = handle
        self.ctx = ctx
        self._refs = refs  # python-side references (the C side holds its own)

    def __del__(self, _destroy=_lib.amg_linop_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None

    @property
    def kind(self):
        k = i32()
        _ck(_lib.amg_linop_kind_of(self.h, C.byref(k)))
        return KINDS[k.value]

    def dims(self):
        r, c = i64(), i64()
        _ck(_lib.amg_linop_dims(self.h, C.byref(r), C.byref(c)))
        return r.value, c.value

    @property
    def nrows(self):
        return self.dims()[0]

    @property
    def ncols(self):
        return self.dims()[1]

    def apply(self, out, rhs):
        """LinOp::apply: out = M rhs (out overwritten)."""
        po, mo, no, ko, lo = _dptr(out)
        pr, mr, nr, kr, lr = _dptr(rhs)
        if mo != mr or ko != kr:
            raise ValueError("out and rhs must live in the same memory with equal columns")
        with _ordered(self.ctx, mo):
            _ck(_lib.amg_linop_apply(self.h, po, lo, pr, lr, ko, mo))
        return out

    def transpose_apply(self, out, rhs):
        po, mo, no, ko, lo = _dptr(out)
        pr, mr, nr, kr, lr = _dptr(rhs)
        with _ordered(self.ctx, mo):
            _ck(_lib.amg_linop_transpose_apply(self.h, po, lo, pr, lr, ko, mo))
        return out

    def apply_in_place(self, rhs):
        """Precond::apply_in_place: rhs <- M rhs."""
        p, m, n, k, ld = _dptr(rhs)
        with _ordered(self.ctx, m):
            _ck(_lib.amg_precond_apply_in_place(self.h, p, ld, k, m))
        return rhs

    def transpose_apply_in_place(self, rhs):
        p, m, n, k, ld = _dptr(rhs)
        with _ordered(self.ctx, m):
            _ck(_lib.amg_precond_transpose_apply_in_place(self.h, p, ld, k, m))
        return rhs

    def __matmul__(self, x):
        """Host convenience: M @ numpy vector (staged through the device)."""
        x = np.ascontiguousarray(x, np.float64)
        out = np.zeros(self.nrows)
        return self.apply(out, x)


class SparseMatOp(LinOp):
    """Device CSR operator (SparseMatOp / ParSpmmOp of the reference)."""

    @classmethod
    def from_arrays(cls, ctx, nrows, ncols, rowptr, col, val):
        rp = np.ascontiguousarray(rowptr, np.int64)
        ci = np.ascontiguousarray(col, np.int64)
        va = np.ascontiguousarray(val, np.float64)
        h = vp()
        _ck(_lib.amg_csr_create(ctx.h, int(nrows), int(ncols), rp.ctypes.data_as(vp),
                                ci.ctypes.data_as(vp), va.ctypes.data_as(vp), C.byref(h)))
        return cls(h, ctx)

    @classmethod
    def from_scipy(cls, ctx, M):
        M = M.tocsr()
        M.sort_indices()
        return cls.from_arrays(ctx, M.shape[0], M.shape[1], M.indptr, M.indices, M.data)

    @classmethod
    def laplace3d_7pt(cls, ctx, nx, ny, nz):
        h = vp()
        _ck(_lib.amg_gen_laplace3d_7pt(ctx.h, nx, ny, nz, C.byref(h)))
        return cls(h, ctx)

    @classmethod
    def aniso27(cls, ctx, nx, ny, nz, ex=1.0, ey=1.0, ez=0.01):
        h = vp()
        _ck(_lib.amg_gen_aniso27(ctx.h, nx, ny, nz, ex, ey, ez, C.byref(h)))
        return cls(h, ctx)

    @classmethod
    def random7(cls, ctx, nx, ny, nz, seed=42, window=4096):
        """Random-coefficient 7-pt SPD operator, symmetrically permuted
        (window < 0 none, 0 all rows, > 0 within windows of that many rows)."""
        h = vp()
        _ck(_lib.amg_gen_random_7pt(ctx.h, nx, ny, nz, seed, window, C.byref(h)))
        return cls(h, ctx)

    @property
    def nnz(self):
        v = i64()
        _ck(_lib.amg_csr_nnz(self.h, C.byref(v)))
        return v.value

    def spmv_info(self):
        """SpMV storage chosen for this matrix (kernel, bytes streamed per SpMV, SELL stats)."""
        info = np.zeros(8, np.int64)
        _ck(_lib.amg_csr_spmv_info(self.h, info.ctypes.data_as(vp)))
        keys = ("kernel", "stream_bytes", "csr_bytes", "slices", "stored_entries",
                "slices_implicit", "slices_u16", "slices_i32")
        d = dict(zip(keys, (int(v) for v in info)))
        d["kernel"] = ("csr-stream", "sell", "vector", "dia", "bsr", "sellp", "classes", "xsell", "gtc")[d["kernel"]]
        vc = np.zeros(2, np.int64)
        _ck(_lib.amg_csr_value_codes(self.h, vc.ctypes.data_as(vp)))
        d["value_bits"], d["value_table"] = int(vc[0]), int(vc[1])
        dr = np.zeros(4, np.int64)
        _ck(_lib.amg_csr_dia_range(self.h, dr.ctypes.data_as(vp)))
        d["dia_rows"] = (int(dr[0]), int(dr[1]))
        d["dia_diagonals"], d["dia_bits"] = int(dr[2]), int(dr[3])
        ci = np.zeros(4, np.int64)
        _ck(_lib.amg_csr_class_info(self.h, ci.ctypes.data_as(vp)))
        d["classes"], d["class_offsets"], d["class_id_bits"] = int(ci[0]), int(ci[1]), int(ci[2])
        g = np.zeros(13, np.int64)
        _ck(_lib.amg_csr_grid_info(self.h, g.ctypes.data_as(vp)))
        d["grid"] = tuple(int(v) for v in g[:3])
        d["grid_source"] = ("none", "given", "inferred")[int(g[10])]
        d["gtc"] = ("none", "P", "R", "P", "R")[int(g[11])]
        d["gtc_kind"] = ("none", "gtc", "gtc", "gtx", "gtx")[int(g[11])]
        d["xstaged"] = bool(g[3])
        if d["xstaged"]:
            d["tile"], d["halo"] = tuple(int(v) for v in g[4:7]), tuple(int(v) for v in g[7:10])
            d["tile_source"] = ("none", "table", "timed", "env", "rule")[int(g[12])]
        return d

    def spmv_epilogue(self, mode, x, y, b=None, d=None):
        """amg_csr_spmv_epilogue on device tensors: mode "set" y = A x, "add" y += A x,
        "resid" y = b - A x, "jacobi" y = x + d (b - A x)."""
        m = {"set": 0, "add": 1, "resid": 2, "jacobi": 3}[mode]
        ptr = lambda t: None if t is None else vp(t.data_ptr())  # noqa: E731
        with _ordered(self.ctx, AMG_MEM_DEVICE):  # y / b / d written on torch's stream
            _ck(_lib.amg_csr_spmv_epilogue(self.h, m, ptr(x), ptr(y), ptr(b), ptr(d)))

    def set_grid(self, nx, ny, nz):
        """Grid hint (amg_csr_set_grid): the rows are an nx x ny x nz grid; re-finalizes the storage."""
        _ck(_lib.amg_csr_set_grid(self.h, nx, ny, nz))

    def arrays(self):
        m, n = self.dims()
        nnz = self.nnz
        rp = np.zeros(m + 1, np.int64)
        ci = np.zeros(max(nnz, 1), np.int64)
        va = np.zeros(max(nnz, 1), np.float64)
        _ck(_lib.amg_csr_download(self.h, rp.ctypes.data_as(vp), ci.ctypes.data_as(vp),
                                  va.ctypes.data_as(vp)))
        return rp, ci[:nnz], va[:nnz]

    def to_scipy(self):
        import scipy.sparse as sp
        rp, ci, va = self.arrays()
        return sp.csr_matrix((va, ci, rp), shape=self.dims())


FLAGS = {"fold_xscs": 0, "dia_dk": 1, "vec_wpr": 2, "gtx_time": 3, "sgs27_march": 4, "xs_pipe": 5, "bsr_kernel": 6,
         "bsr_long": 7,
         "dia7_rp": 8, "fine_fuse": 9, "dense_tail": 10}


def set_flag(name, value):
    """amg_set_flag: a run-time A/B switch (bitwise neutral); multigrids re-capture
    their graphs at the next apply."""
    _ck(_lib.amg_set_flag(FLAGS[name], int(value)))


def get_flag(name):
    v = i64()
    _ck(_lib.amg_get_flag(FLAGS[name], C.byref(v)))
    return v.value


def grid_from_offsets(offsets, n):
    """amg_grid_from_offsets (host only): the (nx, ny, nz) grid the library infers
    for an n-row square operator whose stencil has these col - row offsets, or None."""
    o = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    g = np.zeros(3, np.int64)
    found = C.c_int32(0)
    _ck(_lib.amg_grid_from_offsets(o.ctypes.data_as(vp), len(o), int(n), g.ctypes.data_as(vp), C.byref(found)))
    return tuple(int(v) for v in g) if found.value else None


def _wrap(h, ctx, cls=LinOp, refs=()):
    return cls(h, ctx, refs)


def new_jacobi(A, omega=0.66):
    h = vp()
    _ck(_lib.amg_jacobi_create(A.h, omega, C.byref(h)))
    return _wrap(h, A.ctx)


def new_l1(A):
    h = vp()
    _ck(_lib.amg_l1_create(A.h, C.byref(h)))
    return _wrap(h, A.ctx)


def new_l2(A):
    h = vp()
    _ck(_lib.amg_l2_create(A.h, C.byref(h)))
    return _wrap(h, A.ctx)


def diag(ctx, d):
    d = np.ascontiguousarray(d, np.float64)
    h = vp()
    _ck(_lib.amg_diag_create(ctx.h, len(d), d.ctypes.data_as(vp), C.byref(h)))
    return _wrap(h, ctx)


class SymGaussSeidel(LinOp):
    def __init__(self, A, colors=None):
        h = vp()
        cp = None
        if colors is not None:
            colors = np.ascontiguousarray(colors, np.int32)
            cp = colors.ctypes.data_as(vp)
        _ck(_lib.amg_sgs_create(A.h, cp, C.byref(h)))
        super().__init__(h, A.ctx)

    @property
    def ncolors(self):
        v = i64()
        _ck(_lib.amg_sgs_ncolors(self.h, C.byref(v)))
        return v.value

    def sweep_storage(self):
        """{'colors', 'kernel' ('sell', 'dia', ...), 'diagonals', 'bits'} of the color sweeps."""
        return sgs_info(self)


def sgs_info(S):
    info = np.zeros(4, np.int64)
    _ck(_lib.amg_sgs_info(S.h, info.ctypes.data_as(vp)))
    return {"colors": int(info[0]), "kernel": ("csr-stream", "sell", "vector", "dia", "bsr", "sellp")[int(info[1])],
            "diagonals": int(info[2]), "bits": int(info[3])}


def set_sgs_fused(enable):
    """SGS smoothers built afterwards use the fused plane-parity phases where they
    apply (True / 1: three phases per step, 2: four phases, False / 0: colour launches)."""
    _ck(_lib.amg_set_sgs_fused(int(enable)))


def sgs_fused(S):
    v = i32()
    _ck(_lib.amg_sgs_fused(S.h, C.byref(v)))
    return bool(v.value)


def CoarseCholesky(A):
    """CoarseSolverKind::Cholesky.build_from_sparse (coarse_solvers.rs:22-33)."""
    h = vp()
    _ck(_lib.amg_coarse_chol_create(A.h, C.byref(h)))
    return _wrap(h, A.ctx)


class Multigrid(LinOp):
    """Multigrid (multigrid.rs:171-518)."""

    def __init__(self, op, smoother, _handle=None):
        if _handle is None:
            h = vp()
            _ck(_lib.amg_multigrid_create(op.h, smoother.h, C.byref(h)))
        else:
            h = _handle
        super().__init__(h, op.ctx)

    @classmethod
    def _from_handle(cls, h, ctx):
        obj = cls.__new__(cls)
        LinOp.__init__(obj, h, ctx)
        return obj

    def add_level(self, op, smoother, r, p):
        _ck(_lib.amg_multigrid_add_level(self.h, op.h, smoother.h, r.h, p.h))
        return self

    def with_cycle_type(self, mu):
        self._mu = mu
        _ck(_lib.amg_multigrid_set(self.h, mu, getattr(self, "_steps", 1)))
        return self

    def with_smoothing_steps(self, steps):
        self._steps = steps
        _ck(_lib.amg_multigrid_set(self.h, getattr(self, "_mu", 1), steps))
        return self

    def set_graph(self, enable):
        _ck(_lib.amg_multigrid_set_graph(self.h, 1 if enable else 0))

    def set_reorder(self, mode):
        """Locality reordering of general levels (multigrid option 5): 0 off, 1 auto, 2 force."""
        _ck(_lib.amg_multigrid_set_option(self.h, 5, int(mode)))

    def run_level(self, l):
        """(A, S, R, P) the cycle runs on level l: the renumbered copies of a renumbered level."""
        a, s, r, p = vp(), vp(), vp(), vp()
        _ck(_lib.amg_multigrid_get_run_level(self.h, l, C.byref(a), C.byref(s), C.byref(r), C.byref(p)))
        return (SparseMatOp(a, self.ctx), LinOp(s, self.ctx),
                SparseMatOp(r, self.ctx) if r.value else None,
                SparseMatOp(p, self.ctx) if p.value else None)

    def set_fine_timer(self, which):
        """In-cycle timing of fused fine-level launch `which` (0 / 1; -1 off):
        every cycle records HIP events around it (amg_multigrid_set_fine_timer)."""
        _ck(_lib.amg_multigrid_set_fine_timer(self.h, int(which)))

    def fine_timer_ms(self):
        """Milliseconds of the timed launch in the last completed cycle."""
        v = C.c_float()
        _ck(_lib.amg_multigrid_fine_timer_ms(self.h, C.byref(v)))
        return float(v.value)

    def fine_launch(self, which, out, rhs):
        """One fused fine-level launch as the cycle makes it (amg_multigrid_fine_launch):
        which 0 = residual + restriction, 1 = interpolation + post-smoothing; device
        tensors, asynchronous on the context stream.  False where the cycle has none."""
        import torch
        n = self.nrows
        for t in (rhs,) if out is None else (rhs, out):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
                    and t.numel() == n):
                raise ValueError("fine_launch: contiguous float64 device vectors of the fine level's size")
        st = _lib.amg_multigrid_fine_launch(self.h, int(which), None if out is None else C.c_void_p(out.data_ptr()),
                                            C.c_void_p(rhs.data_ptr()))
        if st == 0:
            return True
        if st == 3:  # AMG_ERR_UNSUPPORTED
            return False
        _ck(st)

    def reordered(self, l):
        """Whether level l runs in a renumbered (locality) numbering."""
        v = i32()
        _ck(_lib.amg_multigrid_level_reordered(self.h, l, C.byref(v)))
        return bool(v.value)

    def set_sgs_residual_form(self, enable):
        """Literal smooth() order for SGS (residual SpMV + SGS(r)) instead of the fused sweep."""
        _ck(_lib.amg_multigrid_set_option(self.h, 1, 1 if enable else 0))

    def set_fold_zero_guess(self, enable):
        """Fold the zero-guess Jacobi step into the residual/correction SpMVs (default on)."""
        _ck(_lib.amg_multigrid_set_option(self.h, 2, 1 if enable else 0))

    def set_restrict_df(self, enable):
        """R on wide grid-transfer classes also writes the next level's first Jacobi step
        from zero (SPMV_SETDF; default on; bitwise the separate d*f pass)."""
        _ck(_lib.amg_multigrid_set_option(self.h, 4, 1 if enable else 0))

    def levels(self):
        v = i64()
        _ck(_lib.amg_multigrid_levels(self.h, C.byref(v)))
        return v.value

    def cycle_plan(self):
        """The launches of one V-cycle in order (amg_multigrid_cycle_plan): list of
        dicts {level, role, kernel, mode, name, rows, bytes, csr_bytes}."""
        n = i64()
        _ck(_lib.amg_multigrid_cycle_plan(self.h, None, 0, C.byref(n)))
        recs = (LaunchRec * max(1, n.value))()
        _ck(_lib.amg_multigrid_cycle_plan(self.h, recs, n.value, C.byref(n)))
        return [{"level": r.level, "role": ROLES.get(r.role, "?"), "kernel": r.kernel,
                 "mode": MODES.get(r.mode, "?"), "name": r.name.decode(), "rows": r.rows,
                 "bytes": r.bytes, "csr_bytes": r.csr_bytes} for r in recs[:n.value]]

    def level(self, l):
        """(A, S, R, P) handles of level l (R, P None on the coarsest)."""
        a, s, r, p = vp(), vp(), vp(), vp()
        _ck(_lib.amg_multigrid_get_level(self.h, l, C.byref(a), C.byref(s), C.byref(r), C.byref(p)))
        return (SparseMatOp(a, self.ctx), LinOp(s, self.ctx),
                SparseMatOp(r, self.ctx) if r.value else None,
                SparseMatOp(p, self.ctx) if p.value else None)


def spgemm(A, B):
    h = vp()
    _ck(_lib.amg_spgemm(A.h, B.h, C.byref(h)))
    return SparseMatOp(h, A.ctx)


def transpose(P_):
    h = vp()
    _ck(_lib.amg_transpose(P_.h, C.byref(h)))
    return SparseMatOp(h, P_.ctx)


def galerkin_rap(R, A, P_):
    h = vp()
    _ck(_lib.amg_galerkin_rap(R.h, A.h, P_.h, C.byref(h)))
    return SparseMatOp(h, A.ctx)


def smooth_interpolation(A, P_, omega=0.66):
    h = vp()
    _ck(_lib.amg_smooth_interpolation(A.h, P_.h, omega, C.byref(h)))
    return SparseMatOp(h, A.ctx)


def sa_tentative(ctx, agg_of, naggs, near_null):
    agg = np.ascontiguousarray(agg_of, np.int64)
    nn = np.ascontiguousarray(near_null, np.float64)
    cnn = np.zeros(naggs)
    h = vp()
    _ck(_lib.amg_sa_tentative(ctx.h, len(agg), agg.ctypes.data_as(vp), naggs,
                              nn.ctypes.data_as(vp), C.byref(h), cnn.ctypes.data_as(vp)))
    return SparseMatOp(h, ctx), cnn


def nn_stationary_l1(A, x, iters=3):
    x = np.array(x, np.float64, copy=True)
    _ck(_lib.amg_nn_stationary_l1(A.h, iters, x.ctypes.data_as(vp)))
    return x


SMOOTHERS = {"jacobi": 0, "l1": 1, "sgs": 2, "block": 3}


def sa_build_box(A, dims, box=(2, 2, 2), coarsest_dim=1000, max_levels=0, omega=0.66,
                 smoother="jacobi"):
    """SA hierarchy + multigrid on a structured grid (Hierarchy::coarsen + Multigrid)."""
    h = vp()
    _ck(_lib.amg_sa_build_box(A.h, dims[0], dims[1], dims[2], box[0], box[1], box[2],
                              coarsest_dim, max_levels, omega, SMOOTHERS[smoother], C.byref(h)))
    return Multigrid._from_handle(h, A.ctx)


class SaConfig(C.Structure):
    """amg_sa_config: AggregationConfig + HierarchyConfig + the smoother choice
    (interpolation/mod.rs:62-79, hierarchy.rs:21-36)."""
    _fields_ = [("block_size", i64), ("candidate_dimension", i64), ("strength_depth", i64),
                ("smoothing_steps", i64), ("coarsest_dim", i64), ("max_levels", i64),
                ("omega", dbl), ("smoother", i32), ("reserved", i32)]

    def __init__(self, **kw):
        super().__init__()
        _ck(_lib.amg_sa_config_default(C.byref(self)))
        for k, v in kw.items():
            if k == "smoother" and isinstance(v, str):
                v = SMOOTHERS[v]
            setattr(self, k, v)


def _colmajor_host(x, nrows):
    x = np.asarray(x, np.float64)
    if x.ndim == 1:
        x = x[:, None]
    x = np.asfortranarray(x)
    if x.shape[0] != nrows:
        raise ValueError("near-null space must have one row per matrix row")
    return x


def smoothed_aggregation(A, near_null, weights=None, **config):
    """SA hierarchy + multigrid for a general SPD matrix (Hierarchy::coarsen with
    AggregationConfig, hierarchy.rs:190-248; interpolation/mod.rs:730-836).
    near_null: n x k candidates; weights: k strength weights (None: 1/v^T A v);
    config: SaConfig fields (block_size, candidate_dimension, strength_depth,
    smoothing_steps, coarsest_dim, max_levels, omega, smoother)."""
    cfg = SaConfig(**config)
    nn = _colmajor_host(near_null, A.nrows)
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    h = vp()
    _ck(_lib.amg_sa_build(A.h, nn.ctypes.data_as(vp), nn.shape[0], nn.shape[1],
                          None if w is None else w.ctypes.data_as(vp), C.byref(cfg), C.byref(h)))
    return Multigrid._from_handle(h, A.ctx)


def strength_graph(A, near_null, weights, depth=1, block_size=1):
    """Node-level strength graph (partitioners/mod.rs:337-393) as scipy CSR."""
    nn = _colmajor_host(near_null, A.nrows)
    w = np.ascontiguousarray(weights, np.float64)
    h = vp()
    _ck(_lib.amg_strength_graph(A.h, nn.ctypes.data_as(vp), nn.shape[0], nn.shape[1],
                                w.ctypes.data_as(vp), depth, block_size, C.byref(h)))
    return HostCsr(h).to_scipy()


def aggregate_mis(G):
    """MIS-seeded aggregates of a strength graph (scipy CSR): (agg_of, naggs)."""
    G = G.tocsr()
    n = G.shape[0]
    tmp = HostCsr(_host_csr_from_scipy(G))
    agg = np.zeros(n, np.int64)
    na = i64()
    _ck(_lib.amg_aggregate_mis(tmp.h, agg.ctypes.data_as(vp), C.byref(na)))
    return agg, na.value


def _host_csr_from_scipy(G):
    G = G.tocsr()
    rp = np.ascontiguousarray(G.indptr, np.int64)
    ci = np.ascontiguousarray(G.indices, np.int64)
    va = np.ascontiguousarray(G.data, np.float64)
    h = vp()
    _ck(_lib.amg_host_csr_create(G.shape[0], G.shape[1], rp.ctypes.data_as(vp), ci.ctypes.data_as(vp),
                                 va.ctypes.data_as(vp), C.byref(h)))
    return h


def sa_tentative_block(ctx, agg_of, naggs, near_null, block_size=1, candidate_dimension=None):
    """Tentative SA interpolation for k candidates (interpolation/mod.rs:754-805):
    returns (P, coarse near-null (naggs*cd) x k)."""
    agg = np.ascontiguousarray(agg_of, np.int64)
    nn = _colmajor_host(near_null, len(agg) * block_size)
    k = nn.shape[1]
    cd = k if candidate_dimension is None else candidate_dimension
    cnn = np.zeros((naggs * cd, k), order="F")
    h = vp()
    _ck(_lib.amg_sa_tentative_block(ctx.h, len(agg), block_size, agg.ctypes.data_as(vp), naggs,
                                    nn.ctypes.data_as(vp), nn.shape[0], k, cd, C.byref(h),
                                    cnn.ctypes.data_as(vp)))
    return SparseMatOp(h, ctx), cnn


def block_jacobi(A, P_, block_size, omega=0.66):
    """block_jacobi P smoothing (interpolation/mod.rs:963-1028)."""
    h = vp()
    _ck(_lib.amg_block_jacobi_smooth(A.h, P_.h, block_size, omega, C.byref(h)))
    return SparseMatOp(h, A.ctx)


def nn_postprocess(A, x, iters=3):
    """Coarse near-null post-processing for k columns (hierarchy.rs:219-228)."""
    x = np.array(_colmajor_host(x, A.nrows), copy=True, order="F")
    _ck(_lib.amg_nn_postprocess(A.h, iters, x.ctypes.data_as(vp), x.shape[0], x.shape[1]))
    return x


def elasticity_q1(elements, contrast=1.0, nu=0.3, seed=42, permute=True):
    """Host CSR of the C5 stand-in: Q1 hex elasticity, block size 3 (gen.cpp).
    permute: False none, True over all nodes, an int W >= 2 within windows of W nodes."""
    ex, ey, ez = elements
    mode = 0 if permute is False else 1 if permute is True else int(permute)
    h = vp()
    _ck(_lib.amg_gen_elasticity_q1(ex, ey, ez, contrast, nu, seed, mode, C.byref(h)))
    return HostCsr(h)


def constant_candidates(n, block_size):
    """block_size constant-per-component near-null vectors, orthonormal (n x bs)."""
    nn = np.zeros((n, block_size), order="F")
    for c in range(block_size):
        nn[c::block_size, c] = 1.0
    return nn / np.sqrt(n // block_size)


def stationary_solve(A, M, b, x, max_iter=100, rel_tol=1e-8):
    """examples/simple_geometric.rs:117-158 on device vectors; returns (iters, hist)."""
    hist = np.zeros(max_iter)
    it = i64()
    with _ordered(A.ctx, AMG_MEM_DEVICE):
        _ck(_lib.amg_stationary_solve(A.h, M.h, vp(b.data_ptr()), vp(x.data_ptr()), max_iter,
                                      rel_tol, hist.ctypes.data_as(vp), C.byref(it)))
    return it.value, hist[:it.value]


def pcg_solve(A, M, b, x, max_iter=1000, rel_tol=1e-8, abs_tol=0.0):
    hist = np.zeros(max(max_iter, 1))
    it = i64()
    with _ordered(A.ctx, AMG_MEM_DEVICE):
        _ck(_lib.amg_pcg_solve(A.h, None if M is None else M.h, vp(b.data_ptr()),
                               vp(x.data_ptr()), max_iter, rel_tol, abs_tol,
                               hist.ctypes.data_as(vp), C.byref(it)))
    return it.value, hist[:min(it.value, max_iter)]


class BlockSmoother(LinOp):
    """BlockSmoother (block_smoothers.rs:80-291): block Jacobi over a node
    partition, diagonally compensated blocks solved exactly."""

    def __init__(self, A, node_partition, naggregates=None, block_size=1):
        part = np.ascontiguousarray(node_partition, np.int64)
        nagg = int(part.max()) + 1 if naggregates is None else int(naggregates)
        h = vp()
        _ck(_lib.amg_block_smoother_create(A.h, part.ctypes.data_as(vp), nagg, int(block_size),
                                           C.byref(h)))
        super().__init__(h, A.ctx, refs=(A,))

    def to_sparse(self):
        """BlockSmoother::into_sparse_mat: the block-diagonal inverse as a SparseMatOp."""
        h = vp()
        _ck(_lib.amg_block_smoother_to_csr(self.h, C.byref(h)))
        return SparseMatOp(h, self.ctx)


class Composite(LinOp):
    """Composite (preconditioners/composite.rs): components c_0..c_{m-1} applied
    c_{m-1}..c_1, c_0, c_1..c_{m-1}, each step out += c(r); r = rhs - A out."""

    def __init__(self, A, components):
        comps = list(components)
        arr = (vp * len(comps))(*[c.h for c in comps])
        h = vp()
        _ck(_lib.amg_composite_create(A.h, arr, len(comps), C.byref(h)))
        super().__init__(h, A.ctx, refs=(A, *comps))

    def push(self, component):
        _ck(_lib.amg_composite_push(self.h, component.h))
        self._refs = tuple(self._refs) + (component,)
        return self

    def ncomponents(self):
        v = i64()
        _ck(_lib.amg_composite_ncomponents(self.h, C.byref(v)))
        return v.value


# ------------------------------------------------------------------ multi-GPU

def rccl_library():
    """Path of the librccl the library bound to ('' if none could be loaded)."""
    return _lib.amg_rccl_library().decode()


def unique_id():
    """ncclUniqueId bytes (create on rank 0, broadcast out of band)."""
    n = _lib.amg_comm_unique_id_size()
    buf = (C.c_char * n)()
    _ck(_lib.amg_comm_get_unique_id(buf))
    return bytes(buf)


class LoopbackHub:
    """In-process transport hub: `nranks` virtual ranks driven by host threads."""

    def __init__(self, nranks):
        h = vp()
        _ck(_lib.amg_loopback_hub_create(nranks, C.byref(h)))
        self.h = h
        self.nranks = nranks

    def __del__(self, _destroy=_lib.amg_loopback_hub_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None


class Comm:
    """Per-process communicator: RCCL (`uid` from unique_id()) or loopback (`hub`)."""

    def __init__(self, ctx, nranks=None, rank=0, uid=None, hub=None):
        h = vp()
        if hub is not None:
            _ck(_lib.amg_comm_create_loopback(ctx.h, hub.h, rank, C.byref(h)))
            self._hub = hub
        else:
            buf = (C.c_char * len(uid)).from_buffer_copy(uid)
            _ck(_lib.amg_comm_create(ctx.h, nranks, rank, buf, C.byref(h)))
        self.h = h
        self.ctx = ctx
        r, n = i32(), i32()
        _ck(_lib.amg_comm_rank(h, C.byref(r), C.byref(n)))
        self.rank, self.nranks = r.value, n.value

    def barrier(self):
        _ck(_lib.amg_comm_barrier(self.h))

    def allreduce_max(self, v):
        d = dbl(v)
        _ck(_lib.amg_comm_allreduce_max(self.h, C.byref(d)))
        return d.value

    def allreduce_sum(self, v):
        d = dbl(v)
        _ck(_lib.amg_comm_allreduce_sum(self.h, C.byref(d)))
        return d.value

    def __del__(self, _destroy=_lib.amg_comm_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None


class DistMultigrid(LinOp):
    """Row-block distributed V-cycle built from a global multigrid on this rank.

    level_splits: list (one per level) of nranks+1 row splits."""

    def __init__(self, comm, mg_global, level_splits, agglomerate_rows=1 << 16):
        s = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int64) for x in level_splits]))
        h = vp()
        _ck(_lib.amg_dist_multigrid_create(comm.h, mg_global.h, s.ctypes.data_as(vp),
                                           int(agglomerate_rows), C.byref(h)))
        super().__init__(h, comm.ctx)
        self.comm = comm
        self.nlevels = len(level_splits)

    def local_rows(self):
        b, e = i64(), i64()
        _ck(_lib.amg_dist_local_rows(self.h, C.byref(b), C.byref(e)))
        return b.value, e.value

    def level_info(self, l):
        info = np.zeros(6, np.int64)
        _ck(_lib.amg_dist_level_info(self.h, l, info.ctypes.data_as(vp)))
        keys = ("n_own", "n_ghost", "n_neighbors", "redundant", "halo_recv", "n_global")
        return dict(zip(keys, (int(v) for v in info)))

    def level_operator(self, l):
        h = vp()
        _ck(_lib.amg_dist_level_operator(self.h, l, C.byref(h)))
        return LinOp(h, self.ctx, refs=(self,))

    def level_matrix(self, l, which="A"):
        """This rank's local CSR of level l (owned rows, [owned | ghost] columns)."""
        h = vp()
        _ck(_lib.amg_dist_level_matrix(self.h, l, {"A": 0, "R": 1, "P": 2}[which], C.byref(h)))
        return SparseMatOp(h, self.ctx, refs=(self,))

    def set_overlap(self, on=True):
        """Overlap halo exchanges with the interior rows of their SpMV (default on)."""
        _ck(_lib.amg_dist_set_option(self.h, 0, 1 if on else 0))
        return self

    def cycle_plan(self, cap=4096):
        """The launches of one distributed V-cycle on this rank (amg_dist_cycle_plan;
        collective: every rank calls it), as Multigrid.cycle_plan."""
        n = i64()
        recs = (LaunchRec * cap)()
        _ck(_lib.amg_dist_cycle_plan(self.h, recs, cap, C.byref(n)))
        return [{"level": r.level, "role": ROLES.get(r.role, "?"), "kernel": r.kernel,
                 "mode": MODES.get(r.mode, "?"), "name": r.name.decode(), "rows": r.rows,
                 "bytes": r.bytes, "csr_bytes": r.csr_bytes} for r in recs[:min(cap, n.value)]]

    def set_graph(self, on=True):
        """hipGraph replay of the distributed cycle (RCCL communicators only; default off)."""
        _ck(_lib.amg_dist_set_option(self.h, 1, 1 if on else 0))
        return self

    def set_per_colour_halo(self, on=True):
        """SGS levels: exchange only the colour swept last before each colour (default on)."""
        _ck(_lib.amg_dist_set_option(self.h, 2, 1 if on else 0))
        return self

    def pcg_solve(self, b, x, max_iter=1000, rel_tol=1e-8, abs_tol=0.0, precondition=True):
        """Distributed PCG (dots all-reduced), one distributed V-cycle per iteration."""
        hist = np.zeros(max(max_iter, 1))
        it = i64()
        with _ordered(self.ctx, AMG_MEM_DEVICE):
            _ck(_lib.amg_dist_pcg_solve(self.h, 1 if precondition else 0, vp(b.data_ptr()),
                                        vp(x.data_ptr()), max_iter, rel_tol, abs_tol,
                                        hist.ctypes.data_as(vp), C.byref(it)))
        return it.value, hist[:min(it.value, max_iter)]

    def stationary_solve(self, b, x, max_iter=100, rel_tol=1e-8):
        hist = np.zeros(max_iter)
        it = i64()
        with _ordered(self.ctx, AMG_MEM_DEVICE):
            _ck(_lib.amg_dist_stationary_solve(self.h, vp(b.data_ptr()), vp(x.data_ptr()),
                                               max_iter, rel_tol, hist.ctypes.data_as(vp),
                                               C.byref(it)))
        return it.value, hist[:it.value]


def _i64(a):
    return np.ascontiguousarray(a, np.int64)


class HaloPlan:
    """Host-side halo plan of one level on one rank (amg_halo_plan_*; no device):
    the library's own planner, driven step by step so any process layout (a gloo
    test, a custom launcher) can exchange the requests itself."""

    def __init__(self, nranks, rank, splits):
        sp_ = _i64(splits)
        if len(sp_) != nranks + 1:
            raise ValueError("splits must have nranks + 1 entries")
        h = vp()
        _ck(_lib.amg_halo_plan_create(nranks, rank, sp_.ctypes.data_as(vp), C.byref(h)))
        self.h, self.nranks, self.rank = h, nranks, rank

    def __del__(self, _destroy=_lib.amg_halo_plan_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None

    def add_columns(self, cols):
        c = _i64(cols)
        _ck(_lib.amg_halo_plan_add_columns(self.h, len(c), c.ctypes.data_as(vp)))

    def requests(self):
        """(ghost ids sorted, ids to request from each rank as a list of arrays)."""
        cnt = np.zeros(self.nranks, np.int64)
        ng = i64()
        _ck(_lib.amg_halo_plan_requests(self.h, cnt.ctypes.data_as(vp), C.byref(ng)))
        ids = np.zeros(max(1, ng.value), np.int64)
        _ck(_lib.amg_halo_plan_ghost_ids(self.h, ids.ctypes.data_as(vp)))
        ids = ids[:ng.value]
        off = np.concatenate([[0], np.cumsum(cnt)])
        return ids, [ids[off[q]:off[q + 1]] for q in range(self.nranks)]

    def set_incoming(self, per_rank_ids):
        cnt = _i64([len(x) for x in per_rank_ids])
        ids = _i64(np.concatenate([np.asarray(x, np.int64) for x in per_rank_ids] + [np.zeros(0, np.int64)]))
        _ck(_lib.amg_halo_plan_set_incoming(self.h, cnt.ctypes.data_as(vp),
                                            ids.ctypes.data_as(vp) if len(ids) else None))

    def info(self):
        v = np.zeros(6, np.int64)
        _ck(_lib.amg_halo_plan_info(self.h, v.ctypes.data_as(vp)))
        return dict(zip(("n_own", "n_ghost", "neighbors", "nsend", "nrecv", "r0"), (int(x) for x in v)))

    def neighbors(self):
        k = self.info()["neighbors"]
        nbr = np.zeros(max(1, k), np.int32)
        arrs = [np.zeros(max(1, k), np.int64) for _ in range(4)]
        _ck(_lib.amg_halo_plan_neighbors(self.h, nbr.ctypes.data_as(vp), *[a.ctypes.data_as(vp) for a in arrs]))
        return {"nbr": nbr[:k], "soff": arrs[0][:k], "scnt": arrs[1][:k], "roff": arrs[2][:k], "rcnt": arrs[3][:k]}

    def send_indices(self):
        n = self.info()["nsend"]
        idx = np.zeros(max(1, n), np.int32)
        _ck(_lib.amg_halo_plan_send_indices(self.h, idx.ctypes.data_as(vp)))
        return idx[:n]

    def remap(self, M):
        """scipy CSR with global columns -> (CSR with [owned | ghost] columns, lo, hi)."""
        import scipy.sparse as sps
        M = M.tocsr()
        rp, ci = _i64(M.indptr), _i64(M.indices)
        out = np.zeros(max(1, len(ci)), np.int32)
        lo, hi = i64(), i64()
        _ck(_lib.amg_halo_plan_remap(self.h, M.shape[0], rp.ctypes.data_as(vp), ci.ctypes.data_as(vp),
                                     out.ctypes.data_as(vp), C.byref(lo), C.byref(hi)))
        inf = self.info()
        L = sps.csr_matrix((M.data.copy(), out[:len(ci)].astype(np.int64), rp.copy()),
                           shape=(M.shape[0], inf["n_own"] + inf["n_ghost"]))
        return L, lo.value, hi.value


def first_redundant_level(level_rows, agglomerate_rows):
    """The first level the distributed multigrid gathers and cycles redundantly."""
    r = _i64(level_rows)
    v = i64()
    _ck(_lib.amg_dist_first_redundant_level(len(r), r.ctypes.data_as(vp), agglomerate_rows, C.byref(v)))
    return v.value


def slab_splits(level_dims, nranks):
    """Row splits per level for a z-slab partition of box-coarsened grids:
    rank p owns planes [floor(p*nz/P), floor((p+1)*nz/P)) of every level."""
    out = []
    for (nx, ny, nz) in level_dims:
        planes = [(p * nz) // nranks for p in range(nranks + 1)]
        out.append([z * nx * ny for z in planes])
    return out


def box_level_dims(dims, box, nlevels):
    d = [tuple(dims)]
    for _ in range(nlevels - 1):
        d.append(tuple(-(-a // b) for a, b in zip(d[-1], box)))
    return d


# ------------------------------------------------------------------ loaders

class HostCsr:
    """Host CSR from a loader (int64 row pointers / columns, f64 values)."""

    def __init__(self, h, owner=None):
        self.h = h
        self._owner = owner  # borrowed from an MfemSystem when set

    def __del__(self, _destroy=_lib.amg_host_csr_destroy):
        if getattr(self, "h", None) and self._owner is None:
            _destroy(self.h)
            self.h = None

    def dims(self):
        m, n, z = i64(), i64(), i64()
        _ck(_lib.amg_host_csr_dims(self.h, C.byref(m), C.byref(n), C.byref(z)))
        return m.value, n.value, z.value

    def arrays(self):
        m, _, z = self.dims()
        rp = np.zeros(m + 1, np.int64)
        ci = np.zeros(z, np.int64)
        va = np.zeros(z, np.float64)
        _ck(_lib.amg_host_csr_arrays(self.h, rp.ctypes.data_as(vp), ci.ctypes.data_as(vp),
                                     va.ctypes.data_as(vp)))
        return rp, ci, va

    def to_scipy(self):
        import scipy.sparse as sps
        m, n, _ = self.dims()
        rp, ci, va = self.arrays()
        return sps.csr_matrix((va, ci, rp), shape=(m, n))

    def upload(self, ctx):
        h = vp()
        _ck(_lib.amg_host_csr_upload(ctx.h, self.h, C.byref(h)))
        return SparseMatOp(h, ctx)


def read_mtx(path):
    """Matrix Market coordinate file -> HostCsr (utils.rs:508-534 semantics)."""
    h = vp()
    _ck(_lib.amg_mtx_read(os.fsencode(path), C.byref(h)))
    return HostCsr(h)


class MfemSystem:
    """dir/name.{mtx,bdy,coords,rhs} (load_mfem_linear_system, utils.rs:269-350)."""

    def __init__(self, directory, name, delete_boundary=True):
        h = vp()
        _ck(_lib.amg_mfem_load(os.fsencode(directory), os.fsencode(name),
                               1 if delete_boundary else 0, C.byref(h)))
        self.h = h
        info = np.zeros(5, np.int64)
        _ck(_lib.amg_mfem_info(self.h, info.ctypes.data_as(vp)))
        self.n, self.rhs_cols, self.coord_dim, self.original_dim, nb = (int(v) for v in info)
        mh = vp()
        _ck(_lib.amg_mfem_matrix(self.h, C.byref(mh)))
        self.matrix = HostCsr(mh, owner=self)
        self.rhs = np.zeros((self.n, self.rhs_cols), order="F")
        self.coords = np.zeros((self.n, self.coord_dim), order="F")
        self.boundary = np.zeros(nb, np.int64)
        self.solution_to_mesh = np.zeros(self.n, np.int64)
        self.mesh_to_solution = np.zeros(self.original_dim, np.int64)
        _ck(_lib.amg_mfem_rhs(self.h, self.rhs.ctypes.data_as(vp), max(1, self.n)))
        _ck(_lib.amg_mfem_coords(self.h, self.coords.ctypes.data_as(vp), max(1, self.n)))
        _ck(_lib.amg_mfem_boundary(self.h, self.boundary.ctypes.data_as(vp)))
        _ck(_lib.amg_mfem_index_maps(self.h, self.solution_to_mesh.ctypes.data_as(vp),
                                     self.mesh_to_solution.ctypes.data_as(vp)))

    def __del__(self, _destroy=_lib.amg_mfem_destroy):
        if getattr(self, "h", None):
            _destroy(self.h)
            self.h = None
