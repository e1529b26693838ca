/*
 * amg.h -- C ABI of the MI355X-native faer-amg V-cycle path (libfaer_amg_amd.so).
 *
 * One handle type, amg_linop, stands for the reference's `Arc<dyn LinOp<f64>>`
 * (faer matrix_free::{LinOp, Precond, BiLinOp, BiPrecond}); every constructor
 * returns one.  Handles are reference counted: amg_linop_destroy drops the
 * caller's reference, and operators that hold other operators (a multigrid
 * holding its A/S/R/P) keep their own.  Each entry point below names the
 * reference interface it replaces (paths relative to the reference root).
 *
 * Errors: every function returns amg_status; AMG_OK is 0.  The message of the
 * last failure on the calling thread is amg_last_error().  The reference
 * panics instead; its binding panics on non-zero status.
 *
 * Memory: vectors are column-major n x k blocks with a leading dimension, as
 * faer MatRef/MatMut.  AMG_MEM_DEVICE pointers are read/written
 * asynchronously on the context's HIP stream (synchronise with
 * amg_ctx_synchronize); AMG_MEM_HOST pointers are staged through the device
 * and the call returns after the result is back on the host.
 *
 * Threading: handles are immutable after construction except through the
 * amg_multigrid_add_level / amg_multigrid_set builders; apply calls on one
 * handle must not run concurrently (workspaces are preallocated).
 */
#ifndef FAER_AMG_AMD_AMG_H
#define FAER_AMG_AMD_AMG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum amg_status {
    AMG_OK = 0,
    AMG_ERR_INVALID = 1,     /* bad argument (null handle, negative size, ...) */
    AMG_ERR_DIM = 2,         /* dimension mismatch (the reference's assert_eq! panics) */
    AMG_ERR_UNSUPPORTED = 3, /* valid input the library does not handle (e.g. nnz >= 2^31) */
    AMG_ERR_NOT_SPD = 4,     /* Cholesky factorization failed */
    AMG_ERR_HIP = 5,         /* HIP runtime error / no device */
    AMG_ERR_RCCL = 6,        /* RCCL error */
    AMG_ERR_OOM = 7          /* device allocation failed */
} amg_status;

typedef enum amg_mem { AMG_MEM_HOST = 0, AMG_MEM_DEVICE = 1 } amg_mem;

typedef enum amg_linop_kind {
    AMG_KIND_CSR = 0,       /* sparse matrix (SparseMatOp / ParSpmmOp / SparseRowMat) */
    AMG_KIND_DIAG = 1,      /* Diag<f64> smoother: Jacobi, L1, L2 */
    AMG_KIND_SGS = 2,       /* multicolor symmetric Gauss-Seidel */
    AMG_KIND_COARSE = 3,    /* coarse Cholesky solve */
    AMG_KIND_MULTIGRID = 4, /* Multigrid */
    AMG_KIND_DIST_CSR = 5,  /* row-block distributed sparse matrix */
    AMG_KIND_DIST_MULTIGRID = 6,
    AMG_KIND_COMPOSITE = 7, /* Composite (preconditioners/composite.rs) */
    AMG_KIND_BLOCK = 8      /* BlockSmoother (preconditioners/block_smoothers.rs) */
} amg_linop_kind;

typedef struct amg_ctx amg_ctx;
typedef struct amg_linop amg_linop;
typedef struct amg_host_csr amg_host_csr; /* host CSR (loaders, generators, strength graphs) */

/* ---- errors, context ------------------------------------------------------ */

/* Thread-local message of the last non-OK status on this thread ("" if none). */
const char *amg_last_error(void);
/* Library version string. */
const char *amg_version(void);

/* Bind device `device` (one process per GPU).  `hip_stream` may be NULL (the
 * library creates its own non-blocking stream) or an existing hipStream_t to
 * order work with the caller's (e.g. torch.cuda.current_stream()). */
amg_status amg_ctx_create(int device, void *hip_stream, amg_ctx **out);
amg_status amg_ctx_destroy(amg_ctx *ctx);
amg_status amg_ctx_synchronize(amg_ctx *ctx);
amg_status amg_ctx_stream(amg_ctx *ctx, void **hip_stream);
/* Order the context stream against another stream (e.g. the caller's
 * torch.cuda.current_stream()): ctx_waits != 0 makes the context stream wait
 * for the work already queued on `other`; ctx_waits == 0 makes `other` wait for
 * the context stream.  Event-based, no host synchronisation. */
amg_status amg_ctx_join_stream(amg_ctx *ctx, void *other, int32_t ctx_waits);
/* SpMV storage policy for matrices built after the call (process-wide):
 * 0 auto -- per matrix the cheapest of: DIA codes (square, <= 32 diagonals or a
 * known run pattern, >= 80 % filled, <= 256 distinct values), 3x3 block storage
 * (block operators), stencil classes (structured Galerkin operators, >= 64
 * offsets; with a grid hint x-staged per grid tile, also for shorter stencils and
 * instead of a > 27-diagonal DIA pattern when that times faster at setup), pattern
 * SELL (structured operators incl. rectangular R/P; the R/P of amg_sa_build_box
 * get the grid-transfer-class overlay, one 8-bit class per row), x-staged
 * SELL (gather-heavy fp64 SELL whose x footprint per 4096 rows fits LDS),
 * SELL-64 with compressed columns and value codes (short regular rows),
 * wave-per-row (rows averaging >= 256 entries), CSR-stream otherwise
 * (DESIGN.md 2); 1 CSR-stream only, 2 SELL-64 whenever rows are <= 256 long,
 * 3 wave-per-row for every matrix.  Results agree to the summation order of the
 * rows (bitwise for rows summed by one lane, which every storage but the
 * long-row CSR-stream / wave-per-row paths does). */
amg_status amg_set_spmv_format(int32_t policy);
/* Value storage of SELL-64 matrices built after the call (process-wide):
 * 1 (default) stores a 4 / 8 / 16-bit code per entry into a per-matrix table of
 * the distinct fp64 bit patterns when the matrix has at most 16 / 256 / 65536 of
 * them (the padding's 0.0 included); 0 always stores fp64 values.  A decoded
 * value is the stored value bit for bit, so results do not change. */
amg_status amg_set_value_codes(int32_t enable);
/* Device allocation policy for buffers allocated after the call: 0 (default)
 * hipMalloc.  1 (physically contiguous buffers >= 16 MiB) is refused with
 * AMG_ERR_UNSUPPORTED: on gfx950 it let kernels read stale data written by the
 * previous kernel on the same stream. */
amg_status amg_set_alloc_policy(int32_t policy);

/* ---- sparse matrices (replaces SparseMatOp::new core.rs:56-74, ParSpmmOp::new
 *      par_spmm.rs:31-96, and the SparseRowMat<usize,f64> LinOp used at
 *      multigrid.rs:137-158) -------------------------------------------------- */

/* Run-time switches (no reference counterpart; measured A/B paths, every
 * setting bitwise neutral): 0 = fold the zero-guess step on x-staged class
 * levels (default 0, env FAMG_FOLD_XSCS), 1 = read a constant coded Jacobi
 * diagonal as one scalar (default 1, env FAMG_DIA_DK), 2 = waves per row of the
 * wave-per-row kernel (0 auto = chosen per matrix at finalize, 1/2/4; env
 * FAMG_VEC_WPR), 3 = where the wide grid-transfer classes (gtx.hip) are kept:
 * 0 wherever they build, 1 where they beat the transfer operator's other storage
 * in a setup-time timing, 2 (default) on operators of >= 2^18 rows (env
 * FAMG_GTX_TIME), 4 = marching
 * 27-point SGS phases (sgs27.hip): 0 = one workgroup per tile and plane, 1 = auto
 * (about one workgroup per CU), n >= 2 = n planes per workgroup (default 1, env
 * FAMG_SGS27_MARCH), 5 = x-staged SELL kernel (xsell.hip): 2 = one burst of
 * loads per row group with LDS-DMA staging (default), 1 = software-pipelined
 * batches, 0 = the round-4 kernel (env FAMG_XS_PIPE), 6 = 3x3-block SpMV kernel
 * (bsr.hip): 0 = the round-2 kernel (default), 1 = node columns first, 4-step
 * batches, 2 = columns first, 2-step batches pipelined, 3 = 4-step pipelined
 * (env FAMG_BSR_KERNEL), 7 = 3x3-block matrices whose slices (64 node rows)
 * average at least this many block steps take the long-row kernel that loads
 * the next 8 steps' node columns ahead (default 48, env FAMG_BSR_LONG; -1
 * never), 8 = row pairs per lane of the constant 7-point DIA kernel: 0 auto
 * (default: 2 for SET, 1 for the cycle's epilogues), 1, 2 or 4 adjacent 512-row
 * blocks per workgroup (env FAMG_DIA7_RP), 9 = the fine level of a constant
 * 7-point box hierarchy as marching fused kernels (fine.hip): 0 = off, 1 = on
 * (default), n >= 2 = n planes per workgroup (env FAMG_FINE_FUSE).  Setting one
 * makes every multigrid re-capture its hipGraph at its next apply.  amg_get_flag
 * reads the current value. */
amg_status amg_set_flag(int32_t which, int64_t value);
amg_status amg_get_flag(int32_t which, int64_t *value);
/* Stencil-class storage of a CSR operator (structured Galerkin operators whose
 * rows repeat up to a shift; replaces the value/column streams of
 * interpolation/mod.rs:828's A_c in SpMV): info4 = {classes, offsets K (padded
 * to 8), class-id bits, dictionary bytes}; zeros when the operator uses another
 * storage. */
amg_status amg_csr_class_info(const amg_linop *op, int64_t *info4);
/* Grid hint (no reference counterpart: the reference's SparseMatOp has no
 * geometry): the rows of the square operator are the points of an nx x ny x nz
 * grid, x fastest.  Stencil-class operators whose nonzero offsets are grid steps
 * that stay inside the grid then run x-staged per grid tile (scs.hip,
 * bitwise the same sums).  Re-finalizes the SpMV storage: call before the
 * operator is used (graphs captured earlier would read released storage).  The
 * stencil generators and amg_sa_build_box set it for the levels they make;
 * 0,0,0 clears it (and stops the inference below).  A square operator created
 * without a hint (amg_csr_create: the drop-in path, multigrid.rs:190-239 /
 * core.rs:56-74 callers) gets one inferred at finalize from the stencil of 64
 * sample rows (amg_grid_from_offsets); every consumer of the hint (x-staged
 * classes, grid-transfer classes in amg_multigrid_add_level, fused SGS phases)
 * checks every entry against it.  FAMG_INFER_GRID=0 turns the inference off. */
amg_status amg_csr_set_grid(amg_linop *op, int64_t nx, int64_t ny, int64_t nz);
/* The grid inference on its own (host only, no device): grid3 = (nx, ny, nz) of
 * an n-row square operator whose stencil has the k offsets offs (col - row,
 * any order, repeats allowed); *found = 0 when no grid explains them. */
amg_status amg_grid_from_offsets(const int64_t *offs, int64_t k, int64_t n, int64_t *grid3, int32_t *found);
/* The fused SpMV epilogues the V-cycle runs (multigrid.rs:337-369, 407-424),
 * on device vectors, asynchronous on the context stream: mode 0 y = A x, 1
 * y += A x, 2 y = b - A x, 3 y = x + d (b - A x) (weighted Jacobi step; d the
 * scaled inverse diagonal).  x != y. */
amg_status amg_csr_spmv_epilogue(const amg_linop *op, int32_t mode, const double *x, double *y,
                                 const double *b, const double *d);
/* info12 (13 entries) = {nx, ny, nz (0: no hint), x-staged (0/1), tile tx, ty,
 * tz, halo rx, ry, rz, hint source (0 none, 1 given, 2 inferred), grid-transfer
 * classes (0 none, 1 as P, 2 as R: 8-bit gtc.hip; 3 as P, 4 as R: 16-bit
 * gtx.hip), how the x-staged tile was chosen (1 the frozen per-shape table of
 * tuning.cpp, 2 timed at setup, 3 FAMG_XSCS_TILE)}. */
amg_status amg_csr_grid_info(const amg_linop *op, int64_t *info12);

/* Copy a host CSR with usize-compatible (int64) row pointers and column indices
 * and fp64 values to the device.  Columns must be sorted ascending within each
 * row and in [0, ncols).  Stored internally with 32-bit indices: returns
 * AMG_ERR_UNSUPPORTED if nrows, ncols or nnz >= 2^31. */
amg_status amg_csr_create(amg_ctx *ctx, int64_t nrows, int64_t ncols, const int64_t *rowptr,
                          const int64_t *colidx, const double *vals, amg_linop **out);
/* Same from device arrays with 32-bit indices (copied). */
amg_status amg_csr_create_device_i32(amg_ctx *ctx, int64_t nrows, int64_t ncols,
                                     const int32_t *rowptr, const int32_t *colidx,
                                     const double *vals, amg_linop **out);
/* Number of stored entries of a CSR operator. */
amg_status amg_csr_nnz(const amg_linop *op, int64_t *nnz);
/* SpMV storage chosen for a CSR operator: info8 = {kernel (0 CSR-stream,
 * 1 SELL-64, 2 vector, 3 DIA codes, 4 3x3 blocks, 5 pattern SELL with lanes per row, 6 stencil
 * classes, 7 x-staged SELL: slices counted as 16-bit when their x is staged in LDS, 32-bit
 * when they escape to global columns), matrix
 * bytes one SpMV streams, CSR bytes (12 nnz +
 * 4 (n+1)), SELL slices, SELL stored entries incl. padding, SELL slices with
 * implicit / 16-bit delta / 32-bit column indices}. */
amg_status amg_csr_spmv_info(const amg_linop *op, int64_t *info8);
/* Value codes of a CSR operator's SpMV storage: info2 = {code bits (0 = fp64
 * values, 4, 8, 16), table entries}. */
amg_status amg_csr_value_codes(const amg_linop *op, int64_t *info2);
/* DIA-code rows of a CSR operator's SpMV storage: info4 = {first row, end row,
 * diagonals, code bits}; all 0 without DIA storage.  The range is the whole
 * matrix (kernel 3 in amg_csr_spmv_info) or one row segment beside SELL / CSR
 * storage (the halo interior of a distributed level). */
amg_status amg_csr_dia_range(const amg_linop *op, int64_t *info4);
/* Copy a CSR operator back to host arrays (rowptr: nrows+1, colidx/vals: nnz). */
amg_status amg_csr_download(const amg_linop *op, int64_t *rowptr, int64_t *colidx, double *vals);
/* Device-side generators for the benchmark operators:
 * 3-D 7-point Laplacian (6 / -1) and 3-D 27-point anisotropic Q1 diffusion on an
 * nx*ny*nz Dirichlet interior grid; row = x + nx*(y + ny*z). */
amg_status amg_gen_laplace3d_7pt(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz,
                                 amg_linop **out);
amg_status amg_gen_aniso27(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz, double ex,
                           double ey, double ez, amg_linop **out);
/* General (non-stencil) SPD operator of the same size: the 7-point graph with
 * edge weights 0.5 + U[0,1) (splitmix64 of the edge and seed), a_ij = -w_ij,
 * a_ii = sum of the six incident weights (1.0 for a missing, Dirichlet
 * neighbour), rows and columns permuted symmetrically by a seeded bijection:
 * window < 0 none, 0 over all rows, > 0 within consecutive windows of that many
 * rows (locality of a mesh numbering without stencil structure). */
amg_status amg_gen_random_7pt(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz, uint64_t seed, int64_t window,
                              amg_linop **out);

/* In-tree stand-in for config C5 (Flan_1565, which cannot be fetched): Q1
 * hexahedral linear elasticity on an ex x ey x ez element box, per-element
 * Young's modulus 10^(contrast (2u - 1)) (u ~ U[0,1) from splitmix64(seed)),
 * Poisson ratio nu, the x = 0 face clamped, free nodes renumbered by a seeded
 * random permutation (permute 0: none, 1: over all nodes, W >= 2: within
 * consecutive windows of W nodes); 3 dofs per node interleaved
 * (block_size 3).  Host CSR (upload with amg_host_csr_upload). */
amg_status amg_gen_elasticity_q1(int64_t ex, int64_t ey, int64_t ez, double contrast, double nu,
                                 uint64_t seed, int32_t permute, amg_host_csr **out);

/* ---- generic LinOp / Precond / BiPrecond (faer matrix_free traits) -------- */

amg_status amg_linop_kind_of(const amg_linop *op, int32_t *kind);
/* LinOp::nrows / ncols */
amg_status amg_linop_dims(const amg_linop *op, int64_t *nrows, int64_t *ncols);
/* LinOp::apply: out = M * rhs, out overwritten (par_spmm.rs:117,151; multigrid.rs:469).
 * out: nrows x k (ld_out), rhs: ncols x k (ld_rhs). */
amg_status amg_linop_apply(amg_linop *op, double *out, int64_t ld_out, const double *rhs,
                           int64_t ld_rhs, int64_t k, amg_mem mem);
/* BiLinOp::transpose_apply.  Supported for the symmetric operators (smoothers,
 * coarse solve, multigrid -- multigrid.rs:487-502) and for CSR matrices. */
amg_status amg_linop_transpose_apply(amg_linop *op, double *out, int64_t ld_out,
                                     const double *rhs, int64_t ld_rhs, int64_t k, amg_mem mem);
/* Precond::apply_in_place: rhs <- M * rhs (coarse_solvers.rs:254; faer Diag). */
amg_status amg_precond_apply_in_place(amg_linop *op, double *rhs, int64_t ld, int64_t k,
                                      amg_mem mem);
/* BiPrecond::transpose_apply_in_place (coarse_solvers.rs:270). */
amg_status amg_precond_transpose_apply_in_place(amg_linop *op, double *rhs, int64_t ld,
                                                int64_t k, amg_mem mem);
/* Drop the caller's reference. */
amg_status amg_linop_destroy(amg_linop *op);

/* ---- smoothers (smoothers.rs:24-86) and coarse solver (coarse_solvers.rs) -- */

/* new_jacobi: d_i = omega / a_ii (smoothers.rs:78-86). */
amg_status amg_jacobi_create(const amg_linop *A, double omega, amg_linop **out);
/* new_l1: d_i = 1 / sum_j |a_ij| (smoothers.rs:63-76). */
amg_status amg_l1_create(const amg_linop *A, amg_linop **out);
/* new_l2 (smoothers.rs:43-61). */
amg_status amg_l2_create(const amg_linop *A, amg_linop **out);
/* Diag from explicit host values (faer Diag<f64>). */
amg_status amg_diag_create(amg_ctx *ctx, int64_t n, const double *d, amg_linop **out);
/* SmootherKind::SymGaussSeidel (smoothers.rs:20,26 -- unimplemented! in the
 * reference; definition in DESIGN.md): multicolor SGS on A e = r from e = 0.
 * colors: host array of nrows colors in [0, ncolors) or NULL for greedy
 * first-fit coloring in row order. */
amg_status amg_sgs_create(const amg_linop *A, const int32_t *colors, amg_linop **out);
/* SGS smoothers built after the call run their sweeps as fused plane-parity
 * phases (sgs27.hip) where that applies -- a 27-point grid operator stored as
 * DIA codes with the parity colouring -- instead of one launch per colour:
 * enable 1 (default) three phases per SGS step, 2 four phases, 0 colour
 * launches (FAMG_SGS_FUSED=0/2 sets the default).  Bitwise the same results. */
amg_status amg_set_sgs_fused(int32_t enable);
/* *fused = 1 if this SGS smoother runs the fused phases. */
amg_status amg_sgs_fused(const amg_linop *op, int32_t *fused);
/* Number of colors of an SGS smoother. */
amg_status amg_sgs_ncolors(const amg_linop *op, int64_t *ncolors);
/* Storage of the color sweeps: info4 = {colors, kernel (as amg_csr_spmv_info:
 * 1 SELL, 3 DIA codes of the color-permuted copy, ...), diagonals, code bits}. */
amg_status amg_sgs_info(const amg_linop *op, int64_t *info4);
/* CoarseSolverKind::Cholesky (coarse_solvers.rs:21-33, SparseCholeskySolve
 * :172-181): exact coarse solve.  Returns AMG_ERR_NOT_SPD if A is not SPD and
 * AMG_ERR_UNSUPPORTED above 16384 rows (dense factor). */
amg_status amg_coarse_chol_create(const amg_linop *A, amg_linop **out);

/* ---- multigrid (multigrid.rs:171-424) -------------------------------------- */

/* Multigrid::new(op, smoother) (multigrid.rs:190-199): mu = 1, steps = 1. */
amg_status amg_multigrid_create(amg_linop *op, amg_linop *smoother, amg_linop **out);
/* Multigrid::add_level(op, smoother, r, p) (multigrid.rs:228-239).  r: n_c x n_f,
 * p: n_f x n_c where n_f is the previous level's size and n_c = op's size;
 * AMG_ERR_DIM otherwise (hierarchy.rs:258-264 asserts). */
amg_status amg_multigrid_add_level(amg_linop *mg, amg_linop *op, amg_linop *smoother,
                                   amg_linop *r, amg_linop *p);
/* with_cycle_type(mu) / with_smoothing_steps(steps) (multigrid.rs:204-214); both > 0. */
amg_status amg_multigrid_set(amg_linop *mg, int64_t mu, int64_t steps);
amg_status amg_multigrid_levels(const amg_linop *mg, int64_t *levels);
/* Enable/disable hipGraph capture of whole V-cycles (default on). */
amg_status amg_multigrid_set_graph(amg_linop *mg, int32_t enable);
/* Options: 0 = hipGraph capture (as above); 1 = SGS smoothing in the literal
 * residual form of smooth() (multigrid.rs:418-423: r = f - A x; x += SGS(r))
 * instead of the fused in-place sweep on x (default 0: fused, one SpMV fewer);
 * 2 = fold the first Jacobi step from v = 0 (v = d f, s = 1) into the residual
 * and correction SpMVs instead of storing it (default 1; bitwise identical), on
 * levels whose operator is fp64 SELL with mostly short columns, x-staged SELL,
 * or DIA codes whose P runs the short-slice kernel; amg_multigrid_cycle_plan
 * reports which levels fold (RESID0 / ADD0 launches); 3 = fused grid transfers:
 * removed in round 5 (measured slower twice); only 0 is accepted.  4 = a
 * restriction stored as wide grid-transfer classes (gtx.hip) also writes the
 * next level's first Jacobi step from zero, d_c f_c, beside f_c (SPMV_SETDF)
 * instead of a separate pass (default 1; bitwise identical). */
amg_status amg_multigrid_set_option(amg_linop *mg, int32_t option, int64_t value);
/* Multigrid option 5 -- locality reordering (reorder.hip; no reference
 * counterpart): the cycle runs a level of a general operator (no grid storage,
 * a diagonal smoother, >= 65536 rows) in a locality numbering of its node graph
 * (its nodes grouped by aggregate in the renumbered coarse level's order, or
 * reverse Cuthill-McKee, whichever touches fewer x cache lines) -- renumbered
 * copies of A_l, its diagonal, R_l and P_l whose rows keep their stored entry
 * order and their original's kind of storage -- with one gather of rhs and one
 * scatter of the result per apply when the fine level is renumbered.  0 off,
 * 1 (default) where the result stays bitwise (every operator whose rows move
 * sums a row independently of its neighbours) and it at least halves the x
 * cache lines an SpMV slice of 64 rows touches, 2 every eligible level (equal
 * to rounding).  amg_multigrid_get_level returns the caller's operators,
 * amg_multigrid_get_run_level the ones the cycle runs (the renumbered copies of
 * a renumbered level); *reordered = 1 when level runs renumbered. */
amg_status amg_multigrid_level_reordered(amg_linop *mg, int64_t level, int32_t *reordered);
amg_status amg_multigrid_get_run_level(amg_linop *mg, int64_t level, amg_linop **A, amg_linop **S,
                                       amg_linop **R, amg_linop **P);
/* Multigrid::apply == amg_linop_apply on a multigrid handle. */
amg_status amg_multigrid_apply(amg_linop *mg, double *out, int64_t ld_out, const double *rhs,
                               int64_t ld_rhs, int64_t k, amg_mem mem);

/* Launch plan of one V-cycle: the kernels the library launches for one
 * amg_multigrid_apply, in launch order, each with the algorithmic bytes of
 * that launch (the bytes its storage streams + the vectors it reads and
 * writes) and the same launch priced with 32-bit CSR matrix bytes
 * (SURVEY.md 8(d)).  Recorded by running one eager (non-graph) cycle on
 * scratch vectors with the recorder on, so fold decisions, SGS colour launches
 * and storage choices are the ones the cycle makes.  recs may be NULL (count
 * only); at most cap records are written, *count = records of the cycle. */
typedef enum amg_role {
    AMG_ROLE_SMOOTH = 0,   /* pre/post smoothing (smooth, multigrid.rs:407-424) */
    AMG_ROLE_RESID = 1,    /* r = f - A v (:341-342), incl. a folded zero-guess step */
    AMG_ROLE_RESTRICT = 2, /* f_c = R r (:343) */
    AMG_ROLE_INTERP = 3,   /* v += P v_c (:349-350), incl. a folded d*f */
    AMG_ROLE_COARSE = 4,   /* coarsest solve (:291) */
    AMG_ROLE_OTHER = 5
} amg_role;
typedef struct amg_launch_rec {
    int32_t level, role, kernel, mode; /* kernel as amg_csr_spmv_info (-1: vector op); mode: SET 0,
                                          ADD 1, RESID 2, JACOBI 3, SGS 4, RESID0 5, ADD0 6,
                                          SETDF 7 = SET + d*y (-1) */
    int64_t rows;                      /* rows this launch updates */
    int64_t bytes;                     /* algorithmic bytes */
    int64_t csr_bytes;                 /* with 12 nnz + 4 (m+1) matrix bytes (= bytes for vector ops) */
    char name[32];                     /* storage kernel ("dia", "sell_short", "dia_sgs", "vec_mul" ...) */
} amg_launch_rec;
amg_status amg_multigrid_cycle_plan(amg_linop *mg, amg_launch_rec *recs, int64_t cap, int64_t *count);
/* One of the fine level's fused launches (no reference counterpart: the fused
 * forms of multigrid.rs:341-343 and 349-369 on a constant 7-point box
 * hierarchy, fine.hip), exactly as amg_multigrid_apply makes it, on the cycle's
 * own workspace, asynchronous on the context stream: which 0 = the folded
 * residual + restriction (rhs in; level 1's f and first Jacobi step written),
 * 1 = interpolation + post-smoothing (rhs and level 1's v in; out written).
 * Device pointers, n = the fine level's rows.  AMG_ERR_UNSUPPORTED where the
 * cycle does not take that launch.  For timing the cycle's dominant kernels
 * on their own (bench.py roofline). */
amg_status amg_multigrid_fine_launch(amg_linop *mg, int32_t which, double *out, const double *rhs);
/* In-cycle timing of one fused fine-level launch (no reference counterpart:
 * measurement): which 0 / 1 as amg_multigrid_fine_launch, -1 off.  While on,
 * every cycle records a pair of HIP events around that launch on the context
 * stream (the cycle then runs its launches eagerly, not as its hipGraph: HIP
 * cannot time events recorded by graph nodes); *ms = the time between the pair
 * of the last completed cycle.  Setting it drops the captured graphs. */
amg_status amg_multigrid_set_fine_timer(amg_linop *mg, int32_t which);
amg_status amg_multigrid_fine_timer_ms(amg_linop *mg, float *ms);
/* The same for a distributed multigrid: one eager cycle (halo exchanges
 * included: collective, every rank calls it) on this rank's scratch vectors;
 * level = global level index (the redundant tail's levels after the
 * distributed ones), rows = this rank's rows. */
amg_status amg_dist_cycle_plan(amg_linop *dist, amg_launch_rec *recs, int64_t cap, int64_t *count);
/* The first 16 hex digits of sha256 over the library's sources (the .hip,
 * .cpp, .hpp and .inc files of csrc in sorted order, then this header) it was built from: the
 * Python package and __graft_entry__.build() compare it with the tree and
 * refuse / rebuild a stale prebuilt library. */
const char *amg_source_hash(void);
/* Launch the marker kernel k_trace_mark(tag) on the context stream: brackets a
 * region of a rocprofv3 kernel trace (bench.py marks its timed V-cycles, and
 * scripts/prof_summary.py keeps the dispatches between the marks). */
amg_status amg_trace_mark(amg_ctx *ctx, int32_t tag);

/* ---- Galerkin setup kernels (interpolation/mod.rs:716-720, 824-828, 927-946) - */

/* C = A * B (faer sparse x sparse). */
amg_status amg_spgemm(const amg_linop *A, const amg_linop *B, amg_linop **out);
/* R = P^T as a CSR (interpolation/mod.rs:824-827). */
amg_status amg_transpose(const amg_linop *P, amg_linop **out);
/* A_c = R * (A * P) (interpolation/mod.rs:828). */
amg_status amg_galerkin_rap(const amg_linop *R, const amg_linop *A, const amg_linop *P,
                            amg_linop **out);
/* smooth_interpolation: P_s = A P scaled by -(omega/a_ii) per row, plus P
 * (interpolation/mod.rs:927-946). */
amg_status amg_smooth_interpolation(const amg_linop *A, const amg_linop *P, double omega,
                                    amg_linop **out);
/* Tentative SA interpolation for one candidate (interpolation/mod.rs:754-805):
 * agg_of[i] in [0,naggs) (host), near_null (host, n); coarse_nn (host, naggs) out. */
amg_status amg_sa_tentative(amg_ctx *ctx, int64_t n, const int64_t *agg_of, int64_t naggs,
                            const double *near_null, amg_linop **P, double *coarse_nn);
/* Coarse near-null post-processing (hierarchy.rs:219-228): L1 StationaryIteration
 * (`iters` steps, smoothers.rs:146-158) then normalization; x is host, in/out. */
amg_status amg_nn_stationary_l1(const amg_linop *A, int64_t iters, double *x);

/* Smoothed-aggregation hierarchy on a structured nx*ny*nz grid with bx*by*bz box
 * aggregates and one constant candidate (Hierarchy::coarsen, hierarchy.rs:190-248,
 * box aggregates standing in for the modularity partitioner -- DESIGN.md).
 * Coarsens until the coarse size <= coarsest_dim or max_levels (0 = unlimited).
 * smoother: 0 Jacobi(omega), 1 L1, 2 SGS (greedy coloring; L1 on levels needing
 * > 32 colors), 3 BlockSmoother over the level's box aggregates, on every level
 * but the coarsest, which gets the Cholesky coarse solve.  Returns the multigrid. */
amg_status amg_sa_build_box(amg_linop *A, int64_t nx, int64_t ny, int64_t nz, int64_t bx,
                            int64_t by, int64_t bz, int64_t coarsest_dim, int64_t max_levels,
                            double omega, int32_t smoother, amg_linop **mg_out);
/* ---- smoothed aggregation on general (unstructured, block) matrices -----------
 * Hierarchy::coarsen (hierarchy.rs:190-248) with AggregationConfig /
 * smoothed_aggregation (interpolation/mod.rs:62-156, 730-836): strength graph
 * (partitioners/mod.rs:337-393, block-reduced :294-301), aggregates seeded by
 * maximal_independent_set (:395-423; stands in for the modularity partitioner,
 * DESIGN.md), tentative P from a per-aggregate thin SVD of the near-null block,
 * P smoothing by Jacobi (block size 1) or block_jacobi (:963-1028), R = P^T,
 * A_c = R A P, coarse near-null by 3 L1 stationary steps + thin QR; the coarse
 * block size is candidate_dimension. */
typedef struct amg_sa_config {
    int64_t block_size;          /* dofs per node of A (SparseMatOp block_size, core.rs:56) */
    int64_t candidate_dimension; /* candidates kept per aggregate (<= near-null columns) */
    int64_t strength_depth;      /* BFS depth of the strength graph (reference: 3) */
    int64_t smoothing_steps;     /* P smoothing steps (AggregationConfig default 1) */
    int64_t coarsest_dim;        /* stop when the coarse size <= this (default 1000) */
    int64_t max_levels;          /* 0 = unlimited */
    double omega;                /* Jacobi smoother weight (smoother 0) */
    int32_t smoother;            /* 0 Jacobi, 1 L1 (default), 2 SGS, 3 BlockSmoother(aggregates) */
    int32_t reserved;
} amg_sa_config;
amg_status amg_sa_config_default(amg_sa_config *cfg);
/* near_null: n x k column-major (leading dimension ld), host; weights: k host
 * values of the strength inner product or NULL for create_weights
 * (examples/amg/main.rs:571-580: 1 / v^T A v).  Returns the multigrid (smoother
 * per cfg on every level but the coarsest, which gets the Cholesky solve). */
amg_status amg_sa_build(amg_linop *A, const double *near_null, int64_t ld, int64_t k, const double *weights,
                        const amg_sa_config *cfg, amg_linop **mg_out);
/* The pieces (for tests and custom hierarchies): node-level strength graph as a
 * host CSR (values = strengths); MIS-seeded aggregates of such a graph;
 * tentative P for k candidates on nnodes nodes of block_size dofs (coarse_nn:
 * (naggs*cd) x k column-major, leading dimension naggs*cd); block_jacobi P
 * smoothing; coarse near-null post-processing of x (n x k, ld) in place. */
amg_status amg_strength_graph(const amg_linop *A, const double *near_null, int64_t ld, int64_t k,
                              const double *weights, int64_t depth, int64_t block_size, amg_host_csr **out);
amg_status amg_aggregate_mis(const amg_host_csr *graph, int64_t *agg_of, int64_t *naggs);
amg_status amg_sa_tentative_block(amg_ctx *ctx, int64_t nnodes, int64_t block_size, const int64_t *agg_of,
                                  int64_t naggs, const double *near_null, int64_t ld, int64_t k, int64_t cd,
                                  amg_linop **P, double *coarse_nn);
amg_status amg_block_jacobi_smooth(const amg_linop *A, const amg_linop *P, int64_t block_size, double omega,
                                   amg_linop **out);
amg_status amg_nn_postprocess(const amg_linop *A, int64_t iters, double *x, int64_t ld, int64_t k);

/* Level accessors of a multigrid: A_l, R_l, P_l (l < levels-1), smoother S_l.
 * Returned handles are new references. */
amg_status amg_multigrid_get_level(const amg_linop *mg, int64_t level, amg_linop **A,
                                   amg_linop **S, amg_linop **R, amg_linop **P);

/* ---- solve drivers (the callers of the hot path) ------- */

/* BlockSmoother (block_smoothers.rs:80-291), BlockSolver(Cholesky) kind:
 * block Jacobi over a partition of the n/block_size nodes (node_partition[i] in
 * 0..naggregates-1); each block is the aggregate's submatrix with the
 * couplings leaving it folded into its diagonal (diagonally_compensate
 * :293-324; block_size > 1: diagonally_compensate_vector :326-400) and is
 * solved exactly (dense LL^T inverse per block, <= 8192 rows per block).
 * AMG_ERR_NOT_SPD if a compensated block is not SPD. */
amg_status amg_block_smoother_create(const amg_linop *A, const int64_t *node_partition,
                                     int64_t naggregates, int64_t block_size, amg_linop **out);
/* BlockSmoother::into_sparse_mat (:122-146): the block-diagonal inverse as CSR. */
amg_status amg_block_smoother_to_csr(const amg_linop *bs, amg_linop **out);
/* Composite (preconditioners/composite.rs:11-83) as a LinOp/Precond on A:
 * components c_0..c_{m-1} are applied c_{m-1},...,c_1,c_0,c_1,...,c_{m-1}
 * (2m-1 steps), each step out += c(r); r = rhs - A out, from out = 0 and
 * r = rhs.  Components are any preconditioning handles (apply_in_place). */
amg_status amg_composite_create(const amg_linop *A, amg_linop *const *components,
                                int64_t ncomponents, amg_linop **out);
/* Composite::push */
amg_status amg_composite_push(amg_linop *composite, const amg_linop *component);
amg_status amg_composite_ncomponents(const amg_linop *composite, int64_t *n);
/* Stationary solver of examples/simple_geometric.rs:117-158 on device vectors:
 * loop { r = b - A x; rho = ||r||/||b||; hist[it] = rho; stop if rho < rel_tol or
 * it+1 >= max_iter; x += M r }.  b, x device pointers (n); hist host (max_iter).
 * *iters = number of residual evaluations. */
amg_status amg_stationary_solve(amg_linop *A, amg_linop *M, const double *b, double *x,
                                int64_t max_iter, double rel_tol, double *hist, int64_t *iters);
/* Preconditioned CG (faer conjugate_gradient caller, utils.rs:600): stops when
 * ||r|| <= max(abs_tol, rel_tol ||b||); M may be NULL (identity).
 * *iters = iterations (max_iter+1 if not converged); hist host (max_iter) gets
 * ||r_k||/||b||. */
amg_status amg_pcg_solve(amg_linop *A, amg_linop *M, const double *b, double *x,
                         int64_t max_iter, double rel_tol, double abs_tol, double *hist,
                         int64_t *iters);

/* ---- multi-GPU (row-block partition + RCCL halo exchange) ------- */

/* The reference has no distributed backend (rayon only).  Here the
 * V-cycle is row-block partitioned: rank p owns a contiguous row range of
 * every level; before each SpMV the ghost entries its rows reference are
 * refreshed by a halo exchange (grouped RCCL send/recv over xGMI); levels with
 * fewer than `agglomerate_rows` rows are gathered (ncclAllGather) and solved
 * redundantly on every rank. */
typedef struct amg_comm amg_comm;
typedef struct amg_loopback_hub amg_loopback_hub;
/* Path of the librccl the library bound to (the one already mapped in the
 * process, e.g. torch's, else $FAMG_RCCL_PATH / librccl.so.1); "" if none loads. */
const char *amg_rccl_library(void);
/* ncclUniqueId size in bytes (128). */
int32_t amg_comm_unique_id_size(void);
/* Fill `id` (amg_comm_unique_id_size() bytes) on rank 0; broadcast it out of band. */
amg_status amg_comm_get_unique_id(void *id);
/* One RCCL communicator per process (one process per GPU). */
amg_status amg_comm_create(amg_ctx *ctx, int32_t nranks, int32_t rank, const void *id,
                           amg_comm **out);
/* In-process transport for validation: `nranks` virtual ranks, each driven by
 * its own host thread with its own context, exchange through device copies. */
amg_status amg_loopback_hub_create(int32_t nranks, amg_loopback_hub **out);
amg_status amg_loopback_hub_destroy(amg_loopback_hub *hub);
amg_status amg_comm_create_loopback(amg_ctx *ctx, amg_loopback_hub *hub, int32_t rank,
                                    amg_comm **out);
amg_status amg_comm_destroy(amg_comm *comm);
amg_status amg_comm_rank(const amg_comm *comm, int32_t *rank, int32_t *nranks);
amg_status amg_comm_barrier(amg_comm *comm);
/* Max / sum over ranks of a host double (reduced on the device). */
amg_status amg_comm_allreduce_max(amg_comm *comm, double *value);
amg_status amg_comm_allreduce_sum(amg_comm *comm, double *value);

/* Distributed multigrid from a global multigrid held by every rank (identical
 * on all ranks, e.g. built redundantly by amg_sa_build_box).  level_splits:
 * nlevels x (nranks+1) row splits (row range of rank p at level l is
 * [s[l*(nranks+1)+p], s[l*(nranks+1)+p+1])).  Levels from the first one with
 * fewer than agglomerate_rows rows down are run redundantly on every rank.
 * Every distributed level must be smoothed by a diagonal (Jacobi/L1/L2) or a
 * multicolor SGS smoother; SGS sweeps the global coloring restricted to the
 * owned rows with one halo exchange before every color (the single-GPU sweep's
 * values on every rank).  apply() maps the rank's owned rows of rhs (n_own) to
 * its owned rows of out. */
amg_status amg_dist_multigrid_create(amg_comm *comm, const amg_linop *mg_global,
                                     const int64_t *level_splits, int64_t agglomerate_rows,
                                     amg_linop **out);
/* Row range [begin, end) of this rank at the finest level. */
amg_status amg_dist_local_rows(const amg_linop *dist, int64_t *begin, int64_t *end);
/* Per-level plan: info[0..5] = n_owned, n_ghost, n_neighbors, redundant (0/1),
 * halo doubles received per exchange, global rows. */
amg_status amg_dist_level_info(const amg_linop *dist, int64_t level, int64_t *info6);
/* The distributed A_l as a LinOp (owned rows in, owned rows out; halo inside). */
amg_status amg_dist_level_operator(const amg_linop *dist, int64_t level, amg_linop **out);
/* This rank's local CSR of a distributed level (which: 0 A_l, 1 R_l, 2 P_l):
 * owned rows, columns in the level's [owned | ghost] numbering. */
amg_status amg_dist_level_matrix(const amg_linop *dist, int64_t level, int32_t which,
                                 amg_linop **out);
/* Options of a distributed multigrid: 0 = overlap each halo exchange with the
 * interior rows of the SpMV that consumes it (default 1; 0 exchanges first);
 * 1 = replay apply() as a captured hipGraph per (out, rhs) pair (default 0;
 * RCCL communicators only -- the loopback transport always runs eagerly);
 * 2 = multicolor SGS levels exchange, before each colour, only the ghost
 * entries of the colour swept just before it (per-colour halo lists; default
 * 1; 0 refreshes the whole halo before every colour).  The plans of
 * amg_dist_cycle_plan carry the exchanges as records of kernel -2 (bytes this
 * rank sends + receives). */
amg_status amg_dist_set_option(amg_linop *dist, int32_t option, int64_t value);
/* Distributed stationary solve (dots all-reduced over ranks): local vectors. */
amg_status amg_dist_stationary_solve(amg_linop *dist_mg, const double *b, double *x,
                                     int64_t max_iter, double rel_tol, double *hist,
                                     int64_t *iters);
/* Distributed PCG on the finest distributed operator, preconditioned by one
 * distributed V-cycle per iteration (precondition = 0: plain CG): the same loop
 * as amg_pcg_solve with every dot all-reduced over the ranks;
 * b, x local (owned rows). */
amg_status amg_dist_pcg_solve(amg_linop *dist_mg, int32_t precondition, const double *b, double *x,
                              int64_t max_iter, double rel_tol, double abs_tol, double *hist,
                              int64_t *iters);

/* ---- host-side distributed planning (no device; faer-amg_amd/csrc/plan.hpp) --
 * The planner amg_dist_multigrid_create runs per level, exported so it can be
 * driven (and tested) from any process layout: rank p owns rows
 * [splits[p], splits[p+1]); add the global column ids of every local matrix
 * that reads the level's vector (A_l, R_l rows and P_{l-1} rows owned here);
 * amg_halo_plan_requests finalises the ghost set (sorted global ids, grouped by
 * owner) and returns how many ids go to each rank; after the ranks have
 * exchanged their request lists, amg_halo_plan_set_incoming builds the send
 * lists (in_ids: the ids every rank requested from this one, concatenated in
 * rank order) and the neighbour table.  amg_halo_plan_remap renumbers a local
 * matrix's columns into [owned | ghost] and returns the interior row segment
 * [lo, hi) (the longest run of rows reading owned entries only). */
typedef struct amg_halo_plan amg_halo_plan;
amg_status amg_halo_plan_create(int32_t nranks, int32_t rank, const int64_t *splits, amg_halo_plan **out);
amg_status amg_halo_plan_destroy(amg_halo_plan *plan);
amg_status amg_halo_plan_add_columns(amg_halo_plan *plan, int64_t nnz, const int64_t *cols);
/* req_counts: nranks entries (may be NULL); *n_ghost: ghost entries. */
amg_status amg_halo_plan_requests(amg_halo_plan *plan, int64_t *req_counts, int64_t *n_ghost);
amg_status amg_halo_plan_ghost_ids(const amg_halo_plan *plan, int64_t *ids);
amg_status amg_halo_plan_set_incoming(amg_halo_plan *plan, const int64_t *in_counts, const int64_t *in_ids);
/* info6 = {n_own, n_ghost, neighbours, entries sent per refresh, entries received, first owned row} */
amg_status amg_halo_plan_info(const amg_halo_plan *plan, int64_t *info6);
/* Per neighbour (rank order): send offset/count into the send list, receive
 * offset/count into the ghost region.  Arrays of `neighbours` entries (any may be NULL). */
amg_status amg_halo_plan_neighbors(const amg_halo_plan *plan, int32_t *nbr, int64_t *soff, int64_t *scnt,
                                   int64_t *roff, int64_t *rcnt);
/* The owned local indices packed for the neighbours (entries sent per refresh). */
amg_status amg_halo_plan_send_indices(const amg_halo_plan *plan, int32_t *idx);
amg_status amg_halo_plan_remap(const amg_halo_plan *plan, int64_t nrows, const int64_t *rowptr, const int64_t *cols,
                               int32_t *local_cols, int64_t *lo, int64_t *hi);
/* The first level cycled redundantly (agglomerated): the first l < nlevels-1
 * with level_rows[l] < agglomerate_rows, else the coarsest. */
amg_status amg_dist_first_redundant_level(int64_t nlevels, const int64_t *level_rows, int64_t agglomerate_rows,
                                          int64_t *level);

/* ---- Dataset loaders (utils.rs:269-534) -------------------
 * Host-side; no device needed.  Matrix Market: sparse coordinate files
 * (real/integer/pattern, general/symmetric), 1-based indices, explicit 0.0
 * entries dropped, symmetric entries mirrored, duplicates summed, columns
 * sorted (load_matrix_triplets, utils.rs:508-534, + faer try_new_from_triplets). */
amg_status amg_mtx_read(const char *path, amg_host_csr **out);
/* Host CSR from arrays (copied; values kept as given, zeros included). */
amg_status amg_host_csr_create(int64_t nrows, int64_t ncols, const int64_t *rowptr, const int64_t *colidx,
                               const double *vals, amg_host_csr **out);
amg_status amg_host_csr_dims(const amg_host_csr *h, int64_t *nrows, int64_t *ncols, int64_t *nnz);
amg_status amg_host_csr_arrays(const amg_host_csr *h, int64_t *rowptr, int64_t *colidx, double *vals);
/* Upload to the device (amg_csr_create). */
amg_status amg_host_csr_upload(amg_ctx *ctx, const amg_host_csr *h, amg_linop **out);
amg_status amg_host_csr_destroy(amg_host_csr *h);

/* MFEM linear system dir/name.{mtx,bdy,coords,rhs} (load_mfem_linear_system,
 * utils.rs:269-350); delete_boundary removes the .bdy rows/columns and
 * renumbers the rest in order (utils.rs:446-480).  The VTK mesh geometry the
 * reference also attaches (visualisation only) is not loaded. */
typedef struct amg_mfem_system amg_mfem_system;
amg_status amg_mfem_load(const char *dir, const char *name, int32_t delete_boundary,
                         amg_mfem_system **out);
/* info5 = {n (after deletion), rhs columns, coordinate dimension, original n,
 * boundary indices (sorted, unique)} */
amg_status amg_mfem_info(const amg_mfem_system *sys, int64_t *info5);
/* The system matrix (borrowed; valid while sys lives). */
amg_status amg_mfem_matrix(const amg_mfem_system *sys, const amg_host_csr **out);
/* rhs (n x k) and coords (n x d), column-major with leading dimension ld. */
amg_status amg_mfem_rhs(const amg_mfem_system *sys, double *out, int64_t ld);
amg_status amg_mfem_coords(const amg_mfem_system *sys, double *out, int64_t ld);
amg_status amg_mfem_boundary(const amg_mfem_system *sys, int64_t *out);
/* solution_to_mesh (n entries), mesh_to_solution (original n entries, -1 =
 * deleted); either may be NULL. */
amg_status amg_mfem_index_maps(const amg_mfem_system *sys, int64_t *solution_to_mesh,
                               int64_t *mesh_to_solution);
amg_status amg_mfem_destroy(amg_mfem_system *sys);

#ifdef __cplusplus
}
#endif
#endif
