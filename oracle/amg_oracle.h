/*
 * amg_oracle.h -- CPU restatement of the faer-amg V-cycle hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product (faer-amg_amd/) never links it.
 *
 * PARITY UNPINNED: the reference (aujxn/faer-amg, Rust) cannot be built here
 * (no cargo/rustc; its faer 0.23.2 path fork is not vendored) and it ships no
 * tests, fixtures or golden vectors.  This restatement is
 * cross-checked against an independent numpy/scipy restatement
 * (oracle/np_oracle.py) and against closed-form answers; see DESIGN.md.
 *
 * Storage mirrors the reference: CSR with usize (int64) row pointers and
 * column indices, fp64 values, ascending columns (faer SparseRowMat<usize,f64>).
 */
#ifndef AMG_ORACLE_H
#define AMG_ORACLE_H
#include <stdint.h>

typedef struct orc_csr {
    int64_t nrows, ncols, nnz;
    int64_t *rowptr, *col;
    double *val;
} orc_csr;

/* ---- CSR handles ---- */
orc_csr *orc_csr_new(int64_t nrows, int64_t ncols, int64_t nnz);
orc_csr *orc_csr_import(int64_t nrows, int64_t ncols, const int64_t *rowptr,
                        const int64_t *col, const double *val);
void orc_csr_free(orc_csr *A);
void orc_csr_dims(const orc_csr *A, int64_t *out3);
void orc_csr_export(const orc_csr *A, int64_t *rowptr, int64_t *col, double *val);

/* ---- generators ---- */
orc_csr *orc_gen_laplace3d_7pt(int64_t nx, int64_t ny, int64_t nz);
void orc_aniso27_stencil(double ex, double ey, double ez, double *c27);
orc_csr *orc_gen_aniso27(int64_t nx, int64_t ny, int64_t nz, double ex, double ey, double ez);
orc_csr *orc_gen_fd1d(int64_t n_elements);
orc_csr *orc_gen_laplace2d_5pt(int64_t n_elements);

/* ---- kernels ---- */
void orc_spmv(const orc_csr *A, const double *x, double *y);
void orc_spmv_omp(const orc_csr *A, const double *x, double *y);
void orc_diag_jacobi(const orc_csr *A, double omega, double *d);
void orc_diag_l1(const orc_csr *A, double *d);
void orc_diag_l2(const orc_csr *A, double *d);
int64_t orc_greedy_coloring(const orc_csr *A, int64_t *color);
void orc_sgs_apply_in_place(const orc_csr *A, const int64_t *color, int64_t ncolors, double *r);

/* ---- dense Cholesky (coarse solver) ---- */
int orc_chol_factor(int64_t n, const double *a_rowmajor, double *L_rowmajor);
void orc_chol_solve(int64_t n, const double *L, double *b);
void orc_csr_to_dense(const orc_csr *A, double *dense_rowmajor);

/* ---- ParSpmmOp restatement (CPU baseline) ---- */
typedef struct orc_parspmm orc_parspmm;
orc_parspmm *orc_parspmm_new(const orc_csr *A);
void orc_parspmm_apply(const orc_parspmm *op, const double *x, double *y);
void orc_parspmm_free(orc_parspmm *op);

/* ---- sparse products / setup ---- */
orc_csr *orc_spgemm(const orc_csr *A, const orc_csr *B);
orc_csr *orc_transpose(const orc_csr *A);
orc_csr *orc_smooth_interpolation(const orc_csr *A, const orc_csr *P, double omega);
orc_csr *orc_rap(const orc_csr *R, const orc_csr *A, const orc_csr *P);
orc_csr *orc_sa_tentative(int64_t n, const int64_t *agg_of, int64_t naggs, const double *nn,
                          double *coarse_nn);
void orc_nn_stationary_l1(const orc_csr *A, int64_t iters, double *x);
int64_t orc_box_aggregates(int64_t nx, int64_t ny, int64_t nz, int64_t bx, int64_t by,
                           int64_t bz, int64_t *agg_of, int64_t *cdims);

/* ---- multigrid ---- */
typedef struct orc_mg orc_mg;
enum { ORC_SM_DIAG = 0, ORC_SM_SGS = 1, ORC_SM_CHOL = 2, ORC_SM_CSR = 3 };
orc_mg *orc_mg_new(int64_t nlevels);
void orc_mg_free(orc_mg *mg);
void orc_mg_set_op(orc_mg *mg, int64_t level, const orc_csr *A);
void orc_mg_set_transfer(orc_mg *mg, int64_t level, const orc_csr *R, const orc_csr *P);
void orc_mg_set_diag(orc_mg *mg, int64_t level, const double *d);
void orc_mg_set_sgs(orc_mg *mg, int64_t level, const int64_t *color, int64_t ncolors);
int orc_mg_set_chol(orc_mg *mg, int64_t level);
/* Smoother given as an explicit sparse matrix M (apply_in_place: r <- M r), e.g.
 * BlockSmoother::into_sparse_mat (block_smoothers.rs:122-146).  M is borrowed. */
void orc_mg_set_csr_smoother(orc_mg *mg, int64_t level, const orc_csr *M);
void orc_mg_set_cycle(orc_mg *mg, int64_t mu, int64_t steps);
void orc_mg_set_parallel(orc_mg *mg, int64_t enable, int64_t nthreads);
void orc_mg_apply(orc_mg *mg, const double *rhs, double *out);

/* ---- solve drivers ---- */
int64_t orc_stationary_solve(const orc_csr *A, orc_mg *mg, const double *b, double *x,
                             int64_t max_iter, double rel_tol, double *hist);
int64_t orc_pcg_solve(const orc_csr *A, orc_mg *mg, const double *diag_pc, const double *b,
                      double *x, int64_t max_iter, double rel_tol, double abs_tol,
                      double *hist);
#endif
