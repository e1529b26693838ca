/*
 * amg_oracle.c -- CPU restatement of the faer-amg V-cycle hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see amg_oracle.h).  PARITY UNPINNED: there is no
 * buildable reference and no reference golden data; this file restates the
 * reference algorithm function by function, citing /root/reference file:line.
 *
 * Arithmetic conventions (shared with the HIP product so that row-sequential
 * kernels agree bit for bit):
 *   - every sparse row sum is  acc = 0.0; for j ascending: acc = fma(a_ij, x_j, acc)
 *   - no other contraction: this file is compiled with -ffp-contract=off
 */
#include "amg_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_DIE(...)                                                                    \
    do {                                                                                \
        fprintf(stderr, "amg_oracle: " __VA_ARGS__);                                    \
        fprintf(stderr, "\n");                                                          \
        abort();                                                                        \
    } while (0)

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) ORC_DIE("out of memory (%zu bytes)", n);
    return p;
}
static void *xcalloc(size_t n, size_t s) {
    void *p = calloc(n ? n : 1, s ? s : 1);
    if (!p) ORC_DIE("out of memory");
    return p;
}

/* ------------------------------------------------------------------ CSR */

orc_csr *orc_csr_new(int64_t nrows, int64_t ncols, int64_t nnz) {
    orc_csr *A = (orc_csr *)xmalloc(sizeof(orc_csr));
    A->nrows = nrows;
    A->ncols = ncols;
    A->nnz = nnz;
    A->rowptr = (int64_t *)xcalloc((size_t)nrows + 1, sizeof(int64_t));
    A->col = (int64_t *)xmalloc((size_t)nnz * sizeof(int64_t));
    A->val = (double *)xmalloc((size_t)nnz * sizeof(double));
    return A;
}

orc_csr *orc_csr_import(int64_t nrows, int64_t ncols, const int64_t *rowptr,
                        const int64_t *col, const double *val) {
    int64_t nnz = rowptr[nrows];
    orc_csr *A = orc_csr_new(nrows, ncols, nnz);
    memcpy(A->rowptr, rowptr, (size_t)(nrows + 1) * sizeof(int64_t));
    memcpy(A->col, col, (size_t)nnz * sizeof(int64_t));
    memcpy(A->val, val, (size_t)nnz * sizeof(double));
    return A;
}

void orc_csr_free(orc_csr *A) {
    if (!A) return;
    free(A->rowptr);
    free(A->col);
    free(A->val);
    free(A);
}

void orc_csr_dims(const orc_csr *A, int64_t *out3) {
    out3[0] = A->nrows;
    out3[1] = A->ncols;
    out3[2] = A->nnz;
}

void orc_csr_export(const orc_csr *A, int64_t *rowptr, int64_t *col, double *val) {
    memcpy(rowptr, A->rowptr, (size_t)(A->nrows + 1) * sizeof(int64_t));
    memcpy(col, A->col, (size_t)A->nnz * sizeof(int64_t));
    memcpy(val, A->val, (size_t)A->nnz * sizeof(double));
}

static double csr_get(const orc_csr *A, int64_t i, int64_t j, int *found) {
    int64_t lo = A->rowptr[i], hi = A->rowptr[i + 1];
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (A->col[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    if (lo < A->rowptr[i + 1] && A->col[lo] == j) {
        *found = 1;
        return A->val[lo];
    }
    *found = 0;
    return 0.0;
}

/* ------------------------------------------------------------ generators */

/* 3-D 7-point Laplacian on an nx*ny*nz Dirichlet interior grid: diagonal 6,
 * off-diagonals -1.  Row index = x + nx*(y + ny*z). */
orc_csr *orc_gen_laplace3d_7pt(int64_t nx, int64_t ny, int64_t nz) {
    int64_t n = nx * ny * nz;
    int64_t nnz = 7 * n - 2 * (ny * nz + nx * nz + nx * ny);
    orc_csr *A = orc_csr_new(n, n, nnz);
    int64_t e = 0;
    for (int64_t z = 0; z < nz; z++)
        for (int64_t y = 0; y < ny; y++)
            for (int64_t x = 0; x < nx; x++) {
                int64_t i = x + nx * (y + ny * z);
                A->rowptr[i] = e;
                if (z > 0) { A->col[e] = i - nx * ny; A->val[e++] = -1.0; }
                if (y > 0) { A->col[e] = i - nx; A->val[e++] = -1.0; }
                if (x > 0) { A->col[e] = i - 1; A->val[e++] = -1.0; }
                A->col[e] = i; A->val[e++] = 6.0;
                if (x + 1 < nx) { A->col[e] = i + 1; A->val[e++] = -1.0; }
                if (y + 1 < ny) { A->col[e] = i + nx; A->val[e++] = -1.0; }
                if (z + 1 < nz) { A->col[e] = i + nx * ny; A->val[e++] = -1.0; }
            }
    A->rowptr[n] = e;
    if (e != nnz) ORC_DIE("7pt nnz mismatch");
    return A;
}

/* 3-D 27-point anisotropic Q1 diffusion:
 *   a(dx,dy,dz) = ex*(T[dx]*M[dy]*M[dz]) + ey*(M[dx]*T[dy]*M[dz]) + ez*(M[dx]*M[dy]*T[dz])
 * with T = {-1, 2, -1}, M = {1/6, 4/6, 1/6}; entries outside the grid dropped. */
void orc_aniso27_stencil(double ex, double ey, double ez, double *c27) {
    const double T[3] = {-1.0, 2.0, -1.0};
    const double M[3] = {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0};
    for (int dz = 0; dz < 3; dz++)
        for (int dy = 0; dy < 3; dy++)
            for (int dx = 0; dx < 3; dx++)
                c27[dx + 3 * (dy + 3 * dz)] = ex * (T[dx] * M[dy] * M[dz]) +
                                              ey * (M[dx] * T[dy] * M[dz]) +
                                              ez * (M[dx] * M[dy] * T[dz]);
}

orc_csr *orc_gen_aniso27(int64_t nx, int64_t ny, int64_t nz, double ex, double ey, double ez) {
    double c27[27];
    orc_aniso27_stencil(ex, ey, ez, c27);
    int64_t n = nx * ny * nz;
    int64_t nnz = (3 * nx - 2) * (3 * ny - 2) * (3 * nz - 2);
    orc_csr *A = orc_csr_new(n, n, nnz);
    int64_t e = 0;
    for (int64_t z = 0; z < nz; z++)
        for (int64_t y = 0; y < ny; y++)
            for (int64_t x = 0; x < nx; x++) {
                int64_t i = x + nx * (y + ny * z);
                A->rowptr[i] = e;
                for (int dz = -1; dz <= 1; dz++)
                    for (int dy = -1; dy <= 1; dy++)
                        for (int dx = -1; dx <= 1; dx++) {
                            int64_t xx = x + dx, yy = y + dy, zz = z + dz;
                            if (xx < 0 || yy < 0 || zz < 0 || xx >= nx || yy >= ny || zz >= nz)
                                continue;
                            A->col[e] = xx + nx * (yy + ny * zz);
                            A->val[e++] = c27[(dx + 1) + 3 * ((dy + 1) + 3 * (dz + 1))];
                        }
            }
    A->rowptr[n] = e;
    if (e != nnz) ORC_DIE("27pt nnz mismatch");
    return A;
}

/* 1-D finite difference of -u'' (reference examples/simple_geometric.rs:96-113). */
orc_csr *orc_gen_fd1d(int64_t n_elements) {
    double h = 1.0 / (double)n_elements;
    double diag_val = 2.0 / (h * h);
    double off_diag_val = -1.0 / (h * h);
    int64_t n = n_elements - 1;
    orc_csr *A = orc_csr_new(n, n, n > 0 ? 3 * n - 2 : 0);
    int64_t e = 0;
    for (int64_t i = 0; i < n; i++) {
        A->rowptr[i] = e;
        if (i > 0) { A->col[e] = i - 1; A->val[e++] = off_diag_val; }
        A->col[e] = i; A->val[e++] = diag_val;
        if (i + 1 < n) { A->col[e] = i + 1; A->val[e++] = off_diag_val; }
    }
    A->rowptr[n] = e;
    return A;
}

/* 2-D analogue of simple_geometric.rs:96-113 (config C1): 5-point stencil of
 * -Laplace(u) with h = 1/n_elements on the (n_elements-1)^2 interior points. */
orc_csr *orc_gen_laplace2d_5pt(int64_t n_elements) {
    double h = 1.0 / (double)n_elements;
    double diag_val = 4.0 / (h * h);
    double off_diag_val = -1.0 / (h * h);
    int64_t m = n_elements - 1, n = m * m;
    orc_csr *A = orc_csr_new(n, n, 5 * n - 4 * m);
    int64_t e = 0;
    for (int64_t y = 0; y < m; y++)
        for (int64_t x = 0; x < m; x++) {
            int64_t i = x + m * y;
            A->rowptr[i] = e;
            if (y > 0) { A->col[e] = i - m; A->val[e++] = off_diag_val; }
            if (x > 0) { A->col[e] = i - 1; A->val[e++] = off_diag_val; }
            A->col[e] = i; A->val[e++] = diag_val;
            if (x + 1 < m) { A->col[e] = i + 1; A->val[e++] = off_diag_val; }
            if (y + 1 < m) { A->col[e] = i + m; A->val[e++] = off_diag_val; }
        }
    A->rowptr[n] = e;
    return A;
}

/* ----------------------------------------------------------------- SpMV */

/* y = A x, out overwritten (faer LinOp::apply semantics, par_spmm.rs:117 fill(0)
 * then accumulate).  Ascending-column accumulation from 0.0. */
void orc_spmv(const orc_csr *A, const double *x, double *y) {
    for (int64_t i = 0; i < A->nrows; i++) {
        double acc = 0.0;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++)
            acc = fma(A->val[e], x[A->col[e]], acc);
        y[i] = acc;
    }
}

void orc_spmv_omp(const orc_csr *A, const double *x, double *y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->nrows; i++) {
        double acc = 0.0;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++)
            acc = fma(A->val[e], x[A->col[e]], acc);
        y[i] = acc;
    }
}

/* -------------------------------------------------------------- smoothers */

/* new_jacobi: d_i = omega / a_ii (smoothers.rs:78-86). */
void orc_diag_jacobi(const orc_csr *A, double omega, double *d) {
    for (int64_t i = 0; i < A->nrows; i++) {
        int found;
        double aii = csr_get(A, i, i, &found);
        if (!found) ORC_DIE("jacobi: missing diagonal at row %lld", (long long)i);
        d[i] = omega / aii;
    }
}

/* new_l1: d_i = 1 / sum_j |a_ij| (smoothers.rs:63-76), triplet order = row order. */
void orc_diag_l1(const orc_csr *A, double *d) {
    for (int64_t i = 0; i < A->nrows; i++) {
        double s = 0.0;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) s += fabs(A->val[e]);
        d[i] = 1.0 / s;
    }
}

/* new_l2: d_i = 1 / sum_j |a_ij| sqrt(a_ii)/sqrt(a_jj) (smoothers.rs:43-61). */
void orc_diag_l2(const orc_csr *A, double *d) {
    int64_t n = A->nrows;
    double *ds = (double *)xmalloc((size_t)n * sizeof(double));
    for (int64_t i = 0; i < n; i++) {
        int found;
        double aii = csr_get(A, i, i, &found);
        if (!found) ORC_DIE("l2: missing diagonal");
        ds[i] = sqrt(aii);
    }
    for (int64_t i = 0; i < n; i++) {
        double s = 0.0;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            double scale = ds[i] / ds[A->col[e]];
            s += fabs(A->val[e]) * scale;
        }
        d[i] = 1.0 / s;
    }
    free(ds);
}

/* Greedy first-fit coloring in row order (SURVEY.md 8(a) a7 build definition):
 * color_i = smallest color not used by an already-colored neighbour j < i.
 * On structured grids this reproduces the parity colorings (2 colors for 7-pt,
 * 8 for 27-pt). Returns the number of colors. */
int64_t orc_greedy_coloring(const orc_csr *A, int64_t *color) {
    int64_t n = A->nrows, ncolors = 0;
    int64_t cap = 64;
    int64_t *mark = (int64_t *)xmalloc((size_t)cap * sizeof(int64_t));
    for (int64_t c = 0; c < cap; c++) mark[c] = -1;
    for (int64_t i = 0; i < n; i++) {
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            int64_t j = A->col[e];
            if (j < i) {
                int64_t c = color[j];
                if (c >= cap) {
                    int64_t nc = cap * 2 > c + 1 ? cap * 2 : c + 1;
                    mark = (int64_t *)realloc(mark, (size_t)nc * sizeof(int64_t));
                    for (int64_t k = cap; k < nc; k++) mark[k] = -1;
                    cap = nc;
                }
                mark[c] = i;
            }
        }
        int64_t c = 0;
        while (c < cap && mark[c] == i) c++;
        if (c >= cap) {
            int64_t nc = cap * 2;
            mark = (int64_t *)realloc(mark, (size_t)nc * sizeof(int64_t));
            for (int64_t k = cap; k < nc; k++) mark[k] = -1;
            cap = nc;
        }
        color[i] = c;
        if (c + 1 > ncolors) ncolors = c + 1;
    }
    free(mark);
    return ncolors;
}

/* Multicolor symmetric Gauss-Seidel as a Precond::apply_in_place (new; the
 * reference has only unimplemented!(), smoothers.rs:26-27).  Solves A e = r
 * approximately from e = 0: forward sweep colors 0..C-1, backward sweep colors
 * C-2..0 (color C-1 would get an exactly-zero correction), row update
 *   acc = sum_j fma(a_ij, e_j, acc);  e_i = e_i + dinv_i * (r_i - acc),
 * dinv_i = 1/a_ii.  Then r <- e. */
static void sgs_color(const orc_csr *A, const int64_t *color, int64_t c, const double *dinv,
                      const double *r, double *e) {
    for (int64_t i = 0; i < A->nrows; i++) {
        if (color[i] != c) continue;
        double acc = 0.0;
        for (int64_t k = A->rowptr[i]; k < A->rowptr[i + 1]; k++)
            acc = fma(A->val[k], e[A->col[k]], acc);
        e[i] = e[i] + dinv[i] * (r[i] - acc);
    }
}

void orc_sgs_apply_in_place(const orc_csr *A, const int64_t *color, int64_t ncolors, double *r) {
    int64_t n = A->nrows;
    double *dinv = (double *)xmalloc((size_t)n * sizeof(double));
    double *e = (double *)xcalloc((size_t)n, sizeof(double));
    for (int64_t i = 0; i < n; i++) {
        int found;
        double aii = csr_get(A, i, i, &found);
        if (!found) ORC_DIE("sgs: missing diagonal");
        dinv[i] = 1.0 / aii;
    }
    for (int64_t c = 0; c < ncolors; c++) sgs_color(A, color, c, dinv, r, e);
    for (int64_t c = ncolors - 2; c >= 0; c--) sgs_color(A, color, c, dinv, r, e);
    memcpy(r, e, (size_t)n * sizeof(double));
    free(dinv);
    free(e);
}

/* ------------------------------------------------------ dense Cholesky */

void orc_csr_to_dense(const orc_csr *A, double *d) {
    memset(d, 0, (size_t)(A->nrows * A->ncols) * sizeof(double));
    for (int64_t i = 0; i < A->nrows; i++)
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++)
            d[i * A->ncols + A->col[e]] += A->val[e];
}

/* A = L L^T (coarse_solvers.rs:66-71 dense; :172-181 sparse LLt -- the sparse
 * factorization's fill-reducing order differs, so agreement is to rounding). */
int orc_chol_factor(int64_t n, const double *a, double *L) {
    memset(L, 0, (size_t)(n * n) * sizeof(double));
    for (int64_t j = 0; j < n; j++) {
        double s = a[j * n + j];
        for (int64_t k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
        if (!(s > 0.0)) return 1;
        double ljj = sqrt(s);
        L[j * n + j] = ljj;
        for (int64_t i = j + 1; i < n; i++) {
            double t = a[i * n + j];
            for (int64_t k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = t / ljj;
        }
    }
    return 0;
}

void orc_chol_solve(int64_t n, const double *L, double *b) {
    for (int64_t i = 0; i < n; i++) {
        double t = b[i];
        for (int64_t k = 0; k < i; k++) t -= L[i * n + k] * b[k];
        b[i] = t / L[i * n + i];
    }
    for (int64_t i = n - 1; i >= 0; i--) {
        double t = b[i];
        for (int64_t k = i + 1; k < n; k++) t -= L[k * n + i] * b[k];
        b[i] = t / L[i * n + i];
    }
}

/* ------------------------------------------ ParSpmmOp (par_spmm.rs:15-133) */

#define PAR_BLOCK_SIZE 8192

typedef struct {
    int64_t ncols;      /* tile width */
    int64_t *colptr;    /* CSC (usize) */
    int64_t *row;
    double *val;
} orc_tile;

typedef struct {
    int64_t ntiles;
    int64_t *block_cols;
    orc_tile *tiles;
} orc_block_row;

struct orc_parspmm {
    int64_t nrows, ncols, nblocks;
    orc_block_row *rows;
};

/* ParSpmmOp::new (par_spmm.rs:31-96): 8192-row block rows, each split into
 * 8192-column CSC tiles.  The reference's row bound uses mat.ncols()
 * (par_spmm.rs:46, a bug for rectangular P/R); this
 * restatement uses nrows so that it computes the correct product. */
orc_parspmm *orc_parspmm_new(const orc_csr *A) {
    orc_parspmm *op = (orc_parspmm *)xmalloc(sizeof(orc_parspmm));
    op->nrows = A->nrows;
    op->ncols = A->ncols;
    op->nblocks = (A->nrows + PAR_BLOCK_SIZE - 1) / PAR_BLOCK_SIZE;
    op->rows = (orc_block_row *)xcalloc((size_t)op->nblocks, sizeof(orc_block_row));
    int64_t ncb = (A->ncols + PAR_BLOCK_SIZE - 1) / PAR_BLOCK_SIZE;
#pragma omp parallel
    {
        int64_t *cnt = (int64_t *)xcalloc((size_t)ncb + 1, sizeof(int64_t));
#pragma omp for schedule(dynamic, 1)
        for (int64_t b = 0; b < op->nblocks; b++) {
            int64_t r0 = b * PAR_BLOCK_SIZE;
            int64_t r1 = r0 + PAR_BLOCK_SIZE < A->nrows ? r0 + PAR_BLOCK_SIZE : A->nrows;
            memset(cnt, 0, (size_t)(ncb + 1) * sizeof(int64_t));
            for (int64_t e = A->rowptr[r0]; e < A->rowptr[r1]; e++) cnt[A->col[e] / PAR_BLOCK_SIZE]++;
            int64_t nt = 0;
            for (int64_t t = 0; t < ncb; t++) nt += cnt[t] > 0;
            orc_block_row *br = &op->rows[b];
            br->ntiles = nt;
            br->block_cols = (int64_t *)xmalloc((size_t)nt * sizeof(int64_t));
            br->tiles = (orc_tile *)xcalloc((size_t)nt, sizeof(orc_tile));
            int64_t k = 0;
            for (int64_t t = 0; t < ncb; t++) {
                if (!cnt[t]) continue;
                int64_t c0 = t * PAR_BLOCK_SIZE;
                int64_t c1 = c0 + PAR_BLOCK_SIZE < A->ncols ? c0 + PAR_BLOCK_SIZE : A->ncols;
                orc_tile *tl = &br->tiles[k];
                br->block_cols[k] = t;
                tl->ncols = c1 - c0;
                tl->colptr = (int64_t *)xcalloc((size_t)tl->ncols + 1, sizeof(int64_t));
                tl->row = (int64_t *)xmalloc((size_t)cnt[t] * sizeof(int64_t));
                tl->val = (double *)xmalloc((size_t)cnt[t] * sizeof(double));
                /* counting sort into CSC, rows ascending within a column */
                for (int64_t i = r0; i < r1; i++)
                    for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
                        int64_t j = A->col[e];
                        if (j >= c0 && j < c1) tl->colptr[j - c0 + 1]++;
                    }
                for (int64_t c = 0; c < tl->ncols; c++) tl->colptr[c + 1] += tl->colptr[c];
                int64_t *pos = (int64_t *)xmalloc((size_t)tl->ncols * sizeof(int64_t));
                memcpy(pos, tl->colptr, (size_t)tl->ncols * sizeof(int64_t));
                for (int64_t i = r0; i < r1; i++)
                    for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
                        int64_t j = A->col[e];
                        if (j >= c0 && j < c1) {
                            int64_t p = pos[j - c0]++;
                            tl->row[p] = i - r0;
                            tl->val[p] = A->val[e];
                        }
                    }
                free(pos);
                k++;
            }
        }
        free(cnt);
    }
    return op;
}

/* ParSpmmOp::implementation + BlockRow::spmm (par_spmm.rs:98-132): parallel over
 * block rows, out.fill(0), then per tile a CSC scatter (Accum::Add, alpha 1).
 * Per output row the contributions arrive in ascending column order, so the
 * result is bit-identical to orc_spmv. */
void orc_parspmm_apply(const orc_parspmm *op, const double *x, double *y) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t b = 0; b < op->nblocks; b++) {
        int64_t r0 = b * PAR_BLOCK_SIZE;
        int64_t nr = r0 + PAR_BLOCK_SIZE < op->nrows ? PAR_BLOCK_SIZE : op->nrows - r0;
        double *out = y + r0;
        memset(out, 0, (size_t)nr * sizeof(double));
        const orc_block_row *br = &op->rows[b];
        for (int64_t t = 0; t < br->ntiles; t++) {
            const orc_tile *tl = &br->tiles[t];
            const double *xs = x + br->block_cols[t] * PAR_BLOCK_SIZE;
            for (int64_t c = 0; c < tl->ncols; c++) {
                double xc = xs[c];
                for (int64_t p = tl->colptr[c]; p < tl->colptr[c + 1]; p++)
                    out[tl->row[p]] = fma(tl->val[p], xc, out[tl->row[p]]);
            }
        }
    }
}

void orc_parspmm_free(orc_parspmm *op) {
    if (!op) return;
    for (int64_t b = 0; b < op->nblocks; b++) {
        orc_block_row *br = &op->rows[b];
        for (int64_t t = 0; t < br->ntiles; t++) {
            free(br->tiles[t].colptr);
            free(br->tiles[t].row);
            free(br->tiles[t].val);
        }
        free(br->tiles);
        free(br->block_cols);
    }
    free(op->rows);
    free(op);
}

/* --------------------------------------------------------- sparse products */

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* C = A B (faer sparse x sparse, interpolation/mod.rs:720,828,938).  Gustavson
 * with a dense accumulator; every structural product is kept (explicit zeros
 * included); per entry the products are accumulated in ascending k:
 *   c_ij = fma(a_ik, b_kj, c_ij) from 0.0.  Columns sorted ascending. */
orc_csr *orc_spgemm(const orc_csr *A, const orc_csr *B) {
    if (A->ncols != B->nrows) ORC_DIE("spgemm dimension mismatch");
    int64_t m = A->nrows, n = B->ncols;
    int64_t *mark = (int64_t *)xmalloc((size_t)(n ? n : 1) * sizeof(int64_t));
    for (int64_t j = 0; j < n; j++) mark[j] = -1;
    int64_t *rowptr = (int64_t *)xcalloc((size_t)m + 1, sizeof(int64_t));
    for (int64_t i = 0; i < m; i++) {
        int64_t cnt = 0;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            int64_t k = A->col[e];
            for (int64_t f = B->rowptr[k]; f < B->rowptr[k + 1]; f++) {
                int64_t j = B->col[f];
                if (mark[j] != i) { mark[j] = i; cnt++; }
            }
        }
        rowptr[i + 1] = rowptr[i] + cnt;
    }
    orc_csr *C = orc_csr_new(m, n, rowptr[m]);
    memcpy(C->rowptr, rowptr, (size_t)(m + 1) * sizeof(int64_t));
    free(rowptr);
    double *acc = (double *)xcalloc((size_t)(n ? n : 1), sizeof(double));
    for (int64_t j = 0; j < n; j++) mark[j] = -1;
    for (int64_t i = 0; i < m; i++) {
        int64_t p = C->rowptr[i];
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            int64_t k = A->col[e];
            for (int64_t f = B->rowptr[k]; f < B->rowptr[k + 1]; f++) {
                int64_t j = B->col[f];
                if (mark[j] != i) { mark[j] = i; C->col[p++] = j; acc[j] = 0.0; }
            }
        }
        qsort(C->col + C->rowptr[i], (size_t)(p - C->rowptr[i]), sizeof(int64_t), cmp_i64);
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            int64_t k = A->col[e];
            double a = A->val[e];
            for (int64_t f = B->rowptr[k]; f < B->rowptr[k + 1]; f++)
                acc[B->col[f]] = fma(a, B->val[f], acc[B->col[f]]);
        }
        for (int64_t q = C->rowptr[i]; q < C->rowptr[i + 1]; q++) C->val[q] = acc[C->col[q]];
    }
    free(acc);
    free(mark);
    return C;
}

/* R = P^T as a row-major matrix (interpolation/mod.rs:824-827). Stable counting
 * sort: entries of each output row in ascending original-row order. */
orc_csr *orc_transpose(const orc_csr *A) {
    orc_csr *T = orc_csr_new(A->ncols, A->nrows, A->nnz);
    for (int64_t e = 0; e < A->nnz; e++) T->rowptr[A->col[e] + 1]++;
    for (int64_t j = 0; j < A->ncols; j++) T->rowptr[j + 1] += T->rowptr[j];
    int64_t *pos = (int64_t *)xmalloc((size_t)(A->ncols ? A->ncols : 1) * sizeof(int64_t));
    memcpy(pos, T->rowptr, (size_t)A->ncols * sizeof(int64_t));
    for (int64_t i = 0; i < A->nrows; i++)
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++) {
            int64_t p = pos[A->col[e]]++;
            T->col[p] = i;
            T->val[p] = A->val[e];
        }
    free(pos);
    return T;
}

/* smooth_interpolation (interpolation/mod.rs:927-946):
 *   S = A P;  S_i* *= -(omega * (1/a_ii));  S += P  (P's pattern within S's). */
orc_csr *orc_smooth_interpolation(const orc_csr *A, const orc_csr *P, double omega) {
    orc_csr *S = orc_spgemm(A, P);
    for (int64_t i = 0; i < A->nrows; i++) {
        int found;
        double aii = csr_get(A, i, i, &found);
        if (!found || !(aii > 1e-6)) ORC_DIE("Diagonal nearly zero at row %lld", (long long)i);
        double scalar = omega * (1.0 / aii);
        for (int64_t e = S->rowptr[i]; e < S->rowptr[i + 1]; e++) S->val[e] = S->val[e] * -scalar;
    }
    for (int64_t i = 0; i < P->nrows; i++)
        for (int64_t e = P->rowptr[i]; e < P->rowptr[i + 1]; e++) {
            int64_t lo = S->rowptr[i], hi = S->rowptr[i + 1];
            while (lo < hi) {
                int64_t mid = (lo + hi) / 2;
                if (S->col[mid] < P->col[e]) lo = mid + 1;
                else hi = mid;
            }
            if (lo >= S->rowptr[i + 1] || S->col[lo] != P->col[e]) ORC_DIE("P pattern not within AP");
            S->val[lo] = S->val[lo] + P->val[e];
        }
    return S;
}

/* Galerkin A_c = R (A P) (interpolation/mod.rs:828). */
orc_csr *orc_rap(const orc_csr *R, const orc_csr *A, const orc_csr *P) {
    orc_csr *AP = orc_spgemm(A, P);
    orc_csr *C = orc_spgemm(R, AP);
    orc_csr_free(AP);
    return C;
}

/* Tentative SA interpolation for one candidate (interpolation/mod.rs:754-805):
 * per aggregate the thin SVD of the local candidate block is q * s * v^T with
 * s = ||local||_2 (sequential sum in ascending fine index), v = +1 (sign fixed
 * positive; the V-cycle is invariant to it), so P_iJ = nn_i / s_J and the coarse
 * candidate is s_J. */
orc_csr *orc_sa_tentative(int64_t n, const int64_t *agg_of, int64_t naggs, const double *nn,
                          double *coarse_nn) {
    double *ss = (double *)xcalloc((size_t)naggs, sizeof(double));
    for (int64_t i = 0; i < n; i++) {
        int64_t J = agg_of[i];
        if (J < 0 || J >= naggs) ORC_DIE("node %lld not aggregated", (long long)i);
        ss[J] = ss[J] + nn[i] * nn[i];
    }
    for (int64_t J = 0; J < naggs; J++) {
        coarse_nn[J] = sqrt(ss[J]);
        if (!(coarse_nn[J] > 0.0)) ORC_DIE("aggregate %lld has a zero candidate", (long long)J);
    }
    orc_csr *P = orc_csr_new(n, naggs, n);
    for (int64_t i = 0; i < n; i++) {
        P->rowptr[i] = i;
        P->col[i] = agg_of[i];
        P->val[i] = nn[i] / coarse_nn[agg_of[i]];
    }
    P->rowptr[n] = n;
    free(ss);
    return P;
}

/* Coarse near-null post-processing (hierarchy.rs:219-228): StationaryIteration
 * with an L1 diagonal, `iters` iterations, applied in place (smoothers.rs:146-158,
 * including its r = x - A x quirk), then the thin-QR Q of the single column,
 * i.e. x / ||x||_2 (sequential sum; sign positive). */
void orc_nn_stationary_l1(const orc_csr *A, int64_t iters, double *x_inout) {
    int64_t n = A->nrows;
    double *d = (double *)xmalloc((size_t)n * sizeof(double));
    double *x = (double *)xmalloc((size_t)n * sizeof(double));
    double *r = (double *)xmalloc((size_t)n * sizeof(double));
    orc_diag_l1(A, d);
    for (int64_t i = 0; i < n; i++) x[i] = d[i] * x_inout[i];
    for (int64_t it = 1; it < iters; it++) {
        orc_spmv(A, x, r);
        for (int64_t i = 0; i < n; i++) {
            double out = d[i] * (x[i] - r[i]);
            x[i] = x[i] + out;
        }
    }
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) s += x[i] * x[i];
    s = sqrt(s);
    for (int64_t i = 0; i < n; i++) x_inout[i] = x[i] / s;
    free(d);
    free(x);
    free(r);
}

/* Box aggregates on a structured grid (documented stand-in for the modularity
 * partitioner): node (x,y,z) -> box (x/bx, y/by, z/bz),
 * boxes numbered lexicographically on the ceil(n/b) coarse grid. */
int64_t orc_box_aggregates(int64_t nx, int64_t ny, int64_t nz, int64_t bx, int64_t by,
                           int64_t bz, int64_t *agg_of, int64_t *cdims) {
    int64_t cx = (nx + bx - 1) / bx, cy = (ny + by - 1) / by, cz = (nz + bz - 1) / bz;
    for (int64_t z = 0; z < nz; z++)
        for (int64_t y = 0; y < ny; y++)
            for (int64_t x = 0; x < nx; x++)
                agg_of[x + nx * (y + ny * z)] = x / bx + cx * (y / by + cy * (z / bz));
    cdims[0] = cx;
    cdims[1] = cy;
    cdims[2] = cz;
    return cx * cy * cz;
}

/* ------------------------------------------------------------ multigrid */

typedef struct {
    int kind;
    double *d;         /* diag smoother */
    int64_t *color;    /* sgs */
    int64_t ncolors;
    double *L;         /* dense Cholesky factor (or the envelope factor's values) */
    int64_t *ep, *fc;  /* envelope factor: row i holds columns fc[i] .. i at L + ep[i] */
    const orc_csr *M;  /* explicit smoother matrix (borrowed) */
} orc_smoother;

/* Envelope (profile) Cholesky A = L L^T for coarse levels above 4096 rows, in
 * the given numbering: row i of L spans columns fc[i] .. i, fc[i] = its first
 * nonzero of A (fill stays inside the envelope).  The reference's
 * SparseCholeskySolve (coarse_solvers.rs:164-206) factors any size with faer's
 * sparse LLt; a dense n^3 / 3 factor stops scaling at a few thousand rows. */
static int orc_env_factor(const orc_csr *A, double **Lp, int64_t **epp, int64_t **fcp) {
    const int64_t n = A->nrows;
    int64_t *fc = (int64_t *)xmalloc((size_t)n * sizeof(int64_t));
    int64_t *ep = (int64_t *)xmalloc((size_t)(n + 1) * sizeof(int64_t));
    ep[0] = 0;
    for (int64_t i = 0; i < n; i++) {
        int64_t f = i;
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++)
            if (A->col[e] < f) f = A->col[e];
        fc[i] = f;
        ep[i + 1] = ep[i] + (i - f + 1);
    }
    double *L = (double *)xcalloc((size_t)ep[n], sizeof(double));
    for (int64_t i = 0; i < n; i++)
        for (int64_t e = A->rowptr[i]; e < A->rowptr[i + 1]; e++)
            if (A->col[e] <= i) L[ep[i] + A->col[e] - fc[i]] += A->val[e];
    for (int64_t i = 0; i < n; i++) {
        double *li = L + ep[i] - fc[i];  /* li[j] = L_ij */
        for (int64_t j = fc[i]; j < i; j++) {
            const double *lj = L + ep[j] - fc[j];
            const int64_t k0 = fc[i] > fc[j] ? fc[i] : fc[j];
            double t = li[j];
            for (int64_t k = k0; k < j; k++) t -= li[k] * lj[k];
            li[j] = t / lj[j];
        }
        double d = li[i];
        for (int64_t k = fc[i]; k < i; k++) d -= li[k] * li[k];
        if (!(d > 0.0)) {
            free(L); free(ep); free(fc);
            return 1;
        }
        li[i] = sqrt(d);
    }
    *Lp = L;
    *epp = ep;
    *fcp = fc;
    return 0;
}

static void orc_env_solve(int64_t n, const double *L, const int64_t *ep, const int64_t *fc, double *b) {
    for (int64_t i = 0; i < n; i++) {
        const double *li = L + ep[i] - fc[i];
        double t = b[i];
        for (int64_t k = fc[i]; k < i; k++) t -= li[k] * b[k];
        b[i] = t / li[i];
    }
    for (int64_t i = n - 1; i >= 0; i--) {
        const double *li = L + ep[i] - fc[i];
        b[i] /= li[i];
        const double x = b[i];
        for (int64_t k = fc[i]; k < i; k++) b[k] -= li[k] * x;
    }
}

struct orc_mg {
    int64_t nlevels, mu, steps;
    int64_t parallel, nthreads;
    const orc_csr **A, **R, **P;
    orc_parspmm **parA, **parR, **parP;
    orc_smoother *S;
};

orc_mg *orc_mg_new(int64_t nlevels) {
    orc_mg *mg = (orc_mg *)xcalloc(1, sizeof(orc_mg));
    mg->nlevels = nlevels;
    mg->mu = 1;
    mg->steps = 1;
    mg->A = (const orc_csr **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->R = (const orc_csr **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->P = (const orc_csr **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->parA = (orc_parspmm **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->parR = (orc_parspmm **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->parP = (orc_parspmm **)xcalloc((size_t)nlevels, sizeof(void *));
    mg->S = (orc_smoother *)xcalloc((size_t)nlevels, sizeof(orc_smoother));
    return mg;
}

static void free_smoother(orc_smoother *s) {
    free(s->d);
    free(s->color);
    free(s->L);
    free(s->ep);
    free(s->fc);
    memset(s, 0, sizeof(*s));
}

void orc_mg_free(orc_mg *mg) {
    if (!mg) return;
    for (int64_t l = 0; l < mg->nlevels; l++) {
        free_smoother(&mg->S[l]);
        orc_parspmm_free(mg->parA[l]);
        orc_parspmm_free(mg->parR[l]);
        orc_parspmm_free(mg->parP[l]);
    }
    free(mg->A); free(mg->R); free(mg->P);
    free(mg->parA); free(mg->parR); free(mg->parP);
    free(mg->S);
    free(mg);
}

void orc_mg_set_op(orc_mg *mg, int64_t level, const orc_csr *A) { mg->A[level] = A; }

void orc_mg_set_transfer(orc_mg *mg, int64_t level, const orc_csr *R, const orc_csr *P) {
    mg->R[level] = R;
    mg->P[level] = P;
}

void orc_mg_set_diag(orc_mg *mg, int64_t level, const double *d) {
    orc_smoother *s = &mg->S[level];
    free_smoother(s);
    int64_t n = mg->A[level]->nrows;
    s->kind = ORC_SM_DIAG;
    s->d = (double *)xmalloc((size_t)n * sizeof(double));
    memcpy(s->d, d, (size_t)n * sizeof(double));
}

void orc_mg_set_sgs(orc_mg *mg, int64_t level, const int64_t *color, int64_t ncolors) {
    orc_smoother *s = &mg->S[level];
    free_smoother(s);
    int64_t n = mg->A[level]->nrows;
    s->kind = ORC_SM_SGS;
    s->ncolors = ncolors;
    s->color = (int64_t *)xmalloc((size_t)n * sizeof(int64_t));
    memcpy(s->color, color, (size_t)n * sizeof(int64_t));
}

int orc_mg_set_chol(orc_mg *mg, int64_t level) {
    orc_smoother *s = &mg->S[level];
    free_smoother(s);
    const orc_csr *A = mg->A[level];
    int64_t n = A->nrows;
    s->kind = ORC_SM_CHOL;
    if (n > 4096) return orc_env_factor(A, &s->L, &s->ep, &s->fc);
    double *dense = (double *)xmalloc((size_t)(n * n) * sizeof(double));
    orc_csr_to_dense(A, dense);
    s->kind = ORC_SM_CHOL;
    s->L = (double *)xmalloc((size_t)(n * n) * sizeof(double));
    int rc = orc_chol_factor(n, dense, s->L);
    free(dense);
    return rc;
}

void orc_mg_set_csr_smoother(orc_mg *mg, int64_t level, const orc_csr *M) {
    orc_smoother *s = &mg->S[level];
    free_smoother(s);
    s->kind = ORC_SM_CSR;
    s->M = M;
}

void orc_mg_set_cycle(orc_mg *mg, int64_t mu, int64_t steps) {
    mg->mu = mu;
    mg->steps = steps;
}

/* Parallel mode = the reference's rayon configuration (multigrid.rs:134-160):
 * every A_l is a ParSpmmOp (core.rs:63-67); R_l/P_l are ParSpmmOps only when both
 * dims exceed PAR_BLOCK_SIZE*threads*4 (multigrid.rs:152-156), otherwise the
 * plain CSR apply with the global parallelism. */
void orc_mg_set_parallel(orc_mg *mg, int64_t enable, int64_t nthreads) {
    mg->parallel = enable;
    mg->nthreads = nthreads;
    if (!enable) return;
    omp_set_num_threads((int)nthreads);
    int64_t thr = (int64_t)PAR_BLOCK_SIZE * nthreads * 4;
    for (int64_t l = 0; l < mg->nlevels; l++) {
        if (!mg->parA[l]) mg->parA[l] = orc_parspmm_new(mg->A[l]);
        if (l + 1 < mg->nlevels && mg->R[l] && mg->R[l]->nrows > thr && mg->R[l]->ncols > thr) {
            if (!mg->parR[l]) mg->parR[l] = orc_parspmm_new(mg->R[l]);
            if (!mg->parP[l]) mg->parP[l] = orc_parspmm_new(mg->P[l]);
        }
    }
}

static void mg_apply_op(const orc_mg *mg, const orc_csr *M, const orc_parspmm *par,
                        const double *x, double *y) {
    if (par) orc_parspmm_apply(par, x, y);
    else if (mg->parallel) orc_spmv_omp(M, x, y);
    else orc_spmv(M, x, y);
}

/* Precond::apply_in_place of the level smoother. */
static void smoother_in_place(const orc_mg *mg, int64_t level, double *r) {
    const orc_smoother *s = &mg->S[level];
    int64_t n = mg->A[level]->nrows;
    switch (s->kind) {
    case ORC_SM_DIAG:
        for (int64_t i = 0; i < n; i++) r[i] = s->d[i] * r[i];
        break;
    case ORC_SM_SGS:
        orc_sgs_apply_in_place(mg->A[level], s->color, s->ncolors, r);
        break;
    case ORC_SM_CHOL:
        if (s->ep) orc_env_solve(n, s->L, s->ep, s->fc, r);
        else orc_chol_solve(n, s->L, r);
        break;
    case ORC_SM_CSR: {
        double *t = (double *)xmalloc((size_t)n * sizeof(double));
        if (mg->parallel) orc_spmv_omp(s->M, r, t);
        else orc_spmv(s->M, r, t);
        memcpy(r, t, (size_t)n * sizeof(double));
        free(t);
        break;
    }
    default:
        ORC_DIE("bad smoother kind");
    }
}

/* smooth (multigrid.rs:407-424): s times  work = A x; r = b - work;
 * pc.apply_in_place(r); x += r.  Fresh temporaries per call as in the
 * reference (:416, :420). */
static void mg_smooth(const orc_mg *mg, int64_t level, double *x, const double *b) {
    int64_t n = mg->A[level]->nrows;
    double *work = (double *)xcalloc((size_t)n, sizeof(double));
    for (int64_t it = 0; it < mg->steps; it++) {
        mg_apply_op(mg, mg->A[level], mg->parA[level], x, work);
        double *r = (double *)xmalloc((size_t)n * sizeof(double));
        for (int64_t i = 0; i < n; i++) r[i] = b[i] - work[i];
        smoother_in_place(mg, level, r);
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + r[i];
        free(r);
    }
    free(work);
}

/* cycle (multigrid.rs:269-380). */
static void mg_cycle(const orc_mg *mg, double *v, const double *f, int64_t level) {
    int64_t n = mg->A[level]->nrows;
    double *work = (double *)xcalloc((size_t)n, sizeof(double)); /* :278 */
    if (level == mg->nlevels - 1) {
        /* smoother.apply(v, f) (:291): out = M f, overwriting v */
        memcpy(v, f, (size_t)n * sizeof(double));
        smoother_in_place(mg, level, v);
        free(work);
        return;
    }
    mg_smooth(mg, level, v, f); /* :314-322 */
    const orc_csr *R = mg->R[level], *P = mg->P[level];
    int64_t nc = R->nrows;
    double *v_coarse = (double *)xcalloc((size_t)nc, sizeof(double)); /* :337 */
    double *f_coarse = (double *)xcalloc((size_t)nc, sizeof(double)); /* :338 */
    mg_apply_op(mg, mg->A[level], mg->parA[level], v, work);         /* :341 */
    for (int64_t i = 0; i < n; i++) work[i] = f[i] - work[i];        /* :342 */
    mg_apply_op(mg, R, mg->parR[level], work, f_coarse);              /* :343 */
    for (int64_t k = 0; k < mg->mu; k++) mg_cycle(mg, v_coarse, f_coarse, level + 1); /* :345-347 */
    mg_apply_op(mg, P, mg->parP[level], v_coarse, work);              /* :349 */
    for (int64_t i = 0; i < n; i++) v[i] = v[i] + work[i];           /* :350 */
    mg_smooth(mg, level, v, f);                                       /* :361-369 */
    free(v_coarse);
    free(f_coarse);
    free(work);
}

/* LinOp::apply for Multigrid (multigrid.rs:469-473, init_cycle :251-267). */
void orc_mg_apply(orc_mg *mg, const double *rhs, double *out) {
    int64_t n = mg->A[0]->nrows;
    if (mg->parallel) omp_set_num_threads((int)mg->nthreads);
    for (int64_t i = 0; i < n; i++) out[i] = 0.0;
    double *v = (double *)xcalloc((size_t)n, sizeof(double));
    mg_cycle(mg, v, rhs, 0);
    for (int64_t i = 0; i < n; i++) out[i] = out[i] + v[i];
    free(v);
}

/* ---------------------------------------------------------- solve drivers */

static double norm2(int64_t n, const double *x) {
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) s += x[i] * x[i];
    return sqrt(s);
}

static double dot(int64_t n, const double *x, const double *y) {
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) s += x[i] * y[i];
    return s;
}

/* stationary_solver (examples/simple_geometric.rs:117-158): records
 * rho_k = ||b - A x_k|| / ||b|| in hist[k-1]; returns the iteration count. */
int64_t orc_stationary_solve(const orc_csr *A, orc_mg *mg, const double *b, double *x,
                             int64_t max_iter, double rel_tol, double *hist) {
    int64_t n = A->nrows, iter = 0;
    double *work = (double *)xcalloc((size_t)n, sizeof(double));
    double *r = (double *)xmalloc((size_t)n * sizeof(double));
    double *z = (double *)xmalloc((size_t)n * sizeof(double));
    double b_norm = norm2(n, b);
    for (;;) {
        /* the residual SpMV in the cycle's parallel mode (same per-row order) */
        if (mg->parallel) orc_spmv_omp(A, x, work);
        else orc_spmv(A, x, work);
        for (int64_t i = 0; i < n; i++) r[i] = b[i] - work[i];
        double rel = norm2(n, r) / b_norm;
        iter += 1;
        if (hist) hist[iter - 1] = rel;
        if (rel < rel_tol || iter >= max_iter) break;
        orc_mg_apply(mg, r, z); /* pc.apply_in_place(r) */
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + z[i];
    }
    free(work);
    free(r);
    free(z);
    return iter;
}

/* Preconditioned CG (the caller side of faer conjugate_gradient, utils.rs:600;
 * simple_geometric.rs:243-268).  faer's own loop is not in this container, so
 * this is the textbook PCG; converged when ||r|| <= max(abs_tol, rel_tol*||b||).
 * Preconditioner: multigrid if mg != NULL, else diagonal diag_pc, else identity.
 * hist[k-1] = ||r_k||/||b||.  Returns the iteration count (max_iter+1 if not
 * converged). */
int64_t orc_pcg_solve(const orc_csr *A, orc_mg *mg, const double *diag_pc, const double *b,
                      double *x, int64_t max_iter, double rel_tol, double abs_tol,
                      double *hist) {
    int64_t n = A->nrows;
    double *r = (double *)xmalloc((size_t)n * sizeof(double));
    double *z = (double *)xmalloc((size_t)n * sizeof(double));
    double *p = (double *)xmalloc((size_t)n * sizeof(double));
    double *Ap = (double *)xmalloc((size_t)n * sizeof(double));
    orc_spmv(A, x, Ap);
    for (int64_t i = 0; i < n; i++) r[i] = b[i] - Ap[i];
    double b_norm = norm2(n, b);
    double tol = rel_tol * b_norm > abs_tol ? rel_tol * b_norm : abs_tol;
    int64_t it = 0;
    if (norm2(n, r) <= tol) goto done;
#define APPLY_PC(src, dst)                                                              \
    do {                                                                                \
        if (mg) orc_mg_apply(mg, src, dst);                                             \
        else if (diag_pc) for (int64_t i_ = 0; i_ < n; i_++) dst[i_] = diag_pc[i_] * src[i_]; \
        else memcpy(dst, src, (size_t)n * sizeof(double));                              \
    } while (0)
    APPLY_PC(r, z);
    memcpy(p, z, (size_t)n * sizeof(double));
    double rz = dot(n, r, z);
    for (it = 1; it <= max_iter; it++) {
        orc_spmv(A, p, Ap);
        double alpha = rz / dot(n, p, Ap);
        for (int64_t i = 0; i < n; i++) {
            x[i] = x[i] + alpha * p[i];
            r[i] = r[i] - alpha * Ap[i];
        }
        double rn = norm2(n, r);
        if (hist) hist[it - 1] = rn / b_norm;
        if (rn <= tol) goto done;
        APPLY_PC(r, z);
        double rz_new = dot(n, r, z);
        double beta = rz_new / rz;
        rz = rz_new;
        for (int64_t i = 0; i < n; i++) p[i] = z[i] + beta * p[i];
    }
#undef APPLY_PC
done:
    free(r);
    free(z);
    free(p);
    free(Ap);
    return it;
}
