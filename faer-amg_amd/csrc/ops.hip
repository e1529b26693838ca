// ops.hip -- LinOp implementations: CSR, diagonal smoothers, multicolor SGS,
// coarse solve, and the multigrid V-cycle (reference
// src/preconditioners/{smoothers,coarse_solvers,multigrid}.rs).
//
// The V-cycle keeps the reference's order of operations exactly
// (multigrid.rs:269-380): pre-smooth, r = f - A v, f_c = R r, mu coarse cycles
// from v_c = 0, v += P v_c, post-smooth; the coarsest level applies its
// smoother (the coarse solve).  What changes is where the work runs and how it
// is fused: every level's vectors are preallocated in HBM, `smooth`'s four
// passes (A x, b - Ax, D r, x + r) are one SpMV with a Jacobi epilogue, the
// residual and the interpolation-correction are SpMV epilogues, the first
// smoothing step from v = 0 skips the SpMV (A 0 = 0 exactly), and a whole
// V-cycle is captured once into a hipGraph and replayed.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

#include "famg.hpp"

namespace famg {

void build_schedule(const std::vector<int64_t> &rp, const std::vector<int64_t> &seg_bounds,
                    std::vector<int32_t> &sched, std::vector<int64_t> &seg_blocks);

Ctx::~Ctx() {
    if (host_red) (void)hipHostFree(host_red);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
}

// ------------------------------------------------------------------ LinOp

void LinOp::apply_in_place(double *rhs) {
    if (inplace_scratch_.size() < (size_t)nrows) inplace_scratch_.resize(nrows);
    vec_copy(inplace_scratch_.get(), rhs, nrows, ctx->stream);
    apply(rhs, inplace_scratch_.get());
}

CsrPtr make_csr(Ctx *ctx) {
    auto p = std::make_shared<CsrOp>();
    p->ctx = ctx;
    return p;
}

void CsrOp::apply(double *out, const double *rhs) {
    spmv(m, rhs, out, SPMV_SET, SpmvEpi{}, ctx->stream);
}

void CsrOp::transpose_apply(double *out, const double *rhs) {
    if (!transpose_) transpose_ = transpose_op(*this);
    transpose_->apply(out, rhs);
}

const double *CsrOp::diagonal() {
    if (!diag_.get()) {
        diag_.resize(m.nrows);
        csr_diagonal(m, diag_.get());
    }
    return diag_.get();
}

// ------------------------------------------------------------- diagonal

void DiagOp::apply(double *out, const double *rhs) { vec_mul(out, d.get(), rhs, nrows, ctx->stream); }
void DiagOp::apply_in_place(double *rhs) { vec_mul(rhs, d.get(), rhs, nrows, ctx->stream); }

__global__ void k_jacobi_diag(const double *aii, double omega, double *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) d[i] = omega / aii[i];
}
__global__ void k_recip(double *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) d[i] = 1.0 / d[i];
}

static std::shared_ptr<DiagOp> new_diag(Ctx *ctx, int64_t n) {
    auto p = std::make_shared<DiagOp>();
    p->ctx = ctx;
    p->nrows = p->ncols = n;
    p->d.resize(n);
    return p;
}

// new_jacobi (smoothers.rs:78-86): d_i = omega / a_ii
std::shared_ptr<DiagOp> make_jacobi(CsrOp &A, double omega) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "jacobi: matrix must be square");
    auto p = new_diag(A.ctx, A.nrows);
    if (A.nrows)
        hipLaunchKernelGGL(k_jacobi_diag, dim3((unsigned)ceil_div(A.nrows, 256)), dim3(256), 0,
                           A.ctx->stream, A.diagonal(), omega, p->d.get(), A.nrows);
    FAMG_CHECK_HIP(hipGetLastError());
    return p;
}

// new_l1 (smoothers.rs:63-76): d_i = 1 / sum_j |a_ij|
std::shared_ptr<DiagOp> make_l1(CsrOp &A) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "l1: matrix must be square");
    auto p = new_diag(A.ctx, A.nrows);
    csr_abs_row_sums(A.m, p->d.get());
    if (A.nrows)
        hipLaunchKernelGGL(k_recip, dim3((unsigned)ceil_div(A.nrows, 256)), dim3(256), 0,
                           A.ctx->stream, p->d.get(), A.nrows);
    FAMG_CHECK_HIP(hipGetLastError());
    return p;
}

// new_l2 (smoothers.rs:43-61): d_i = 1 / sum_j |a_ij| sqrt(a_ii)/sqrt(a_jj)
__global__ void k_l2(const int64_t *rp, const int32_t *col, const double *val, const double *aii,
                     double *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double si = sqrt(aii[i]);
    double s = 0.0;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
        const double scale = si / sqrt(aii[col[e]]);
        s += fabs(val[e]) * scale;
    }
    d[i] = 1.0 / s;
}

std::shared_ptr<DiagOp> make_l2(CsrOp &A) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "l2: matrix must be square");
    auto p = new_diag(A.ctx, A.nrows);
    if (A.nrows)
        hipLaunchKernelGGL(k_l2, dim3((unsigned)ceil_div(A.nrows, 256)), dim3(256), 0, A.ctx->stream,
                           A.m.rp64.get(), A.m.col.get(), A.m.val.get(), A.diagonal(), p->d.get(),
                           A.nrows);
    FAMG_CHECK_HIP(hipGetLastError());
    return p;
}

// --------------------------------------------------------- multicolor SGS

int64_t greedy_coloring(const GpuCsr &A, std::vector<int32_t> &color) {
    std::vector<int64_t> rp(A.nrows + 1);
    std::vector<int32_t> col(A.nnz);
    hipStream_t s = A.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(rp.data(), A.rp64.get(), (A.nrows + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    if (A.nnz) FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), A.col.get(), A.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    color.assign(A.nrows, 0);
    std::vector<int64_t> mark(64, -1);
    int64_t nc = 0;
    for (int64_t i = 0; i < A.nrows; i++) {
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int64_t j = col[e];
            if (j < i) {
                const int32_t c = color[j];
                if ((size_t)c >= mark.size()) mark.resize(2 * (c + 1), -1);
                mark[c] = i;
            }
        }
        int32_t c = 0;
        while ((size_t)c < mark.size() && mark[c] == i) c++;
        if ((size_t)c >= mark.size()) mark.resize(2 * mark.size(), -1);
        color[i] = c;
        nc = std::max<int64_t>(nc, c + 1);
    }
    return nc;
}

__global__ void k_perm_counts(const int64_t *rp, const int32_t *perm, int64_t n, int64_t *cnt) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p < n) cnt[p] = rp[perm[p] + 1] - rp[perm[p]];
}
__global__ void k_perm_rows(const int64_t *rp, const int32_t *col, const double *val,
                            const int32_t *perm, int64_t n, const int64_t *prp, int32_t *pcol,
                            double *pval, const double *aii, double *dinv) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int32_t i = perm[p];
    int64_t o = prp[p];
    for (int64_t e = rp[i]; e < rp[i + 1]; e++, o++) {
        pcol[o] = col[e];
        pval[o] = val[e];
    }
    dinv[p] = 1.0 / aii[i];
}
// first forward color from e = 0: e_i = 0 + dinv (r_i - 0) = dinv r_i
__global__ void k_sgs_first(const int32_t *perm, const double *dinv, const double *r, double *e,
                            int64_t p0, int64_t p1) {
    const int64_t p = p0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p < p1) {
        const int32_t i = perm[p];
        e[i] = dinv[p] * r[i];
    }
}

// The color-permuted copy Ap (rows grouped by color, stable within a color),
// perm and 1/a_ii of op->A for the coloring op->host_colors / op->ncolors.
// A may be rectangular (the owned rows of a distributed level over the
// [owned | ghost] columns); its diagonal then comes from op.aii_.
static void sgs_permuted_copy(SgsOp &op) {
    const CsrPtr &A = op.A;
    Ctx *ctx = A->ctx;
    hipStream_t s = ctx->stream;
    const int64_t n = A->nrows;
    const std::vector<int32_t> &color = op.host_colors;
    // stable counting sort of rows by color
    op.color_ptr.assign(op.ncolors + 1, 0);
    for (int64_t i = 0; i < n; i++) op.color_ptr[color[i] + 1]++;
    for (int64_t c = 0; c < op.ncolors; c++) op.color_ptr[c + 1] += op.color_ptr[c];
    std::vector<int32_t> perm(n);
    {
        std::vector<int64_t> pos(op.color_ptr.begin(), op.color_ptr.end() - 1);
        for (int64_t i = 0; i < n; i++) perm[pos[color[i]]++] = (int32_t)i;
    }
    op.perm.resize(std::max<int64_t>(1, n));
    if (n) FAMG_CHECK_HIP(hipMemcpyAsync(op.perm.get(), perm.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, s));
    DevBuf<int64_t> cnt(std::max<int64_t>(1, n));
    const unsigned g = (unsigned)std::max<int64_t>(1, ceil_div(n, 256));
    if (n) hipLaunchKernelGGL(k_perm_counts, dim3(g), dim3(256), 0, s, A->m.rp64.get(), op.perm.get(), n, cnt.get());
    DevBuf<int64_t> prp(n + 1);
    const int64_t nnz = scan_counts(cnt.get(), prp.get(), n, *ctx);
    csr_alloc(op.Ap, ctx, n, A->ncols, nnz);
    op.Ap.rp64 = std::move(prp);
    op.Ap.no_bsr = true;  // swept in SGS mode only
    op.Ap.no_sellp = true;
    op.dinv.resize(std::max<int64_t>(1, n));
    const double *aii = op.aii_ ? op.aii_ : A->diagonal();
    if (n)
        hipLaunchKernelGGL(k_perm_rows, dim3(g), dim3(256), 0, s, A->m.rp64.get(), A->m.col.get(),
                           A->m.val.get(), op.perm.get(), n, op.Ap.rp64.get(), op.Ap.col.get(),
                           op.Ap.val.get(), aii, op.dinv.get());
    FAMG_CHECK_HIP(hipGetLastError());
    csr_finalize(op.Ap, &op.color_ptr);  // one row segment per color
    FAMG_REQUIRE(op.Ap.spmv_ready(), AMG_ERR_UNSUPPORTED, "sgs: nnz must be < 2^31");
}

std::shared_ptr<SgsOp> make_sgs_slice(const CsrPtr &A, const int32_t *colors, int64_t ncolors, const double *aii) {
    FAMG_REQUIRE(A->nrows <= A->ncols, AMG_ERR_DIM, "sgs slice: more rows than columns");
    auto op = std::make_shared<SgsOp>();
    op->ctx = A->ctx;
    op->A = A;
    op->nrows = op->ncols = A->nrows;
    op->ncolors = ncolors;
    op->host_colors.assign(colors, colors + A->nrows);
    for (int32_t c : op->host_colors)
        FAMG_REQUIRE(c >= 0 && c < ncolors, AMG_ERR_INVALID, "sgs slice: color out of range");
    op->aii_ = aii;
    sgs_permuted_copy(*op);
    op->aii_ = nullptr;
    return op;
}

void SgsOp::first_color(double *e, const double *r) {
    const int64_t p0 = color_ptr[0], p1 = color_ptr[1];
    if (p1 > p0) log_launch("sgs_first", -1, -1, p1 - p0, 28 * (p1 - p0));
    if (p1 > p0)
        hipLaunchKernelGGL(k_sgs_first, dim3((unsigned)ceil_div(p1 - p0, 256)), dim3(256), 0, ctx->stream,
                           perm.get(), dinv.get(), r, e, p0, p1);
    FAMG_CHECK_HIP(hipGetLastError());
}

std::shared_ptr<SgsOp> make_sgs(const CsrPtr &A, const int32_t *colors, bool validate) {
    FAMG_REQUIRE(A->nrows == A->ncols, AMG_ERR_DIM, "sgs: matrix must be square");
    Ctx *ctx = A->ctx;
    auto op = std::make_shared<SgsOp>();
    op->ctx = ctx;
    op->A = A;
    op->nrows = op->ncols = A->nrows;
    const int64_t n = A->nrows;
    std::vector<int32_t> color;
    if (colors) {
        color.assign(colors, colors + n);
        op->ncolors = 0;
        for (int64_t i = 0; i < n; i++) {
            FAMG_REQUIRE(color[i] >= 0, AMG_ERR_INVALID, "negative color");
            op->ncolors = std::max<int64_t>(op->ncolors, color[i] + 1);
        }
        if (validate) {  // no two coupled rows may share a color
            std::vector<int64_t> rp(n + 1), col(A->m.nnz);
            std::vector<double> val(A->m.nnz);
            csr_to_host(A->m, rp.data(), col.data(), val.data());
            for (int64_t i = 0; i < n; i++)
                for (int64_t e = rp[i]; e < rp[i + 1]; e++)
                    FAMG_REQUIRE(col[e] == i || color[col[e]] != color[i], AMG_ERR_INVALID,
                                 "coloring couples two rows of the same color");
        }
    } else {
        op->ncolors = greedy_coloring(A->m, color);
    }
    op->host_colors = std::move(color);
    sgs_permuted_copy(*op);
    build_dia_sgs(op->Ap, op->perm.get());  // constant-stencil operators: DIA codes for the sweeps
    op->e_.resize(n);
    sgs27_setup(*op);  // 27-point grid operators: fused plane-parity phases
    return op;
}

// e = SGS(r) from e = 0: forward colors 0..C-1, backward C-2..0.
void SgsOp::sweep(double *e, const double *r) {
    hipStream_t s = ctx->stream;
    const int64_t n = nrows;
    if (!n) return;
    if (sgs27_applies(*this, e, r)) {
        sgs27_sweep(*this, e, r, true);
        return;
    }
    vec_fill(e, 0.0, n, s);
    first_color(e, r);
    SpmvEpi epi;
    epi.b = r;
    epi.d = dinv.get();
    epi.perm = perm.get();
    for (int64_t c = 1; c < ncolors; c++) spmv(Ap, e, e, SPMV_SGS, epi, s, c);
    for (int64_t c = ncolors - 2; c >= 0; c--) spmv(Ap, e, e, SPMV_SGS, epi, s, c);
}

// One smoothing step x <- x + SGS(b - A x) done directly on x (no residual
// vector): the same color sweeps with b in place of r.  Equal to the
// residual form in exact arithmetic; saves one SpMV with A per step.
void SgsOp::sweep_x(double *x, const double *b) {
    hipStream_t s = ctx->stream;
    if (!nrows) return;
    if (sgs27_applies(*this, x, b)) {
        sgs27_sweep(*this, x, b, false);
        return;
    }
    SpmvEpi epi;
    epi.b = b;
    epi.d = dinv.get();
    epi.perm = perm.get();
    for (int64_t c = 0; c < ncolors; c++) spmv(Ap, x, x, SPMV_SGS, epi, s, c);
    for (int64_t c = ncolors - 2; c >= 0; c--) spmv(Ap, x, x, SPMV_SGS, epi, s, c);
}

void SgsOp::apply(double *out, const double *rhs) {
    if (out == rhs) { apply_in_place(out); return; }
    sweep(out, rhs);
}

void SgsOp::apply_in_place(double *rhs) {
    sweep(e_.get(), rhs);
    vec_copy(rhs, e_.get(), nrows, ctx->stream);
}

// ------------------------------------------------------------ coarse solve

// Dense Cholesky on the host (setup) and the explicit inverse; the solve on the
// device is one GEMV (8 n^2 bytes, L2/MALL resident for n <= ~2000).  Larger
// coarsest levels (FAMG_COARSE_DENSE_MAX, default 8192 rows) take chol.hip's
// envelope factor.
static int64_t coarse_dense_max() {
    static const int64_t v = [] {
        const char *e = getenv("FAMG_COARSE_DENSE_MAX");
        return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)8192;
    }();
    return v;
}

std::shared_ptr<CoarseCholOp> make_coarse_chol_env(CsrOp &A);  // chol.hip
void chol_env_apply(const CoarseCholOp &op, double *out, const double *rhs, hipStream_t s);

std::shared_ptr<CoarseCholOp> make_coarse_chol(CsrOp &A) {
    FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "coarse solve: matrix must be square");
    const int64_t n = A.nrows;
    // above 8192 rows: the envelope Cholesky factor, block triangular solves (chol.hip)
    if (n > coarse_dense_max()) return make_coarse_chol_env(A);
    std::vector<int64_t> rp(n + 1), col(A.m.nnz);
    std::vector<double> val(A.m.nnz);
    csr_to_host(A.m, rp.data(), col.data(), val.data());
    std::vector<double> L((size_t)n * n, 0.0);
    for (int64_t i = 0; i < n; i++)
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) L[(size_t)i * n + col[e]] += val[e];
    // in-place lower Cholesky (row-major), left-looking
    for (int64_t j = 0; j < n; j++) {
        double sjj = L[(size_t)j * n + j];
        for (int64_t k = 0; k < j; k++) sjj -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
        FAMG_REQUIRE(sjj > 0.0, AMG_ERR_NOT_SPD, "coarse matrix is not SPD (Cholesky pivot <= 0)");
        const double ljj = std::sqrt(sjj);
        L[(size_t)j * n + j] = ljj;
#pragma omp parallel for schedule(static)
        for (int64_t i = j + 1; i < n; i++) {
            double t = L[(size_t)i * n + j];
            for (int64_t k = 0; k < j; k++) t -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
            L[(size_t)i * n + j] = t / ljj;
        }
    }
    // inverse: column j = L^-T L^-1 e_j ; stored row-major (symmetric)
    std::vector<double> inv((size_t)n * n, 0.0);
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t j = 0; j < n; j++) {
        std::vector<double> y(n, 0.0);
        y[j] = 1.0;
        for (int64_t i = j; i < n; i++) {
            double t = y[i];
            for (int64_t k = j; k < i; k++) t -= L[(size_t)i * n + k] * y[k];
            y[i] = t / L[(size_t)i * n + i];
        }
        for (int64_t i = n - 1; i >= 0; i--) {
            double t = y[i];
            for (int64_t k = i + 1; k < n; k++) t -= L[(size_t)k * n + i] * y[k];
            y[i] = t / L[(size_t)i * n + i];
        }
        for (int64_t i = 0; i < n; i++) inv[(size_t)i * n + j] = y[i];
    }
    auto op = std::make_shared<CoarseCholOp>();
    op->ctx = A.ctx;
    op->nrows = op->ncols = n;
    op->inv.resize((size_t)n * n);
    FAMG_CHECK_HIP(hipMemcpyAsync(op->inv.get(), inv.data(), inv.size() * sizeof(double),
                                  hipMemcpyHostToDevice, A.ctx->stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(A.ctx->stream));
    return op;
}

void CoarseCholOp::apply(double *out, const double *rhs) {
    if (out == rhs) { LinOp::apply_in_place(out); return; }
    if (nb > 0) chol_env_apply(*this, out, rhs, ctx->stream);
    else dense_gemv(inv.get(), rhs, out, nrows, ctx->stream);
}

// --------------------------------------------------------------- multigrid

MultigridOp::~MultigridOp() {
    invalidate_graphs();
    for (auto &e : fine_ev)
        if (e) (void)hipEventDestroy(e);
}

void MultigridOp::invalidate_graphs() {
    for (auto &g : graphs_) (void)hipGraphExecDestroy(g.exec);
    graphs_.clear();
    tail_key_ = ~uint64_t(0);  // operators, options or switches changed: the dense tail is rebuilt
}

void MultigridOp::add_level(LinOpPtr A, LinOpPtr S, LinOpPtr R, LinOpPtr P) {
    FAMG_REQUIRE(!levels.empty(), AMG_ERR_INVALID, "add_level on an empty multigrid");
    undo_reorder();  // renumbered again at the next apply, over every level
    FAMG_REQUIRE(A && S && R && P, AMG_ERR_INVALID, "add_level: null operator");
    const int64_t nf = levels.back().A->nrows, nc = A->nrows;
    FAMG_REQUIRE(A->nrows == A->ncols, AMG_ERR_DIM, "add_level: op must be square");
    FAMG_REQUIRE(S->nrows == nc && S->ncols == nc, AMG_ERR_DIM, "add_level: smoother size != op size");
    FAMG_REQUIRE(P->nrows == nf && P->ncols == nc, AMG_ERR_DIM, "add_level: p must be n_fine x n_coarse");
    FAMG_REQUIRE(R->nrows == nc && R->ncols == nf, AMG_ERR_DIM, "add_level: r must be n_coarse x n_fine");
    // the drop-in path (amg_csr_create per level, then add_level) gets the same
    // grid-transfer storage as sa_build_box: attached when A_l and A_{l+1} carry
    // grid hints of a 2x2x2 box relation (inferred at finalize), rows verified
    {
        auto *Af = dynamic_cast<CsrOp *>(levels.back().A.get());
        auto *Ac = dynamic_cast<CsrOp *>(A.get());
        auto *Rc = dynamic_cast<CsrOp *>(R.get());
        auto *Pc = dynamic_cast<CsrOp *>(P.get());
        if (Af && Ac && Rc && Pc) attach_box_transfers(Af->m, Ac->m, Rc->m, Pc->m);
    }
    levels.back().R = R;
    levels.back().P = P;
    MgLevel L;
    L.A = A;
    L.S = S;
    levels.push_back(std::move(L));
    workspace_ready_ = false;
    invalidate_graphs();
}

void MultigridOp::ensure_workspace() {
    if (workspace_ready_) return;
    if (!reorder_done_) reorder_levels();
    for (size_t l = 0; l < levels.size(); l++) {
        const int64_t n = levels[l].A->nrows;
        MgLevel &L = levels[l];
        if (l > 0) { L.v.resize(n); L.f.resize(n); }
        L.t.resize(n);
        L.r.resize(n);
    }
    // 8-bit codes of the Jacobi diagonals (bitwise the same d), before any graph capture
    for (auto &L : levels) {
        auto *D = dynamic_cast<DiagOp *>(L.S.get());
        if (D && !D->codes_tried) {
            array_codes_u8(D->d.get(), D->nrows, *ctx, D->dcode, D->dtab, &D->dconst);
            D->codes_tried = true;
        }
    }
    workspace_ready_ = true;
}

// smooth (multigrid.rs:407-424), `steps` times: x <- x + S (b - A x).
// Fused forms per smoother; the first step from x = 0 needs no SpMV.
// v/t are the two buffers of the level; Jacobi ping-pongs between them.
// FAMG_FOLD_DIA=1: fold the zero-guess step on DIA levels too (A/B switch)
// FAMG_FOLD_DIA: unset -- fold on a DIA level whose P runs the short-slice
// kernel (P_0 of a box hierarchy: its d*b epilogue streams dc and b instead of
// v, the same bytes); 1 -- every DIA level; 0 -- none
static int fold_dia_mode() {
    static const int v = [] {
        const char *e = getenv("FAMG_FOLD_DIA");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    return v;
}

void MultigridOp::smooth(int64_t l, double *&v, double *&t, const double *f, bool v_zero, bool pre_df) {
    MgLevel &L = levels[l];
    const int64_t n = L.A->nrows;
    hipStream_t s = ctx->stream;
    auto *A = dynamic_cast<CsrOp *>(L.A.get());
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    auto *G = dynamic_cast<SgsOp *>(L.S.get());
    log_at(l, AMG_ROLE_SMOOTH);
    for (int64_t it = 0; it < steps; it++) {
        const bool zero = v_zero && it == 0;
        if (A && D) {
            if (zero && pre_df) {
                // t = d*f was written by the restriction (SPMV_SETDF)
            } else if (zero) {
                if (D->dcode.get()) vec_mul_coded(t, D->dcode.get(), D->dtab.get(), f, n, s);
                else vec_mul(t, D->d.get(), f, n, s);  // 0 + d (f - A 0)
            } else {
                SpmvEpi epi;
                epi.b = f;
                epi.d = D->d.get();
                epi.dc = D->dcode.get();
                epi.dt = D->dtab.get();
                epi.dk = D->dconst;
                spmv(A->m, v, t, SPMV_JACOBI, epi, s);
            }
            std::swap(v, t);
        } else if (A && G) {
            if (zero) {
                G->sweep(v, f);  // e = SGS(f - A 0); v = 0 + e
            } else if (sgs_residual_form) {
                SpmvEpi epi;
                epi.b = f;
                spmv(A->m, v, L.r.get(), SPMV_RESID, epi, s);
                G->sweep(t, L.r.get());
                vec_add_inplace(v, t, n, s);
            } else {
                G->sweep_x(v, f);  // fused: x <- x + SGS(f - A x)
            }
        } else {
            if (zero) {
                L.S->apply(v, f);
            } else {
                L.A->apply(t, v);
                vec_sub(L.r.get(), f, t, n, s);
                L.S->apply_in_place(L.r.get());
                vec_add_inplace(v, L.r.get(), n, s);
            }
        }
    }
}

// One Jacobi step from v = 0 gives v = d*f; with s = 1 nothing else reads v
// before the correction, so the residual gathers d*f on the fly (RESID0) and the
// correction writes d*f + P v_c (ADD0): the same rounded values, 16n bytes and
// one launch fewer per level.  Where that pays (measured per storage, below) --
// the decision of MultigridOp::cycle and of the distributed cycle's levels.
bool fold_level(const CsrOp *A, const DiagOp *D, const CsrOp *P, bool fold_zero_guess, bool v_zero, int64_t steps) {
    const bool gather_cheap = A && 2 * A->m.sell_mode_slices[2] < A->m.nslices;
    // x-staged stencil classes (levels 1-3 of the box hierarchies): d*f can be
    // staged with the window (1-B codes of d per staged point) and the
    // correction's d*f epilogue streams dc and f in place of v, saving the
    // 24n-byte d*f pass and its launch.  Measured a net loss on the C2 cycle
    // (profiles/r03/ab_fold_xscs_{on,off_wpr1}.txt: dependent code -> table loads lengthen
    // the staging, RESID0 44.4 vs 33.3 + 8.5 us on A_1; ADD0 on P_1 49.5 vs
    // 46.5 us), so off by default; FAMG_FOLD_XSCS=1 turns it on (also for the
    // small wave-per-row levels below, which lose 0.6 us the same way).
    const bool fold_xscs = flag(FLAG_FOLD_XSCS) != 0;
    const bool p_add0 = P && (P->m.kernel == SPMV_KERNEL_SELL || P->m.kernel == SPMV_KERNEL_SELLP ||
                              P->m.kernel == SPMV_KERNEL_STREAM || P->m.kernel == SPMV_KERNEL_VECTOR || P->m.gtc_on);
    // every fold writes the correction d*f + P v_c with P's ADD0 epilogue (the 3x3-block
    // kernel has none: a level with a block-stored P never folds)
    return fold_zero_guess && v_zero && steps == 1 && A && D && P && p_add0 &&
                      ((A->m.kernel == SPMV_KERNEL_SELL && A->m.sell_vbits == 0 && gather_cheap) ||
                       A->m.kernel == SPMV_KERNEL_XS ||  // x-staged: d*x staged with x, no extra gather
                       (fold_xscs && A->m.kernel == SPMV_KERNEL_SCS && A->m.xscs && p_add0) ||
                       // wave-per-row levels small enough that x and d stay in L2 (A_4 of the
                       // box hierarchies: 4096 rows): d gathered beside x costs no HBM bytes
                       (fold_xscs && A->m.kernel == SPMV_KERNEL_VECTOR && A->m.ncols <= 65536 && p_add0) ||
                       (A->m.kernel == SPMV_KERNEL_DIA &&
                        (fold_dia_mode() == 1 ||
                         (fold_dia_mode() < 0 &&
                          ((P->m.kernel == SPMV_KERNEL_SELL && P->m.sell_short) || P->m.gtc_on)))));
}

// cycle (multigrid.rs:269-380).  The result ends in the buffer v points to on
// entry (Jacobi ping-pong flips an even number of times: 2*steps).
// FAMG_SETDF=0: the next level's first Jacobi step from zero as its own d*f pass
bool setdf_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_SETDF");
        return !(e && e[0] == '0');
    }();
    return on;
}

// gather rhs into the renumbered fine level's order and run the cycle there; where
// level 0 takes its first Jacobi step from zero unfolded (smooth(): t = d*f), the
// gather writes that step too (one pass, one launch fewer: the t buffer cycle(0)
// smooths into, as SPMV_SETDF does for coarser levels)
void MultigridOp::gather_fine(const double *rhs, hipStream_t s) {
    MgLevel &L = levels[0];
    const int64_t n = L.A->nrows;
    auto *A = dynamic_cast<CsrOp *>(L.A.get());
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    auto *P = dynamic_cast<CsrOp *>(L.P.get());
    const bool df = levels.size() > 1 && A && D && steps >= 1 && !fold_level(A, D, P, fold_zero_guess, true, steps);
    if (df) {
        perm_gather_df(perm_f0_.get(), L.t.get(), rhs, L.perm.get(), *D, n, s);
    } else {
        perm_gather(perm_f0_.get(), rhs, L.perm.get(), n, s);
    }
    cycle(0, perm_v0_.get(), perm_f0_.get(), true, perm_v0_.get(), df);
}

void MultigridOp::ensure_tail() {
    const int64_t lim = flag(FLAG_DENSE_TAIL);
    const uint64_t key = ((uint64_t)mu << 48) ^ ((uint64_t)steps << 40) ^ ((uint64_t)levels.size() << 32) ^
                         (uint64_t)std::max<int64_t>(lim, 0);
    if (key == tail_key_) return;
    tail_key_ = key;
    tail_level = -1;
    tail_M_.release();
    if (lim <= 0 || mu != 1 || levels.size() < 3) return;
    int64_t l0 = -1;
    for (int64_t l = 1; l + 1 < (int64_t)levels.size(); l++)
        if (levels[l].A->nrows <= lim) {
            l0 = l;
            break;
        }
    if (l0 < 0) return;
    const int64_t n = levels[l0].A->nrows;
    hipStream_t s = ctx->stream;
    // column j of M = the tail's v for f = e_j (eager launches, before any capture)
    DevBuf<double> Mt(n * n), e(n);
    LaunchLog *saved = g_launch_log;
    g_launch_log = nullptr;
    for (int64_t j = 0; j < n; j++) {
        unit_vector(e.get(), n, j, s);
        cycle(l0, Mt.get() + j * n, e.get(), true, nullptr, false);
    }
    g_launch_log = saved;
    tail_M_.resize(n * n);
    dense_transpose(Mt.get(), tail_M_.get(), n, s);
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    tail_level = l0;
}

void MultigridOp::cycle(int64_t l, double *v, const double *f, bool v_zero, double *, bool pre_df) {
    MgLevel &L = levels[l];
    hipStream_t s = ctx->stream;
    const int64_t n = L.A->nrows;
    if (l == tail_level && v_zero) {  // the dense tail: this level and every coarser one as v = M f
        log_at(l, AMG_ROLE_COARSE);
        dense_gemv(tail_M_.get(), f, v, n, s);
        return;
    }
    if (l == (int64_t)levels.size() - 1) {
        log_at(l, AMG_ROLE_COARSE);
        L.S->apply(v, f);  // smoother.apply(v, f) (:291)
        return;
    }
    double *v0 = v;
    double *t = (v == L.t.get()) ? L.v.get() : L.t.get();
    auto *A = dynamic_cast<CsrOp *>(L.A.get());
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    auto *P = dynamic_cast<CsrOp *>(L.P.get());
    // One Jacobi step from v = 0 gives v = d*f; with s = 1 nothing else reads
    // v before the correction, so the residual gathers d*f on the fly and the
    // correction writes d*f + P v_c: the same rounded values, 16n bytes and one
    // launch fewer per level.  Only for bandwidth-bound storage (SELL with fp64
    // values): value-code SELL and the wave-per-row kernel are latency-bound,
    // and gathering d beside x cost more there than the separate streaming
    // pass (measured on the 256^3 hierarchy).
    // DIA storage folds where P runs the short-slice kernel (P_0 of the 256^3
    // cycle): the residual gathers d beside x (115 us vs 91 + 51 for RESID + the
    // d*f pass) and the correction's d*f epilogue costs 117 vs 99 us -- 9 us net.
    // With the generic value-code SELL P (level 1) it lost: 58 + 49 vs 44 + 9 + 46.
    // Not where most slices carry 32-bit columns (unstructured operators): the
    // residual then gathers d as randomly as x, and that doubled gather cost more
    // than the pass it saves (Q1 elasticity 1.57M rows: 640 vs 388 + 15 us).
    const bool fold = fold_level(A, D, P, fold_zero_guess, v_zero, steps);
    MgLevel &C = levels[l + 1];
    // R on grid-transfer classes (either width) also writes the next level's first Jacobi
    // step from zero (d_c * f_c, what smooth() would compute first) into the
    // buffer that step writes: one launch and 24 n_c bytes fewer, same values
    bool df = false;
    auto *Rc = dynamic_cast<CsrOp *>(L.R.get());
    SpmvEpi epic;  // the SETDF epilogue: level l + 1's d, y2 = d_c f_c
    if (l + 2 < (int64_t)levels.size() && l + 1 != tail_level && restrict_df && setdf_enabled()) {
        auto *Ac = dynamic_cast<CsrOp *>(C.A.get());
        auto *Dc = dynamic_cast<DiagOp *>(C.S.get());
        auto *Pc = dynamic_cast<CsrOp *>(C.P.get());
        df = r_has_setdf(Rc) && Ac && Dc && steps >= 1 &&
             !fold_level(Ac, Dc, Pc, fold_zero_guess, true, steps);
        if (df) {
            epic.d = Dc->d.get();
            epic.dc = Dc->dcode.get();
            epic.dt = Dc->dtab.get();
            epic.dk = Dc->dconst;
            epic.y2 = C.t.get();  // cycle(l + 1, C.v, ...) smooths into C.t first
        }
    }
    SpmvEpi epi0;  // the folded residual's epilogue
    if (fold) {
        epi0.b = f;
        epi0.d = D->d.get();
        epi0.dc = D->dcode.get();  // DIA: 1-B codes of d gathered instead of d
        epi0.dt = D->dtab.get();
        epi0.dk = D->dconst;
    }
    if (fold && df && fine_resid_restrict_ok(A->m, Rc->m, epi0, epic)) {
        // the folded residual and the restriction in one marching launch
        // (fine.hip): r stays in LDS, f_c and d_c f_c land where SETDF writes them
        log_at(l, AMG_ROLE_RESID);
        if (fine_timer == 0) FAMG_CHECK_HIP(hipEventRecord(fine_ev[0], s));
        fine_resid_restrict(A->m, Rc->m, f, D->dconst, C.f.get(), epic, s);
        if (fine_timer == 0) FAMG_CHECK_HIP(hipEventRecord(fine_ev[1], s));
    } else {
        if (fold) {
            log_at(l, AMG_ROLE_RESID);
            spmv(A->m, f, L.r.get(), SPMV_RESID0, epi0, s);  // work = f - A (d f)
        } else {
            smooth(l, v, t, f, v_zero, pre_df);
            log_at(l, AMG_ROLE_RESID);
            if (A) {
                SpmvEpi epi;
                epi.b = f;
                spmv(A->m, v, L.r.get(), SPMV_RESID, epi, s);  // work = f - A v (:341-342)
            } else {
                L.A->apply(L.r.get(), v);
                vec_sub(L.r.get(), f, L.r.get(), n, s);
            }
        }
        log_at(l, AMG_ROLE_RESTRICT);
        if (df) spmv(Rc->m, L.r.get(), C.f.get(), SPMV_SETDF, epic, s);
        else L.R->apply(C.f.get(), L.r.get());  // f_c = R work (:343)
    }
    for (int64_t k = 0; k < mu; k++) cycle(l + 1, C.v.get(), C.f.get(), k == 0, nullptr, df && k == 0);
    log_at(l, AMG_ROLE_INTERP);
    if (fold) {
        SpmvEpi epi;
        epi.b = f;
        epi.d = D->d.get();
        epi.dc = D->dcode.get();
        epi.dt = D->dtab.get();
        epi.dk = D->dconst;
        if (steps == 1 && fine_interp_jacobi_ok(A->m, P->m, epi)) {
            // v = d f + P v_c and the post-smoothing step in one marching launch
            // (fine.hip): v stays in LDS, the result lands in v0
            if (fine_timer == 1) FAMG_CHECK_HIP(hipEventRecord(fine_ev[0], s));
            fine_interp_jacobi(A->m, P->m, C.v.get(), f, D->dconst, v0, s);
            if (fine_timer == 1) FAMG_CHECK_HIP(hipEventRecord(fine_ev[1], s));
            return;
        }
        spmv(P->m, C.v.get(), t, SPMV_ADD0, epi, s);  // v = d f + P v_c
        std::swap(v, t);                               // (where smooth() would have left v)
    } else if (P) {
        spmv(P->m, C.v.get(), v, SPMV_ADD, SpmvEpi{}, s);  // v += P v_c (:349-350)
    } else {
        L.P->apply(L.r.get(), C.v.get());
        vec_add_inplace(v, L.r.get(), n, s);
    }
    smooth(l, v, t, f, false);  // post-smoothing (:361-369)
    log_at(l, AMG_ROLE_OTHER);
    if (v != v0) vec_copy(v0, v, n, s);
}

bool MultigridOp::fine_launch(int which, double *out, const double *rhs) {
    std::lock_guard<std::mutex> lk(mtx);
    ensure_workspace();
    if (levels.size() < 3 || levels[0].permuted) return false;
    MgLevel &L = levels[0], &C = levels[1];
    auto *A = dynamic_cast<CsrOp *>(L.A.get());
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    auto *P = dynamic_cast<CsrOp *>(L.P.get());
    auto *Rc = dynamic_cast<CsrOp *>(L.R.get());
    if (!A || !D || !P || !Rc || !fold_level(A, D, P, fold_zero_guess, true, steps) || steps != 1) return false;
    SpmvEpi epi0;
    epi0.b = rhs;
    epi0.d = D->d.get();
    epi0.dc = D->dcode.get();
    epi0.dt = D->dtab.get();
    epi0.dk = D->dconst;
    hipStream_t s = ctx->stream;
    if (which == 1) {
        if (!fine_interp_jacobi_ok(A->m, P->m, epi0)) return false;
        fine_interp_jacobi(A->m, P->m, C.v.get(), rhs, D->dconst, out, s);
        return true;
    }
    auto *Ac = dynamic_cast<CsrOp *>(C.A.get());
    auto *Dc = dynamic_cast<DiagOp *>(C.S.get());
    auto *Pc = dynamic_cast<CsrOp *>(C.P.get());
    if (!(restrict_df && setdf_enabled() && r_has_setdf(Rc) && Ac && Dc &&
          !fold_level(Ac, Dc, Pc, fold_zero_guess, true, steps)))
        return false;
    SpmvEpi epic;
    epic.d = Dc->d.get();
    epic.dc = Dc->dcode.get();
    epic.dt = Dc->dtab.get();
    epic.dk = Dc->dconst;
    epic.y2 = C.t.get();
    if (!fine_resid_restrict_ok(A->m, Rc->m, epi0, epic)) return false;
    fine_resid_restrict(A->m, Rc->m, rhs, D->dconst, C.f.get(), epic, s);
    return true;
}

// LinOp::apply for Multigrid (multigrid.rs:469-473 / init_cycle :251-267):
// out = V-cycle(rhs) from a zero guess.
void MultigridOp::apply(double *out, const double *rhs) {
    std::lock_guard<std::mutex> lk(mtx);
    FAMG_REQUIRE(!levels.empty(), AMG_ERR_INVALID, "empty multigrid");
    FAMG_REQUIRE(out != rhs, AMG_ERR_INVALID, "multigrid apply: out must not alias rhs");
    for (size_t l = 0; l + 1 < levels.size(); l++)
        FAMG_REQUIRE(levels[l].R && levels[l].P, AMG_ERR_INVALID, "multigrid level without R/P");
    ensure_workspace();
    if (flags_gen_ != flags_generation()) {  // a switch changed: graphs recorded the old launches
        invalidate_graphs();
        flags_gen_ = flags_generation();
    }
    ensure_tail();
    hipStream_t s = ctx->stream;
    auto run = [&]() {
        if (levels[0].permuted) {  // the fine level runs in its numbering: rhs in, result out
            const int64_t n = levels[0].A->nrows;
            gather_fine(rhs, s);
            perm_scatter(out, perm_v0_.get(), levels[0].perm.get(), n, s);
        } else {
            cycle(0, out, rhs, true, out);
        }
    };
    // (the in-cycle launch timer runs the cycle eagerly: events recorded by graph
    // nodes cannot be read back with hipEventElapsedTime)
    if (!use_graph || s == nullptr || fine_timer >= 0) {
        run();
        return;
    }
    for (auto &g : graphs_)
        if (g.out == out && g.rhs == rhs) {
            FAMG_CHECK_HIP(hipGraphLaunch(g.exec, s));
            return;
        }
    hipGraph_t graph = nullptr;
    FAMG_CHECK_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
        run();
    } catch (...) {
        (void)hipStreamEndCapture(s, &graph);
        if (graph) (void)hipGraphDestroy(graph);
        throw;
    }
    FAMG_CHECK_HIP(hipStreamEndCapture(s, &graph));
    hipGraphExec_t exec = nullptr;
    FAMG_CHECK_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    (void)hipGraphDestroy(graph);
    if (graphs_.size() >= 8) {
        (void)hipGraphExecDestroy(graphs_.front().exec);
        graphs_.erase(graphs_.begin());
    }
    graphs_.push_back({out, rhs, exec});
    FAMG_CHECK_HIP(hipGraphLaunch(exec, s));
}

// Launch plan of one V-cycle (amg_multigrid_cycle_plan): one eager cycle on
// scratch vectors (b = 1) with the launch recorder on.
std::vector<LaunchRec> MultigridOp::cycle_plan() {
    std::lock_guard<std::mutex> lk(mtx);
    FAMG_REQUIRE(!levels.empty(), AMG_ERR_INVALID, "empty multigrid");
    ensure_workspace();
    ensure_tail();
    const int64_t n = levels[0].A->nrows;
    DevBuf<double> b(std::max<int64_t>(1, n)), z(std::max<int64_t>(1, n));
    vec_fill(b.get(), 1.0, n, ctx->stream);
    LaunchLog log;
    g_launch_log = &log;
    try {
        if (levels[0].permuted) {
            gather_fine(b.get(), ctx->stream);
            perm_scatter(z.get(), perm_v0_.get(), levels[0].perm.get(), n, ctx->stream);
        } else {
            cycle(0, z.get(), b.get(), true, z.get());
        }
    } catch (...) {
        g_launch_log = nullptr;
        throw;
    }
    g_launch_log = nullptr;
    FAMG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return log.recs;
}

// empty: only its name and grid (1 block per tag unit) show in a kernel trace
__global__ void k_trace_mark() {}

void trace_mark(Ctx &ctx, int32_t tag) {
    hipLaunchKernelGGL(k_trace_mark, dim3((unsigned)std::max<int32_t>(1, tag)), dim3(64), 0, ctx.stream);
    FAMG_CHECK_HIP(hipGetLastError());
}

// ------------------------------------------------------------------- setup

// Tentative SA interpolation, one candidate (interpolation/mod.rs:754-805).
CsrPtr sa_tentative(Ctx *ctx, int64_t n, const int64_t *agg_of, int64_t naggs, const double *nn,
                    double *coarse_nn) {
    std::vector<double> ss(naggs, 0.0);
    for (int64_t i = 0; i < n; i++) {
        const int64_t J = agg_of[i];
        FAMG_REQUIRE(J >= 0 && J < naggs, AMG_ERR_INVALID, "node not aggregated");
        ss[J] = ss[J] + nn[i] * nn[i];
    }
    for (int64_t J = 0; J < naggs; J++) {
        coarse_nn[J] = std::sqrt(ss[J]);
        FAMG_REQUIRE(coarse_nn[J] > 0.0, AMG_ERR_INVALID, "aggregate with a zero candidate");
    }
    std::vector<int64_t> rp(n + 1), col(n);
    std::vector<double> val(n);
    for (int64_t i = 0; i < n; i++) {
        rp[i] = i;
        col[i] = agg_of[i];
        val[i] = nn[i] / coarse_nn[agg_of[i]];
    }
    rp[n] = n;
    auto P = make_csr(ctx);
    csr_from_host(P->m, ctx, n, naggs, rp.data(), col.data(), val.data());
    P->nrows = n;
    P->ncols = naggs;
    return P;
}

static CsrPtr wrap(Ctx *ctx, GpuCsr &&m) {
    auto p = make_csr(ctx);
    p->m = std::move(m);
    p->nrows = p->m.nrows;
    p->ncols = p->m.ncols;
    return p;
}

CsrPtr spgemm_op(const CsrOp &A, const CsrOp &B) {
    GpuCsr C;
    spgemm(A.m, B.m, C);
    return wrap(A.ctx, std::move(C));
}

CsrPtr transpose_op(const CsrOp &P) {
    GpuCsr T;
    transpose(P.m, T);
    return wrap(P.ctx, std::move(T));
}

// smooth_interpolation (interpolation/mod.rs:927-946)
CsrPtr smooth_interpolation(CsrOp &A, const CsrOp &P, double omega) {
    FAMG_REQUIRE(A.nrows == A.ncols && A.ncols == P.nrows, AMG_ERR_DIM, "smooth_interpolation dims");
    GpuCsr S;
    spgemm(A.m, P.m, S, false);  // finalized by the fixup
    smooth_interp_fixup(S, P.m, A.diagonal(), omega);
    return wrap(A.ctx, std::move(S));
}

// A_c = R (A P) (interpolation/mod.rs:828)
CsrPtr galerkin_rap(const CsrOp &R, const CsrOp &A, const CsrOp &P, const int64_t *grid) {
    FAMG_REQUIRE(R.ncols == A.nrows && A.ncols == P.nrows && R.nrows == P.ncols, AMG_ERR_DIM,
                 "galerkin_rap dims");
    GpuCsr AP, C;
    spgemm(A.m, P.m, AP, false);
    spgemm(R.m, AP, C, false);
    if (grid)
        for (int q = 0; q < 3; q++) C.grid[q] = grid[q];
    if (grid) C.grid_src = 1;
    csr_finalize(C);
    return wrap(A.ctx, std::move(C));
}

__global__ void k_divs(double *x, double s, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = x[i] / s;
}

// hierarchy.rs:219-228 + smoothers.rs:146-158 (r = x - A x quirk) + thin QR
void nn_stationary_l1(CsrOp &A, int64_t iters, double *x_host) {
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    const int64_t n = A.nrows;
    auto d = make_l1(A);
    DevBuf<double> x(n), xin(n), r(n);
    FAMG_CHECK_HIP(hipMemcpyAsync(xin.get(), x_host, n * sizeof(double), hipMemcpyHostToDevice, s));
    vec_mul(x.get(), d->d.get(), xin.get(), n, s);
    for (int64_t it = 1; it < iters; it++) {
        spmv(A.m, x.get(), r.get(), SPMV_SET, SpmvEpi{}, s);
        vec_nn_step(x.get(), d->d.get(), r.get(), n, s);
    }
    const double nrm = std::sqrt(vec_dot(x.get(), x.get(), n, ctx));
    if (n) hipLaunchKernelGGL(k_divs, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, x.get(), nrm, n);
    FAMG_CHECK_HIP(hipMemcpyAsync(x_host, x.get(), n * sizeof(double), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
}

// ---- box-aggregate setup kernels (device-resident: no host pass over the
// fine rows; the 512^3 global setup copy of the distributed bench has 134M)

// agg[i] = box index of row i (x fastest)
__global__ void k_box_agg(int64_t cx, int64_t cy, int64_t cz, int64_t bx, int64_t by, int64_t bz, int64_t ncx,
                          int64_t ncy, int32_t *agg) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= cx * cy * cz) return;
    const int64_t x = i % cx, y = (i / cx) % cy, z = i / (cx * cy);
    agg[i] = (int32_t)(x / bx + ncx * (y / by + ncy * (z / bz)));
}

// coarse candidate of box J: sqrt(sum nn_i^2) over its nodes in ascending index
// order (the host loop of sa_tentative, bit for bit); *bad = 1 on a zero candidate
__global__ void k_box_norm(const double *nn, int64_t cx, int64_t cy, int64_t cz, int64_t bx, int64_t by, int64_t bz,
                           int64_t ncx, int64_t ncy, int64_t na, double *cnn, int *bad) {
    const int64_t J = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (J >= na) return;
    const int64_t ax = J % ncx, ay = (J / ncx) % ncy, az = J / (ncx * ncy);
    double ss = 0.0;
    for (int64_t z = az * bz; z < min(cz, (az + 1) * bz); z++)
        for (int64_t y = ay * by; y < min(cy, (ay + 1) * by); y++)
            for (int64_t x = ax * bx; x < min(cx, (ax + 1) * bx); x++) {
                const double v = nn[x + cx * (y + cy * z)];
                ss = ss + v * v;
            }
    cnn[J] = sqrt(ss);
    if (!(cnn[J] > 0.0)) *bad = 1;
}

// tentative P for one candidate: row i has one entry nn_i / cnn[agg_i] at agg_i
__global__ void k_tent_fill(const int32_t *agg, const double *nn, const double *cnn, int64_t n, int64_t *rp,
                            int32_t *col, double *val) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    rp[i] = i;
    if (i < n) {
        col[i] = agg[i];
        val[i] = nn[i] / cnn[agg[i]];
    }
}

// hierarchy.rs:219-228 on a device vector (nn_stationary_l1 without the host copies)
static void nn_stationary_l1_dev(CsrOp &A, int64_t iters, double *x) {
    Ctx &ctx = *A.ctx;
    hipStream_t s = ctx.stream;
    const int64_t n = A.nrows;
    auto d = make_l1(A);
    DevBuf<double> xin(n), r(n);
    vec_copy(xin.get(), x, n, s);
    vec_mul(x, d->d.get(), xin.get(), n, s);
    for (int64_t it = 1; it < iters; it++) {
        spmv(A.m, x, r.get(), SPMV_SET, SpmvEpi{}, s);
        vec_nn_step(x, d->d.get(), r.get(), n, s);
    }
    const double nrm = std::sqrt(vec_dot(x, x, n, ctx));
    if (n) hipLaunchKernelGGL(k_divs, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, x, nrm, n);
    FAMG_CHECK_HIP(hipGetLastError());
}

// Hierarchy::coarsen (hierarchy.rs:190-248) with box aggregates, then a
// Multigrid assembled as Multigrid::new / add_level (multigrid.rs:190-239).
// Every per-row pass runs on the device; the results are those of the host
// sa_tentative / nn_stationary_l1 (same operation order).
std::shared_ptr<MultigridOp> sa_build_box(const CsrPtr &A, int64_t nx, int64_t ny, int64_t nz,
                                          int64_t bx, int64_t by, int64_t bz,
                                          int64_t coarsest_dim, int64_t max_levels,
                                          double omega, int smoother) {
    FAMG_REQUIRE(nx * ny * nz == A->nrows, AMG_ERR_DIM, "grid dims do not match the matrix");
    FAMG_REQUIRE(bx > 0 && by > 0 && bz > 0, AMG_ERR_INVALID, "box sizes must be positive");
    Ctx *ctx = A->ctx;
    hipStream_t s = ctx->stream;
    if (max_levels <= 0) max_levels = INT64_MAX;
    std::vector<CsrPtr> As{A}, Rs, Ps;
    DevBuf<double> nn(std::max<int64_t>(1, A->nrows));
    vec_fill(nn.get(), 1.0, A->nrows, s);
    int64_t cx = nx, cy = ny, cz = nz;
    int64_t level = 1, coarse_dim = -1;
    std::vector<std::vector<int64_t>> aggs;  // per coarsened level (block smoother partition)
    std::vector<int64_t> naggs;
    DevBuf<int> bad(1);
    while ((coarse_dim < 0 || coarse_dim > coarsest_dim) && level < max_levels) {
        CsrPtr cur = As.back();
        const int64_t n = cur->nrows;
        const int64_t ncx = ceil_div(cx, bx), ncy = ceil_div(cy, by), ncz = ceil_div(cz, bz);
        const int64_t na = ncx * ncy * ncz;
        DevBuf<int32_t> agg(std::max<int64_t>(1, n));
        DevBuf<double> cnn(std::max<int64_t>(1, na));
        FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
        hipLaunchKernelGGL(k_box_agg, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, cx, cy, cz, bx, by, bz,
                           ncx, ncy, agg.get());
        hipLaunchKernelGGL(k_box_norm, dim3((unsigned)ceil_div(na, 256)), dim3(256), 0, s, nn.get(), cx, cy, cz, bx,
                           by, bz, ncx, ncy, na, cnn.get(), bad.get());
        int h = 0;
        FAMG_CHECK_HIP(hipMemcpyAsync(&h, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        FAMG_REQUIRE(h == 0, AMG_ERR_INVALID, "aggregate with a zero candidate");
        // tentative P (interpolation/mod.rs:754-805), one candidate: only the
        // SpGEMM reads it, so it gets no SpMV storage
        auto Pt = make_csr(ctx);
        csr_alloc(Pt->m, ctx, n, na, n);
        hipLaunchKernelGGL(k_tent_fill, dim3((unsigned)ceil_div(n + 1, 256)), dim3(256), 0, s, agg.get(), nn.get(),
                           cnn.get(), n, Pt->m.rp64.get(), Pt->m.col.get(), Pt->m.val.get());
        FAMG_CHECK_HIP(hipGetLastError());
        Pt->nrows = n;
        Pt->ncols = na;
        CsrPtr P = smooth_interpolation(*cur, *Pt, omega);
        Pt.reset();
        CsrPtr R = transpose_op(*P);
        {  // R and P as grid-transfer classes (1 B per row) where their rows fit the boxes
            const int64_t fg[3] = {cx, cy, cz}, cg[3] = {ncx, ncy, ncz};
            if (bx == 2 && by == 2 && bz == 2) {
                gtc_attach(P->m, fg, cg, 0);
                gtc_attach(R->m, fg, cg, 1);
                // the wider classes where the 8-bit ones do not fit (levels >= 1), or everywhere (FAMG_GTX=2)
                if (!P->m.gtc_on || gtx_mode() == 2) gtx_attach(P->m, fg, cg, 0);
                if (!R->m.gtc_on || gtx_mode() == 2) gtx_attach(R->m, fg, cg, 1);
            }
        }
        const int64_t cgrid[3] = {ncx, ncy, ncz};  // the coarse grid (x-staged stencil kernels)
        CsrPtr Ac = galerkin_rap(*R, *cur, *P, cgrid);
        nn_stationary_l1_dev(*Ac, 3, cnn.get());
        if (smoother == 3) {
            std::vector<int32_t> a32(n);
            FAMG_CHECK_HIP(hipMemcpyAsync(a32.data(), agg.get(), n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            FAMG_CHECK_HIP(hipStreamSynchronize(s));
            aggs.emplace_back(a32.begin(), a32.end());
            naggs.push_back(na);
        }
        Rs.push_back(R);
        Ps.push_back(P);
        As.push_back(Ac);
        nn = std::move(cnn);
        cx = ncx; cy = ncy; cz = ncz;
        coarse_dim = Ac->nrows;
        level++;
    }
    auto make_smoother = [&](const CsrPtr &M, size_t l) -> LinOpPtr {
        switch (smoother) {
        case 0: return make_jacobi(*M, omega);
        case 1: return make_l1(*M);
        case 2: {
            // multicolor SGS where the greedy coloring exposes parallelism
            // (<= SGS_MAX_COLORS colors); L1 on the dense Galerkin levels, whose
            // colorings need hundreds of colors (one launch per color)
            std::vector<int32_t> colors;
            const int64_t nc = greedy_coloring(M->m, colors);
            if (nc <= SGS_MAX_COLORS) return make_sgs(M, colors.data(), false);
            return make_l1(*M);
        }
        case 3:  // BlockSmoother over the level's box aggregates (block_smoothers.rs)
            return make_block_smoother(*M, aggs[l].data(), naggs[l], 1);
        default: fail(AMG_ERR_INVALID, "unknown smoother kind");
        }
    };
    auto mg = std::make_shared<MultigridOp>();
    mg->ctx = ctx;
    mg->nrows = mg->ncols = A->nrows;
    MgLevel L0;
    L0.A = A;
    L0.S = As.size() == 1 ? LinOpPtr(make_coarse_chol(*A)) : make_smoother(A, 0);
    mg->levels.push_back(std::move(L0));
    for (size_t l = 1; l < As.size(); l++) {
        LinOpPtr S = (l + 1 == As.size()) ? LinOpPtr(make_coarse_chol(*As[l])) : make_smoother(As[l], l);
        mg->add_level(As[l], S, Rs[l - 1], Ps[l - 1]);
    }
    return mg;
}

}  // namespace famg
