// solve.cpp -- solve loops, Composite, and their C ABI (include/amg.h).
#include "solve.hpp"

#include <cmath>

#include "handles.hpp"

using namespace famg;

namespace famg {

void residual(LinOp &A, double *r, const double *b, const double *x) {
    hipStream_t s = A.ctx->stream;
    if (auto *c = dynamic_cast<CsrOp *>(&A)) {
        SpmvEpi epi;
        epi.b = b;
        spmv(c->m, x, r, SPMV_RESID, epi, s);
        return;
    }
    A.apply(r, x);
    vec_sub(r, b, r, A.nrows, s);
}

// x in a buffer of the operator's allocation length (the caller's when that is n)
static double *padded_x(const SolveOps &o, double *x, DevBuf<double> &xp) {
    if (o.n_alloc <= o.n) return x;
    xp.resize(o.n_alloc);
    vec_copy(xp.get(), x, o.n, o.ctx->stream);
    return xp.get();
}

int64_t stationary_impl(const SolveOps &o, const double *b, double *x_user, int64_t max_iter, double rel_tol,
                        double *hist) {
    hipStream_t s = o.ctx->stream;
    const int64_t n = o.n;
    DevBuf<double> r(std::max<int64_t>(1, n)), z(std::max<int64_t>(1, n)), xp;
    double *x = padded_x(o, x_user, xp);
    const double bn = std::sqrt(o.dot(b, b));
    int64_t it = 0;
    for (;;) {
        o.resid(r.get(), b, x);
        const double rel = std::sqrt(o.dot(r.get(), r.get())) / bn;
        it++;
        if (hist) hist[it - 1] = rel;
        if (rel < rel_tol || it >= max_iter) break;
        o.M(z.get(), r.get());
        vec_add_inplace(x, z.get(), n, s);
    }
    if (x != x_user) vec_copy(x_user, x, n, s);
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return it;
}

int64_t pcg_impl(const SolveOps &o, const double *b, double *x, int64_t max_iter, double rel_tol, double abs_tol,
                 double *hist) {
    hipStream_t s = o.ctx->stream;
    const int64_t n = o.n;
    const int64_t nb = std::max<int64_t>(1, n);
    DevBuf<double> r(nb), z(nb), p(std::max(nb, o.n_alloc)), Ap(nb), xp;
    o.resid(r.get(), b, padded_x(o, x, xp));  // x itself only moves by axpys below
    const double bn = std::sqrt(o.dot(b, b));
    const double tol = std::max(rel_tol * bn, abs_tol);
    int64_t it = 0;
    if (std::sqrt(o.dot(r.get(), r.get())) > tol) {
        auto pc = [&](double *dst, const double *src) {
            if (o.M) o.M(dst, src);
            else vec_copy(dst, src, n, s);
        };
        pc(z.get(), r.get());
        vec_copy(p.get(), z.get(), n, s);
        double rz = o.dot(r.get(), z.get());
        for (it = 1; it <= max_iter; it++) {
            o.A(Ap.get(), p.get());
            const double alpha = rz / o.dot(p.get(), Ap.get());
            vec_axpy(x, alpha, p.get(), n, s);
            vec_axpy(r.get(), -alpha, Ap.get(), n, s);
            const double rn = std::sqrt(o.dot(r.get(), r.get()));
            if (hist) hist[it - 1] = rn / bn;
            if (rn <= tol) break;
            pc(z.get(), r.get());
            const double rzn = o.dot(r.get(), z.get());
            const double beta = rzn / rz;
            rz = rzn;
            vec_xpay(p.get(), beta, z.get(), n, s);
        }
    }
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    return it;
}

void CompositeOp::apply(double *out, const double *rhs) {
    std::lock_guard<std::mutex> lk(mtx);
    hipStream_t s = ctx->stream;
    const int64_t n = nrows;
    if (ws.size() < (size_t)std::max<int64_t>(1, n)) ws.resize(std::max<int64_t>(1, n));
    vec_fill(out, 0.0, n, s);
    vec_copy(ws.get(), rhs, n, s);
    auto step = [&](LinOp &c) {
        c.apply_in_place(ws.get());
        vec_add_inplace(out, ws.get(), n, s);
        residual(*A, ws.get(), rhs, out);
    };
    for (size_t k = comps.size(); k-- > 0;) step(*comps[k]);
    for (size_t k = 1; k < comps.size(); k++) step(*comps[k]);
}

}  // namespace famg

namespace {

LinOp &need_op(const amg_linop *h) {
    FAMG_REQUIRE(h && h->op, AMG_ERR_INVALID, "null amg_linop handle");
    return *h->op;
}

SolveOps single_gpu_ops(LinOp &a, LinOp *m) {
    SolveOps o;
    o.ctx = a.ctx;
    o.n = a.nrows;
    o.n_alloc = a.nrows;
    o.A = [&a](double *out, double *x) { a.apply(out, x); };
    o.resid = [&a](double *r, const double *b, double *x) { residual(a, r, b, x); };
    if (m) o.M = [m](double *out, const double *r) { m->apply(out, r); };
    Ctx *ctx = a.ctx;
    const int64_t n = a.nrows;
    o.dot = [ctx, n](const double *u, const double *v) { return vec_dot(u, v, n, *ctx); };
    return o;
}

}  // namespace

extern "C" {

amg_status amg_composite_create(const amg_linop *A, amg_linop *const *components, int64_t ncomponents,
                                amg_linop **out) {
    return guard([&] {
        LinOp &a = need_op(A);
        FAMG_REQUIRE(out && ncomponents >= 1 && components, AMG_ERR_INVALID, "need at least one component");
        FAMG_REQUIRE(a.nrows == a.ncols, AMG_ERR_DIM, "Composite needs a square operator");
        auto c = std::make_shared<CompositeOp>();
        c->ctx = a.ctx;
        c->A = A->op;
        c->nrows = c->ncols = a.nrows;
        for (int64_t k = 0; k < ncomponents; k++) {
            LinOp &p = need_op(components[k]);
            FAMG_REQUIRE(p.nrows == a.nrows && p.ncols == a.nrows, AMG_ERR_DIM, "component dims");
            FAMG_REQUIRE(p.ctx == a.ctx, AMG_ERR_INVALID, "component on another context");
            c->comps.push_back(components[k]->op);
        }
        *out = new amg_linop{c};
    });
}

amg_status amg_composite_push(amg_linop *composite, const amg_linop *component) {
    return guard([&] {
        need_op(composite);
        auto c = std::dynamic_pointer_cast<CompositeOp>(composite->op);
        FAMG_REQUIRE(c, AMG_ERR_INVALID, "not a Composite");
        LinOp &p = need_op(component);
        FAMG_REQUIRE(p.nrows == c->nrows && p.ncols == c->nrows, AMG_ERR_DIM, "component dims");
        std::lock_guard<std::mutex> lk(c->mtx);
        c->comps.push_back(component->op);
    });
}

amg_status amg_composite_ncomponents(const amg_linop *composite, int64_t *n) {
    return guard([&] {
        auto *c = dynamic_cast<CompositeOp *>(&need_op(composite));
        FAMG_REQUIRE(c && n, AMG_ERR_INVALID, "not a Composite");
        *n = (int64_t)c->comps.size();
    });
}

amg_status amg_stationary_solve(amg_linop *A, amg_linop *M, const double *b, double *x, int64_t max_iter,
                                double rel_tol, double *hist, int64_t *iters) {
    return guard([&] {
        LinOp &a = need_op(A);
        LinOp &m = need_op(M);
        FAMG_REQUIRE(b && x && iters && max_iter > 0, AMG_ERR_INVALID, "bad argument");
        FAMG_REQUIRE(a.nrows == a.ncols && m.nrows == a.nrows, AMG_ERR_DIM, "solver dims");
        a.ctx->set_device();
        *iters = stationary_impl(single_gpu_ops(a, &m), b, x, max_iter, rel_tol, hist);
    });
}

amg_status amg_pcg_solve(amg_linop *A, amg_linop *M, const double *b, double *x, int64_t max_iter,
                         double rel_tol, double abs_tol, double *hist, int64_t *iters) {
    return guard([&] {
        LinOp &a = need_op(A);
        FAMG_REQUIRE(b && x && iters && max_iter >= 0, AMG_ERR_INVALID, "bad argument");
        LinOp *m = M ? &need_op(M) : nullptr;
        FAMG_REQUIRE(a.nrows == a.ncols && (!m || m->nrows == a.nrows), AMG_ERR_DIM, "solver dims");
        a.ctx->set_device();
        *iters = pcg_impl(single_gpu_ops(a, m), b, x, max_iter, rel_tol, abs_tol, hist);
    });
}

}  // extern "C"
