// solve.hpp -- device-resident solve loops and the Composite preconditioner.
//
// The loops keep every vector in HBM; only the scalars of each iteration (dots)
// come back to the host.  They are written once over a small set of callbacks so
// the single-GPU and distributed (dots all-reduced over ranks) drivers share the
// arithmetic exactly.
#pragma once

#include <functional>
#include <mutex>

#include "famg.hpp"

namespace famg {

struct SolveOps {
    Ctx *ctx = nullptr;
    int64_t n = 0;                                                          // local rows
    // allocation length of the vectors A and resid read (>= n): a distributed
    // operator keeps its halo entries behind the owned rows, so the loops keep
    // x and p in buffers of this length and A reads them in place
    int64_t n_alloc = 0;
    std::function<void(double *out, double *x)> A;                          // out = A x (x: n_alloc, halo written)
    std::function<void(double *r, const double *b, double *x)> resid;        // r = b - A x (x: n_alloc)
    std::function<void(double *out, const double *r)> M;                    // out = M r (empty: identity)
    std::function<double(const double *, const double *)> dot;              // global dot
};

// Stationary iteration (examples/simple_geometric.rs:117-158): rho_k =
// ||b - A x_k|| / ||b||, stop below rel_tol or at max_iter, else x += M r.
int64_t stationary_impl(const SolveOps &o, const double *b, double *x, int64_t max_iter, double rel_tol,
                        double *hist);

// Preconditioned CG (the counterpart of faer conjugate_gradient as called by
// utils.rs:600-609): stop when ||r|| <= max(rel_tol ||b||, abs_tol).
int64_t pcg_impl(const SolveOps &o, const double *b, double *x, int64_t max_iter, double rel_tol, double abs_tol,
                 double *hist);

// Composite (preconditioners/composite.rs:11-83): components c_0..c_{m-1}
// applied c_{m-1}, ..., c_1, c_0, c_1, ..., c_{m-1}; each step
// out += c(r); r = rhs - A out, starting from out = 0, r = rhs.
struct CompositeOp : LinOp {
    LinOpPtr A;
    std::vector<LinOpPtr> comps;
    DevBuf<double> ws;
    std::mutex mtx;
    Kind kind() const override { return Kind::Composite; }
    bool is_precond() const override { return true; }
    void apply(double *out, const double *rhs) override;
};

// r = b - A x using the fused residual SpMV when A is a CSR matrix.
void residual(LinOp &A, double *r, const double *b, const double *x);

}  // namespace famg
