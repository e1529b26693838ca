// capi.cpp -- extern "C" boundary (include/amg.h).  Converts library
// exceptions to amg_status + a thread-local message; handles are thin boxes
// around shared_ptr<LinOp> so operators keep what they reference alive (the
// reference's Arc<dyn LinOp> ownership, core.rs:9-17).
#include <atomic>
#include <cmath>
#include <cstring>
#include <string>

#include "handles.hpp"

using namespace famg;

namespace {
thread_local std::string g_last_error;
}

amg_status famg::set_last_error(amg_status s, const char *msg) {
    g_last_error = msg;
    return s;
}

namespace {
amg_linop *box(LinOpPtr p) { return new amg_linop{std::move(p)}; }

LinOp &need(const amg_linop *h) {
    FAMG_REQUIRE(h && h->op, AMG_ERR_INVALID, "null amg_linop handle");
    return *h->op;
}

CsrPtr need_csr(const amg_linop *h) {
    need(h);
    auto p = std::dynamic_pointer_cast<CsrOp>(h->op);
    FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not a CSR matrix");
    return p;
}

std::shared_ptr<MultigridOp> need_mg(const amg_linop *h) {
    need(h);
    auto p = std::dynamic_pointer_cast<MultigridOp>(h->op);
    FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not a multigrid");
    return p;
}

amg_ctx *ctx_of(const LinOp &op) {
    // Ctx is the first member of amg_ctx
    return reinterpret_cast<amg_ctx *>(op.ctx);
}

// Run f(out_col, rhs_col) for each of k columns, staging host memory.
template <typename F>
void for_columns(LinOp &op, double *out, int64_t ld_out, const double *rhs, int64_t ld_rhs,
                 int64_t k, amg_mem mem, int64_t out_rows, int64_t rhs_rows, F &&f) {
    FAMG_REQUIRE(k >= 0, AMG_ERR_INVALID, "negative column count");
    if (k == 0) return;
    FAMG_REQUIRE(out && rhs, AMG_ERR_INVALID, "null vector");
    FAMG_REQUIRE(ld_out >= out_rows && ld_rhs >= rhs_rows, AMG_ERR_INVALID, "leading dimension too small");
    Ctx &ctx = *op.ctx;
    ctx.set_device();
    if (mem == AMG_MEM_DEVICE) {
        for (int64_t c = 0; c < k; c++) f(out + c * ld_out, rhs + c * ld_rhs);
        return;
    }
    FAMG_REQUIRE(mem == AMG_MEM_HOST, AMG_ERR_INVALID, "bad amg_mem");
    amg_ctx *ac = ctx_of(op);
    if (ac->stage_in.size() < (size_t)rhs_rows) ac->stage_in.resize(rhs_rows);
    if (ac->stage_out.size() < (size_t)out_rows) ac->stage_out.resize(out_rows);
    for (int64_t c = 0; c < k; c++) {
        FAMG_CHECK_HIP(hipMemcpyAsync(ac->stage_in.get(), rhs + c * ld_rhs, rhs_rows * sizeof(double),
                                      hipMemcpyHostToDevice, ctx.stream));
        f(ac->stage_out.get(), ac->stage_in.get());
        FAMG_CHECK_HIP(hipMemcpyAsync(out + c * ld_out, ac->stage_out.get(), out_rows * sizeof(double),
                                      hipMemcpyDeviceToHost, ctx.stream));
        FAMG_CHECK_HIP(hipStreamSynchronize(ctx.stream));
    }
}

}  // namespace

namespace famg {
void export_plan(const std::vector<LaunchRec> &plan, amg_launch_rec *recs, int64_t cap, int64_t *count) {
    *count = (int64_t)plan.size();
    if (!recs) return;
    for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)plan.size()); i++) {
        const LaunchRec &r = plan[i];
        amg_launch_rec &o = recs[i];
        o.level = r.level;
        o.role = r.role;
        o.kernel = r.kernel;
        o.mode = r.mode;
        o.rows = r.rows;
        o.bytes = r.bytes;
        o.csr_bytes = r.csr_bytes;
        std::memset(o.name, 0, sizeof(o.name));
        std::strncpy(o.name, r.name, sizeof(o.name) - 1);
    }
}
}  // namespace famg

namespace famg {
static std::atomic<int64_t> g_flag_val[FLAG_COUNT] = {
    {[] { const char *e = getenv("FAMG_FOLD_XSCS"); return (int64_t)(e && e[0] == '1'); }()},
    {[] { const char *e = getenv("FAMG_DIA_DK"); return (int64_t)!(e && e[0] == '0'); }()},
    {[] {
        const char *e = getenv("FAMG_VEC_WPR");
        const int w = e ? atoi(e) : 0;
        return (int64_t)((w == 1 || w == 2 || w == 4) ? w : 0);
    }()},
    {[] { const char *e = getenv("FAMG_GTX_TIME"); return (int64_t)(e ? atoi(e) : 2); }()},
    {[] { const char *e = getenv("FAMG_SGS27_MARCH"); return (int64_t)(e ? atoi(e) : 1); }()},
    {[] { const char *e = getenv("FAMG_XS_PIPE"); return (int64_t)(e ? atoi(e) : 2); }()},
    {[] { const char *e = getenv("FAMG_BSR_KERNEL"); return (int64_t)(e ? atoi(e) : 0); }()},
    {[] { const char *e = getenv("FAMG_BSR_LONG"); return (int64_t)(e ? atoll(e) : 48); }()},
    {[] { const char *e = getenv("FAMG_DIA7_RP"); return (int64_t)(e ? atoi(e) : 0); }()},
    {[] { const char *e = getenv("FAMG_FINE_FUSE"); return (int64_t)(e ? atoi(e) : 1); }()},
    {[] { const char *e = getenv("FAMG_DENSE_TAIL"); return (int64_t)(e ? atoll(e) : 4096); }()}};
static std::atomic<uint64_t> g_flag_gen{0};
int64_t flag(FlagId f) { return g_flag_val[f].load(std::memory_order_relaxed); }
void set_flag(FlagId f, int64_t v) {
    g_flag_val[f].store(v);
    g_flag_gen.fetch_add(1);
}
uint64_t flags_generation() { return g_flag_gen.load(); }
}  // namespace famg

extern "C" {

const char *amg_last_error(void) { return g_last_error.c_str(); }
const char *amg_version(void) { return "faer-amg_amd 0.1.0 (gfx950)"; }

amg_status amg_ctx_create(int device, void *hip_stream, amg_ctx **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output pointer");
        int ndev = 0;
        FAMG_CHECK_HIP(hipGetDeviceCount(&ndev));
        FAMG_REQUIRE(device >= 0 && device < ndev, AMG_ERR_INVALID, "device index out of range");
        auto *c = new amg_ctx();
        c->ctx.device = device;
        try {
            c->ctx.set_device();
            if (hip_stream) {
                c->ctx.stream = static_cast<hipStream_t>(hip_stream);
            } else {
                FAMG_CHECK_HIP(hipStreamCreateWithFlags(&c->ctx.stream, hipStreamNonBlocking));
                c->ctx.own_stream = true;
            }
            hipDeviceProp_t prop;
            FAMG_CHECK_HIP(hipGetDeviceProperties(&prop, device));
            c->ctx.num_cus = prop.multiProcessorCount;
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

amg_status amg_ctx_destroy(amg_ctx *ctx) {
    return guard([&] {
        if (!ctx) return;
        ctx->ctx.set_device();
        if (ctx->ctx.stream) (void)hipStreamSynchronize(ctx->ctx.stream);
        delete ctx;
    });
}

amg_status amg_ctx_synchronize(amg_ctx *ctx) {
    return guard([&] {
        FAMG_REQUIRE(ctx, AMG_ERR_INVALID, "null context");
        ctx->ctx.set_device();
        FAMG_CHECK_HIP(hipStreamSynchronize(ctx->ctx.stream));
    });
}

amg_status amg_ctx_stream(amg_ctx *ctx, void **hip_stream) {
    return guard([&] {
        FAMG_REQUIRE(ctx && hip_stream, AMG_ERR_INVALID, "null argument");
        *hip_stream = ctx->ctx.stream;
    });
}

amg_status amg_ctx_join_stream(amg_ctx *ctx, void *other, int32_t ctx_waits) {
    return guard([&] {
        FAMG_REQUIRE(ctx, AMG_ERR_INVALID, "null context");
        hipStream_t o = static_cast<hipStream_t>(other);
        if (o == ctx->ctx.stream) return;
        ctx->ctx.set_device();
        if (!ctx->join_event) FAMG_CHECK_HIP(hipEventCreateWithFlags(&ctx->join_event, hipEventDisableTiming));
        if (ctx_waits) {
            FAMG_CHECK_HIP(hipEventRecord(ctx->join_event, o));
            FAMG_CHECK_HIP(hipStreamWaitEvent(ctx->ctx.stream, ctx->join_event, 0));
        } else {
            FAMG_CHECK_HIP(hipEventRecord(ctx->join_event, ctx->ctx.stream));
            FAMG_CHECK_HIP(hipStreamWaitEvent(o, ctx->join_event, 0));
        }
    });
}

amg_status amg_set_alloc_policy(int32_t policy) {
    return guard([&] {
        FAMG_REQUIRE(policy == 0 || policy == 1, AMG_ERR_INVALID, "policy must be 0 or 1");
        FAMG_REQUIRE(policy == 0 || g_alloc_experiment > 0, AMG_ERR_UNSUPPORTED,
                     "contiguous allocations read stale data across kernels on gfx950 (DESIGN.md 3)");
        g_alloc_policy = policy;
    });
}

amg_status amg_set_value_codes(int32_t enable) {
    return guard([&] {
        FAMG_REQUIRE(enable >= 0 && enable <= 2, AMG_ERR_INVALID, "enable must be 0, 1 or 2");
        g_value_codes = enable;
    });
}

amg_status amg_set_sgs_fused(int32_t enable) {
    return guard([&] {
        FAMG_REQUIRE(enable >= 0 && enable <= 2, AMG_ERR_INVALID, "enable must be 0, 1 or 2");
        g_sgs_fused = enable;
    });
}

amg_status amg_sgs_fused(const amg_linop *op, int32_t *fused) {
    return guard([&] {
        FAMG_REQUIRE(fused, AMG_ERR_INVALID, "null output");
        auto p = std::dynamic_pointer_cast<SgsOp>(need(op).shared_from_this());
        FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not an SGS smoother");
        *fused = p->fused27 ? 1 : 0;
    });
}

amg_status amg_set_spmv_format(int32_t policy) {
    return guard([&] {
        FAMG_REQUIRE(policy >= 0 && policy <= 3, AMG_ERR_INVALID, "policy must be 0..3");
        g_spmv_format_policy = policy;
    });
}

// ------------------------------------------------------------------ CSR

amg_status amg_csr_create(amg_ctx *ctx, int64_t nrows, int64_t ncols, const int64_t *rowptr,
                          const int64_t *colidx, const double *vals, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out, AMG_ERR_INVALID, "null argument");
        FAMG_REQUIRE(nrows >= 0 && ncols >= 0, AMG_ERR_INVALID, "negative dimension");
        ctx->ctx.set_device();
        auto p = make_csr(&ctx->ctx);
        csr_from_host(p->m, &ctx->ctx, nrows, ncols, rowptr, colidx, vals);
        p->nrows = nrows;
        p->ncols = ncols;
        *out = box(p);
    });
}

__attribute__((visibility("default"))) amg_status amg_csr_create_device_i32(
    amg_ctx *ctx, int64_t nrows, int64_t ncols, const int32_t *rowptr, const int32_t *colidx,
    const double *vals, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out && rowptr, AMG_ERR_INVALID, "null argument");
        ctx->ctx.set_device();
        hipStream_t s = ctx->ctx.stream;
        std::vector<int32_t> rp32(nrows + 1);
        FAMG_CHECK_HIP(hipMemcpyAsync(rp32.data(), rowptr, (nrows + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        std::vector<int64_t> rp(rp32.begin(), rp32.end());
        const int64_t nnz = rp[nrows];
        auto p = make_csr(&ctx->ctx);
        csr_alloc(p->m, &ctx->ctx, nrows, ncols, nnz);
        FAMG_CHECK_HIP(hipMemcpyAsync(p->m.rp64.get(), rp.data(), (nrows + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
        if (nnz) {
            FAMG_CHECK_HIP(hipMemcpyAsync(p->m.col.get(), colidx, nnz * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
            FAMG_CHECK_HIP(hipMemcpyAsync(p->m.val.get(), vals, nnz * sizeof(double), hipMemcpyDeviceToDevice, s));
        }
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        csr_finalize(p->m);
        p->nrows = nrows;
        p->ncols = ncols;
        *out = box(p);
    });
}

amg_status amg_csr_nnz(const amg_linop *op, int64_t *nnz) {
    return guard([&] {
        FAMG_REQUIRE(nnz, AMG_ERR_INVALID, "null argument");
        *nnz = need_csr(op)->m.nnz;
    });
}

amg_status amg_csr_spmv_info(const amg_linop *op, int64_t *info8) {
    return guard([&] {
        FAMG_REQUIRE(info8, AMG_ERR_INVALID, "null argument");
        const GpuCsr &m = need_csr(op)->m;
        info8[0] = m.kernel;
        info8[1] = m.stream_bytes();
        info8[2] = m.index_bytes();
        info8[3] = m.nslices;
        info8[4] = m.sell_steps * 64;
        info8[5] = m.sell_mode_slices[0];
        info8[6] = m.sell_mode_slices[1];
        info8[7] = m.sell_mode_slices[2];
        if (m.kernel == SPMV_KERNEL_XS) {  // slices with LDS indices as "u16", escape slices as "i32"
            info8[3] = (int64_t)m.xs_desc.size();
            info8[4] = m.xs_steps * 64;
            info8[5] = 0;
            info8[6] = info8[3] - m.xs_escape_slices;
            info8[7] = m.xs_escape_slices;
        }
        if (m.gtx_on) {  // the wide grid-transfer overlay (gtx.hip; served first)
            info8[0] = SPMV_KERNEL_GTC;
            info8[1] = 2 * m.nrows + 12 * m.gtx_nent + 8 * m.gtx_nclass;
        } else if (m.gtc_on) {  // the grid-transfer overlay (its modes; the storage above serves the rest)
            info8[0] = SPMV_KERNEL_GTC;
            info8[1] = m.nrows + 2 * (int64_t)m.gtc_nce + 8 * (int64_t)m.gtc_ntab;
        }
    });
}

amg_status amg_csr_value_codes(const amg_linop *op, int64_t *info2) {
    return guard([&] {
        FAMG_REQUIRE(info2, AMG_ERR_INVALID, "null argument");
        const GpuCsr &m = need_csr(op)->m;
        if (m.kernel == SPMV_KERNEL_DIA) {
            info2[0] = m.dia_vbits;
            info2[1] = m.dia_ntab;
        } else {
            if (m.kernel == SPMV_KERNEL_SELLP) {
                info2[0] = m.sellp_vbits;
                info2[1] = m.sellp_ntab;
                return;
            }
            const bool coded = m.kernel == SPMV_KERNEL_SELL || m.kernel == SPMV_KERNEL_VECTOR;
            info2[0] = !coded ? 0 : m.kernel == SPMV_KERNEL_SELL ? m.sell_vbits : m.vec_vbits;
            info2[1] = coded && info2[0] ? m.sell_ntab : 0;
        }
    });
}

amg_status amg_csr_class_info(const amg_linop *op, int64_t *info4) {
    return guard([&] {
        FAMG_REQUIRE(info4, AMG_ERR_INVALID, "null argument");
        const GpuCsr &m = need_csr(op)->m;
        const bool on = m.has_scs();
        info4[0] = on ? m.scs_nclass : 0;
        info4[1] = on ? m.scs_k : 0;
        info4[2] = on ? 8 * m.scs_ib : 0;
        info4[3] = on ? 8 * m.scs_k * m.scs_nclass : 0;
    });
}

amg_status amg_csr_set_grid(amg_linop *op, int64_t nx, int64_t ny, int64_t nz) {
    return guard([&] {
        auto p = need_csr(op);
        FAMG_REQUIRE(nx >= 0 && ny >= 0 && nz >= 0, AMG_ERR_INVALID, "grid dims must be >= 0");
        FAMG_REQUIRE((nx == 0 && ny == 0 && nz == 0) || (p->m.nrows == p->m.ncols && nx * ny * nz == p->m.nrows),
                     AMG_ERR_DIM, "grid dims do not match the square matrix");
        p->m.grid[0] = nx;
        p->m.grid[1] = ny;
        p->m.grid[2] = nz;
        p->m.grid_src = 1;  // also a cleared hint: nothing is inferred then
        csr_finalize(p->m, &p->m.seg_rows);
    });
}


amg_status amg_set_flag(int32_t which, int64_t value) {
    return guard([&] {
        FAMG_REQUIRE(which >= 0 && which < FLAG_COUNT, AMG_ERR_INVALID, "unknown flag");
        if (which == FLAG_DIA7_RP)
            FAMG_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, AMG_ERR_INVALID,
                         "row pairs per lane must be 0 (auto), 1, 2 or 4");
        if (which == FLAG_VEC_WPR)
            FAMG_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, AMG_ERR_INVALID,
                         "waves per row must be 0 (auto), 1, 2 or 4");
        set_flag((FlagId)which, value);
    });
}

amg_status amg_get_flag(int32_t which, int64_t *value) {
    return guard([&] {
        FAMG_REQUIRE(which >= 0 && which < FLAG_COUNT && value, AMG_ERR_INVALID, "bad argument");
        *value = flag((FlagId)which);
    });
}

amg_status amg_grid_from_offsets(const int64_t *offs, int64_t k, int64_t n, int64_t *grid3, int32_t *found) {
    return guard([&] {
        FAMG_REQUIRE((offs || k == 0) && grid3 && found && k >= 0 && n >= 0, AMG_ERR_INVALID, "bad argument");
        std::vector<int64_t> o(offs, offs + k);
        grid3[0] = grid3[1] = grid3[2] = 0;
        *found = grid_from_offsets(o, n, grid3) ? 1 : 0;
    });
}

amg_status amg_csr_grid_info(const amg_linop *op, int64_t *info12) {
    return guard([&] {
        FAMG_REQUIRE(info12, AMG_ERR_INVALID, "null argument");
        const GpuCsr &m = need_csr(op)->m;
        for (int q = 0; q < 13; q++) info12[q] = 0;
        for (int q = 0; q < 3; q++) info12[q] = m.grid[q];
        info12[10] = m.grid_src;
        info12[12] = m.xscs ? m.xscs_tile_src : 0;
        info12[11] = m.gtx_on ? (m.gtx_r ? 4 : 3) : m.gtc_on ? (m.gtc_r ? 2 : 1) : 0;
        const bool on = m.has_scs() && m.xscs;
        info12[3] = on ? 1 : 0;
        for (int q = 0; q < 3; q++) {
            info12[4 + q] = on ? m.xscs_t[q] : 0;
            info12[7 + q] = on ? m.xscs_r[q] : 0;
        }
    });
}

amg_status amg_csr_dia_range(const amg_linop *op, int64_t *info4) {
    return guard([&] {
        FAMG_REQUIRE(info4, AMG_ERR_INVALID, "null argument");
        const GpuCsr &m = need_csr(op)->m;
        const bool on = m.has_dia();
        info4[0] = on ? m.dia_r0 : 0;
        info4[1] = on ? m.dia_r1 : 0;
        info4[2] = on ? m.dia_k : 0;
        info4[3] = on ? m.dia_vbits : 0;
    });
}

amg_status amg_csr_spmv_epilogue(const amg_linop *op, int32_t mode, const double *x, double *y, const double *b,
                                 const double *d) {
    return guard([&] {
        auto p = need_csr(op);
        FAMG_REQUIRE(mode >= SPMV_SET && mode <= SPMV_JACOBI, AMG_ERR_INVALID, "mode must be SET, ADD, RESID or JACOBI");
        FAMG_REQUIRE(x && y && x != y, AMG_ERR_INVALID, "x and y must be distinct device vectors");
        FAMG_REQUIRE((mode != SPMV_RESID && mode != SPMV_JACOBI) || b, AMG_ERR_INVALID, "b required");
        FAMG_REQUIRE(mode != SPMV_JACOBI || d, AMG_ERR_INVALID, "d required");
        SpmvEpi e;
        e.b = b;
        e.d = d;
        spmv(p->m, x, y, (SpmvMode)mode, e, p->ctx->stream);
    });
}

amg_status amg_csr_download(const amg_linop *op, int64_t *rowptr, int64_t *colidx, double *vals) {
    return guard([&] {
        auto p = need_csr(op);
        FAMG_REQUIRE(rowptr && (p->m.nnz == 0 || (colidx && vals)), AMG_ERR_INVALID, "null array");
        p->ctx->set_device();
        csr_to_host(p->m, rowptr, colidx, vals);
    });
}

amg_status amg_gen_laplace3d_7pt(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out, AMG_ERR_INVALID, "null argument");
        ctx->ctx.set_device();
        static const int offs[21] = {0, 0, -1, 0, -1, 0, -1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1};
        static const double coef[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
        auto p = make_csr(&ctx->ctx);
        gen_stencil(p->m, &ctx->ctx, nx, ny, nz, offs, coef, 7);
        p->nrows = p->ncols = p->m.nrows;
        *out = box(p);
    });
}

amg_status amg_gen_random_7pt(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz, uint64_t seed, int64_t window,
                              amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out, AMG_ERR_INVALID, "null argument");
        ctx->ctx.set_device();
        auto p = make_csr(&ctx->ctx);
        gen_random_7pt(p->m, &ctx->ctx, nx, ny, nz, seed, window);
        p->nrows = p->ncols = p->m.nrows;
        *out = box(p);
    });
}

amg_status amg_gen_aniso27(amg_ctx *ctx, int64_t nx, int64_t ny, int64_t nz, double ex, double ey,
                           double ez, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out, AMG_ERR_INVALID, "null argument");
        ctx->ctx.set_device();
        const double T[3] = {-1.0, 2.0, -1.0};
        const double M[3] = {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0};
        int offs[81];
        double coef[27];
        int k = 0;
        for (int dz = 0; dz < 3; dz++)
            for (int dy = 0; dy < 3; dy++)
                for (int dx = 0; dx < 3; dx++, k++) {
                    offs[3 * k] = dx - 1;
                    offs[3 * k + 1] = dy - 1;
                    offs[3 * k + 2] = dz - 1;
                    coef[k] = ex * (T[dx] * M[dy] * M[dz]) + ey * (M[dx] * T[dy] * M[dz]) +
                              ez * (M[dx] * M[dy] * T[dz]);
                }
        auto p = make_csr(&ctx->ctx);
        gen_stencil(p->m, &ctx->ctx, nx, ny, nz, offs, coef, 27);
        p->nrows = p->ncols = p->m.nrows;
        *out = box(p);
    });
}

// ------------------------------------------------------------ generic ops

amg_status amg_linop_kind_of(const amg_linop *op, int32_t *kind) {
    return guard([&] {
        FAMG_REQUIRE(kind, AMG_ERR_INVALID, "null argument");
        *kind = static_cast<int32_t>(need(op).kind());
    });
}

amg_status amg_linop_dims(const amg_linop *op, int64_t *nrows, int64_t *ncols) {
    return guard([&] {
        const LinOp &o = need(op);
        if (nrows) *nrows = o.nrows;
        if (ncols) *ncols = o.ncols;
    });
}

// k > 1 columns of a CSR operator: one SpMM (the matrix streamed once per 8
// columns) instead of k SpMVs; host blocks are staged whole.
static bool csr_multi_apply(LinOp &o, double *out, int64_t ld_out, const double *rhs, int64_t ld_rhs, int64_t k,
                            amg_mem mem) {
    auto *c = dynamic_cast<CsrOp *>(&o);
    if (!c || k <= 1) return false;
    FAMG_REQUIRE(out && rhs, AMG_ERR_INVALID, "null vector");
    FAMG_REQUIRE(ld_out >= o.nrows && ld_rhs >= o.ncols, AMG_ERR_INVALID, "leading dimension too small");
    Ctx &ctx = *o.ctx;
    ctx.set_device();
    if (mem == AMG_MEM_DEVICE) {
        spmm(c->m, rhs, ld_rhs, out, ld_out, k, ctx.stream);
        return true;
    }
    FAMG_REQUIRE(mem == AMG_MEM_HOST, AMG_ERR_INVALID, "bad amg_mem");
    amg_ctx *ac = ctx_of(o);
    const int64_t m = std::max<int64_t>(1, o.nrows), n = std::max<int64_t>(1, o.ncols);
    if (ac->stage_in.size() < (size_t)(n * k)) ac->stage_in.resize(n * k);
    if (ac->stage_out.size() < (size_t)(m * k)) ac->stage_out.resize(m * k);
    FAMG_CHECK_HIP(hipMemcpy2DAsync(ac->stage_in.get(), n * sizeof(double), rhs, ld_rhs * sizeof(double),
                                    o.ncols * sizeof(double), k, hipMemcpyHostToDevice, ctx.stream));
    spmm(c->m, ac->stage_in.get(), n, ac->stage_out.get(), m, k, ctx.stream);
    FAMG_CHECK_HIP(hipMemcpy2DAsync(out, ld_out * sizeof(double), ac->stage_out.get(), m * sizeof(double),
                                    o.nrows * sizeof(double), k, hipMemcpyDeviceToHost, ctx.stream));
    FAMG_CHECK_HIP(hipStreamSynchronize(ctx.stream));
    return true;
}

amg_status amg_linop_apply(amg_linop *op, double *out, int64_t ld_out, const double *rhs,
                           int64_t ld_rhs, int64_t k, amg_mem mem) {
    return guard([&] {
        LinOp &o = need(op);
        if (csr_multi_apply(o, out, ld_out, rhs, ld_rhs, k, mem)) return;
        for_columns(o, out, ld_out, rhs, ld_rhs, k, mem, o.nrows, o.ncols,
                    [&](double *y, const double *x) { o.apply(y, x); });
    });
}

amg_status amg_linop_transpose_apply(amg_linop *op, double *out, int64_t ld_out, const double *rhs,
                                     int64_t ld_rhs, int64_t k, amg_mem mem) {
    return guard([&] {
        LinOp &o = need(op);
        for_columns(o, out, ld_out, rhs, ld_rhs, k, mem, o.ncols, o.nrows,
                    [&](double *y, const double *x) { o.transpose_apply(y, x); });
    });
}

amg_status amg_precond_apply_in_place(amg_linop *op, double *rhs, int64_t ld, int64_t k, amg_mem mem) {
    return guard([&] {
        LinOp &o = need(op);
        FAMG_REQUIRE(o.nrows == o.ncols, AMG_ERR_DIM, "apply_in_place needs a square operator");
        if (mem == AMG_MEM_DEVICE) {
            o.ctx->set_device();
            FAMG_REQUIRE(k >= 0 && (k == 0 || rhs) && ld >= o.nrows, AMG_ERR_INVALID, "bad vector");
            for (int64_t c = 0; c < k; c++) o.apply_in_place(rhs + c * ld);
        } else {
            for_columns(o, rhs, ld, rhs, ld, k, mem, o.nrows, o.ncols,
                        [&](double *y, const double *x) { o.apply(y, x); });
        }
    });
}

amg_status amg_precond_transpose_apply_in_place(amg_linop *op, double *rhs, int64_t ld, int64_t k,
                                                amg_mem mem) {
    // every preconditioner of this library is symmetric (BiPrecond impls of the
    // reference forward transpose to apply: coarse_solvers.rs:266-276)
    return amg_precond_apply_in_place(op, rhs, ld, k, mem);
}

amg_status amg_linop_destroy(amg_linop *op) {
    return guard([&] {
        if (!op) return;
        if (op->op && op->op->ctx) op->op->ctx->set_device();
        delete op;
    });
}

// ------------------------------------------------------------- smoothers

amg_status amg_jacobi_create(const amg_linop *A, double omega, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *out = box(make_jacobi(*a, omega));
    });
}

amg_status amg_l1_create(const amg_linop *A, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *out = box(make_l1(*a));
    });
}

amg_status amg_l2_create(const amg_linop *A, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *out = box(make_l2(*a));
    });
}

amg_status amg_diag_create(amg_ctx *ctx, int64_t n, const double *d, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(ctx && out && (n == 0 || d) && n >= 0, AMG_ERR_INVALID, "bad argument");
        ctx->ctx.set_device();
        auto p = std::make_shared<DiagOp>();
        p->ctx = &ctx->ctx;
        p->nrows = p->ncols = n;
        p->d.resize(n);
        if (n) {
            FAMG_CHECK_HIP(hipMemcpyAsync(p->d.get(), d, n * sizeof(double), hipMemcpyHostToDevice, ctx->ctx.stream));
            FAMG_CHECK_HIP(hipStreamSynchronize(ctx->ctx.stream));
        }
        *out = box(p);
    });
}

amg_status amg_sgs_create(const amg_linop *A, const int32_t *colors, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *out = box(make_sgs(a, colors));
    });
}

amg_status amg_sgs_ncolors(const amg_linop *op, int64_t *ncolors) {
    return guard([&] {
        FAMG_REQUIRE(ncolors, AMG_ERR_INVALID, "null output");
        auto p = std::dynamic_pointer_cast<SgsOp>(need(op).shared_from_this());
        FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not an SGS smoother");
        *ncolors = p->ncolors;
    });
}

amg_status amg_sgs_info(const amg_linop *op, int64_t *info4) {
    return guard([&] {
        FAMG_REQUIRE(info4, AMG_ERR_INVALID, "null output");
        auto p = std::dynamic_pointer_cast<SgsOp>(need(op).shared_from_this());
        FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not an SGS smoother");
        const bool dia = p->Ap.has_dia() && p->Ap.dia_rowid;
        info4[0] = p->ncolors;
        info4[1] = dia ? SPMV_KERNEL_DIA : p->Ap.kernel;
        info4[2] = dia ? p->Ap.dia_k : 0;
        info4[3] = dia ? p->Ap.dia_vbits : 0;
    });
}

amg_status amg_coarse_chol_create(const amg_linop *A, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *out = box(make_coarse_chol(*a));
    });
}

// -------------------------------------------------------------- multigrid

amg_status amg_multigrid_create(amg_linop *op, amg_linop *smoother, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        LinOp &A = need(op);
        LinOp &S = need(smoother);
        FAMG_REQUIRE(A.nrows == A.ncols, AMG_ERR_DIM, "multigrid: op must be square");
        FAMG_REQUIRE(S.nrows == A.nrows && S.ncols == A.ncols, AMG_ERR_DIM, "multigrid: smoother size");
        auto mg = std::make_shared<MultigridOp>();
        mg->ctx = A.ctx;
        mg->nrows = mg->ncols = A.nrows;
        MgLevel L;
        L.A = op->op;
        L.S = smoother->op;
        mg->levels.push_back(std::move(L));
        *out = box(mg);
    });
}

amg_status amg_multigrid_add_level(amg_linop *mg, amg_linop *op, amg_linop *smoother, amg_linop *r,
                                   amg_linop *p) {
    return guard([&] {
        auto m = need_mg(mg);
        need(op); need(smoother); need(r); need(p);
        std::lock_guard<std::mutex> lk(m->mtx);
        m->add_level(op->op, smoother->op, r->op, p->op);
    });
}

amg_status amg_multigrid_set(amg_linop *mg, int64_t mu, int64_t steps) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(mu > 0 && steps > 0, AMG_ERR_INVALID, "mu and steps must be > 0");
        std::lock_guard<std::mutex> lk(m->mtx);
        m->mu = mu;
        m->steps = steps;
        m->invalidate_graphs();
    });
}

amg_status amg_multigrid_levels(const amg_linop *mg, int64_t *levels) {
    return guard([&] {
        FAMG_REQUIRE(levels, AMG_ERR_INVALID, "null output");
        *levels = (int64_t)need_mg(mg)->levels.size();
    });
}

amg_status amg_multigrid_set_graph(amg_linop *mg, int32_t enable) {
    return guard([&] {
        auto m = need_mg(mg);
        std::lock_guard<std::mutex> lk(m->mtx);
        m->use_graph = enable != 0;
        m->invalidate_graphs();
    });
}

amg_status amg_multigrid_set_option(amg_linop *mg, int32_t option, int64_t value) {
    return guard([&] {
        auto m = need_mg(mg);
        std::lock_guard<std::mutex> lk(m->mtx);
        switch (option) {
        case 0: m->use_graph = value != 0; break;
        case 1: m->sgs_residual_form = value != 0; break;
        case 2: m->fold_zero_guess = value != 0; break;
        case 3: FAMG_REQUIRE(value == 0, AMG_ERR_UNSUPPORTED, "fused grid transfers were removed (DESIGN.md 3)"); break;
        case 4: m->restrict_df = value != 0; break;
        case 5:
            FAMG_REQUIRE(value >= 0 && value <= 2, AMG_ERR_INVALID, "reorder: 0, 1 or 2");
            if (m->reorder == (int)value) return;  // unchanged: keep the copies and the graphs
            m->undo_reorder();
            m->reorder = (int)value;
            break;
        default: fail(AMG_ERR_INVALID, "unknown multigrid option");
        }
        m->invalidate_graphs();
    });
}

amg_status amg_multigrid_apply(amg_linop *mg, double *out, int64_t ld_out, const double *rhs,
                               int64_t ld_rhs, int64_t k, amg_mem mem) {
    return guard([&] {
        auto m = need_mg(mg);
        for_columns(*m, out, ld_out, rhs, ld_rhs, k, mem, m->nrows, m->ncols,
                    [&](double *y, const double *x) { m->apply(y, x); });
    });
}

amg_status amg_multigrid_cycle_plan(amg_linop *mg, amg_launch_rec *recs, int64_t cap, int64_t *count) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(count && cap >= 0, AMG_ERR_INVALID, "bad argument");
        m->ctx->set_device();
        export_plan(m->cycle_plan(), recs, cap, count);
    });
}

amg_status amg_multigrid_fine_launch(amg_linop *mg, int32_t which, double *out, const double *rhs) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE((which == 0 || which == 1) && rhs && (out || which == 0), AMG_ERR_INVALID, "bad argument");
        m->ctx->set_device();
        FAMG_REQUIRE(m->fine_launch(which, out, rhs), AMG_ERR_UNSUPPORTED,
                     "the cycle takes no fused fine-level launch of this kind");
    });
}

amg_status amg_multigrid_set_fine_timer(amg_linop *mg, int32_t which) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(which >= -1 && which <= 1, AMG_ERR_INVALID, "bad argument");
        std::lock_guard<std::mutex> lk(m->mtx);
        m->ctx->set_device();
        for (auto &e : m->fine_ev)
            if (!e) FAMG_CHECK_HIP(hipEventCreate(&e));
        m->fine_timer = which;
        m->invalidate_graphs();
    });
}

amg_status amg_multigrid_fine_timer_ms(amg_linop *mg, float *ms) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(ms && m->fine_timer >= 0, AMG_ERR_INVALID, "no fine-level timer set");
        FAMG_CHECK_HIP(hipEventSynchronize(m->fine_ev[1]));
        FAMG_CHECK_HIP(hipEventElapsedTime(ms, m->fine_ev[0], m->fine_ev[1]));
    });
}

amg_status amg_trace_mark(amg_ctx *ctx, int32_t tag) {
    return guard([&] {
        FAMG_REQUIRE(ctx, AMG_ERR_INVALID, "null context");
        ctx->ctx.set_device();
        trace_mark(ctx->ctx, tag);
    });
}

amg_status amg_multigrid_get_level(const amg_linop *mg, int64_t level, amg_linop **A, amg_linop **S,
                                   amg_linop **R, amg_linop **P) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(level >= 0 && level < (int64_t)m->levels.size(), AMG_ERR_INVALID, "level out of range");
        const MgLevel &L = m->levels[level];  // the caller's operators (not a renumbered copy)
        if (A) *A = box(L.origA());
        if (S) *S = box(L.origS());
        if (R) *R = L.origR() ? box(L.origR()) : nullptr;
        if (P) *P = L.origP() ? box(L.origP()) : nullptr;
    });
}

amg_status amg_multigrid_get_run_level(amg_linop *mg, int64_t level, amg_linop **A, amg_linop **S, amg_linop **R,
                                       amg_linop **P) {
    return guard([&] {
        auto m = need_mg(mg);
        std::lock_guard<std::mutex> lk(m->mtx);
        FAMG_REQUIRE(level >= 0 && level < (int64_t)m->levels.size(), AMG_ERR_INVALID, "level out of range");
        m->ensure_workspace();  // the renumbering is decided with the workspaces
        const MgLevel &L = m->levels[level];
        if (A) *A = box(L.A);
        if (S) *S = box(L.S);
        if (R) *R = L.R ? box(L.R) : nullptr;
        if (P) *P = L.P ? box(L.P) : nullptr;
    });
}

amg_status amg_multigrid_level_reordered(amg_linop *mg, int64_t level, int32_t *reordered) {
    return guard([&] {
        auto m = need_mg(mg);
        FAMG_REQUIRE(reordered, AMG_ERR_INVALID, "null output");
        std::lock_guard<std::mutex> lk(m->mtx);
        FAMG_REQUIRE(level >= 0 && level < (int64_t)m->levels.size(), AMG_ERR_INVALID, "level out of range");
        m->ensure_workspace();  // the renumbering is decided with the workspaces
        *reordered = m->levels[level].permuted ? 1 : 0;
    });
}

// ------------------------------------------------------------------ setup

amg_status amg_spgemm(const amg_linop *A, const amg_linop *B, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A), b = need_csr(B);
        FAMG_REQUIRE(a->ctx == b->ctx, AMG_ERR_INVALID, "operands on different contexts");
        a->ctx->set_device();
        *out = box(spgemm_op(*a, *b));
    });
}

amg_status amg_transpose(const amg_linop *P, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto p = need_csr(P);
        p->ctx->set_device();
        *out = box(transpose_op(*p));
    });
}

amg_status amg_galerkin_rap(const amg_linop *R, const amg_linop *A, const amg_linop *P, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto r = need_csr(R), a = need_csr(A), p = need_csr(P);
        a->ctx->set_device();
        *out = box(galerkin_rap(*r, *a, *p));
    });
}

amg_status amg_smooth_interpolation(const amg_linop *A, const amg_linop *P, double omega, amg_linop **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A), p = need_csr(P);
        a->ctx->set_device();
        *out = box(smooth_interpolation(*a, *p, omega));
    });
}

amg_status amg_sa_tentative(amg_ctx *ctx, int64_t n, const int64_t *agg_of, int64_t naggs,
                            const double *near_null, amg_linop **P, double *coarse_nn) {
    return guard([&] {
        FAMG_REQUIRE(ctx && P && coarse_nn && (n == 0 || (agg_of && near_null)), AMG_ERR_INVALID, "null argument");
        FAMG_REQUIRE(n >= 0 && naggs > 0, AMG_ERR_INVALID, "bad sizes");
        ctx->ctx.set_device();
        *P = box(sa_tentative(&ctx->ctx, n, agg_of, naggs, near_null, coarse_nn));
    });
}

amg_status amg_nn_stationary_l1(const amg_linop *A, int64_t iters, double *x) {
    return guard([&] {
        auto a = need_csr(A);
        FAMG_REQUIRE(x && iters >= 1, AMG_ERR_INVALID, "bad argument");
        a->ctx->set_device();
        nn_stationary_l1(*a, iters, x);
    });
}

amg_status amg_sa_build_box(amg_linop *A, int64_t nx, int64_t ny, int64_t nz, int64_t bx, int64_t by,
                            int64_t bz, int64_t coarsest_dim, int64_t max_levels, double omega,
                            int32_t smoother, amg_linop **mg_out) {
    return guard([&] {
        FAMG_REQUIRE(mg_out, AMG_ERR_INVALID, "null output");
        auto a = need_csr(A);
        a->ctx->set_device();
        *mg_out = box(sa_build_box(a, nx, ny, nz, bx, by, bz, coarsest_dim, max_levels, omega, smoother));
    });
}

// ------------------------------------------------------------ solve drivers

}  // extern "C"
