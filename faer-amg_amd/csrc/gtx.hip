// gtx.hip -- wide grid-transfer classes: SpMV storage for R and P of every level
// of a 2 x 2 x 2-box hierarchy, the generalisation of gtc.hip.
//
// gtc.hip stores P_0 / R_0 of the 256^3 cycle as 8-bit class ids into an LDS
// dictionary of (value index, step slot) pairs: at most 256 classes, 256
// distinct values, steps {-1,0,1}^3 (P) / {-1,..,2}^3 (R).  The transfer
// operators of the Galerkin levels do not fit: smoothing the tentative P with a
// radius-2 A_1 gives P_1 rows at coarse steps {-1,0,1}^3 but in 5832 classes
// (parity x boundary distance) with ~2000 distinct values, and R_1 rows of 88
// entries at fine steps {-2,..,3}^3 (profiles/r04: levels 1-3 grow to steps
// {-5,..,6}^3 and 35428 values).  Here:
//   * one 16-bit class id per row (2 B / row instead of 10-16 B of value-code
//     SELL), the dictionary in global memory (L2-resident: <= 1 MB);
//   * a dictionary entry is (int32 window offset, fp64 value): the offset is
//     precomputed for the kernel's window at setup, so a term is one LDS read
//     at row base + offset -- no slot -> lookup -> window chain;
//   * waves cover points of one parity class (P: a wave holds x = px + 2i,
//     y = py + 2j of one plane), so every interior wave is class-uniform and
//     reads its dictionary entries through scalar loads (the offset and value
//     broadcast from SGPRs); boundary waves read them per lane;
//   * R's epilogue can also write the next level's first Jacobi step from zero
//     (y2 = d * y, SPMV_SETDF), which removes that level's d*f pass.
// Row sums walk the stored entries in ascending column order with fma:
// bitwise the oracle's CSR sums (and gtc's).  Rank-local matrices of a
// distributed level use the same slab frames / z-tile segments as gtc.
#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "famg.hpp"

namespace famg {

struct GtxArgs;
// class peeling on mixed waves (scalar walks per distinct class) measured far slower than per-lane
// dictionary loads: a boundary wave of the small Galerkin levels holds dozens of classes
__device__ __forceinline__ constexpr bool gtx_peel() { return false; }

struct GtxArgs {
    const uint16_t *cls;    // class id per row
    const int32_t *dptr;    // per class: first dictionary entry
    const int32_t *dlen;    // per class: entries (a multiple of 4)
    const int32_t *doff;    // per entry: window offset from the row's base (32-bit: scalar loads)
    const double *dval;     // per entry: value
    int rx, ry, rz;         // row grid (rz: owned row planes)
    int kx, ky, kz;         // column grid (kz: owned column planes)
    int tx, ty, tz;         // tile (rows)
    int wx, wy, wz;         // window (columns)
    int lox, loy, loz;      // the lowest step per axis
    int ntx, nty, tile0;
    int kz_lo, kz_hi, rz0, kz0;  // as GtcArgs (slab frames; single GPU 0, kz, 0, 0)
    int64_t add_lo, add_hi;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
    int dconst;
    double dk;
    double *y2;  // SETDF: y2 = d * y
    float rwx, rwy, rtx, rty;  // 1 / wx, wy, tx, ty for fdiv_rcp (host-checked exact)
};

// stage the column window [w0, w0 + w) into LDS (0.0 outside the grid / the
// loadable planes): every load of a lane issued before its stores -- PF is
// chosen per matrix so one round covers the window (a round per memory latency
// is what the staging costs; the gtc kernels' compile-time windows do the same)
template <int PF>
__device__ __forceinline__ void gtx_stage(const GtxArgs &a, double *win, int wx0, int wy0, int wz0) {
    const int W = a.wx * a.wy * a.wz;
    const int64_t cplane = (int64_t)a.kx * a.ky;
    for (int q0 = threadIdx.x; q0 < W; q0 += 256 * PF) {
        double v[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int q = q0 + 256 * u;
            const int q1 = fdiv_rcp(q, a.rwx), q2 = fdiv_rcp(q1, a.rwy);
            const int X = wx0 + q - q1 * a.wx, Y = wy0 + q1 - q2 * a.wy, Z = wz0 + q2;
            const bool in = q < W && (unsigned)X < (unsigned)a.kx && (unsigned)Y < (unsigned)a.ky && Z >= a.kz_lo &&
                            Z < a.kz_hi;
            const int64_t zb = (int64_t)Z * cplane + (Z < 0 ? a.add_lo : Z >= a.kz ? a.add_hi : 0);
            v[u] = in ? a.x[zb + (int64_t)Y * a.kx + X] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < PF; u++)
            if (q0 + 256 * u < W) win[q0 + 256 * u] = v[u];
    }
}

// Row sums over a class's entries in stored order (fma, ascending columns).
// gtx_rows_u: NB rows of one wave-uniform class cu -- each entry (offset, value)
// is one scalar load shared by the NB rows, which run NB independent fma chains.
// gtx_row_v: one row of a per-lane class (vector loads; boundary waves).
template <int NB>
__device__ __forceinline__ void gtx_rows_u(const GtxArgs &a, const double *win, const int *base, int cu,
                                           double *acc) {
    const int e0 = a.dptr[cu], n = a.dlen[cu];
#pragma unroll
    for (int r = 0; r < NB; r++) acc[r] = 0.0;
    for (int k = 0; k < n; k += 4) {
        int o[4];
        double v[4], w[NB][4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            o[u] = a.doff[e0 + k + u];
            v[u] = a.dval[e0 + k + u];
        }
#pragma unroll
        for (int r = 0; r < NB; r++)
#pragma unroll
            for (int u = 0; u < 4; u++) w[r][u] = win[base[r] + o[u]];
#pragma unroll
        for (int r = 0; r < NB; r++)
#pragma unroll
            for (int u = 0; u < 4; u++) acc[r] = fma(v[u], w[r][u], acc[r]);
    }
}

// A row of a wave whose rows mix classes (boundary tiles): the wave peels
// its classes one at a time -- the first pending lane's class cu is walked
// with scalar dictionary loads by every lane of that class -- so boundary waves
// also read the dictionary from SGPRs, once per distinct class.
__device__ __forceinline__ double gtx_row_peel(const GtxArgs &a, const double *win, int base, int c, bool live) {
    double acc = 0.0;
    bool pending = live;
    while (__any(pending)) {
        if (pending) {
            const int cu = __builtin_amdgcn_readfirstlane(c);
            if (c == cu) {
                double r[1];
                const int b[1] = {base};
                gtx_rows_u<1>(a, win, b, cu, r);
                acc = r[0];
                pending = false;
            }
        }
    }
    return acc;
}

__device__ __forceinline__ double gtx_row_v(const GtxArgs &a, const double *win, int base, int e0, int n) {
    double acc = 0.0;
    for (int k = 0; k < n; k += 4) {
        int o[4];
        double v[4], w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            o[u] = a.doff[e0 + k + u];
            v[u] = a.dval[e0 + k + u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) w[u] = win[base + o[u]];
#pragma unroll
        for (int u = 0; u < 4; u++) acc = fma(v[u], w[u], acc);
    }
    return acc;
}

// P v_c over a fine tile of 32 x 8 x TZ points.  Wave wv holds x parity wv & 1,
// y parity wv >> 1: lane l is the point (px + 2 (l & 15), py + 2 (l >> 4)),
// and each lane walks TZ planes -- every wave of an interior tile is one class
// per plane.
template <int MODE, int TZ, int PF>
__global__ __launch_bounds__(256) void k_gtx_interp(GtxArgs a) {
    extern __shared__ double win[];
    __shared__ double sdt[256];
    const int tid = threadIdx.x;
    const int t = a.tile0 + xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int x0 = tix * 32, y0 = tiy * 8, z0 = tiz * TZ;
    const int wv = tid >> 6, l = tid & 63;
    const int lx = (wv & 1) + 2 * (l & 15), ly = (wv >> 1) + 2 * (l >> 4);
    const int gx = x0 + lx, gy = y0 + ly;
    const int az0 = ((a.rz0 + z0) >> 1) - a.kz0;  // local coarse plane of the tile's first anchor (rz0 even)
    const int64_t fplane = (int64_t)a.rx * a.ry;
    int cl[TZ], dci[TZ];
    double yb[TZ];
    bool live[TZ];
    if constexpr (MODE == SPMV_ADD0)
        if (a.dc && !a.dconst) sdt[tid] = a.dt[tid];
#pragma unroll
    for (int j = 0; j < TZ; j++) {
        const int gz = z0 + j;
        live[j] = gx < a.rx && gy < a.ry && gz < a.rz;
        const int64_t i = live[j] ? (int64_t)gz * fplane + (int64_t)gy * a.rx + gx : 0;
        cl[j] = live[j] ? (int)a.cls[i] : -1;
        yb[j] = 0.0;
        dci[j] = 0;
        if (live[j]) {
            if constexpr (MODE == SPMV_ADD) yb[j] = a.y[i];
            if constexpr (MODE == SPMV_ADD0) {
                yb[j] = a.b[i];
                if (a.dconst) yb[j] = a.dk * yb[j];  // d*b (vec_mul's product)
                else if (a.dc) dci[j] = a.dc[i];
                else yb[j] = a.d[i] * yb[j];
            }
        }
    }
    // per-lane dictionary ranges (boundary waves), loaded under the staging
    int e0[TZ], en[TZ];
#pragma unroll
    for (int j = 0; j < TZ; j++) {
        e0[j] = live[j] ? a.dptr[cl[j]] : 0;
        en[j] = live[j] ? a.dlen[cl[j]] : 0;
    }
    gtx_stage<PF>(a, win, (x0 >> 1) + a.lox, (y0 >> 1) + a.loy, az0 + a.loz);
    __syncthreads();
    int base[TZ];
#pragma unroll
    for (int j = 0; j < TZ; j++) base[j] = ((j >> 1) * a.wy + (ly >> 1)) * a.wx + (lx >> 1);
    double acc[TZ];
    // planes j and j + 2 share their z parity, hence (inside the grid) their class
#pragma unroll
    for (int j0 = 0; j0 < (TZ == 4 ? 2 : TZ); j0++) {
        constexpr int NB = TZ == 4 ? 2 : 1;
        const int cu = __builtin_amdgcn_readfirstlane(cl[j0]);
        bool uni = cu >= 0;
#pragma unroll
        for (int r = 0; r < NB; r++) uni = uni && __all(cl[j0 + 2 * r] == cu);
        if (uni) {
            int bs[NB];
            double ac[NB];
#pragma unroll
            for (int r = 0; r < NB; r++) bs[r] = base[j0 + 2 * r];
            gtx_rows_u<NB>(a, win, bs, cu, ac);
#pragma unroll
            for (int r = 0; r < NB; r++) acc[j0 + 2 * r] = ac[r];
        } else {
#pragma unroll
            for (int r = 0; r < NB; r++) {
                const int j = j0 + 2 * r;
                acc[j] = gtx_peel() ? gtx_row_peel(a, win, base[j], cl[j], live[j])
                                    : (live[j] ? gtx_row_v(a, win, base[j], e0[j], en[j]) : 0.0);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TZ; j++) {
        if (!live[j]) continue;
        if constexpr (MODE == SPMV_ADD0)
            if (a.dc && !a.dconst) yb[j] = sdt[dci[j]] * yb[j];
        const int64_t i = (int64_t)(z0 + j) * fplane + (int64_t)gy * a.rx + gx;
        if constexpr (MODE == SPMV_SET) a.y[i] = acc[j];
        else a.y[i] = yb[j] + acc[j];  // ADD, ADD0
    }
}

// R r over a coarse tile of tx x ty x tz rows (RL rows per lane); SETDF also
// writes y2 = d * y (the next level's first Jacobi step from zero).
template <int MODE, int RL, int PF>
__global__ __launch_bounds__(256) void k_gtx_restrict(GtxArgs a) {
    extern __shared__ double win[];
    __shared__ double sdt[256];
    const int tid = threadIdx.x;
    const int t = a.tile0 + xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int X0 = tix * a.tx, Y0 = tiy * a.ty, Z0 = tiz * a.tz;
    const int T = a.tx * a.ty * a.tz;
    const int64_t cplane = (int64_t)a.rx * a.ry;
    if constexpr (MODE == SPMV_SETDF)
        if (a.dc && !a.dconst) sdt[tid] = a.dt[tid];
    int cl[RL], base[RL];
    int64_t J[RL];
    bool live[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) {
        const int lt = tid + 256 * j;
        const int lq = fdiv_rcp(lt, a.rtx), lz = fdiv_rcp(lq, a.rty);
        const int lx = lt - lq * a.tx, ly = lq - lz * a.ty;
        const int X = X0 + lx, Y = Y0 + ly, Z = Z0 + lz;
        live[j] = lt < T && X < a.rx && Y < a.ry && Z < a.rz;
        J[j] = live[j] ? (int64_t)Z * cplane + (int64_t)Y * a.rx + X : 0;
        cl[j] = live[j] ? (int)a.cls[J[j]] : -1;
        base[j] = ((2 * lz) * a.wy + 2 * ly) * a.wx + 2 * lx;
    }
    int e0[RL], en[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) {
        e0[j] = live[j] ? a.dptr[cl[j]] : 0;
        en[j] = live[j] ? a.dlen[cl[j]] : 0;
    }
    gtx_stage<PF>(a, win, 2 * X0 + a.lox, 2 * Y0 + a.loy, 2 * (a.rz0 + Z0) - a.kz0 + a.loz);
    __syncthreads();
    double acc[RL];
    const int cu = __builtin_amdgcn_readfirstlane(cl[0]);
    bool uni = cu >= 0;
#pragma unroll
    for (int j = 0; j < RL; j++) uni = uni && __all(cl[j] == cu);
    if (uni) {  // interior waves: one class for all their rows
        gtx_rows_u<RL>(a, win, base, cu, acc);
    } else {
#pragma unroll
        for (int j = 0; j < RL; j++)
            acc[j] = gtx_peel() ? gtx_row_peel(a, win, base[j], cl[j], live[j])
                                : (live[j] ? gtx_row_v(a, win, base[j], e0[j], en[j]) : 0.0);
    }
#pragma unroll
    for (int j = 0; j < RL; j++) {
        if (!live[j]) continue;
        a.y[J[j]] = acc[j];
        if constexpr (MODE == SPMV_SETDF) {
            const double dd = a.dconst ? a.dk : a.dc ? sdt[a.dc[J[j]]] : a.d[J[j]];
            a.y2[J[j]] = dd * acc[j];  // vec_mul(_coded)'s product
        }
    }
}

// ------------------------------------------------------------ build / dispatch

void gtx_release(GpuCsr &m) {
    m.gtx_cls.release();
    m.gtx_dptr.release();
    m.gtx_dlen.release();
    m.gtx_doff.release();
    m.gtx_dval.release();
    m.gtx_on = m.gtx_r = false;
    m.gtx_nclass = m.gtx_nent = 0;
}

// FAMG_GTX: 0 off; 1 (default) levels whose R/P the 8-bit grid-transfer classes
// (gtc.hip) cannot take; 2 every box level (A/B against gtc on level 0)
int gtx_mode() {
    static const int v = [] {
        const char *e = getenv("FAMG_GTX");
        return e ? atoi(e) : 1;
    }();
    return v;
}

// flag FLAG_GTX_TIME (FAMG_GTX_TIME, amg_set_flag(3, v)): 0 = keep the classes
// wherever they build; 1 = time them against the storage underneath; 2 (default)
// = keep them on transfer operators of >= 2^18 rows (P: fine rows, R: coarse
// rows), the levels where the timing chose them on the 256^3 cycles (P_1, R_1,
// P_2) -- deterministic, so two builds of one hierarchy take the same storages
// (the timing could flip on noise between a 2-lane pattern SELL and the classes,
// whose row sums differ in rounding)
static bool gtx_beats_storage(GpuCsr &m) {
    const int64_t how = flag(FLAG_GTX_TIME);
    if (how == 0 || gtx_mode() == 2) return true;
    // a rank-local matrix of a distributed level (rframe on) is sized by its global
    // operator's rows, so every rank keeps the storage -- and the rounding -- of
    // the single-GPU cycle
    const int64_t rows = m.rframe.on() ? m.rframe.nx * m.rframe.ny * m.rframe.gz : m.nrows;
    if (how != 1) return rows >= (int64_t(1) << 18);
    // R of the small levels (<= 65536 coarse rows of hundreds of entries) loses in the cycle
    // even where an isolated timing has it ahead (R_2 of the 256^3 cycle: 32.5 vs 21.9 + 4.6 us)
    if (m.gtx_r && m.nrows <= 65536) return false;
    hipStream_t s = m.ctx->stream;
    DevBuf<double> x(m.ncols), y(m.nrows), y2(m.nrows);
    FAMG_CHECK_HIP(hipMemsetAsync(x.get(), 0, m.ncols * sizeof(double), s));
    FAMG_CHECK_HIP(hipMemsetAsync(y.get(), 0, m.nrows * sizeof(double), s));
    hipEvent_t e0, e1;
    FAMG_CHECK_HIP(hipEventCreate(&e0));
    FAMG_CHECK_HIP(hipEventCreate(&e1));
    float ms[2] = {0.f, 0.f};
    for (int k = 0; k < 2; k++) {
        m.gtx_on = k == 1;
        auto run = [&] {
            spmv(m, x.get(), y.get(), SPMV_SET, SpmvEpi{}, s);
            if (m.gtx_r && k == 0) vec_mul(y2.get(), y.get(), y.get(), m.nrows, s);  // the d*f pass SETDF saves
        };
        run();
        FAMG_CHECK_HIP(hipEventRecord(e0, s));
        for (int r = 0; r < 5; r++) run();
        FAMG_CHECK_HIP(hipEventRecord(e1, s));
        FAMG_CHECK_HIP(hipEventSynchronize(e1));
        FAMG_CHECK_HIP(hipEventElapsedTime(&ms[k], e0, e1));
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    m.gtx_on = true;
    return ms[1] < 0.9f * ms[0];  // a clear win only (launch-bound small levels time noisily)
}

bool gtx_attach(GpuCsr &m, const int64_t *fg, const int64_t *cg, int which) {
    gtx_release(m);
    m.gtx_tried = true;
    if (gtx_mode() == 0 || m.nnz >= (int64_t(1) << 31) || m.nrows <= 0 || m.nnz <= 0) return false;
    const bool is_r = which < 0 ? m.nrows < m.ncols : which == 1;
    const int64_t rx = is_r ? cg[0] : fg[0], ry = is_r ? cg[1] : fg[1], rz = is_r ? cg[2] : fg[2];  // row grid
    const int64_t kx = is_r ? fg[0] : cg[0], ky = is_r ? fg[1] : cg[1], kz = is_r ? fg[2] : cg[2];  // column grid
    if (cg[0] != (fg[0] + 1) / 2 || cg[1] != (fg[1] + 1) / 2 || cg[2] != (fg[2] + 1) / 2) return false;
    if (rx >= 32768 || ry >= 32768 || kx >= 32768 || ky >= 32768) return false;
    const SlabFrame &RF = m.rframe, &CF = m.cframe;
    if (RF.on() != CF.on()) return false;
    const int64_t n = m.nrows, nnz = m.nnz;
    if (RF.on()) {
        if (RF.nx != rx || RF.ny != ry || RF.gz != rz || CF.nx != kx || CF.ny != ky || CF.gz != kz) return false;
        if (RF.n_own() != n || CF.n_own() + (CF.gl + CF.gh) * CF.pl() != m.ncols) return false;
        if (!is_r && (RF.z0 & 1)) return false;  // P tiles: four fine planes on two coarse planes
    } else if (rx * ry * rz != n || kx * ky * kz != m.ncols) {
        return false;
    }
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    hipStream_t s = m.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(rp.data(), m.rp64.get(), (n + 1) * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), m.col.get(), nnz * 4, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), m.val.get(), nnz * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    // steps (dx, dy, dz) of every entry from its row's anchor (global coordinates)
    std::vector<int8_t> st(3 * nnz);
    bool ok = true;
    int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
#pragma omp parallel
    {
        int llo[3] = {127, 127, 127}, lhi[3] = {-128, -128, -128};
        bool lok = true;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; i++) {
            const int64_t x = i % rx, y = (i / rx) % ry, z = i / (rx * ry) + (RF.on() ? RF.z0 : 0);
            const int64_t ax = is_r ? 2 * x : x / 2, ay = is_r ? 2 * y : y / 2, az = is_r ? 2 * z : z / 2;
            int64_t prev = -1;
            for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
                const int64_t j = col[e];
                const int64_t jp = CF.on() ? CF.in_plane(j) : j % (kx * ky);
                const int64_t jz = CF.on() ? CF.plane_of(j) : j / (kx * ky);
                const int64_t d[3] = {jp % kx - ax, jp / kx - ay, jz - az};
                for (int q = 0; q < 3; q++) {
                    if (d[q] < -8 || d[q] > 8) lok = false;
                    llo[q] = std::min<int>(llo[q], (int)d[q]);
                    lhi[q] = std::max<int>(lhi[q], (int)d[q]);
                    st[3 * e + q] = (int8_t)std::max<int64_t>(-8, std::min<int64_t>(8, d[q]));
                }
                // ascending columns = ascending (dz, dy, dx) (the stored order is the sum order)
                const int64_t key = ((d[2] + 8) * 17 + d[1] + 8) * 17 + d[0] + 8;
                if (key <= prev) lok = false;
                prev = key;
            }
        }
#pragma omp critical
        {
            ok = ok && lok;
            for (int q = 0; q < 3; q++) {
                lo[q] = std::min(lo[q], llo[q]);
                hi[q] = std::max(hi[q], lhi[q]);
            }
        }
    }
    if (!ok) return false;
    // tile and window: P 32 x 8 x TZ fine points, R the largest of a few coarse
    // tiles whose fine window fits 64 KB of LDS
    int tile[3] = {0, 0, 0}, wdim[3] = {0, 0, 0};
    if (!is_r) {
        // four fine planes per lane, or two where that leaves fewer than 1024 tiles
        // (P_2 of the 256^3 cycle: 256 workgroups of 4 planes cover the chip once and
        // leave its cold misses exposed; FAMG_GTX_PTZ=4 / 2 forces)
        static const int ptz = [] {
            const char *e = getenv("FAMG_GTX_PTZ");
            return e ? atoi(e) : 0;
        }();
        const int64_t tiles4 = ((rx + 31) / 32) * ((ry + 7) / 8) * ((n / (rx * ry) + 3) / 4);
        const int first = ptz == 2 || (ptz == 0 && tiles4 < 1024) ? 2 : 4;
        for (int tzc : {first, 2}) {
            const int w0 = 16 + hi[0] - lo[0], w1 = 4 + hi[1] - lo[1], w2 = tzc / 2 + hi[2] - lo[2];
            if ((int64_t)w0 * w1 * w2 * 8 <= 64 * 1024) {
                tile[0] = 32; tile[1] = 8; tile[2] = tzc;
                wdim[0] = w0; wdim[1] = w1; wdim[2] = w2;
                break;
            }
        }
    } else {
        static const int cands[][3] = {{16, 8, 4}, {16, 4, 4}, {16, 8, 2}, {16, 8, 1}, {16, 4, 1},
                                       {8, 4, 1},  {8, 2, 1},  {4, 2, 1}};
        for (const auto &c : cands) {
            const int w0 = 2 * c[0] - 1 + hi[0] - lo[0], w1 = 2 * c[1] - 1 + hi[1] - lo[1],
                      w2 = 2 * c[2] - 1 + hi[2] - lo[2];
            if ((int64_t)w0 * w1 * w2 * 8 <= 64 * 1024) {
                for (int q = 0; q < 3; q++) tile[q] = c[q];
                wdim[0] = w0; wdim[1] = w1; wdim[2] = w2;
                break;
            }
        }
    }
    if (!tile[0] || (int64_t)wdim[0] * wdim[1] * wdim[2] > 65535) return false;
    // classes: rows with equal (steps, value bits) lists
    std::vector<uint64_t> h(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        uint64_t hh = 0x9E3779B97F4A7C15ull ^ (uint64_t)(rp[i + 1] - rp[i]);
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            uint64_t bits;
            std::memcpy(&bits, &val[e], 8);
            const uint64_t sk = (uint64_t)(uint8_t)st[3 * e] | (uint64_t)(uint8_t)st[3 * e + 1] << 8 |
                                (uint64_t)(uint8_t)st[3 * e + 2] << 16;
            hh = (hh ^ sk) * 0x100000001B3ull;
            hh = (hh ^ bits) * 0xFF51AFD7ED558CCDull;
            hh ^= hh >> 29;
        }
        h[i] = hh;
    }
    auto same = [&](int64_t i, int64_t j) {
        if (rp[i + 1] - rp[i] != rp[j + 1] - rp[j]) return false;
        for (int64_t p = rp[i], q = rp[j]; p < rp[i + 1]; p++, q++)
            if (st[3 * p] != st[3 * q] || st[3 * p + 1] != st[3 * q + 1] || st[3 * p + 2] != st[3 * q + 2] ||
                std::memcmp(&val[p], &val[q], 8) != 0)
                return false;
        return true;
    };
    std::unordered_map<uint64_t, std::vector<int>> by_hash;
    std::vector<int64_t> rep;
    std::vector<uint16_t> cls(n);
    int64_t last_i = -1;
    int last_c = -1;
    for (int64_t i = 0; i < n; i++) {
        int c = -1;
        if (last_c >= 0 && h[i] == h[last_i] && same(last_i, i)) c = last_c;
        if (c < 0) {
            auto &cands = by_hash[h[i]];
            for (int q : cands)
                if (same(rep[q], i)) { c = q; break; }
            if (c < 0) {
                c = (int)rep.size();
                if (c >= 65536) return false;
                rep.push_back(i);
                cands.push_back(c);
            }
        }
        cls[i] = (uint16_t)c;
        last_i = i;
        last_c = c;
    }
    // dictionary: per class its entries (window offset from the row's base, value), padded to
    // a multiple of 4 with +0.0 at offset 0 (a +0.0 term leaves the sum unchanged)
    const int64_t C = (int64_t)rep.size();
    std::vector<int32_t> dptr(C), dlen(C);
    std::vector<int32_t> doff;
    std::vector<double> dval;
    for (int64_t c = 0; c < C; c++) {
        const int64_t i = rep[c];
        dptr[c] = (int32_t)doff.size();
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int off = ((st[3 * e + 2] - lo[2]) * wdim[1] + (st[3 * e + 1] - lo[1])) * wdim[0] + (st[3 * e] - lo[0]);
            doff.push_back(off);
            dval.push_back(val[e]);
        }
        while ((doff.size() - dptr[c]) % 4) {
            doff.push_back(0);
            dval.push_back(0.0);
        }
        dlen[c] = (int32_t)(doff.size() - dptr[c]);
        if (doff.size() >= (size_t)INT32_MAX / 2) return false;
    }
    m.gtx_cls.resize(n);
    m.gtx_dptr.resize(C);
    m.gtx_dlen.resize(C);
    m.gtx_doff.resize(doff.size() + 4);
    m.gtx_dval.resize(dval.size() + 4);
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtx_cls.get(), cls.data(), n * 2, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtx_dptr.get(), dptr.data(), C * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtx_dlen.get(), dlen.data(), C * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtx_doff.get(), doff.data(), doff.size() * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtx_dval.get(), dval.data(), dval.size() * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.gtx_nclass = C;
    m.gtx_nent = (int64_t)doff.size();
    for (int q = 0; q < 3; q++) {
        m.gtx_tile[q] = tile[q];
        m.gtx_win[q] = wdim[q];
        m.gtx_lo[q] = lo[q];
        m.gtx_fg[q] = fg[q];
        m.gtx_cg[q] = cg[q];
    }
    m.gtx_r = is_r;
    {  // the staging loops' float-reciprocal divisions, checked once at build
        const int wx = wdim[0], wy = wdim[1], wz = wdim[2], tx = std::max(tile[0], 1), ty = std::max(tile[1], 1);
        m.gtx_fdiv = fdiv_exact(wx * wy * wz + 256 * 8, wx, 1.0f / (float)wx) &&
                     fdiv_exact((wx * wy * wz + 256 * 8) / wx + 1, wy, 1.0f / (float)wy) &&
                     fdiv_exact(1024, tx, 1.0f / (float)tx) && fdiv_exact(1024 / tx + 1, ty, 1.0f / (float)ty);
    }
    m.gtx_on = true;
    // keep the classes only where they beat the storage underneath (timed on
    // scratch vectors; R is charged with the d*f pass its SETDF epilogue saves):
    // the small Galerkin levels' long rows (R_3: ~490 entries, P_4 from a 16^3
    // grid: 8 tiles) run a lane per row and lose to the lanes-per-row kernels
    if (!gtx_beats_storage(m)) {
        gtx_release(m);
        return false;
    }
    return true;
}

bool gtx_supports(const GpuCsr &m, SpmvMode mode) {
    return m.gtx_r ? (mode == SPMV_SET || mode == SPMV_SETDF)
                   : (mode == SPMV_SET || mode == SPMV_ADD || mode == SPMV_ADD0);
}

// the z-tile range of a launch (as spmv_gtc): all, or (rank-local) 1 = tiles whose
// window reads no ghost plane, 0 / 2 = those before / after
template <typename F>
static void gtx_tiles(int ntz, int64_t seg, int wz, int kz, int kz_lo, int kz_hi, F w0, int &z0, int &z1) {
    z0 = 0;
    z1 = ntz;
    if (seg < 0) return;
    int ta = 0;
    while (ta < ntz && w0(ta) < 0 && kz_lo < 0) ta++;
    int tb = ta;
    while (tb < ntz && !(w0(tb) + wz > kz && kz_hi > kz)) tb++;
    z0 = seg == 0 ? 0 : seg == 1 ? ta : tb;
    z1 = seg == 0 ? ta : seg == 1 ? tb : ntz;
}

void spmv_gtx(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg) {
    FAMG_REQUIRE(gtx_supports(m, mode), AMG_ERR_UNSUPPORTED, "wide grid-transfer classes: unsupported epilogue");
    GtxArgs a{};
    a.cls = m.gtx_cls.get();
    a.dptr = m.gtx_dptr.get();
    a.dlen = m.gtx_dlen.get();
    a.doff = m.gtx_doff.get();
    a.dval = m.gtx_dval.get();
    const int64_t *rg = m.gtx_r ? m.gtx_cg : m.gtx_fg, *kg = m.gtx_r ? m.gtx_fg : m.gtx_cg;
    a.rx = (int)rg[0]; a.ry = (int)rg[1]; a.rz = (int)rg[2];
    a.kx = (int)kg[0]; a.ky = (int)kg[1]; a.kz = (int)kg[2];
    a.tx = m.gtx_tile[0]; a.ty = m.gtx_tile[1]; a.tz = m.gtx_tile[2];
    a.wx = m.gtx_win[0]; a.wy = m.gtx_win[1]; a.wz = m.gtx_win[2];
    a.lox = m.gtx_lo[0]; a.loy = m.gtx_lo[1]; a.loz = m.gtx_lo[2];
    a.rwx = 1.0f / (float)a.wx; a.rwy = 1.0f / (float)a.wy;
    a.rtx = 1.0f / (float)std::max(a.tx, 1); a.rty = 1.0f / (float)std::max(a.ty, 1);
    FAMG_REQUIRE(m.gtx_fdiv, AMG_ERR_UNSUPPORTED, "wide grid-transfer classes: window too large for the float divisions");
    a.kz_lo = 0; a.kz_hi = a.kz; a.rz0 = 0; a.kz0 = 0; a.add_lo = a.add_hi = 0;
    if (m.rframe.on()) {
        a.rz = (int)m.rframe.nz;
        a.rz0 = (int)m.rframe.z0;
        a.kz = (int)m.cframe.nz;
        a.kz0 = (int)m.cframe.z0;
        a.kz_lo = (int)-m.cframe.gl;
        a.kz_hi = (int)(m.cframe.nz + m.cframe.gh);
        a.add_lo = m.cframe.add_lo();
        a.add_hi = m.cframe.add_hi();
    }
    a.x = x;
    a.y = y;
    a.b = epi.b;
    a.d = epi.d;
    a.dc = epi.dc;
    a.dt = epi.dt;
    a.dconst = epi.dc && epi.dk != 0.0 && flag(FLAG_DIA_DK) != 0;
    a.dk = epi.dk;
    a.y2 = epi.y2;
    a.ntx = (int)ceil_div(a.rx, a.tx);
    a.nty = (int)ceil_div(a.ry, a.ty);
    const int ntz = (int)ceil_div(a.rz, a.tz);
    const size_t lds = (size_t)a.wx * a.wy * a.wz * sizeof(double);
    int z0 = 0, z1 = ntz;
    if (m.gtx_r) {
        FAMG_REQUIRE(mode != SPMV_SETDF || (epi.y2 && (epi.d || epi.dc || epi.dk != 0.0)), AMG_ERR_INVALID,
                     "SETDF needs y2 and d");
        gtx_tiles(ntz, seg, a.wz, a.kz, a.kz_lo, a.kz_hi,
                  [&](int t) { return 2 * (a.rz0 + t * a.tz) - a.kz0 + a.loz; }, z0, z1);
        if (z1 <= z0) return;
        a.tile0 = a.ntx * a.nty * z0;
        const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * (z1 - z0))), block(256);
        const int T = a.tx * a.ty * a.tz;
        const int rl = T <= 256 ? 1 : 2;
        const int W = a.wx * a.wy * a.wz, pf = W <= 256 * 8 ? 8 : W <= 256 * 16 ? 16 : 32;
#define FAMG_GTXR2(M, PF)                                                                          \
    if (rl == 1) k_gtx_restrict<M, 1, PF><<<grid, block, lds, s>>>(a);                             \
    else k_gtx_restrict<M, 2, PF><<<grid, block, lds, s>>>(a);
#define FAMG_GTXR(M)                                                                               \
    if (pf == 8) { FAMG_GTXR2(M, 8) }                                                              \
    else if (pf == 16) { FAMG_GTXR2(M, 16) }                                                       \
    else { FAMG_GTXR2(M, 32) }
        if (mode == SPMV_SETDF) { FAMG_GTXR(SPMV_SETDF) }
        else { FAMG_GTXR(SPMV_SET) }
#undef FAMG_GTXR
#undef FAMG_GTXR2
    } else {
        gtx_tiles(ntz, seg, a.wz, a.kz, a.kz_lo, a.kz_hi,
                  [&](int t) { return ((a.rz0 + t * a.tz) >> 1) - a.kz0 + a.loz; }, z0, z1);
        if (z1 <= z0) return;
        a.tile0 = a.ntx * a.nty * z0;
        const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * (z1 - z0))), block(256);
        const int W = a.wx * a.wy * a.wz, pf = W <= 256 * 4 ? 4 : W <= 256 * 8 ? 8 : 16;
#define FAMG_GTXP2(TZ, PF)                                                                         \
    switch (mode) {                                                                                \
    case SPMV_SET: k_gtx_interp<SPMV_SET, TZ, PF><<<grid, block, lds, s>>>(a); break;              \
    case SPMV_ADD: k_gtx_interp<SPMV_ADD, TZ, PF><<<grid, block, lds, s>>>(a); break;              \
    case SPMV_ADD0: k_gtx_interp<SPMV_ADD0, TZ, PF><<<grid, block, lds, s>>>(a); break;            \
    default: break;                                                                                \
    }
#define FAMG_GTXP(TZ)                                                                              \
    if (pf == 4) { FAMG_GTXP2(TZ, 4) }                                                             \
    else if (pf == 8) { FAMG_GTXP2(TZ, 8) }                                                        \
    else { FAMG_GTXP2(TZ, 16) }
        if (a.tz == 4) { FAMG_GTXP(4) }
        else { FAMG_GTXP(2) }
#undef FAMG_GTXP
#undef FAMG_GTXP2
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
