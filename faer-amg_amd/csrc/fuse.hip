// fuse.hip -- the fine-level grid transfers of a V-cycle fused with their
// neighbouring SpMVs, for a level whose operator is a stencil on a structured
// grid ("Fused grid transfers").
//
// Multigrid::cycle (multigrid.rs:337-369) runs on such a level
//   r = f - A v            (residual; v = d*f when the zero-guess step is folded)
//   f_c = R r              (restriction)
//   ...coarse cycle...
//   v = v + P v_c          (interpolate-add; d*f + P v_c when folded)
//   v = v + d (f - A v)    (one post-smoothing Jacobi step)
// and each line is one launch streaming its vectors through HBM: r and the
// corrected v are written only to be read back by the next launch.  Here two
// single-pass launches replace the four; one workgroup per 3-D grid tile keeps
// the intermediate in LDS and recomputes it on the tile's halo:
//   k_fuse_resid_restrict: a 16 x 4 x 2 coarse tile stages the residual's x
//     operand (the iterate, or d*f) over 36 x 12 x 8 fine points, computes r on
//     the 34 x 10 x 6 points R reads, then the tile's restriction;
//   k_fuse_interp_jacobi: a 32 x 8 x 4 fine tile stages v_c over its coarse
//     window, computes the corrected v on the tile and a halo of one (34 x 10 x 6),
//     then the Jacobi step of the tile.
// (A first version marched plane by plane with an LDS ring: every plane step
// waited for a global round trip at 2-3 workgroups per CU, 257 / 189 us against
// 146 / 202 us for the separate launches on the 256^3 cycle.)  R and P are read
// through their grid-transfer classes (gtc.hip: one 8-bit class per row, coded
// (value, step) dictionaries); A is the level's DIA codes.
//
// Arithmetic is the unfused launches' exactly: each row sum is the fma chain
// over the stored entries in ascending column order (for a grid step that is
// ascending (dz, dy, dx)), absent or out-of-grid terms multiply +0.0 (codes
// of +0.0 are checked at setup for every entry leaving the grid), and the
// epilogues are the DIA / grid-transfer ones (b - acc; y + acc with y = d*f or
// v; v + d (f - acc)) -- bitwise equal to the oracle's row sums.
#include <algorithm>
#include <cstring>

#include "famg.hpp"

namespace famg {

// FAMG_FUSE=1 enables the fused transfers for multigrids created afterwards
// (default off until measured faster)
int g_fuse_transfers = [] {
    const char *e = getenv("FAMG_FUSE");
    return (e && e[0] == '1') ? 1 : 0;
}();

struct TransferFuse {
    int fx = 0, fy = 0, fz = 0, cx = 0, cy = 0, cz = 0;
    int K = 0;
    int8_t adx[32] = {}, ady[32] = {}, adz[32] = {};
    const GpuCsr *R = nullptr, *P = nullptr;  // their grid-transfer overlays
    bool pre = false, post = false;
};

// ---------------------------------------------------------------- kernels

constexpr int FR_CX = 16, FR_CY = 4, FR_CZ = 2;                       // coarse tile (restriction)
constexpr int FR_RX = 2 * FR_CX + 2, FR_RY = 2 * FR_CY + 2, FR_RZ = 2 * FR_CZ + 2;  // residual 34 x 10 x 6
constexpr int FR_XX = FR_RX + 2, FR_XY = FR_RY + 2, FR_XZ = FR_RZ + 2;  // x operand 36 x 12 x 8
constexpr int FI_TX = 32, FI_TY = 8, FI_TZ = 4;                         // fine tile (interpolation)
constexpr int FI_VX = FI_TX + 2, FI_VY = FI_TY + 2, FI_VZ = FI_TZ + 2;  // corrected v 34 x 10 x 6
constexpr int FI_WX = FI_TX / 2 + 4, FI_WY = FI_TY / 2 + 4, FI_WZ = FI_TZ / 2 + 4;  // v_c window 20 x 8 x 6
constexpr int F_DMAX = 2048;  // class dictionary entries (nclass * ke) staged in LDS

struct FuseArgs {
    const uint32_t *codes;
    const double *vtab;
    int ntab, K;
    int8_t adx[32], ady[32], adz[32];
    const double *f;      // the level's right-hand side
    const double *x;      // restriction: the iterate (XM 0); interpolation: v before the correction (ADD)
    const uint8_t *dc;    // 8-bit codes of the Jacobi diagonal into dt (or null: d)
    const double *dt;
    const double *d;
    const uint8_t *cls;   // R (restriction) or P (interpolation) grid-transfer classes
    const uint16_t *dict; // value index << 8 | step slot, ke per class
    const double *ctab;   // their values
    int ke, nce, nctab;
    const double *vc;     // interpolation: the coarse correction
    double *out;          // restriction: f_c; interpolation: the smoothed v
    int fx, fy, fz, cx, cy, cz;
    int ntx, nty;
};

// tables into LDS with every load of a lane issued before its stores
__device__ __forceinline__ void fuse_stage_tables(const FuseArgs &a, double *stab, int nstab, double *sdt,
                                                  uint16_t *sd, double *sct) {
    constexpr int PF = F_DMAX / 256;
    const int tid = threadIdx.x;
    uint16_t v[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) v[u] = a.dict[min(tid + 256 * u, a.nce - 1)];
    const double t0 = a.vtab[min(tid, a.ntab - 1)];
    const double t1 = a.ctab[min(tid, a.nctab - 1)];
    const double t2 = sdt ? a.dt[tid] : 0.0;
#pragma unroll
    for (int u = 0; u < PF; u++)
        if (tid + 256 * u < a.nce) sd[tid + 256 * u] = v[u];
    if (tid < a.ntab && tid < nstab) stab[tid] = t0;
    if (tid < a.nctab) sct[tid] = t1;
    if (sdt) sdt[tid] = t2;
}

// XM: the residual's x operand -- 0 the iterate x, 1 d*f with coded d, 2 d*f with fp64 d
template <int VB, int CW, int XM>
__global__ __launch_bounds__(256) void k_fuse_resid_restrict(FuseArgs a) {
    constexpr int RN = FR_RX * FR_RY * FR_RZ, XN = FR_XX * FR_XY * FR_XZ;
    constexpr int NX = (XN + 255) / 256, NR = (RN + 255) / 256;
    constexpr int KM = (CW * 32 / VB) < 27 ? (CW * 32 / VB) : 27;
    constexpr uint32_t MASK = (1u << VB) - 1;
    __shared__ double xo[XN];
    __shared__ double rr[RN];
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[XM == 1 ? 256 : 1];
    __shared__ uint16_t sd[F_DMAX];
    __shared__ double sct[256];
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int X0 = tix * FR_CX, Y0 = tiy * FR_CY, Z0 = tiz * FR_CZ;
    const int rx0 = 2 * X0 - 1, ry0 = 2 * Y0 - 1, rz0 = 2 * Z0 - 1;  // residual region origin (fine)
    const int64_t plane = (int64_t)a.fx * a.fy, cplane = (int64_t)a.cx * a.cy;
    fuse_stage_tables(a, stab, VB == 4 ? 16 : 256, XM == 1 ? sdt : nullptr, sd, sct);
    // the coarse row's class (restriction lanes)
    const int lx = tid % FR_CX, ly = (tid / FR_CX) % FR_CY, lz = tid / (FR_CX * FR_CY);
    const int X = X0 + lx, Y = Y0 + ly, Z = Z0 + lz;
    const bool rlive = tid < FR_CX * FR_CY * FR_CZ && X < a.cx && Y < a.cy && Z < a.cz;
    const int64_t J = rlive ? (int64_t)Z * cplane + (int64_t)Y * a.cx + X : 0;
    const int rc = a.cls[J];
    // the residual points' codes and f, the x operand's loads
    uint32_t w[NR][CW];
    double fb[NR];
#pragma unroll
    for (int u = 0; u < NR; u++) {
        const int q = min(tid + 256 * u, RN - 1);
        const int gx = rx0 + q % FR_RX, gy = ry0 + (q / FR_RX) % FR_RY, gz = rz0 + q / (FR_RX * FR_RY);
        const bool in = (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy && (unsigned)gz < (unsigned)a.fz;
        const int64_t p = in ? (int64_t)gz * plane + (int64_t)gy * a.fx + gx : 0;
#pragma unroll
        for (int c = 0; c < CW; c++) w[u][c] = a.codes[p * CW + c];
        fb[u] = a.f[p];
    }
    double xv[NX];
    int xc[NX];
#pragma unroll
    for (int u = 0; u < NX; u++) {
        const int q = min(tid + 256 * u, XN - 1);
        const int gx = rx0 - 1 + q % FR_XX, gy = ry0 - 1 + (q / FR_XX) % FR_XY, gz = rz0 - 1 + q / (FR_XX * FR_XY);
        const bool in = (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy && (unsigned)gz < (unsigned)a.fz;
        const int64_t p = in ? (int64_t)gz * plane + (int64_t)gy * a.fx + gx : 0;
        if constexpr (XM == 0) xv[u] = in ? a.x[p] : 0.0;
        else if constexpr (XM == 1) {
            xv[u] = in ? a.f[p] : 0.0;
            xc[u] = a.dc[p];
        } else xv[u] = in ? a.d[p] * a.f[p] : 0.0;
    }
    __syncthreads();  // tables
#pragma unroll
    for (int u = 0; u < NX; u++) {
        const int q = tid + 256 * u;
        if (q < XN) xo[q] = XM == 1 ? sdt[xc[u]] * xv[u] : xv[u];  // vec_mul's d*f (0 * 0.0 outside)
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NR; u++) {
        const int q = tid + 256 * u;
        if (q >= RN) continue;
        const int qx = q % FR_RX, qy = (q / FR_RX) % FR_RY, qz = q / (FR_RX * FR_RY);
        const int gx = rx0 + qx, gy = ry0 + qy, gz = rz0 + qz;
        const bool in = (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy && (unsigned)gz < (unsigned)a.fz;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KM; k++) {
            const uint32_t code = (w[u][(k * VB) >> 5] >> ((k * VB) & 31)) & MASK;
            const double xk = xo[((qz + 1 + a.adz[k]) * FR_XY + qy + 1 + a.ady[k]) * FR_XX + qx + 1 + a.adx[k]];
            const double f0 = fma(stab[code], xk, acc);
            acc = k < a.K ? f0 : acc;
        }
        rr[q] = in ? fb[u] - acc : 0.0;
    }
    __syncthreads();
    if (!rlive) return;
    const int base = ((2 * lz + 1) * FR_RY + 2 * ly + 1) * FR_RX + 2 * lx + 1;
    const uint16_t *e = sd + rc * a.ke;
    double acc = 0.0;
    for (int k = 0; k < a.ke; k += 8) {
        double cv[8], rv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int c = e[k + u], sl = c & 255;
            cv[u] = sct[c >> 8];
            rv[u] = rr[base + ((sl >> 4) - 1) * (FR_RY * FR_RX) + (((sl >> 2) & 3) - 1) * FR_RX + (sl & 3) - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc = fma(cv[u], rv[u], acc);
    }
    a.out[J] = acc;
}

// FOLD: v = d*f + P v_c (the folded zero-guess step), else v = x + P v_c;
// DC: d from 8-bit codes (dc, dt), else fp64 d
template <int VB, int CW, bool FOLD, bool DC>
__global__ __launch_bounds__(256) void k_fuse_interp_jacobi(FuseArgs a) {
    constexpr int VN = FI_VX * FI_VY * FI_VZ, WN = FI_WX * FI_WY * FI_WZ;
    constexpr int NV = (VN + 255) / 256, NW = (WN + 255) / 256;
    constexpr int KM = (CW * 32 / VB) < 27 ? (CW * 32 / VB) : 27;
    constexpr uint32_t MASK = (1u << VB) - 1;
    __shared__ double vr[VN];
    __shared__ double cw[WN];
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[DC ? 256 : 1];
    __shared__ uint16_t sd[F_DMAX];
    __shared__ double sct[256];
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int x0 = tix * FI_TX, y0 = tiy * FI_TY, z0 = tiz * FI_TZ;
    const int wx0 = x0 / 2 - 2, wy0 = y0 / 2 - 2, wz0 = z0 / 2 - 2;  // v_c window origin (coarse)
    const int64_t plane = (int64_t)a.fx * a.fy, cplane = (int64_t)a.cx * a.cy;
    fuse_stage_tables(a, stab, VB == 4 ? 16 : 256, DC ? sdt : nullptr, sd, sct);
    // loads: the v_c window, the corrected-v points' classes and bases, the Jacobi rows
    double wv[NW];
#pragma unroll
    for (int u = 0; u < NW; u++) {
        const int q = min(tid + 256 * u, WN - 1);
        const int Xc = wx0 + q % FI_WX, Yc = wy0 + (q / FI_WX) % FI_WY, Zc = wz0 + q / (FI_WX * FI_WY);
        const bool in = (unsigned)Xc < (unsigned)a.cx && (unsigned)Yc < (unsigned)a.cy && (unsigned)Zc < (unsigned)a.cz;
        wv[u] = in ? a.vc[(int64_t)Zc * cplane + (int64_t)Yc * a.cx + Xc] : 0.0;
    }
    int cl[NV], vd[NV];
    double vb[NV];
#pragma unroll
    for (int u = 0; u < NV; u++) {
        const int q = min(tid + 256 * u, VN - 1);
        const int gx = x0 - 1 + q % FI_VX, gy = y0 - 1 + (q / FI_VX) % FI_VY, gz = z0 - 1 + q / (FI_VX * FI_VY);
        const bool in = (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy && (unsigned)gz < (unsigned)a.fz;
        const int64_t p = in ? (int64_t)gz * plane + (int64_t)gy * a.fx + gx : 0;
        cl[u] = in ? (int)a.cls[p] : -1;
        if constexpr (FOLD) {
            vb[u] = a.f[p];
            if constexpr (DC) vd[u] = a.dc[p];
            else vb[u] = a.d[p] * vb[u];  // the ADD0 epilogue's d*b
        } else {
            vb[u] = a.x[p];
        }
    }
    constexpr int NJ = FI_TZ;  // the lane's Jacobi rows: (x, y) fixed, z0 .. z0+3
    const int jx = tid % FI_TX, jy = tid / FI_TX;
    uint32_t w[NJ][CW];
    double fj[NJ], dj[NJ];
    int dcj[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        const int gx = x0 + jx, gy = y0 + jy, gz = z0 + j;
        const bool in = gx < a.fx && gy < a.fy && gz < a.fz;
        const int64_t p = in ? (int64_t)gz * plane + (int64_t)gy * a.fx + gx : 0;
#pragma unroll
        for (int c = 0; c < CW; c++) w[j][c] = a.codes[p * CW + c];
        fj[j] = a.f[p];
        if constexpr (DC) dcj[j] = a.dc[p];
        else dj[j] = a.d[p];
    }
#pragma unroll
    for (int u = 0; u < NW; u++)
        if (tid + 256 * u < WN) cw[tid + 256 * u] = wv[u];
    __syncthreads();  // tables and the window
#pragma unroll
    for (int u = 0; u < NV; u++) {
        const int q = tid + 256 * u;
        if (q >= VN) continue;
        double out = 0.0;
        if (cl[u] >= 0) {
            const int gx = x0 - 1 + q % FI_VX, gy = y0 - 1 + (q / FI_VX) % FI_VY, gz = z0 - 1 + q / (FI_VX * FI_VY);
            const int base = (((gz >> 1) - wz0) * FI_WY + (gy >> 1) - wy0) * FI_WX + (gx >> 1) - wx0;
            const uint16_t *e = sd + cl[u] * a.ke;
            double acc = 0.0;
            for (int k = 0; k < a.ke; k += 4) {
                double cv[4], vv[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int c = e[k + i], sl = c & 255;
                    cv[i] = sct[c >> 8];
                    vv[i] = cw[base + (sl / 9 - 1) * (FI_WY * FI_WX) + ((sl / 3) % 3 - 1) * FI_WX + sl % 3 - 1];
                }
#pragma unroll
                for (int i = 0; i < 4; i++) acc = fma(cv[i], vv[i], acc);
            }
            double y0v = vb[u];
            if constexpr (FOLD && DC) y0v = sdt[vd[u]] * y0v;  // d*b
            out = y0v + acc;
        }
        vr[q] = out;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        const int gx = x0 + jx, gy = y0 + jy, gz = z0 + j;
        if (gx >= a.fx || gy >= a.fy || gz >= a.fz) continue;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KM; k++) {
            const uint32_t code = (w[j][(k * VB) >> 5] >> ((k * VB) & 31)) & MASK;
            const double xk = vr[((j + 1 + a.adz[k]) * FI_VY + jy + 1 + a.ady[k]) * FI_VX + jx + 1 + a.adx[k]];
            const double f0 = fma(stab[code], xk, acc);
            acc = k < a.K ? f0 : acc;
        }
        const double xr = vr[((j + 1) * FI_VY + jy + 1) * FI_VX + jx + 1];
        const double dr = DC ? sdt[dcj[j]] : dj[j];
        a.out[(int64_t)gz * plane + (int64_t)gy * a.fx + gx] = xr + dr * (fj[j] - acc);  // DIA JACOBI
    }
}

// every entry of a DIA operator on the grid whose step leaves the grid carries
// the +0.0 code (the fused kernels read 0.0 there, the DIA kernels some x value)
__global__ void k_fuse_check_dia(const uint32_t *codes, int cw, int vb, int K, const int8_t *steps, int zcode,
                                 int fx, int fy, int fz, int *bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = (int64_t)fx * fy * fz;
    if (i >= n) return;
    const int x = (int)(i % fx), y = (int)((i / fx) % fy), z = (int)(i / ((int64_t)fx * fy));
    const uint32_t mask = (1u << vb) - 1;
    for (int k = 0; k < K; k++) {
        const int X = x + steps[3 * k], Y = y + steps[3 * k + 1], Z = z + steps[3 * k + 2];
        const bool in = X >= 0 && X < fx && Y >= 0 && Y < fy && Z >= 0 && Z < fz;
        const uint32_t c = (codes[i * cw + ((k * vb) >> 5)] >> ((k * vb) & 31)) & mask;
        if (!in && (int)c != zcode) bad[0] = 1;
    }
}

// ---------------------------------------------------------------- setup

static bool fuse_kernel_shape(const GpuCsr &m) {
    return (m.dia_vbits == 4 && (m.dia_cw == 1 || m.dia_cw == 4)) || (m.dia_vbits == 8 && (m.dia_cw == 2 || m.dia_cw == 8));
}

// Decide and build the fused transfers of level l (A_l on a grid as DIA codes
// with steps in {-1,0,1}^3, the next level on the 2 x 2 x 2 box grid, R/P as
// grid-transfer classes).  Setup only (before any graph capture).
void fuse_setup(MultigridOp &mg, size_t l) {
    MgLevel &L = mg.levels[l];
    L.fuse.reset();
    if (!mg.fuse_transfers || l + 1 >= mg.levels.size()) return;
    auto *A = dynamic_cast<CsrOp *>(L.A.get());
    auto *R = dynamic_cast<CsrOp *>(L.R.get());
    auto *P = dynamic_cast<CsrOp *>(L.P.get());
    auto *Ac = dynamic_cast<CsrOp *>(mg.levels[l + 1].A.get());
    if (!A || !R || !P || !Ac) return;
    const GpuCsr &m = A->m;
    if (m.kernel != SPMV_KERNEL_DIA || !m.has_dia() || m.dia_rowid || m.dia_r0 != 0 || m.dia_r1 != m.nrows ||
        m.dia_k > 27 || !fuse_kernel_shape(m) || m.nrows != m.ncols)
        return;
    const int64_t fx = m.grid[0], fy = m.grid[1], fz = m.grid[2];
    const int64_t cx = Ac->m.grid[0], cy = Ac->m.grid[1], cz = Ac->m.grid[2];
    if (fx <= 2 || fy <= 2 || fz <= 2 || fx * fy * fz != m.nrows || cx != ceil_div(fx, 2) || cy != ceil_div(fy, 2) ||
        cz != ceil_div(fz, 2) || cx * cy * cz != Ac->m.nrows || fx * fy * fz >= (int64_t(1) << 31))
        return;
    auto F = std::make_shared<TransferFuse>();
    F->fx = (int)fx; F->fy = (int)fy; F->fz = (int)fz;
    F->cx = (int)cx; F->cy = (int)cy; F->cz = (int)cz;
    F->K = m.dia_k;
    std::vector<int8_t> steps(3 * 32, 0);
    for (int k = 0; k < m.dia_k; k++) {
        const int64_t o = m.dia_off[k];
        int64_t dx = ((o % fx) + fx) % fx;
        if (dx > fx / 2) dx -= fx;
        const int64_t q = (o - dx) / fx;
        int64_t dy = ((q % fy) + fy) % fy;
        if (dy > fy / 2) dy -= fy;
        const int64_t dz = (q - dy) / fy;
        if (std::abs(dx) > 1 || std::abs(dy) > 1 || std::abs(dz) > 1) return;
        F->adx[k] = (int8_t)dx; F->ady[k] = (int8_t)dy; F->adz[k] = (int8_t)dz;
        steps[3 * k] = (int8_t)dx; steps[3 * k + 1] = (int8_t)dy; steps[3 * k + 2] = (int8_t)dz;
    }
    // the +0.0 code (the table is sorted by bit pattern) on every entry leaving the grid
    std::vector<double> tab(m.dia_ntab);
    hipStream_t s = mg.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(tab.data(), m.dia_vtab.get(), tab.size() * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    int zcode = -1;
    for (size_t q = 0; q < tab.size(); q++) {
        uint64_t bits;
        std::memcpy(&bits, &tab[q], 8);
        if (bits == 0) zcode = (int)q;
    }
    if (zcode < 0) return;
    {
        DevBuf<int> bad(1);
        DevBuf<int8_t> dsteps(steps.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(dsteps.get(), steps.data(), steps.size(), hipMemcpyHostToDevice, s));
        FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
        hipLaunchKernelGGL(k_fuse_check_dia, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s,
                           m.dia_codes.get(), m.dia_cw, m.dia_vbits, m.dia_k, dsteps.get(), zcode, (int)fx, (int)fy,
                           (int)fz, bad.get());
        FAMG_CHECK_HIP(hipGetLastError());
        int hbad = 1;
        FAMG_CHECK_HIP(hipMemcpyAsync(&hbad, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        if (hbad) return;
    }
    // R and P through their grid-transfer overlays (gtc.hip), built for the same grids
    auto same_grids = [&](const GpuCsr &M) {
        return M.gtc_on && M.gtc_nce <= F_DMAX && M.gtc_fg[0] == fx && M.gtc_fg[1] == fy && M.gtc_fg[2] == fz &&
               M.gtc_cg[0] == cx && M.gtc_cg[1] == cy && M.gtc_cg[2] == cz;
    };
    F->R = &R->m;
    F->P = &P->m;
    F->pre = same_grids(R->m) && R->m.gtc_r;
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    F->post = D && same_grids(P->m) && !P->m.gtc_r;
    if (F->pre || F->post) L.fuse = F;
}

bool fuse_has_pre(const MgLevel &L) { return L.fuse && L.fuse->pre && L.fuse->R->gtc_on; }
bool fuse_has_post(const MgLevel &L) { return L.fuse && L.fuse->post && L.fuse->P->gtc_on; }

static void fuse_common(FuseArgs &a, const TransferFuse &F, const GpuCsr &m, const GpuCsr &T) {
    a.codes = m.dia_codes.get();
    a.vtab = m.dia_vtab.get();
    a.ntab = (int)m.dia_ntab;
    a.K = F.K;
    std::memcpy(a.adx, F.adx, 32);
    std::memcpy(a.ady, F.ady, 32);
    std::memcpy(a.adz, F.adz, 32);
    a.fx = F.fx; a.fy = F.fy; a.fz = F.fz;
    a.cx = F.cx; a.cy = F.cy; a.cz = F.cz;
    a.cls = T.gtc_cls.get();
    a.dict = T.gtc_dict.get();
    a.ctab = T.gtc_vtab.get();
    a.ke = T.gtc_ke;
    a.nce = T.gtc_nce;
    a.nctab = T.gtc_ntab;
}

// f_c = R (f - A x): x = the iterate, or (x null) the folded zero-guess iterate d*f
void fuse_resid_restrict(const TransferFuse &F, const GpuCsr &m, const double *f, const double *x,
                         const DiagOp *D, double *fc, hipStream_t s) {
    FuseArgs a{};
    fuse_common(a, F, m, *F.R);
    a.f = f;
    a.x = x;
    const bool dc = D && D->dcode.get();
    if (!x) {
        FAMG_REQUIRE(D, AMG_ERR_INVALID, "fused restriction: folded step without a diagonal");
        a.dc = D->dcode.get();
        a.dt = D->dtab.get();
        a.d = D->d.get();
    }
    a.out = fc;
    a.ntx = (int)ceil_div(F.cx, FR_CX);
    a.nty = (int)ceil_div(F.cy, FR_CY);
    const int ntz = (int)ceil_div(F.cz, FR_CZ);
    const int64_t n = (int64_t)F.fx * F.fy * F.fz, nc = (int64_t)F.cx * F.cy * F.cz;
    // bytes: A's codes, f (and d's codes) or x, the classes, f_c written
    if (g_launch_log)
        log_launch("fuse_resid_restrict", SPMV_KERNEL_DIA, x ? SPMV_RESID : SPMV_RESID0, n,
                   4 * (int64_t)m.dia_cw * n + 8 * n + (x ? 8 * n : (dc ? 1 : 8) * n) + nc + 8 * nc);
    const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * ntz)), block(256);
    const int xm = x ? 0 : dc ? 1 : 2;
#define FAMG_FRR(VB, CW)                                                                           \
    if (xm == 0) k_fuse_resid_restrict<VB, CW, 0><<<grid, block, 0, s>>>(a);                       \
    else if (xm == 1) k_fuse_resid_restrict<VB, CW, 1><<<grid, block, 0, s>>>(a);                  \
    else k_fuse_resid_restrict<VB, CW, 2><<<grid, block, 0, s>>>(a);
    if (m.dia_vbits == 4 && m.dia_cw == 1) { FAMG_FRR(4, 1) }
    else if (m.dia_vbits == 4) { FAMG_FRR(4, 4) }
    else if (m.dia_cw == 2) { FAMG_FRR(8, 2) }
    else { FAMG_FRR(8, 8) }
#undef FAMG_FRR
    FAMG_CHECK_HIP(hipGetLastError());
}

// out = Jacobi step from v = (x null: d*f | x) + P v_c
void fuse_interp_jacobi(const TransferFuse &F, const GpuCsr &m, const double *vc, const double *f, const double *x,
                        const DiagOp &D, double *out, hipStream_t s) {
    FAMG_REQUIRE(out != x && out != f && out != vc, AMG_ERR_INVALID, "fused interpolation: aliased output");
    FuseArgs a{};
    fuse_common(a, F, m, *F.P);
    a.f = f;
    a.x = x;
    a.dc = D.dcode.get();
    a.dt = D.dtab.get();
    a.d = D.d.get();
    a.vc = vc;
    a.out = out;
    a.ntx = (int)ceil_div(F.fx, FI_TX);
    a.nty = (int)ceil_div(F.fy, FI_TY);
    const int ntz = (int)ceil_div(F.fz, FI_TZ);
    const int64_t n = (int64_t)F.fx * F.fy * F.fz, nc = (int64_t)F.cx * F.cy * F.cz;
    const bool dc = a.dc != nullptr;
    // bytes: classes, v_c, f, d (codes), x (ADD), A's codes, out written
    if (g_launch_log)
        log_launch("fuse_interp_jacobi", SPMV_KERNEL_DIA, x ? SPMV_ADD : SPMV_ADD0, n,
                   n + 8 * nc + 8 * n + (dc ? 1 : 8) * n + (x ? 8 * n : 0) + 4 * (int64_t)m.dia_cw * n + 8 * n);
    const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * ntz)), block(256);
#define FAMG_FIJ(VB, CW)                                                                           \
    if (!x && dc) k_fuse_interp_jacobi<VB, CW, true, true><<<grid, block, 0, s>>>(a);              \
    else if (!x) k_fuse_interp_jacobi<VB, CW, true, false><<<grid, block, 0, s>>>(a);              \
    else if (dc) k_fuse_interp_jacobi<VB, CW, false, true><<<grid, block, 0, s>>>(a);              \
    else k_fuse_interp_jacobi<VB, CW, false, false><<<grid, block, 0, s>>>(a);
    if (m.dia_vbits == 4 && m.dia_cw == 1) { FAMG_FIJ(4, 1) }
    else if (m.dia_vbits == 4) { FAMG_FIJ(4, 4) }
    else if (m.dia_cw == 2) { FAMG_FIJ(8, 2) }
    else { FAMG_FIJ(8, 8) }
#undef FAMG_FIJ
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
