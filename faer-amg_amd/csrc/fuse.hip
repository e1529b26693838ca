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
// launches replace the four.  Both march one workgroup's tile through the grid
// plane by plane and keep the intermediate (r, or the corrected v) in an LDS
// ring of planes:
//   k_fuse_resid_restrict: per coarse plane Z, the fine residual planes
//     2Z+1, 2Z+2 of a 34 x 18 region (16 x 8 coarse points and the reach of R)
//     from an LDS ring of x-operand planes (the iterate, or d*f), then the
//     restriction of the tile's coarse points from the residual ring;
//   k_fuse_interp_jacobi: per fine plane z, the corrected v of plane z+1 over
//     a 34 x 18 region (32 x 16 points and a halo of one) from an LDS window of
//     v_c, then the Jacobi step of plane z from the ring of v planes.
// R and P are read as grid-transfer classes: for 2 x 2 x 2 box aggregates a
// row's entries sit at fixed grid steps from its anchor (P: the coarse point
// of its box, steps in {-1,0,1}^3; R: the box's first fine point, steps in
// {-1,..,2}^3), so a row is one 8-bit class id into a dictionary of (step,
// value) lists -- 1 B per row instead of P_0's 12.5 B of SELL storage.  A is
// the level's DIA codes (4 B per row for the 7-point operator).
//
// Arithmetic is the unfused launches' exactly: each row sum is the fma chain
// over the stored entries in ascending column order (for a grid step that is
// ascending (dz, dy, dx)), absent or out-of-grid terms multiply +0.0 (codes
// of +0.0 are checked at setup for every entry leaving the grid), and the
// epilogues are the DIA / SELL ones (b - acc; y + acc with y = d*f or v;
// v + d (f - acc)) -- bitwise equal to the four launches.
#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "famg.hpp"

namespace famg {

// FAMG_FUSE=1 enables the fused transfers process-wide (default off: measured
// slower than the separate launches so far)
int g_fuse_transfers = [] {
    const char *e = getenv("FAMG_FUSE");
    return (e && e[0] == '1') ? 1 : 0;
}();

struct TransferFuse {
    int fx = 0, fy = 0, fz = 0, cx = 0, cy = 0, cz = 0;
    int K = 0;
    int8_t adx[32] = {}, ady[32] = {}, adz[32] = {};
    DevBuf<uint8_t> pcls, rcls;
    DevBuf<int16_t> poff, roff;  // per class entry: its position in the kernel's LDS layout (below)
    DevBuf<double> pval, rval;
    int pke = 0, rke = 0, pnc = 0, rnc = 0;
    bool pre = false, post = false;
};

// ---------------------------------------------------------------- kernels

constexpr int FR_CTX = 16, FR_CTY = 8;                      // coarse tile of the restriction
constexpr int FR_RX = 2 * FR_CTX + 2, FR_RY = 2 * FR_CTY + 2;  // residual region 34 x 18
constexpr int FR_XX = FR_RX + 2, FR_XY = FR_RY + 2;          // x-operand region 36 x 20
constexpr int FI_TX = 32, FI_TY = 16;                       // fine tile of the interpolation
constexpr int FI_VX = FI_TX + 2, FI_VY = FI_TY + 2;          // corrected-v region 34 x 18
constexpr int FI_WX = FI_TX / 2 + 4, FI_WY = FI_TY / 2 + 4;  // v_c window 20 x 12 (x 3 planes)
constexpr int F_DMAX = 1024;  // class entries staged in LDS (nclass * ke)
// R entry at step (dx, dy, dz) from the box's first fine point: (dz + 1) << 12 |
// (dy * FR_RX + dx + 2048), relative to that point's position in a residual plane
__host__ __device__ constexpr int fr_pack(int dx, int dy, int dz) { return ((dz + 1) << 12) | (dy * FR_RX + dx + 2048); }
// P entry at coarse step (dx, dy, dz) from the anchor: its offset in the v_c window
__host__ __device__ constexpr int fi_pack(int dx, int dy, int dz) { return (dz * FI_WY + dy) * FI_WX + dx; }

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
    const uint8_t *cls;   // R (restriction) or P (interpolation) classes
    const double *cval;   // class entries: values and LDS positions, ke per class
    const int16_t *coff;
    int ke, nce;          // entries per class (a multiple of 8 / 4), nclass * ke
    const double *vc;     // interpolation: the coarse correction
    double *out;          // restriction: f_c; interpolation: the smoothed v
    int fx, fy, fz, cx, cy, cz;
    int ntx, nty, zchunk;
};

// XM: the residual's x operand -- 0 the iterate x, 1 d*f with coded d, 2 d*f with fp64 d
template <int VB, int CW, int XM>
__global__ __launch_bounds__(256) void k_fuse_resid_restrict(FuseArgs a) {
    constexpr int RPL = FR_RX * FR_RY, XPL = FR_XX * FR_XY;
    constexpr int KM = (CW * 32 / VB) < 27 ? (CW * 32 / VB) : 27;
    constexpr uint32_t MASK = (1u << VB) - 1;
    constexpr int NX = (2 * XPL + 255) / 256, NR = (2 * RPL + 255) / 256;
    __shared__ double xo[4][XPL];
    __shared__ double rr[4][RPL];
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[XM == 1 ? 256 : 1];
    __shared__ double sval[F_DMAX];
    __shared__ int16_t soff[F_DMAX];
    const int tid = threadIdx.x;
    {  // class dictionary: all loads of a lane before its stores
        constexpr int PF = F_DMAX / 256;
        double v[PF];
        int16_t o[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int q = min(tid + 256 * u, a.nce - 1);
            v[u] = a.cval[q];
            o[u] = a.coff[q];
        }
#pragma unroll
        for (int u = 0; u < PF; u++)
            if (tid + 256 * u < a.nce) {
                sval[tid + 256 * u] = v[u];
                soff[tid + 256 * u] = o[u];
            }
    }
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int X0 = tix * FR_CTX, Y0 = tiy * FR_CTY, Z0 = tiz * a.zchunk, Z1 = min(Z0 + a.zchunk, a.cz);
    const int rx0 = 2 * X0 - 1, ry0 = 2 * Y0 - 1;  // residual region origin (fine)
    const int64_t plane = (int64_t)a.fx * a.fy;
    if (tid < a.ntab) stab[tid] = a.vtab[tid];
    if constexpr (XM == 1) sdt[tid] = a.dt[tid];
    __syncthreads();

    // x operand planes z2, z2+1 of the 36 x 20 region: loads, then LDS stores
    auto load_xo = [&](int z2, double (&v)[NX]) {
#pragma unroll
        for (int u = 0; u < NX; u++) {
            const int q = tid + 256 * u;
            const int pl = q >= XPL ? 1 : 0, w = q - pl * XPL;
            const int zz = z2 + pl, gx = rx0 - 1 + w % FR_XX, gy = ry0 - 1 + w / FR_XX;
            const bool in = q < 2 * XPL && (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy &&
                            (unsigned)zz < (unsigned)a.fz;
            const int64_t p = in ? (int64_t)zz * plane + (int64_t)gy * a.fx + gx : 0;
            if constexpr (XM == 0) v[u] = in ? a.x[p] : 0.0;
            else if constexpr (XM == 1) v[u] = in ? sdt[a.dc[p]] * a.f[p] : 0.0;  // vec_mul's d*f
            else v[u] = in ? a.d[p] * a.f[p] : 0.0;
        }
    };
    auto store_xo = [&](int z2, const double (&v)[NX]) {
#pragma unroll
        for (int u = 0; u < NX; u++) {
            const int q = tid + 256 * u;
            const int pl = q >= XPL ? 1 : 0;
            if (q < 2 * XPL) xo[(z2 + pl + 4) & 3][q - pl * XPL] = v[u];
        }
    };
    // residual planes z2, z2+1 of the 34 x 18 region: codes and f loaded first
    auto load_r = [&](int z2, uint32_t (&w)[NR][CW], double (&fb)[NR]) {
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int q = tid + 256 * u;
            const int pl = q >= RPL ? 1 : 0, wq = q - pl * RPL;
            const int zz = z2 + pl, gx = rx0 + wq % FR_RX, gy = ry0 + wq / FR_RX;
            const bool in = q < 2 * RPL && (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy &&
                            (unsigned)zz < (unsigned)a.fz;
            const int64_t p = in ? (int64_t)zz * plane + (int64_t)gy * a.fx + gx : 0;
#pragma unroll
            for (int c = 0; c < CW; c++) w[u][c] = a.codes[p * CW + c];
            fb[u] = in ? a.f[p] : 0.0;
        }
    };
    auto comp_r = [&](int z2, const uint32_t (&w)[NR][CW], const double (&fb)[NR]) {
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int q = tid + 256 * u;
            if (q >= 2 * RPL) continue;
            const int pl = q >= RPL ? 1 : 0, wq = q - pl * RPL;
            const int zz = z2 + pl, lx = wq % FR_RX, ly = wq / FR_RX;
            const int gx = rx0 + lx, gy = ry0 + ly;
            const bool in = (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy && (unsigned)zz < (unsigned)a.fz;
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < KM; k++) {
                const uint32_t code = (w[u][(k * VB) >> 5] >> ((k * VB) & 31)) & MASK;
                const double xv = xo[(zz + a.adz[k] + 4) & 3][(ly + 1 + a.ady[k]) * FR_XX + lx + 1 + a.adx[k]];
                const double f0 = fma(stab[code], xv, acc);
                acc = k < a.K ? f0 : acc;
            }
            rr[(zz + 4) & 3][wq] = in ? fb[u] - acc : 0.0;
        }
    };
    auto restrict_plane = [&](int Z) {
        if (tid >= FR_CTX * FR_CTY) return;
        const int lx = tid % FR_CTX, ly = tid / FR_CTX, X = X0 + lx, Y = Y0 + ly;
        if (X >= a.cx || Y >= a.cy) return;
        const int64_t J = ((int64_t)Z * a.cy + Y) * a.cx + X;
        const int c0 = a.cls[J] * a.ke;
        const int base = (2 * ly + 1) * FR_RX + 2 * lx + 1 - 2048;
        double acc = 0.0;
        for (int e0 = 0; e0 < a.ke; e0 += 8) {
            double cv[8], rv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int o = soff[c0 + e0 + u];
                cv[u] = sval[c0 + e0 + u];
                rv[u] = rr[(2 * Z + (o >> 12) - 1 + 4) & 3][base + (o & 4095)];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) acc = fma(cv[u], rv[u], acc);
        }
        a.out[J] = acc;
    };

    double v[NX];
    uint32_t w[NR][CW];
    double fb[NR];
    // prologue: x operand planes 2Z0-2 .. 2Z0+1, residual planes 2Z0-1, 2Z0
    load_xo(2 * Z0 - 2, v);
    store_xo(2 * Z0 - 2, v);
    load_xo(2 * Z0, v);
    load_r(2 * Z0 - 1, w, fb);
    store_xo(2 * Z0, v);
    __syncthreads();
    comp_r(2 * Z0 - 1, w, fb);
    __syncthreads();
    for (int Z = Z0; Z < Z1; Z++) {
        // x operand planes 2Z+2, 2Z+3 (over those of 2Z-2, 2Z-1) and the loads of
        // residual planes 2Z+1, 2Z+2, beside the restriction of Z-1
        load_xo(2 * Z + 2, v);
        load_r(2 * Z + 1, w, fb);
        store_xo(2 * Z + 2, v);
        __syncthreads();
        comp_r(2 * Z + 1, w, fb);  // over residual planes 2Z-3, 2Z-2 (read by Z-1)
        __syncthreads();
        restrict_plane(Z);
    }
}

// FOLD: v = d*f + P v_c (the folded zero-guess step), else v = x + P v_c;
// DC: d from 8-bit codes (dc, dt), else fp64 d
template <int VB, int CW, bool FOLD, bool DC>
__global__ __launch_bounds__(256) void k_fuse_interp_jacobi(FuseArgs a) {
    constexpr int VPL = FI_VX * FI_VY, WPL = FI_WX * FI_WY, TPL = FI_TX * FI_TY;
    constexpr int KM = (CW * 32 / VB) < 27 ? (CW * 32 / VB) : 27;
    constexpr uint32_t MASK = (1u << VB) - 1;
    constexpr int NV = (VPL + 255) / 256, NW = (3 * WPL + 255) / 256, NJ = (TPL + 255) / 256;
    __shared__ double vr[3][VPL];
    __shared__ double cw[3 * WPL];
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double sdt[DC ? 256 : 1];
    __shared__ double sval[F_DMAX];
    __shared__ int16_t soff[F_DMAX];
    const int tid = threadIdx.x;
    {  // class dictionary: all loads of a lane before its stores
        constexpr int PF = F_DMAX / 256;
        double v[PF];
        int16_t o[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int q = min(tid + 256 * u, a.nce - 1);
            v[u] = a.cval[q];
            o[u] = a.coff[q];
        }
#pragma unroll
        for (int u = 0; u < PF; u++)
            if (tid + 256 * u < a.nce) {
                sval[tid + 256 * u] = v[u];
                soff[tid + 256 * u] = o[u];
            }
    }
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int x0 = tix * FI_TX, y0 = tiy * FI_TY, z0 = tiz * a.zchunk, z1 = min(z0 + a.zchunk, a.fz);
    const int wx0 = x0 / 2 - 2, wy0 = y0 / 2 - 2;  // v_c window origin (coarse)
    const int64_t plane = (int64_t)a.fx * a.fy, cplane = (int64_t)a.cx * a.cy;
    if (tid < a.ntab) stab[tid] = a.vtab[tid];
    if constexpr (DC) sdt[tid] = a.dt[tid];
    __syncthreads();
    auto dget = [&](int64_t p) {
        if constexpr (DC) return sdt[a.dc[p]];
        else return a.d[p];
    };

    // loads for v plane zz: the v_c window (coarse planes zz/2 - 1 .. + 1) and
    // the region's classes and correction bases
    struct VLoad {
        double win[NW];
        int cl[NV];
        double base[NV];
    };
    auto load_v = [&](int zz, VLoad &L) {
        const int wz0 = (zz >> 1) - 1;
#pragma unroll
        for (int u = 0; u < NW; u++) {
            const int q = tid + 256 * u;
            const int pz = q / WPL, r = q - pz * WPL;
            const int X = wx0 + r % FI_WX, Y = wy0 + r / FI_WX, Z = wz0 + pz;
            const bool in = q < 3 * WPL && (unsigned)X < (unsigned)a.cx && (unsigned)Y < (unsigned)a.cy &&
                            (unsigned)Z < (unsigned)a.cz;
            L.win[u] = in ? a.vc[(int64_t)Z * cplane + (int64_t)Y * a.cx + X] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < NV; u++) {
            const int q = tid + 256 * u;
            const int gx = x0 - 1 + q % FI_VX, gy = y0 - 1 + q / FI_VX;
            const bool in = q < VPL && (unsigned)gx < (unsigned)a.fx && (unsigned)gy < (unsigned)a.fy &&
                            (unsigned)zz < (unsigned)a.fz;
            const int64_t p = in ? (int64_t)zz * plane + (int64_t)gy * a.fx + gx : 0;
            L.cl[u] = in ? (int)a.cls[p] : -1;
            if constexpr (FOLD) L.base[u] = in ? dget(p) * a.f[p] : 0.0;  // the ADD0 epilogue's d*b
            else L.base[u] = in ? a.x[p] : 0.0;
        }
    };
    auto store_win = [&](const VLoad &L) {
#pragma unroll
        for (int u = 0; u < NW; u++) {
            const int q = tid + 256 * u;
            if (q < 3 * WPL) cw[q] = L.win[u];
        }
    };
    auto comp_v = [&](int zz, const VLoad &L) {
#pragma unroll
        for (int u = 0; u < NV; u++) {
            const int q = tid + 256 * u;
            if (q >= VPL) continue;
            double out = 0.0;
            if (L.cl[u] >= 0) {
                const int gx = x0 - 1 + q % FI_VX, gy = y0 - 1 + q / FI_VX;
                const int base = (FI_WY + (gy >> 1) - wy0) * FI_WX + (gx >> 1) - wx0;  // the anchor, window plane 1
                const int c0 = L.cl[u] * a.ke;
                double acc = 0.0;
                for (int e0 = 0; e0 < a.ke; e0 += 4) {
                    double cv[4], wv[4];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        cv[e] = sval[c0 + e0 + e];
                        wv[e] = cw[base + soff[c0 + e0 + e]];
                    }
#pragma unroll
                    for (int e = 0; e < 4; e++) acc = fma(cv[e], wv[e], acc);
                }
                out = L.base[u] + acc;
            }
            vr[(zz + 3) % 3][q] = out;
        }
    };

    VLoad L;
    // prologue: v planes z0-1 and z0
    load_v(z0 - 1, L);
    store_win(L);
    __syncthreads();
    comp_v(z0 - 1, L);
    __syncthreads();
    load_v(z0, L);
    store_win(L);
    __syncthreads();
    comp_v(z0, L);
    __syncthreads();
    for (int z = z0; z < z1; z++) {
        // loads of v plane z+1 and of the Jacobi rows of plane z
        load_v(z + 1, L);
        uint32_t w[NJ][CW];
        double fb[NJ], db[NJ];
#pragma unroll
        for (int u = 0; u < NJ; u++) {
            const int q = tid + 256 * u;
            const int gx = x0 + q % FI_TX, gy = y0 + q / FI_TX;
            const bool in = q < TPL && gx < a.fx && gy < a.fy;
            const int64_t p = in ? (int64_t)z * plane + (int64_t)gy * a.fx + gx : 0;
#pragma unroll
            for (int c = 0; c < CW; c++) w[u][c] = a.codes[p * CW + c];
            fb[u] = in ? a.f[p] : 0.0;
            db[u] = in ? dget(p) : 0.0;
        }
        store_win(L);
        __syncthreads();
        comp_v(z + 1, L);  // over v plane z-2 (read by the Jacobi rows of z-1)
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NJ; u++) {
            const int q = tid + 256 * u;
            const int lx = q % FI_TX, ly = q / FI_TX;
            const int gx = x0 + lx, gy = y0 + ly;
            if (q >= TPL || gx >= a.fx || gy >= a.fy) continue;
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < KM; k++) {
                const uint32_t code = (w[u][(k * VB) >> 5] >> ((k * VB) & 31)) & MASK;
                const double xv = vr[(z + a.adz[k] + 3) % 3][(ly + 1 + a.ady[k]) * FI_VX + lx + 1 + a.adx[k]];
                const double f0 = fma(stab[code], xv, acc);
                acc = k < a.K ? f0 : acc;
            }
            const double xr = vr[z % 3][(ly + 1) * FI_VX + lx + 1];
            a.out[(int64_t)z * plane + (int64_t)gy * a.fx + gx] = xr + db[u] * (fb[u] - acc);  // DIA JACOBI
        }
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

// Grid-transfer classes of P (rows on the fine grid, is_r = false) or R (rows
// on the coarse grid) for 2 x 2 x 2 boxes; false if an entry is not at such a
// step, the columns are not ascending, or there are more than 256 classes.
static bool build_gtc(const GpuCsr &M, bool is_r, const TransferFuse &F, DevBuf<uint8_t> &dcls,
                      DevBuf<double> &dval, DevBuf<int16_t> &doff, int &ke_out, int &nc_out) {
    const int64_t fg[3] = {F.fx, F.fy, F.fz}, cg[3] = {F.cx, F.cy, F.cz};
    std::vector<uint8_t> cls;
    std::vector<std::vector<std::pair<uint8_t, double>>> dict;
    if (!gtc_classes(M, is_r, fg, cg, cls, dict)) return false;
    const int64_t n = M.nrows;
    hipStream_t s = M.ctx->stream;
    const int C = (int)dict.size();
    int ke = 1;
    for (int c = 0; c < C; c++) ke = std::max<int>(ke, (int)dict[c].size());
    const int gran = is_r ? 8 : 4;  // the kernels' load groups
    ke = (ke + gran - 1) / gran * gran;
    if ((int64_t)C * ke > F_DMAX) return false;
    // entries as the kernels' LDS positions; padding: +0.0 at the anchor itself
    // (after the row's entries: a +0.0 term leaves the accumulator unchanged)
    auto pack = [&](int sl) {
        if (is_r) return fr_pack(sl % 4 - 1, (sl / 4) % 4 - 1, sl / 16 - 1);
        return fi_pack(sl % 3 - 1, (sl / 3) % 3 - 1, sl / 9 - 1);
    };
    const int16_t centre = (int16_t)(is_r ? fr_pack(0, 0, 0) : fi_pack(0, 0, 0));
    std::vector<double> hv((size_t)C * ke, 0.0);
    std::vector<int16_t> ho((size_t)C * ke, centre);
    for (int c = 0; c < C; c++)
        for (size_t k = 0; k < dict[c].size(); k++) {
            hv[(size_t)c * ke + k] = dict[c][k].second;
            ho[(size_t)c * ke + k] = (int16_t)pack(dict[c][k].first);
        }
    dcls.resize(n);
    dval.resize(hv.size());
    doff.resize(ho.size());
    FAMG_CHECK_HIP(hipMemcpyAsync(dcls.get(), cls.data(), n, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(dval.get(), hv.data(), hv.size() * 8, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(doff.get(), ho.data(), ho.size() * 2, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    ke_out = ke;
    nc_out = C;
    return true;
}

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
    F->pre = build_gtc(R->m, true, *F, F->rcls, F->rval, F->roff, F->rke, F->rnc);
    auto *D = dynamic_cast<DiagOp *>(L.S.get());
    F->post = D && build_gtc(P->m, false, *F, F->pcls, F->pval, F->poff, F->pke, F->pnc);
    if (F->pre || F->post) L.fuse = F;
}

bool fuse_has_pre(const MgLevel &L) { return L.fuse && L.fuse->pre; }
bool fuse_has_post(const MgLevel &L) { return L.fuse && L.fuse->post; }

static void fuse_common(FuseArgs &a, const TransferFuse &F, const GpuCsr &m) {
    a.codes = m.dia_codes.get();
    a.vtab = m.dia_vtab.get();
    a.ntab = (int)m.dia_ntab;
    a.K = F.K;
    std::memcpy(a.adx, F.adx, 32);
    std::memcpy(a.ady, F.ady, 32);
    std::memcpy(a.adz, F.adz, 32);
    a.fx = F.fx; a.fy = F.fy; a.fz = F.fz;
    a.cx = F.cx; a.cy = F.cy; a.cz = F.cz;
}

// f_c = R (f - A x): x = the iterate, or (x null) the folded zero-guess iterate d*f
void fuse_resid_restrict(const TransferFuse &F, const GpuCsr &m, const double *f, const double *x,
                         const DiagOp *D, double *fc, hipStream_t s) {
    FuseArgs a{};
    fuse_common(a, F, m);
    a.f = f;
    a.x = x;
    const bool dc = D && D->dcode.get();
    if (!x) {
        FAMG_REQUIRE(D, AMG_ERR_INVALID, "fused restriction: folded step without a diagonal");
        a.dc = D->dcode.get();
        a.dt = D->dtab.get();
        a.d = D->d.get();
    }
    a.cls = F.rcls.get();
    a.cval = F.rval.get();
    a.coff = F.roff.get();
    a.ke = F.rke;
    a.nce = F.rke * F.rnc;
    a.out = fc;
    a.ntx = (int)ceil_div(F.cx, FR_CTX);
    a.nty = (int)ceil_div(F.cy, FR_CTY);
    a.zchunk = 8;
    const int nch = (int)ceil_div(F.cz, a.zchunk);
    const int64_t n = (int64_t)F.fx * F.fy * F.fz, nc = (int64_t)F.cx * F.cy * F.cz;
    // bytes: A's codes, f (and d's codes) or x, the classes, f_c written
    if (g_launch_log)
        log_launch("fuse_resid_restrict", SPMV_KERNEL_DIA, x ? SPMV_RESID : SPMV_RESID0, n,
                   4 * (int64_t)m.dia_cw * n + 8 * n + (x ? 8 * n : (dc ? 1 : 8) * n) + nc + 8 * nc);
    const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * nch)), block(256);
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
    fuse_common(a, F, m);
    a.f = f;
    a.x = x;
    a.dc = D.dcode.get();
    a.dt = D.dtab.get();
    a.d = D.d.get();
    a.cls = F.pcls.get();
    a.cval = F.pval.get();
    a.coff = F.poff.get();
    a.ke = F.pke;
    a.nce = F.pke * F.pnc;
    a.vc = vc;
    a.out = out;
    a.ntx = (int)ceil_div(F.fx, FI_TX);
    a.nty = (int)ceil_div(F.fy, FI_TY);
    a.zchunk = 16;
    const int nch = (int)ceil_div(F.fz, a.zchunk);
    const int64_t n = (int64_t)F.fx * F.fy * F.fz, nc = (int64_t)F.cx * F.cy * F.cz;
    const bool dc = a.dc != nullptr;
    // bytes: classes, v_c, f, d (codes), x (ADD), A's codes, out written
    if (g_launch_log)
        log_launch("fuse_interp_jacobi", SPMV_KERNEL_DIA, x ? SPMV_ADD : SPMV_ADD0, n,
                   n + 8 * nc + 8 * n + (dc ? 1 : 8) * n + (x ? 8 * n : 0) + 4 * (int64_t)m.dia_cw * n + 8 * n);
    const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * nch)), block(256);
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
