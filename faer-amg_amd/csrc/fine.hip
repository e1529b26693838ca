// fine.hip -- the fine level of a box hierarchy whose operator is the constant
// 7-point stencil (C2: A_0 of the 256^3 Laplacian), its interpolation and
// post-smoothing as ONE marching kernel.
//
// The cycle's last two fine launches (multigrid.rs:349-350 and 361-369, the
// zero-guess step folded: v = d f + P v_c, then one Jacobi step
// z = v + d (f - A v)) stream f and v_c in, v out, then v and f in again and z
// out: 704 MB per cycle at 256^3.  v is an intermediate: computed on the fly per
// fine plane (with its one-point x/y halo) and kept in an LDS ring of planes, it
// never reaches HBM -- f, v_c and z cross it once, 285 MB.
//
// k_fine_interp_jacobi: a workgroup takes a 64 x 16 fine (x, y) tile through a
// run of jper planes (one round of workgroups over the chip).  Per plane z:
//   v(z + 1) on the 66 x 18 window: d f + the grid-transfer class walk of P's
//     row over the coarse window (gtc.hip's dictionary in LDS, the coarse
//     planes in a ring of four slots), into the v ring (slot (z + 1) & 3);
//   barrier;
//   z(z) = v + d (f - A v) from the v ring (planes z - 1, z, z + 1), the row's
//     own v and f from registers.
// f and the class ids of plane z + 3 and the coarse plane v(z + 3) adds are
// fetched into registers while plane z is summed (two planes in flight).  Every sum is the unfused kernels' fma
// chain over the same operands (k_gtc_interp ADD0 with a one-value d;
// spmv_dia_kernel's constant 7-point JACOBI), so z is bitwise the two-launch
// result (test_fine_fused_bitwise).
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include "famg.hpp"

namespace famg {

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef double dbl2u_t __attribute__((ext_vector_type(2), aligned(8)));  // 8-B aligned 16-B loads

constexpr int FP_TX = 64, FP_TY = 16;                                            // fine tile (x, y)
constexpr int FP_VX = FP_TX + 2, FP_VY = FP_TY + 2, FP_VPL = FP_VX * FP_VY;      // v window 66 x 18
constexpr int FP_CX = FP_TX / 2 + 4, FP_CY = FP_TY / 2 + 4, FP_CPL = FP_CX * FP_CY;  // coarse window 36 x 12
constexpr int FP_PF = (FP_VPL + 255) / 256;                                      // window points per lane (5)
constexpr int FP_CPF = (FP_CPL + 255) / 256;                                     // coarse points per lane (2)
constexpr int FP_DMAX = 2048;                                                    // P dictionary entries in LDS

struct FinePjArgs {
    const uint8_t *cls;    // P's class id per fine row (gtc.hip)
    const uint16_t *dict;  // nclass x ke entries: value index << 8 | slot
    const double *vtab;
    int ke, nce, ntab;
    int nx, ny, nz;  // fine grid
    int cx, cy, cz;  // coarse grid
    int ntx, nty, jper;
    const double *vc;  // coarse correction v_c
    const double *f;   // fine rhs
    double *out;       // z
    double dk;         // the one value of the Jacobi diagonal d
    double cst[7];     // A's interior stencil, ascending offsets (z-, y-, x-, 0, x+, y+, z+)
};

// coarse plane Z of the tile's window (0.0 outside the coarse grid) into registers
__device__ __forceinline__ void fp_coarse_fetch(const FinePjArgs &a, int cwx0, int cwy0, int Z, double (&v)[FP_CPF]) {
    const int64_t cpl = (int64_t)a.cx * a.cy;
#pragma unroll
    for (int u = 0; u < FP_CPF; u++) {
        const int p = threadIdx.x + 256 * u;
        const int X = cwx0 + p % FP_CX, Y = cwy0 + p / FP_CX;
        const bool in = p < FP_CPL && (unsigned)X < (unsigned)a.cx && (unsigned)Y < (unsigned)a.cy &&
                        (unsigned)Z < (unsigned)a.cz;
        v[u] = in ? a.vc[(int64_t)Z * cpl + (int64_t)Y * a.cx + X] : 0.0;
    }
}

__device__ __forceinline__ void fp_coarse_store(double *cring, int Z, const double (&v)[FP_CPF]) {
#pragma unroll
    for (int u = 0; u < FP_CPF; u++) {
        const int p = threadIdx.x + 256 * u;
        if (p < FP_CPL) cring[(Z & 3) * FP_CPL + p] = v[u];
    }
}

// f, P's class ids and v of one fine plane at a lane's window points
struct FpSet {
    double F[FP_PF], V[FP_PF];
    int C[FP_PF];
};

__global__ __launch_bounds__(256) void k_fine_interp_jacobi(FinePjArgs a) {
    __shared__ double vring[4 * FP_VPL];
    __shared__ double cring[4 * FP_CPL];
    __shared__ uint16_t sd[FP_DMAX];
    __shared__ double st[256];
    __shared__ int16_t lut[4][27];  // [Zc & 3][slot]: coarse ring offset of step (dx, dy, dz)
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int x0 = (txy % a.ntx) * FP_TX, y0 = (txy / a.ntx) * FP_TY;
    const int zb = chunk * a.jper, ze = min(zb + a.jper, a.nz);
    const int cwx0 = (x0 >> 1) - 2, cwy0 = (y0 >> 1) - 2;
    const int64_t fpl = (int64_t)a.nx * a.ny;

    // the lane's window points q = tid + 256 u: (gx, gy) = (x0 - 1 + q % 66, y0 - 1 + q / 66)
    int gxq[FP_PF], gyq[FP_PF], cb[FP_PF];
    bool inq[FP_PF], jac[FP_PF];
#pragma unroll
    for (int u = 0; u < FP_PF; u++) {
        const int q = tid + 256 * u, wx = q % FP_VX, wy = q / FP_VX;
        gxq[u] = x0 - 1 + wx;
        gyq[u] = y0 - 1 + wy;
        inq[u] = q < FP_VPL && (unsigned)gxq[u] < (unsigned)a.nx && (unsigned)gyq[u] < (unsigned)a.ny;
        jac[u] = inq[u] && wx >= 1 && wx <= FP_TX && wy >= 1 && wy <= FP_TY;
        cb[u] = inq[u] ? ((gyq[u] >> 1) - cwy0) * FP_CX + (gxq[u] >> 1) - cwx0 : 0;
    }
    // f and the class ids of fine plane z at the lane's window points (0 outside the grid)
    auto fetch = [&](int z, double (&F)[FP_PF], int (&C)[FP_PF]) {
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            const bool in = inq[u] && (unsigned)z < (unsigned)a.nz;
            const int64_t i = in ? (int64_t)z * fpl + (int64_t)gyq[u] * a.nx + gxq[u] : 0;
            F[u] = in ? a.f[i] : 0.0;
            C[u] = in ? (int)a.cls[i] : 0;
        }
    };
    // v = d f + P v_c of fine plane z at the window points (k_gtc_interp's ADD0 sum)
    auto interp = [&](int z, const double (&F)[FP_PF], const int (&C)[FP_PF], double (&V)[FP_PF]) {
        const bool zin = (unsigned)z < (unsigned)a.nz;
        const int16_t *lz = lut[(z >> 1) & 3];
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            double v = 0.0;
            if (zin && inq[u]) {
                const uint16_t *e = sd + C[u] * a.ke;
                double acc = 0.0;
                for (int k = 0; k < a.ke; k += 4) {
                    double cv[4], w[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint16_t c = e[k + j];
                        cv[j] = st[c >> 8];
                        w[j] = cring[cb[u] + lz[c & 255]];
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) acc = fma(cv[j], w[j], acc);
                }
                v = a.dk * F[u] + acc;  // d*b (vec_mul's product) + P v_c
            }
            V[u] = v;
            if (tid + 256 * u < FP_VPL) vring[(z & 3) * FP_VPL + tid + 256 * u] = v;
        }
    };

    // the dictionary, value table and ring lookup
    for (int b = tid; b < a.nce; b += 256) sd[b] = a.dict[b];
    if (tid < a.ntab) st[tid] = a.vtab[tid];
    if (tid < 4 * 27) {
        const int r = tid / 27, s = tid % 27;
        const int dz = s / 9 - 1, dy = (s / 3) % 3 - 1, dx = s % 3 - 1;
        lut[r][s] = (int16_t)(((r + dz) & 3) * FP_CPL + dy * FP_CX + dx);
    }
    // coarse planes zb/2 - 2 .. zb/2 + 1 (those of v(zb - 1) .. v(zb + 1); zb is even)
    const int Zb = zb >> 1;
    for (int Z = Zb - 2; Z <= Zb + 1; Z++) {
        double cv[FP_CPF];
        fp_coarse_fetch(a, cwx0, cwy0, Z, cv);
        fp_coarse_store(cring, Z, cv);
    }
    // register sets of four consecutive planes (set = plane mod 4, renamed by
    // unrolling): at plane z the Jacobi sum reads set z, v(z + 1) is computed
    // from set z + 1, set z + 2 is in flight and set z + 3 is issued -- f and
    // the class ids arrive two planes after their loads are issued
    FpSet S0, S1, S2, S3;
    fetch(zb - 1, S3.F, S3.C);
    fetch(zb, S0.F, S0.C);
    __syncthreads();
    interp(zb - 1, S3.F, S3.C, S3.V);  // plane zb - 1: only its ring slot is read
    interp(zb, S0.F, S0.C, S0.V);      // plane zb: ring slot and (registers) the row's own v
    fetch(zb + 1, S1.F, S1.C);
    fetch(zb + 2, S2.F, S2.C);
    // the coarse plane v(zb + 2) adds, stored at the first step (its slot held zb/2 - 2)
    int cmax = Zb + 2;
    bool cpend = true;
    double cp[FP_CPF];
    fp_coarse_fetch(a, cwx0, cwy0, cmax, cp);
    __syncthreads();  // the prologue's reads of plane zb/2 - 2 before its slot is reused

    auto step = [&](int z, FpSet &sz, FpSet &s1, FpSet &s3) {
        interp(z + 1, s1.F, s1.C, s1.V);  // v(z + 1)
        if (cpend) fp_coarse_store(cring, cmax, cp);  // the plane v(z + 2) adds (slot of cmax - 4: unread)
        cpend = false;
        // issued now: f / classes of plane z + 3, the coarse plane v(z + 3) adds
        if (z + 3 <= ze) fetch(z + 3, s3.F, s3.C);
        if (((z + 3) >> 1) + 1 > cmax) {
            cmax++;
            fp_coarse_fetch(a, cwx0, cwy0, cmax, cp);
            cpend = true;
        }
        __syncthreads();  // v(z + 1) in the ring
        // z(z) = v + d (f - A v): spmv_dia_kernel's constant 7-point JACOBI sum
        const double *vm = vring + ((z - 1) & 3) * FP_VPL, *v0 = vring + (z & 3) * FP_VPL,
                     *vp = vring + ((z + 1) & 3) * FP_VPL;
        const bool zlo = z > 0, zhi = z < a.nz - 1;
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            if (!jac[u]) continue;
            const int q = tid + 256 * u, gx = gxq[u], gy = gyq[u];
            const double y[7] = {vm[q], v0[q - FP_VX], v0[q - 1], sz.V[u], v0[q + 1], v0[q + FP_VX], vp[q]};
            const bool in[7] = {zlo, gy > 0, gx > 0, true, gx + 1 < a.nx, gy < a.ny - 1, zhi};
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) acc = fma(a.cst[k], in[k] ? y[k] : 0.0, acc);
            a.out[(int64_t)z * fpl + (int64_t)gy * a.nx + gx] = sz.V[u] + a.dk * (sz.F[u] - acc);
        }
    };
    for (int z = zb; z < ze; z += 4) {
        step(z, S0, S1, S3);
        if (z + 1 < ze) step(z + 1, S1, S2, S0);
        if (z + 2 < ze) step(z + 2, S2, S3, S1);
        if (z + 3 < ze) step(z + 3, S3, S0, S2);
    }
}


// k_fine_resid_restrict: the fine residual from the zero guess (RESID0,
// multigrid.rs:341-342 with the first Jacobi step folded: r = f - A (d f)) and
// the restriction f_c = R r with the next level's first step d_c f_c (SETDF) in
// one marching launch -- r never reaches HBM (f in, f_c and d_c f_c out: 168 MB
// instead of 440 MB at 256^3).  A workgroup takes a 32 x 8 coarse tile through a
// run of jper coarse planes, walking the fine planes p = 2 Zb - 1 .. 2 Ze once:
//   r(p) on the 68 x 18 fine window (row pairs, f gathered as
//   spmv_dia_kernel's constant 7-point RESID0 does) into one of two LDS slots;
//   barrier;
//   every coarse row adds the entries of its R row that lie in plane p to the
//   fma chain of the coarse plane they belong to (p = 2Z - 1, 2Z, 2Z + 1,
//   2Z + 2: two chains in flight per row); a chain is complete at p = 2Z + 2
//   (then its +0.0 padding terms, as the grid-transfer kernel adds them).
// R's entries ascend in (dz, dy, dx), so the chain is k_gtc_restrict_march's, term
// for term: f_c and d_c f_c are bitwise the two-launch result.
constexpr int FR_TX = 32, FR_TY = 8;                                  // coarse tile
constexpr int FR_WX = 2 * FR_TX + 4, FR_WY = 2 * FR_TY + 2;           // r window 68 x 18 (pairs aligned)
constexpr int FR_WPL = FR_WX * FR_WY, FR_NP = FR_WPL / 2;             // 612 row pairs per plane
constexpr int FR_PP = (FR_NP + 255) / 256;                            // pairs per lane (3)
constexpr int FR_DMAX = 4096;

struct FineRrArgs {
    const uint8_t *cls;    // R's class per coarse row
    const uint16_t *dict;  // nclass x ke entries: value index << 8 | slot
    const double *vtab;
    const uint8_t *kdz;    // per class: first entry of dz = -1, 0, 1, 2, and the real entry count
    int ke, nce, ntab, nclass;
    int nx, ny, nz, cx, cy, cz;
    int ntx, nty, jper;
    const double *f;
    double *fc, *dfc;
    const uint8_t *dcc;    // the coarse level's d: codes into dtc, or plain dpc, or one value dkc
    const double *dtc, *dpc;
    double dkc;
    int dmode;             // 0 one value, 1 codes, 2 plain
    double dk;             // the fine level's one-value d
    double cst[7];
};

// x operands of rows (r, r + 1) at column c (dia_gx2) and the x run x[c .. c + 3] (dia_gx4)
__device__ __forceinline__ void fr_gx2(const double *x, int64_t c, int64_t n, double &x0, double &x1) {
    const int64_t cc = min(max(c, (int64_t)0), n - 2);
    const dbl2_t v = *reinterpret_cast<const dbl2u_t *>(x + cc);
    x0 = c > n - 2 ? v.y : v.x;
    x1 = c < 0 ? v.x : v.y;
}
__device__ __forceinline__ void fr_gx4(const double *x, int64_t c, int64_t n, double (&v)[4]) {
    const int64_t p0 = min(max(c, (int64_t)0), n - 2), p1 = min(max(c + 2, (int64_t)0), n - 2);
    const dbl2_t q0 = *reinterpret_cast<const dbl2u_t *>(x + p0);
    const dbl2_t q1 = *reinterpret_cast<const dbl2u_t *>(x + p1);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t t = c + j;
        v[j] = t == p0 ? q0.x : t == p0 + 1 ? q0.y : t == p1 ? q1.x : q1.y;
    }
}

__global__ __launch_bounds__(256) void k_fine_resid_restrict(FineRrArgs a) {
    __shared__ __attribute__((aligned(16))) double rs[2 * FR_WPL];
    __shared__ uint16_t sd[FR_DMAX];
    __shared__ double st[256];
    __shared__ double sdt[256];
    __shared__ int16_t lut[16];
    extern __shared__ uint8_t skdz[];  // nclass x 5
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int X0 = (txy % a.ntx) * FR_TX, Y0 = (txy / a.ntx) * FR_TY;
    const int Zb = chunk * a.jper, Ze = min(Zb + a.jper, a.cz);
    const int64_t fpl = (int64_t)a.nx * a.ny, n = fpl * a.nz, cpl = (int64_t)a.cx * a.cy;
    const int wx0 = 2 * X0 - 2, wy0 = 2 * Y0 - 1;  // fine window origin (x even: row pairs aligned)
    for (int b = tid; b < a.nce; b += 256) sd[b] = a.dict[b];
    for (int b = tid; b < 5 * a.nclass; b += 256) skdz[b] = a.kdz[b];
    if (tid < a.ntab) st[tid] = a.vtab[tid];
    if (a.dmode == 1) sdt[tid] = a.dtc[tid];
    if (tid < 16) lut[tid] = (int16_t)(((tid >> 2) - 1) * FR_WX + (tid & 3) - 1);
    // the lane's row pairs of the window: pair q -> (wx, wy) = (2 (q % 34), q / 34)
    int gxp[FR_PP], gyp[FR_PP];
    bool inp[FR_PP];
#pragma unroll
    for (int u = 0; u < FR_PP; u++) {
        const int q = tid + 256 * u;
        gxp[u] = wx0 + 2 * (q % (FR_WX / 2));
        gyp[u] = wy0 + q / (FR_WX / 2);
        inp[u] = q < FR_NP && (unsigned)gxp[u] < (unsigned)a.nx && (unsigned)gyp[u] < (unsigned)a.ny;
    }
    // the lane's coarse row
    const int lx = tid % FR_TX, ly = tid / FR_TX, X = X0 + lx, Y = Y0 + ly;
    const bool live = X < a.cx && Y < a.cy;
    const int base = (2 * ly + 1) * FR_WX + 2 * lx + 2;  // window position of the anchor (2X, 2Y)
    double acc[2] = {0.0, 0.0}, ra[2] = {0.0, 0.0};
    int cl[2] = {0, 0};
    __syncthreads();
    for (int p = 2 * Zb - 1; p <= 2 * Ze; p++) {
        // r(p) = f - A (d f) on the window's row pairs: spmv_dia_kernel<DIA_RESID0_DK, CST>
        double rr[FR_PP][2];
        {
            double xs[FR_PP][4][2], xq[FR_PP][4];
            const bool pin = (unsigned)p < (unsigned)a.nz;
#pragma unroll
            for (int u = 0; u < FR_PP; u++) {
                const int64_t i = (pin && inp[u]) ? (int64_t)p * fpl + (int64_t)gyp[u] * a.nx + gxp[u] : 0;
                fr_gx2(a.f, i - fpl, n, xs[u][0][0], xs[u][0][1]);
                fr_gx2(a.f, i - a.nx, n, xs[u][1][0], xs[u][1][1]);
                fr_gx4(a.f, i - 1, n, xq[u]);
                fr_gx2(a.f, i + a.nx, n, xs[u][2][0], xs[u][2][1]);
                fr_gx2(a.f, i + fpl, n, xs[u][3][0], xs[u][3][1]);
            }
            const bool zlo = p > 0, zhi = p < a.nz - 1;
#pragma unroll
            for (int u = 0; u < FR_PP; u++) {
                const double b0 = xq[u][1], b1 = xq[u][2];  // f of the pair (the epilogue's b)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) xs[u][i][j] = a.dk * xs[u][i][j];
#pragma unroll
                for (int j = 0; j < 4; j++) xq[u][j] = a.dk * xq[u][j];
                const int gx = gxp[u], gy = gyp[u];
                const bool ylo = gy > 0, yhi = gy < a.ny - 1, xlo = gx > 0, xhi = gx + 2 < a.nx;
                double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
                for (int k = 0; k < 7; k++) {
                    const double y0 = k < 2 ? xs[u][k][0] : k < 5 ? xq[u][k - 2] : xs[u][k - 3][0];
                    const double y1 = k < 2 ? xs[u][k][1] : k < 5 ? xq[u][k - 1] : xs[u][k - 3][1];
                    const bool in = k == 0 ? zlo : k == 1 ? ylo : k == 5 ? yhi : k == 6 ? zhi : true;
                    const bool in0 = in && (k != 2 || xlo), in1 = in && (k != 4 || xhi);
                    acc0 = fma(a.cst[k], in0 ? y0 : 0.0, acc0);
                    acc1 = fma(a.cst[k], in1 ? y1 : 0.0, acc1);
                }
                const bool ok = pin && inp[u];
                rr[u][0] = ok ? b0 - acc0 : 0.0;
                rr[u][1] = ok ? b1 - acc1 : 0.0;
            }
        }
        double *rp = rs + (p & 1) * FR_WPL;
#pragma unroll
        for (int u = 0; u < FR_PP; u++) {
            const int q = tid + 256 * u;
            if (q < FR_NP) *reinterpret_cast<dbl2_t *>(rp + 2 * q) = dbl2_t{rr[u][0], rr[u][1]};
        }
        __syncthreads();
        // the plane's terms of the two coarse chains it belongs to
        if (live) {
            // p odd: Z = (p + 1) / 2 starts (dz = -1), Z - 1 continues (dz = +1);
            // p even: Z = p / 2 continues (dz = 0), Z - 1 ends (dz = +2, then the padding)
            const int Zn = (p + 1) >> 1, Zo = Zn - 1;
            const int gn = (p & 1) ? 0 : 1, go = (p & 1) ? 2 : 3;
            for (int w = 0; w < 2; w++) {
                const int Z = w == 0 ? Zn : Zo, g = w == 0 ? gn : go;
                if (Z < Zb || Z >= Ze) continue;
                const int s = Z & 1;
                if (g == 0) {
                    cl[s] = a.cls[(int64_t)Z * cpl + (int64_t)Y * a.cx + X];
                    acc[s] = 0.0;
                }
                const uint8_t *kz = skdz + 5 * cl[s];
                const uint16_t *e = sd + cl[s] * a.ke;
                double ac = acc[s];
                for (int k = kz[g]; k < kz[g + 1]; k++) {
                    const uint16_t c = e[k];
                    ac = fma(st[c >> 8], rp[base + lut[c & 15]], ac);
                }
                if (g == 1) ra[s] = rp[base];  // r at the anchor: the padding entries' operand
                if (g == 3) {
                    for (int k = kz[4]; k < a.ke; k++) ac = fma(st[e[k] >> 8], ra[s], ac);
                    const int64_t J = (int64_t)Z * cpl + (int64_t)Y * a.cx + X;
                    a.fc[J] = ac;
                    const double dd = a.dmode == 0 ? a.dkc : a.dmode == 1 ? sdt[a.dcc[J]] : a.dpc[J];
                    a.dfc[J] = dd * ac;  // vec_mul(_coded)'s product
                }
                acc[s] = ac;
            }
        }
    }
}

// ------------------------------------------------------------ host side

// workgroups of k_fine_interp_jacobi per CU (cached)
static int fine_pj_occupancy() {
    static std::once_flag once;
    static int n = 1;
    std::call_once(once, [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k_fine_interp_jacobi, 256, 0) == hipSuccess && v >= 1)
            n = v;
        else
            (void)hipGetLastError();
    });
    return n;
}

// workgroups of k_fine_resid_restrict per CU with dyn bytes of class table (cached)
static int fine_rr_occupancy(size_t dyn) {
    static std::mutex mu;
    static std::unordered_map<size_t, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dyn);
    if (it != cache.end()) return it->second;
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k_fine_resid_restrict, 256, dyn) != hipSuccess || v < 1) {
        (void)hipGetLastError();
        v = 1;
    }
    cache[dyn] = v;
    return v;
}

bool fine_resid_restrict_ok(const GpuCsr &A, const GpuCsr &R, const SpmvEpi &epi, const SpmvEpi &epic) {
    if (flag(FLAG_FINE_FUSE) == 0 || !dia7_cst_dk(A, epi)) return false;
    if (!R.gtc_on || !R.gtc_r || R.rframe.on() || R.cframe.on() || R.gtc_nce > FR_DMAX || R.gtc_ntab > 256 ||
        !R.gtc_kdz.get() || R.gtc_ke % 8 != 0)
        return false;
    if (!epic.y2 || !(epic.dk != 0.0 || epic.dc || epic.d)) return false;
    for (int q = 0; q < 3; q++)
        if (R.gtc_fg[q] != A.dia_cst_n[q] || R.gtc_cg[q] != (R.gtc_fg[q] + 1) / 2) return false;
    return A.nrows == R.ncols && R.nrows == R.gtc_cg[0] * R.gtc_cg[1] * R.gtc_cg[2];
}

void fine_resid_restrict(const GpuCsr &A, const GpuCsr &R, const double *f, double dk, double *fc,
                         const SpmvEpi &epic, hipStream_t s) {
    FineRrArgs a{};
    a.cls = R.gtc_cls.get();
    a.dict = R.gtc_dict.get();
    a.vtab = R.gtc_vtab.get();
    a.kdz = R.gtc_kdz.get();
    a.ke = R.gtc_ke;
    a.nce = R.gtc_nce;
    a.ntab = R.gtc_ntab;
    a.nclass = R.gtc_nclass;
    a.nx = (int)R.gtc_fg[0]; a.ny = (int)R.gtc_fg[1]; a.nz = (int)R.gtc_fg[2];
    a.cx = (int)R.gtc_cg[0]; a.cy = (int)R.gtc_cg[1]; a.cz = (int)R.gtc_cg[2];
    a.ntx = (int)ceil_div(a.cx, FR_TX);
    a.nty = (int)ceil_div(a.cy, FR_TY);
    a.f = f;
    a.fc = fc;
    a.dfc = epic.y2;
    // the coarse level's d as the SETDF epilogue reads it (k_gtc_restrict_march)
    if (epic.dc && epic.dk != 0.0 && flag(FLAG_DIA_DK) != 0) {
        a.dmode = 0;
        a.dkc = epic.dk;
    } else if (epic.dc) {
        a.dmode = 1;
        a.dcc = epic.dc;
        a.dtc = epic.dt;
    } else {
        a.dmode = 2;
        a.dpc = epic.d;
    }
    a.dk = dk;
    for (int k = 0; k < 7; k++) a.cst[k] = A.dia_cst_v[k];
    const size_t dyn = (size_t)5 * a.nclass;
    const int64_t ntxy = (int64_t)a.ntx * a.nty;
    const int64_t want = (int64_t)fine_rr_occupancy(dyn) * std::max(A.ctx ? A.ctx->num_cus : 256, 1);
    a.jper = (int)std::max<int64_t>(1, ceil_div((int64_t)a.cz * ntxy, want));
    if (flag(FLAG_FINE_FUSE) > 1) a.jper = (int)std::max<int64_t>(1, flag(FLAG_FINE_FUSE) / 2);
    const dim3 grid((unsigned)(ntxy * ceil_div(a.cz, a.jper)));
    k_fine_resid_restrict<<<grid, dim3(256), dyn, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
    const int64_t n = A.nrows, nc = R.nrows;
    // f in once, f_c and d_c f_c out, R's class ids (1 B per coarse row; a coded d_c: 1 B more);
    // CSR-equivalent: A's RESID0 (x, b = f; r out; d gathered) + R's SETDF
    log_launch("fine-rr", SPMV_KERNEL_DIA, -1, n, 8 * n + 16 * nc + nc + (a.dmode == 1 ? nc : a.dmode == 2 ? 8 * nc : 0),
               (12 * A.nnz + 4 * (n + 1) + 32 * n) + (12 * R.nnz + 4 * (nc + 1) + 8 * n + 16 * nc));
}

bool fine_interp_jacobi_ok(const GpuCsr &A, const GpuCsr &P, const SpmvEpi &epi) {
    if (flag(FLAG_FINE_FUSE) == 0 || !dia7_cst_dk(A, epi)) return false;
    if (!P.gtc_on || P.gtc_r || P.rframe.on() || P.cframe.on() || P.gtc_nce > FP_DMAX || P.gtc_ke % 4 != 0 ||
        P.gtc_ntab > 256)
        return false;
    for (int q = 0; q < 3; q++)
        if (P.gtc_fg[q] != A.dia_cst_n[q] || P.gtc_cg[q] != (P.gtc_fg[q] + 1) / 2) return false;
    return A.nrows == P.nrows && P.ncols == P.gtc_cg[0] * P.gtc_cg[1] * P.gtc_cg[2];
}

void fine_interp_jacobi(const GpuCsr &A, const GpuCsr &P, const double *vc, const double *f, double dk, double *out,
                        hipStream_t s) {
    FinePjArgs a{};
    a.cls = P.gtc_cls.get();
    a.dict = P.gtc_dict.get();
    a.vtab = P.gtc_vtab.get();
    a.ke = P.gtc_ke;
    a.nce = P.gtc_nce;
    a.ntab = P.gtc_ntab;
    a.nx = (int)P.gtc_fg[0]; a.ny = (int)P.gtc_fg[1]; a.nz = (int)P.gtc_fg[2];
    a.cx = (int)P.gtc_cg[0]; a.cy = (int)P.gtc_cg[1]; a.cz = (int)P.gtc_cg[2];
    a.ntx = (int)ceil_div(a.nx, FP_TX);
    a.nty = (int)ceil_div(a.ny, FP_TY);
    a.vc = vc;
    a.f = f;
    a.out = out;
    a.dk = dk;
    for (int k = 0; k < 7; k++) a.cst[k] = A.dia_cst_v[k];
    // one round of workgroups over the chip; an even run of planes per workgroup
    const int64_t ntxy = (int64_t)a.ntx * a.nty;
    const int64_t want = (int64_t)fine_pj_occupancy() * std::max(A.ctx ? A.ctx->num_cus : 256, 1);
    int jper = (int)std::max<int64_t>(2, ceil_div((int64_t)a.nz * ntxy, want));
    if (flag(FLAG_FINE_FUSE) > 1) jper = (int)flag(FLAG_FINE_FUSE);
    a.jper = jper + (jper & 1);
    const dim3 grid((unsigned)(ntxy * ceil_div(a.nz, a.jper)));
    k_fine_interp_jacobi<<<grid, dim3(256), 0, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
    const int64_t n = A.nrows;
    // f and z once, v_c once, the class ids (1 B per row); CSR-equivalent: P's ADD0 + A's JACOBI
    log_launch("fine-pj", SPMV_KERNEL_DIA, -1, n, 8 * n + 8 * P.ncols + 8 * n + n,
               (12 * P.nnz + 4 * (n + 1) + 8 * P.ncols + 16 * n) + (12 * A.nnz + 4 * (n + 1) + 32 * n));
}

}  // namespace famg
