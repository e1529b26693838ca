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
#include <type_traits>
#include <unordered_map>

#include "famg.hpp"

namespace famg {

// A workgroup barrier that orders LDS only: __syncthreads() also waits for every
// outstanding global load, which would drain the next planes' register prefetch
// at each plane step
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef double dbl2u_t __attribute__((ext_vector_type(2), aligned(8)));  // 8-B aligned 16-B loads

constexpr int FP_TX = 64, FP_TY = 16;                                            // fine tile (x, y)
constexpr int FP_VX = FP_TX + 2, FP_VY = FP_TY + 2, FP_VPL = FP_VX * FP_VY;      // v window 66 x 18
constexpr int FP_CX = FP_TX / 2 + 4, FP_CY = FP_TY / 2 + 4, FP_CPL = FP_CX * FP_CY;  // coarse window 36 x 12
constexpr int FP_PF = (FP_VPL + 255) / 256;                                      // window points per lane (5)
constexpr int FP_CPF = (FP_CPL + 255) / 256;                                     // coarse points per lane (2)

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
        v[u] = a.vc[in ? (int64_t)Z * cpl + (int64_t)Y * a.cx + X : 0];  // raw: the store selects
    }
}

// (the 0.0 outside the coarse grid is selected here, where the load is consumed:
// a select next to the load would make every later wait include it)
__device__ __forceinline__ void fp_coarse_store(const FinePjArgs &a, double *cring, int cwx0, int cwy0, int Z,
                                                const double (&v)[FP_CPF]) {
#pragma unroll
    for (int u = 0; u < FP_CPF; u++) {
        const int p = threadIdx.x + 256 * u;
        const int X = cwx0 + p % FP_CX, Y = cwy0 + p / FP_CX;
        const bool in = (unsigned)X < (unsigned)a.cx && (unsigned)Y < (unsigned)a.cy && (unsigned)Z < (unsigned)a.cz;
        if (p < FP_CPL) cring[(Z & 3) * FP_CPL + p] = in ? v[u] : 0.0;
    }
}

// f, P's class ids and v of one fine plane at a lane's window points
struct FpSet {
    double F[FP_PF], V[FP_PF];
    int C[FP_PF];
};

template <int KE>
__global__ __launch_bounds__(256) void k_fine_interp_jacobi(FinePjArgs a) {
    __shared__ double vring[4 * FP_VPL];
    __shared__ double cring[4 * FP_CPL];
    __shared__ double st[256];
    // P's dictionary decoded for the four coarse-ring phases: dec[r][e] = value
    // index << 16 | (int16) coarse-window offset of entry e when the row's coarse
    // plane sits in ring slot r (so a term is two LDS reads and no arithmetic)
    extern __shared__ uint32_t dec[];
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int x0 = (txy % a.ntx) * FP_TX, y0 = (txy / a.ntx) * FP_TY;
    const int zb = chunk * a.jper, ze = min(zb + a.jper, a.nz);
    const int cwx0 = (x0 >> 1) - 2, cwy0 = (y0 >> 1) - 2;
    const int64_t fpl = (int64_t)a.nx * a.ny;

    // the lane's window points q = tid + 256 u: (gx, gy) = (x0 - 1 + q % 66, y0 - 1 + q / 66);
    // po = its offset in a plane (32-bit; an in-grid point for points outside the grid)
    int cb[FP_PF], po[FP_PF], gxq[FP_PF], gyq[FP_PF];
    bool inq[FP_PF], jac[FP_PF];
#pragma unroll
    for (int u = 0; u < FP_PF; u++) {
        const int q = tid + 256 * u, wx = q % FP_VX, wy = q / FP_VX;
        gxq[u] = x0 - 1 + wx;
        gyq[u] = y0 - 1 + wy;
        inq[u] = q < FP_VPL && (unsigned)gxq[u] < (unsigned)a.nx && (unsigned)gyq[u] < (unsigned)a.ny;
        jac[u] = inq[u] && wx >= 1 && wx <= FP_TX && wy >= 1 && wy <= FP_TY;
        // (in-range coarse-window reads for points outside the grid)
        cb[u] = inq[u] ? ((gyq[u] >> 1) - cwy0) * FP_CX + (gxq[u] >> 1) - cwx0 : FP_CX + 1;
        po[u] = inq[u] ? gyq[u] * a.nx + gxq[u] : 0;
    }
    // f and the class ids of fine plane z at the lane's window points: one uniform
    // plane pointer (clamped plane) and 32-bit offsets; unconditional loads, no
    // select -- interp() zeroes v outside the grid, the Jacobi sum reads f at grid points
    auto fetch = [&](int z, double (&F)[FP_PF], int (&C)[FP_PF]) {
        const int zc = min(max(z, 0), a.nz - 1);
        const double *fz = a.f + (int64_t)zc * fpl;
        const uint8_t *cz = a.cls + (int64_t)zc * fpl;
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            F[u] = fz[po[u]];
            C[u] = (int)cz[po[u]];
        }
    };
    // v = d f + P v_c of fine plane z at the window points (k_gtc_interp's ADD0
    // sum); KE (the dictionary width) compile-time, all FP_PF x KE terms in flight
    auto interp = [&](int z, const double (&F)[FP_PF], const int (&C)[FP_PF], double (&V)[FP_PF]) {
        const bool zin = (unsigned)z < (unsigned)a.nz;
        const uint32_t *dz = dec + ((z >> 1) & 3) * a.nce;
        uint32_t e[FP_PF][KE];
#pragma unroll
        for (int u = 0; u < FP_PF; u++)
#pragma unroll
            for (int j = 0; j < KE; j += 4) {
                const uint4 q = *reinterpret_cast<const uint4 *>(dz + C[u] * KE + j);
                e[u][j] = q.x;
                e[u][j + 1] = q.y;
                e[u][j + 2] = q.z;
                e[u][j + 3] = q.w;
            }
        double cv[FP_PF][KE], w[FP_PF][KE];
#pragma unroll
        for (int u = 0; u < FP_PF; u++)
#pragma unroll
            for (int j = 0; j < KE; j++) {
                cv[u][j] = st[e[u][j] >> 16];
                w[u][j] = cring[cb[u] + (int)(int16_t)(e[u][j] & 0xffffu)];
            }
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < KE; j++) acc = fma(cv[u][j], w[u][j], acc);
            const double v = (zin && inq[u]) ? a.dk * F[u] + acc : 0.0;  // d*b (vec_mul's product) + P v_c
            V[u] = v;
            if (tid + 256 * u < FP_VPL) vring[(z & 3) * FP_VPL + tid + 256 * u] = v;
        }
    };

    // the decoded dictionary and the value table
    for (int b = tid; b < 4 * a.nce; b += 256) {
        const int r = b / a.nce, e = b - r * a.nce;
        const uint32_t c = a.dict[e], sl = c & 255u;
        const int dzs = (int)(sl / 9u) - 1, dys = (int)((sl / 3u) % 3u) - 1, dxs = (int)(sl % 3u) - 1;
        const int off = ((r + dzs) & 3) * FP_CPL + dys * FP_CX + dxs;
        dec[b] = (c >> 8) << 16 | ((uint32_t)off & 0xffffu);
    }
    if (tid < a.ntab) st[tid] = a.vtab[tid];
    // coarse planes zb/2 - 2 .. zb/2 + 1 (those of v(zb - 1) .. v(zb + 1); zb is even)
    const int Zb = zb >> 1;
    for (int Z = Zb - 2; Z <= Zb + 1; Z++) {
        double cv[FP_CPF];
        fp_coarse_fetch(a, cwx0, cwy0, Z, cv);
        fp_coarse_store(a, cring, cwx0, cwy0, Z, cv);
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
    // the coarse plane v(zb + 2) adds, stored at the first step (its slot held
    // zb/2 - 2); issued before f as in every step, so the loop's waits match
    int cmax = Zb + 2;
    double cp[FP_CPF];
    fp_coarse_fetch(a, cwx0, cwy0, cmax, cp);
    fetch(zb + 1, S1.F, S1.C);
    fetch(zb + 2, S2.F, S2.C);
    __syncthreads();  // the prologue's reads of plane zb/2 - 2 before its slot is reused

    // every step of the unrolled loop runs unconditionally (a step past ze only
    // skips its stores): a conditional step would join its loads' registers and
    // drain the prefetch at the join
    auto step = [&](int z, FpSet &sz, FpSet &s1, FpSet &s3) {
        interp(z + 1, s1.F, s1.C, s1.V);  // v(z + 1)
        fp_coarse_store(a, cring, cwx0, cwy0, cmax, cp);  // the plane v(z + 2) adds (slot of cmax - 4: unread;
                                                          // or cmax again: the same values)
        // issued now: the coarse plane v(z + 3) adds (first: it is stored one
        // plane later, and a wait for it then must not wait for the f below),
        // f / classes of plane z + 3
        // (both unconditional: a load under a branch is drained at the join)
        cmax = ((z + 3) >> 1) + 1;
        fp_coarse_fetch(a, cwx0, cwy0, cmax, cp);
        fetch(min(z + 3, ze), s3.F, s3.C);
        lds_barrier();  // v(z + 1) in the ring (the prefetches stay in flight)
        // z(z) = v + d (f - A v): spmv_dia_kernel's constant 7-point JACOBI sum
        const double *vm = vring + ((z - 1) & 3) * FP_VPL, *v0 = vring + (z & 3) * FP_VPL,
                     *vp = vring + ((z + 1) & 3) * FP_VPL;
        // (a neighbour outside the grid -- x, y or a plane past either end -- holds
        // the +0.0 interp() wrote: the constant kernel's `in ? x : 0.0` without selects)
        const bool zon = z < ze;
        double *oz = a.out + (int64_t)min(z, a.nz - 1) * fpl;
#pragma unroll
        for (int u = 0; u < FP_PF; u++) {
            if (!jac[u] || !zon) continue;
            const int q = tid + 256 * u;
            const double y[7] = {vm[q], v0[q - FP_VX], v0[q - 1], sz.V[u], v0[q + 1], v0[q + FP_VX], vp[q]};
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) acc = fma(a.cst[k], y[k], acc);
            oz[po[u]] = sz.V[u] + a.dk * (sz.F[u] - acc);
        }
    };
    for (int z = zb; z < ze; z += 4) {
        step(z, S0, S1, S3);
        step(z + 1, S1, S2, S0);
        step(z + 2, S2, S3, S1);
        step(z + 3, S3, S0, S2);
    }
}


// k_fine_resid_restrict: the fine residual from the zero guess (RESID0,
// multigrid.rs:341-342 with the first Jacobi step folded: r = f - A (d f)) and
// the restriction f_c = R r with the next level's first step d_c f_c (SETDF) in
// one marching launch -- r never reaches HBM (f in, f_c and d_c f_c out: 172 MB
// instead of 440 MB at 256^3).  A workgroup takes a 32 x 8 coarse tile through a
// run of jper coarse planes, walking the fine planes p = 2 Zb - 1 .. 2 Ze once:
//   f of each fine plane (72 x 20 window) reaches an LDS ring of four planes
//     through registers, loaded two planes ahead (16-B loads);
//   r(p) on the 68 x 18 window from the ring (row pairs, the constant 7-point
//     RESID0 sum of spmv_dia_kernel: d f at the seven neighbours, +0.0 where a
//     neighbour leaves the grid) into one of two LDS slots;
//   barrier;
//   every coarse row adds the entries of its R row that lie in plane p to the
//   fma chain of the coarse plane they belong to (p = 2Z - 1, 2Z, 2Z + 1,
//   2Z + 2: two chains in flight per row); a chain is complete at p = 2Z + 2
//   (then its +0.0 padding terms, as the grid-transfer kernel adds them).
// R's entries ascend in (dz, dy, dx), so the chain is k_gtc_restrict_march's, term
// for term: f_c and d_c f_c are bitwise the two-launch result.
constexpr int FR_TX = 32, FR_TY = 8;                                  // coarse tile
constexpr int FR_WX = 2 * FR_TX + 4, FR_WY = 2 * FR_TY + 2;           // r window 68 x 18 (x from 2 X0 - 2)
constexpr int FR_WPL = FR_WX * FR_WY, FR_NP = FR_WPL / 2;             // 612 row pairs per plane
constexpr int FR_PP = (FR_NP + 255) / 256;                            // pairs per lane (3)
constexpr int FF_WX = FR_WX + 4, FF_WY = FR_WY + 2;                   // f window 72 x 20 (x from 2 X0 - 4)
constexpr int FF_PL = FF_WX * FF_WY, FF_NU = FF_PL / 2;               // 720 16-B units per plane
constexpr int FF_PU = (FF_NU + 255) / 256;                            // units per lane (3)
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
    int dbg;               // timing experiments only (FAMG_FINE_DBG): 1 skips the R sums, 2 the residual
};

// f of fine plane p at the lane's 16-B units of the window (0.0 outside the grid)
__device__ __forceinline__ void fr_fetch(const FineRrArgs &a, int gx0, int gy0, int p, dbl2_t (&v)[FF_PU]) {
    const int64_t fpl = (int64_t)a.nx * a.ny;
#pragma unroll
    for (int u = 0; u < FF_PU; u++) {
        const int q = threadIdx.x + 256 * u;
        const int gx = gx0 + 2 * (q % (FF_WX / 2)), gy = gy0 + q / (FF_WX / 2);
        const bool in = q < FF_NU && (unsigned)gx < (unsigned)a.nx && (unsigned)gy < (unsigned)a.ny &&
                        (unsigned)p < (unsigned)a.nz;
        // an unconditional load at a clamped address, no select here: a select (or
        // a branch) next to the load makes the compiler drain every load in flight
        v[u] = *reinterpret_cast<const dbl2_t *>(a.f + (in ? (int64_t)p * fpl + (int64_t)gy * a.nx + gx : 0));
    }
}

// the 0.0 outside the grid selected where the prefetched plane is consumed
__device__ __forceinline__ void fr_store(const FineRrArgs &a, int gx0, int gy0, double *fring, int p,
                                         const dbl2_t (&v)[FF_PU]) {
#pragma unroll
    for (int u = 0; u < FF_PU; u++) {
        const int q = threadIdx.x + 256 * u;
        const int gx = gx0 + 2 * (q % (FF_WX / 2)), gy = gy0 + q / (FF_WX / 2);
        const bool in = (unsigned)gx < (unsigned)a.nx && (unsigned)gy < (unsigned)a.ny && (unsigned)p < (unsigned)a.nz;
        if (q < FF_NU) *reinterpret_cast<dbl2_t *>(fring + (p & 3) * FF_PL + 2 * q) = in ? v[u] : dbl2_t{0.0, 0.0};
    }
}

// one coarse row's fma chain and its class's position tables (registers)
struct RrChain {
    uint4 iw[4];   // per plane group: the 16 positions' value indices (bytes)
    uint2 mk;      // per plane group: 16-bit position masks
    double ac, ra;
    int npad, c;
};

__global__ __launch_bounds__(256) void k_fine_resid_restrict(FineRrArgs a) {
    __shared__ __attribute__((aligned(16))) double fring[4 * FF_PL];
    __shared__ __attribute__((aligned(16))) double rs[2 * FR_WPL];
    __shared__ double st[256];
    __shared__ double sdt[256];
    // nclass x 5 plane-group starts, the position tables, then the class ids and
    // (coded d_c) diagonal codes of the run's coarse rows (256 per plane, jper planes):
    // no global load in the plane loop waits behind the f prefetch
    extern __shared__ __attribute__((aligned(16))) uint8_t sdyn[];
    uint8_t *skdz = sdyn;
    uint8_t *stab = skdz + ((5 * a.nclass + 15) & ~15);      // 64 B per class (16-B aligned)
    uint16_t *smk = reinterpret_cast<uint16_t *>(stab + 64 * a.nclass);
    uint8_t *scl = reinterpret_cast<uint8_t *>(smk + 4 * a.nclass);
    uint8_t *sdc = scl + 256 * a.jper;
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int X0 = (txy % a.ntx) * FR_TX, Y0 = (txy / a.ntx) * FR_TY;
    const int Zb = chunk * a.jper, Ze = min(Zb + a.jper, a.cz);
    const int64_t cpl = (int64_t)a.cx * a.cy;
    const int wx0 = 2 * X0 - 2, wy0 = 2 * Y0 - 1;  // r window origin (x even: row pairs aligned)
    for (int b = tid; b < 5 * a.nclass; b += 256) skdz[b] = a.kdz[b];
    // per class and plane group: the value index of each of the 16 in-plane
    // positions (bytes) and which positions hold an entry (16-bit masks)
    for (int b = tid; b < 16 * a.nclass; b += 256) reinterpret_cast<uint32_t *>(stab)[b] = 0u;
    for (int b = tid; b < 4 * a.nclass; b += 256) smk[b] = 0;
    __syncthreads();
    for (int b = tid; b < 4 * a.nclass; b += 256) {
        const int c = b >> 2, g = b & 3;
        uint32_t m = 0;
        for (int k = a.kdz[5 * c + g]; k < a.kdz[5 * c + g + 1]; k++) {
            const uint32_t e = a.dict[c * a.ke + k], pos = e & 15u;
            stab[64 * c + 16 * g + pos] = (uint8_t)(e >> 8);
            m |= 1u << pos;
        }
        smk[b] = (uint16_t)m;
    }
    if (tid < a.ntab) st[tid] = a.vtab[tid];
    if (a.dmode == 1) sdt[tid] = a.dtc[tid];
    // the lane's row pairs of the r window: pair q -> (wx, wy) = (2 (q % 34), q / 34)
    int gxp[FR_PP], gyp[FR_PP], fo[FR_PP];
    bool inp[FR_PP];
#pragma unroll
    for (int u = 0; u < FR_PP; u++) {
        const int q = tid + 256 * u;
        const int wx = 2 * (q % (FR_WX / 2)), wy = q / (FR_WX / 2);
        gxp[u] = wx0 + wx;
        gyp[u] = wy0 + wy;
        inp[u] = q < FR_NP && (unsigned)gxp[u] < (unsigned)a.nx && (unsigned)gyp[u] < (unsigned)a.ny;
        fo[u] = q < FR_NP ? (wy + 1) * FF_WX + wx + 2 : FF_WX + 2;  // its position in the f window
    }
    // the lane's coarse row
    const int lx = tid % FR_TX, ly = tid / FR_TX, X = X0 + lx, Y = Y0 + ly;
    const bool live = X < a.cx && Y < a.cy;
    for (int Z = Zb; Z < Ze; Z++) {
        const int64_t J = live ? (int64_t)Z * cpl + (int64_t)Y * a.cx + X : 0;
        const uint8_t c = a.cls[J];
        scl[(Z - Zb) * 256 + tid] = c;
        if (a.dmode == 1) sdc[(Z - Zb) * 256 + tid] = a.dcc[J];
    }
    const int base = (2 * ly + 1) * FR_WX + 2 * lx + 2;  // window position of the anchor (2X, 2Y)
    const int p0 = 2 * Zb - 1, p1 = 2 * Ze;
    const int fgx0 = 2 * X0 - 4, fgy0 = 2 * Y0 - 2;
    {
        dbl2_t v[FF_PU];
        for (int p = p0 - 1; p <= p0 + 1; p++) {
            fr_fetch(a, fgx0, fgy0, p, v);
            fr_store(a, fgx0, fgy0, fring, p, v);
        }
    }
    dbl2_t pa[FF_PU], pb[FF_PU];  // f of planes p + 2 (even p: pa) and p + 3 in flight
    fr_fetch(a, fgx0, fgy0, p0 + 2, (p0 & 1) ? pb : pa);
    fr_fetch(a, fgx0, fgy0, p0 + 3, (p0 & 1) ? pa : pb);
    __syncthreads();

    RrChain ch[2];
    auto step = [&](int p, dbl2_t (&pn)[FF_PU], auto ph) {
        // r(p) = f - A (d f) on the window's row pairs: spmv_dia_kernel<DIA_RESID0_DK, CST>
        const double *fm = fring + ((p - 1) & 3) * FF_PL, *f0 = fring + (p & 3) * FF_PL,
                     *fp = fring + ((p + 1) & 3) * FF_PL;
        const bool pin = (unsigned)p < (unsigned)a.nz;
        double *rp = rs + (p & 1) * FR_WPL;
#pragma unroll
        for (int u = 0; u < FR_PP; u++) {
            if (a.dbg & 2) break;
            const int o = fo[u];
            const dbl2_t zm = *reinterpret_cast<const dbl2_t *>(fm + o), ym = *reinterpret_cast<const dbl2_t *>(f0 + o - FF_WX);
            const dbl2_t xc = *reinterpret_cast<const dbl2_t *>(f0 + o), yp = *reinterpret_cast<const dbl2_t *>(f0 + o + FF_WX);
            const dbl2_t zp = *reinterpret_cast<const dbl2_t *>(fp + o);
            const double xl = f0[o - 1], xr = f0[o + 2];
            const double b0 = xc.x, b1 = xc.y;  // f of the pair (the epilogue's b)
            const double dk = a.dk;
            // every neighbour outside the grid (x, y, or a plane past either end) is
            // +0.0 in the ring: dk * 0.0 is a zero whose term leaves the sum as the
            // constant kernel's `in ? d x : 0.0` does (an accumulator that starts at
            // +0.0 never becomes -0.0), so no selects
            const double y0[7] = {dk * zm.x, dk * ym.x, dk * xl, dk * xc.x, dk * xc.y, dk * yp.x, dk * zp.x};
            const double y1[7] = {dk * zm.y, dk * ym.y, dk * xc.x, dk * xc.y, dk * xr, dk * yp.y, dk * zp.y};
            double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                acc0 = fma(a.cst[k], y0[k], acc0);
                acc1 = fma(a.cst[k], y1[k], acc1);
            }
            const bool ok = pin && inp[u];
            const int q = tid + 256 * u;
            if (q < FR_NP) *reinterpret_cast<dbl2_t *>(rp + 2 * q) = dbl2_t{ok ? b0 - acc0 : 0.0, ok ? b1 - acc1 : 0.0};
        }
        fr_store(a, fgx0, fgy0, fring, p + 2, pn);            // f(p + 2): the slot of p - 2 (unread now)
        fr_fetch(a, fgx0, fgy0, min(p + 4, p1 + 1), pn);      // in flight two planes (unconditional)
        lds_barrier();
        if (!live || (a.dbg & 1)) return;
        // the plane's terms of the two coarse chains it belongs to: chain n (coarse
        // plane Zn = (p + 1) / 2: dz = -1 at odd p, 0 at even p) and chain o (Zn - 1:
        // dz = +1, then +2 and the padding); PH = (p - p0) % 4 fixes each chain's
        // register slot and group at compile time
        constexpr int PH = decltype(ph)::value;
        constexpr int sn = (PH >> 1) & 1, so = sn ^ 1, gn = PH & 1, go = 2 + (PH & 1);
        const int Zn = (p + 1) >> 1, Zo = Zn - 1;
        const bool nl = Zn < Ze, ol = Zo >= Zb;
        if (gn == 0 && nl) {  // chain n starts: its class's position tables into registers
            const int c = scl[(Zn - Zb) * 256 + tid];
            const uint4 *tw = reinterpret_cast<const uint4 *>(stab) + 4 * c;
#pragma unroll
            for (int g = 0; g < 4; g++) ch[sn].iw[g] = tw[g];
            ch[sn].mk = *reinterpret_cast<const uint2 *>(smk + 4 * c);
            ch[sn].npad = a.ke - skdz[5 * c + 4];
            ch[sn].c = c;
            ch[sn].ac = 0.0;
        }
        // r(p) at the 4 x 4 in-plane positions (dy, dx) in -1..2 of the row's anchor,
        // shared by both chains; a position's values through its class's byte index
        double w[16];
#pragma unroll
        for (int dy = 0; dy < 4; dy++) {
            const double *rr = rp + base + (dy - 1) * FR_WX;
            const dbl2_t m = *reinterpret_cast<const dbl2_t *>(rr);
            w[4 * dy + 0] = rr[-1];
            w[4 * dy + 1] = m.x;
            w[4 * dy + 2] = m.y;
            w[4 * dy + 3] = rr[2];
        }
        auto terms = [&](RrChain &c, int g) {
            const uint4 iw = c.iw[g];
            const uint32_t mk = ((g < 2 ? c.mk.x : c.mk.y) >> (16 * (g & 1))) & 0xffffu;
            const uint32_t wd[4] = {iw.x, iw.y, iw.z, iw.w};
            double v[16];
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = st[(wd[j >> 2] >> (8 * (j & 3))) & 255u];
            double ac = c.ac;
#pragma unroll
            for (int j = 0; j < 16; j++) ac = (mk >> j) & 1u ? fma(v[j], w[j], ac) : ac;
            c.ac = ac;
        };
        if (nl) {
            terms(ch[sn], gn);
            if (gn == 1) ch[sn].ra = w[5];  // r at the anchor: the padding entries' operand
        }
        if (ol) {
            terms(ch[so], go);
            if (go == 3) {
                double ac = ch[so].ac;
                for (int k = 0; k < ch[so].npad; k++) ac = fma(0.0, ch[so].ra, ac);  // +0.0 padding
                const int64_t J = (int64_t)Zo * cpl + (int64_t)Y * a.cx + X;
                a.fc[J] = ac;
                const double dd = a.dmode == 0 ? a.dkc : sdt[sdc[(Zo - Zb) * 256 + tid]];
                a.dfc[J] = dd * ac;  // vec_mul(_coded)'s product
            }
        }
    };
    // planes p0 .. p1 (p0 = 2 Zb - 1 odd, an even count): f(p + 2) in pb for odd p, pa for even p
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    int p = p0;
    for (; p + 3 <= p1; p += 4) {
        step(p, pb, P0{});
        step(p + 1, pa, P1{});
        step(p + 2, pb, P2{});
        step(p + 3, pa, P3{});
    }
    if (p < p1) {
        step(p, pb, P0{});
        step(p + 1, pa, P1{});
    }
}

// k_fine_rr: the same launch (r = f - A (d f), f_c = R r, d_c f_c) with the
// work per fine plane cut where the counters put it (round 6: 100.7 us of which
// the R sums ~44 us, the residual ~23 us):
//   R's terms without value-table lookups or masks: every class's entries lie in
//     the 32 slots (dz, dy, dx) a 2 x 2 x 2 box smoothed by the 7-point stencil
//     reaches (4 at dz = -1, 12 at dz = 0, 12 at dz = 1, 4 at dz = 2), so each
//     class is 32 fp64 weights in LDS (gtc_wt, +0.0 where the class has no
//     entry) and a plane adds 4 or 12 fma terms per chain: an absent slot adds
//     fma(+0.0, r, acc) = acc (r finite, the accumulator never -0.0), so every
//     chain is the class's entries in ascending (dz, dy, dx) order, bitwise
//     k_gtc_restrict_march's; the two chains of a plane interleave;
//   g = d f once per point, when a plane arrives (the seven-point sum is
//     spmv_dia_kernel's fma chain over d x_j): the z neighbours and the centre
//     from the lane's registers (every lane keeps the same 16-B units of the
//     window through the march), only the plane itself in LDS (two slots);
//   windows start at an odd x (2 X0 - 3 for f, 2 X0 - 1 for r), so a coarse
//     row's four r values per (dz, dy) are two aligned 16-B LDS reads;
//   the class ids and d_c codes of the next coarse plane load with the f plane
//     two steps ahead (no LDS staging, no wait of their own).
// Three workgroups per CU.  Even nx: a unit (x, x + 1) with x odd straddles the
// grid only at x = -1 and x = nx - 1, loaded from the clamped pair and shifted.
constexpr int R2_TX = 32, R2_TY = 8;                        // coarse tile
constexpr int R2_UX = R2_TX + 3, R2_UY = 2 * R2_TY + 4;     // f/g window: 35 units x 20 rows (x from 2 X0 - 3, y from 2 Y0 - 2)
constexpr int R2_NU = R2_UX * R2_UY, R2_PU = (R2_NU + 255) / 256;  // 700 units, 3 per lane
constexpr int R2_RX = R2_TX + 1, R2_RY = 2 * R2_TY + 2;     // r window: 33 units x 18 rows (x from 2 X0 - 1, y from 2 Y0 - 1)
constexpr int R2_NR = R2_RX * R2_RY;                        // 594
constexpr int R2_WS = 34;                                   // LDS doubles per class (32 weights, padded against bank repeats)
constexpr int R2_CMAX = 32;                                 // classes (LDS: 8.7 KB)

struct FineRr2Args {
    const uint8_t *cls;  // R's class per coarse row
    const double *wt;    // nclass x 32 weights (the 32-slot pattern)
    int nclass;
    int nx, ny, nz, cx, cy, cz;
    int ntx, nty, jper;
    const double *f;
    double *fc, *dfc;
    const uint8_t *dcc;  // the coarse level's d: codes into dtc, or one value dkc
    const double *dtc;
    double dkc;
    int dmode;  // 0 one value, 1 codes
    double dk;  // the fine level's one-value d
    double cst[7];
    int dbg;  // timing experiments only (FAMG_FINE_DBG): 1 skips the R sums, 2 the residual
};

struct Rr2Set {
    dbl2_t F[R2_PU], G[R2_PU];  // f (shifted, 0.0 outside the grid) and d f of one plane at the lane's units
};

__global__ __launch_bounds__(256, 3) void k_fine_rr(FineRr2Args a) {
    __shared__ __attribute__((aligned(16))) double gs[2 * 2 * R2_NU];   // d f of planes p, p + 1
    __shared__ __attribute__((aligned(16))) double rs2[2 * 2 * R2_NR];  // r of planes p, p - 1
    __shared__ double sdt[256];
    extern __shared__ __attribute__((aligned(16))) double sw[];  // the classes' weights, R2_WS per class
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int X0 = (txy % a.ntx) * R2_TX, Y0 = (txy / a.ntx) * R2_TY;
    const int Zb = chunk * a.jper, Ze = min(Zb + a.jper, a.cz);
    const int64_t cpl = (int64_t)a.cx * a.cy, fpl = (int64_t)a.nx * a.ny;
    for (int b = tid; b < a.nclass * 32; b += 256) sw[(b >> 5) * R2_WS + (b & 31)] = a.wt[b];
    if (a.dmode == 1) sdt[tid] = a.dtc[tid];
    // the lane's units: load offset in a plane (32-bit), shift code, residual slot
    int off[R2_PU], ri[R2_PU];
    bool sa[R2_PU], sb[R2_PU], sc[R2_PU], rin[R2_PU], v0[R2_PU], v1[R2_PU];
#pragma unroll
    for (int u = 0; u < R2_PU; u++) {
        const int q = tid + 256 * u, ux = q % R2_UX, uy = q / R2_UX;
        const int x = 2 * X0 - 3 + 2 * ux, y = 2 * Y0 - 2 + uy;
        const bool yin = q < R2_NU && (unsigned)y < (unsigned)a.ny;
        const bool any = yin && x >= -1 && x <= a.nx - 1;
        sa[u] = any && x >= 0 && x + 1 < a.nx;  // both points: (f[x], f[x + 1])
        sb[u] = any && x == a.nx - 1;           // loaded (nx - 2, nx - 1): (.y, 0)
        sc[u] = any && x == -1;                 // loaded (0, 1): (0, .x)
        off[u] = any ? y * a.nx + min(max(x, 0), a.nx - 2) : 0;
        rin[u] = q < R2_NU && ux >= 1 && ux <= R2_RX && uy >= 1 && uy <= R2_RY;
        ri[u] = rin[u] ? (uy - 1) * R2_RX + ux - 1 : 0;
        v0[u] = yin && x >= 0 && x < a.nx;
        v1[u] = yin && x + 1 >= 0 && x + 1 < a.nx;
    }
    // the lane's coarse row
    const int lx = tid % R2_TX, ly = tid / R2_TX, X = X0 + lx, Y = Y0 + ly;
    const bool live = X < a.cx && Y < a.cy;
    const int64_t Jxy = live ? (int64_t)Y * a.cx + X : 0;
    const int p0 = 2 * Zb - 1, p1 = 2 * Ze;
    auto fetch = [&](int p, Rr2Set &S) {
        const double *fz = a.f + (int64_t)min(max(p, 0), a.nz - 1) * fpl;
#pragma unroll
        for (int u = 0; u < R2_PU; u++) S.F[u] = *reinterpret_cast<const dbl2u_t *>(fz + off[u]);
    };
    // class id and d_c code of coarse plane Z (clamped: a plane past the run is never used)
    int ncls = 0, ndc = 0;
    auto fetch_cls = [&](int Z) {
        const int64_t J = (int64_t)min(Z, a.cz - 1) * cpl + Jxy;
        ncls = a.cls[J];
        if (a.dmode == 1) ndc = a.dcc[J];
    };
    // the arrived plane: shift / zero in place, d f beside it
    auto settle = [&](int p, Rr2Set &S) {
        const bool pin = (unsigned)p < (unsigned)a.nz;
#pragma unroll
        for (int u = 0; u < R2_PU; u++) {
            const dbl2_t v = S.F[u];
            const double x0 = sa[u] ? v.x : sb[u] ? v.y : 0.0;
            const double x1 = sa[u] ? v.y : sc[u] ? v.x : 0.0;
            S.F[u] = pin ? dbl2_t{x0, x1} : dbl2_t{0.0, 0.0};
            S.G[u] = a.dk * S.F[u];
        }
    };
    auto publish = [&](int p, const Rr2Set &S) {
        double *g = gs + (p & 1) * 2 * R2_NU;
#pragma unroll
        for (int u = 0; u < R2_PU; u++) {
            const int q = tid + 256 * u;
            if (q < R2_NU) *reinterpret_cast<dbl2_t *>(g + 2 * q) = S.G[u];
        }
    };
    Rr2Set S0, S1, S2, S3;  // plane p0 + k in set k mod 4
    fetch(p0 - 1, S3);
    fetch(p0, S0);
    fetch(p0 + 1, S1);
    fetch_cls(Zb);
    settle(p0 - 1, S3);
    settle(p0, S0);
    publish(p0, S0);
    fetch(p0 + 2, S2);
    __syncthreads();

    double acc[2] = {0.0, 0.0};
    int cb[2] = {0, 0}, dq[2] = {0, 0};  // per chain: its class's weights in sw, its d_c code
    // step p: Sm = plane p - 1 (its G), S0 = p, S1 = p + 1 (arrived), S3 = p + 3 (issued here; the set of p - 1)
    auto step = [&](int p, Rr2Set &Sm, Rr2Set &Sp, Rr2Set &S1p, Rr2Set &S3p, auto ph) {
        constexpr int PH = decltype(ph)::value;
        constexpr int sn = (PH >> 1) & 1, so = sn ^ 1, gn = PH & 1, go = 2 + (PH & 1);
        settle(p + 1, S1p);
        publish(p + 1, S1p);  // the slot of p - 1: its in-plane reads ended before the last barrier
        const double *g0 = gs + (p & 1) * 2 * R2_NU;
        double *rp = rs2 + (p & 1) * 2 * R2_NR;
        const bool pin = (unsigned)p < (unsigned)a.nz;
#pragma unroll
        for (int u = 0; u < R2_PU; u++) {
            if (!rin[u] || (a.dbg & 2)) continue;
            const int q = tid + 256 * u;
            const dbl2_t ym = *reinterpret_cast<const dbl2_t *>(g0 + 2 * (q - R2_UX));
            const dbl2_t yp = *reinterpret_cast<const dbl2_t *>(g0 + 2 * (q + R2_UX));
            const double xl = g0[2 * q - 1], xr = g0[2 * q + 2];
            const dbl2_t gm = Sm.G[u], gc = Sp.G[u], gp = S1p.G[u];
            const double y0[7] = {gm.x, ym.x, xl, gc.x, gc.y, yp.x, gp.x};
            const double y1[7] = {gm.y, ym.y, gc.x, gc.y, xr, yp.y, gp.y};
            double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                acc0 = fma(a.cst[k], y0[k], acc0);
                acc1 = fma(a.cst[k], y1[k], acc1);
            }
            const dbl2_t b = Sp.F[u];
            *reinterpret_cast<dbl2_t *>(rp + 2 * ri[u]) =
                dbl2_t{pin && v0[u] ? b.x - acc0 : 0.0, pin && v1[u] ? b.y - acc1 : 0.0};
        }
        fetch(min(p + 3, p1 + 1), S3p);  // in flight two planes
        const int Zn = (p + 1) >> 1, Zo = Zn - 1;
        const bool nl = Zn < Ze, ol = Zo >= Zb;
        if (gn == 0 && nl) {  // chain n starts: its class (loaded two steps ago); the next one's load
            cb[sn] = ncls * R2_WS;
            dq[sn] = ndc;
            acc[sn] = 0.0;
            fetch_cls(Zn + 1);
        }
        lds_barrier();
        if (!live || (a.dbg & 1)) return;
        // r(p) at the 4 x 4 positions (dy, dx) in -1..2 of the anchor (2X, 2Y): units lx, lx + 1 of rows 2 ly + dy
        double w[16];
#pragma unroll
        for (int dy = 0; dy < 4; dy++) {
            const double *rr = rp + 2 * ((2 * ly + dy) * R2_RX + lx);
            const dbl2_t m0 = *reinterpret_cast<const dbl2_t *>(rr);
            const dbl2_t m1 = *reinterpret_cast<const dbl2_t *>(rr + 2);
            w[4 * dy + 0] = m0.x;
            w[4 * dy + 1] = m0.y;
            w[4 * dy + 2] = m1.x;
            w[4 * dy + 3] = m1.y;
        }
        // the slots of a plane group: 4 (dz = -1, 2) or 12 (dz = 0, 1), as w indices
        constexpr int P4[4] = {5, 6, 9, 10};
        constexpr int P12[12] = {1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 13, 14};
        constexpr int NN = (gn == 0) ? 4 : 12, NO = (go == 3) ? 4 : 12;
        constexpr int ON = (gn == 0) ? 0 : 4, OO = (go == 2) ? 16 : 28;
        double wn[NN], wo[NO];
        if (nl) {
#pragma unroll
            for (int k = 0; k < NN; k += 2) {
                const dbl2_t v = *reinterpret_cast<const dbl2_t *>(sw + cb[sn] + ON + k);
                wn[k] = v.x;
                wn[k + 1] = v.y;
            }
        }
        if (ol) {
#pragma unroll
            for (int k = 0; k < NO; k += 2) {
                const dbl2_t v = *reinterpret_cast<const dbl2_t *>(sw + cb[so] + OO + k);
                wo[k] = v.x;
                wo[k + 1] = v.y;
            }
        }
        double an = acc[sn], ao = acc[so];
#pragma unroll
        for (int k = 0; k < 12; k++) {
            if (nl && k < NN) an = fma(wn[k], w[NN == 4 ? P4[k % 4] : P12[k]], an);
            if (ol && k < NO) ao = fma(wo[k], w[NO == 4 ? P4[k % 4] : P12[k]], ao);
        }
        acc[sn] = an;
        acc[so] = ao;
        if (go == 3 && ol) {
            const int64_t J = (int64_t)Zo * cpl + Jxy;
            a.fc[J] = ao;
            const double dd = a.dmode == 0 ? a.dkc : sdt[dq[so]];
            a.dfc[J] = dd * ao;  // vec_mul(_coded)'s product
        }
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    int p = p0;
    for (; p + 3 <= p1; p += 4) {
        step(p, S3, S0, S1, S3, P0{});
        step(p + 1, S0, S1, S2, S0, P1{});
        step(p + 2, S1, S2, S3, S1, P2{});
        step(p + 3, S2, S3, S0, S2, P3{});
    }
    if (p < p1) {
        step(p, S3, S0, S1, S3, P0{});
        step(p + 1, S0, S1, S2, S0, P1{});
    }
}

// k_fine_pj: the same launch as k_fine_interp_jacobi (v = d f + P v_c, then
// z = v + d (f - A v)) on 16-B units -- two x-adjacent fine points, x even, in
// one box, so one coarse window anchor -- the way k_fine_rr cut its plane work:
//   per lane three units of the 68 x 18 v window (x from x0 - 2, y from y0 - 1):
//     f and the two class bytes of a unit in one load each (16 B, 2 B);
//   v of planes z - 1, z, z + 1 stay in the lane's registers (the Jacobi sum's
//     z neighbours and centre), only plane z in LDS for the in-plane neighbours
//     (two slots);
//   P's dictionary decoded per class: its KE = 4 fp64 weights (two 16-B LDS
//     reads) and, per coarse-ring phase, its four coarse-window offsets (one
//     8-B read) -- the fma chain over the KE entries in dictionary order, padding
//     +0.0 terms included, is k_gtc_interp's ADD0 sum;
//   the output tile's 512 units as 16-B stores.
// Bitwise k_fine_interp_jacobi (test_fine_fused_bitwise).  Even nx.
constexpr int J2_NT = 1024;                                 // threads per workgroup
constexpr int J2_TX = 256, J2_TY = 16;                      // fine tile (x, y): whole grid rows at 256^3
constexpr int J2_UX = J2_TX / 2 + 2, J2_UY = J2_TY + 2;     // v window: 130 units x 18 rows
constexpr int J2_NU = J2_UX * J2_UY, J2_PU = (J2_NU + J2_NT - 1) / J2_NT;  // 2340 units, 3 per lane
constexpr int J2_CX = J2_TX / 2 + 4, J2_CY = J2_TY / 2 + 4, J2_CPL = J2_CX * J2_CY;  // coarse window 132 x 12
constexpr int J2_CPF = (J2_CPL + J2_NT - 1) / J2_NT;        // coarse points per lane (2)
constexpr int J2_CMAX = 128;                                // classes

struct FinePj2Args {
    const uint8_t *cls;    // P's class id per fine row
    const uint16_t *dict;  // nclass x 4 entries: value index << 8 | slot
    const double *vtab;
    int nclass;
    int nx, ny, nz, cx, cy, cz;
    int ntx, nty, jper;
    const double *vc;  // coarse correction v_c
    const double *f;   // fine rhs
    double *out;       // z
    double dk;
    double cst[7];
    int dbg;  // timing experiments only (FAMG_FINE_DBG): 1 no stores, 2 no P sums, 4 no Jacobi sums
};

struct Pj2Set {
    dbl2_t F[J2_PU], V[J2_PU];
    int C[J2_PU];  // the unit's two class bytes (x even: low byte)
};

__global__ __launch_bounds__(J2_NT) void k_fine_pj(FinePj2Args a) {
    __shared__ __attribute__((aligned(16))) double vr[2 * 2 * J2_NU];  // v of planes z, z + 1
    __shared__ double cring[4 * J2_CPL];
    __shared__ __attribute__((aligned(16))) double pw[J2_CMAX * 4];    // per class its 4 weights
    __shared__ __attribute__((aligned(8))) int16_t po[4 * J2_CMAX * 4];  // per ring phase and class: 4 offsets
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int x0 = (txy % a.ntx) * J2_TX, y0 = (txy / a.ntx) * J2_TY;
    const int zb = chunk * a.jper, ze = min(zb + a.jper, a.nz);
    const int cwx0 = (x0 >> 1) - 2, cwy0 = (y0 >> 1) - 2;
    const int64_t fpl = (int64_t)a.nx * a.ny;
    for (int b = tid; b < 4 * a.nclass; b += J2_NT) {
        const uint32_t e = a.dict[b], sl = e & 255u;
        pw[b] = a.vtab[e >> 8];
        const int dzs = (int)(sl / 9u) - 1, dys = (int)((sl / 3u) % 3u) - 1, dxs = (int)(sl % 3u) - 1;
#pragma unroll
        for (int r = 0; r < 4; r++) po[r * 4 * a.nclass + b] = (int16_t)(((r + dzs) & 3) * J2_CPL + dys * J2_CX + dxs);
    }
    // the lane's units: plane offset (32-bit, an in-grid unit for units outside),
    // coarse anchor, whether in the grid / in the output tile
    int off[J2_PU], cb[J2_PU];
    bool inq[J2_PU], jac[J2_PU];
#pragma unroll
    for (int u = 0; u < J2_PU; u++) {
        const int q = tid + J2_NT * u, ux = q % J2_UX, uy = q / J2_UX;
        const int x = x0 - 2 + 2 * ux, y = y0 - 1 + uy;
        inq[u] = q < J2_NU && (unsigned)x < (unsigned)a.nx && (unsigned)y < (unsigned)a.ny;
        jac[u] = inq[u] && ux >= 1 && ux <= J2_TX / 2 && uy >= 1 && uy <= J2_TY;
        off[u] = inq[u] ? y * a.nx + x : 0;
        cb[u] = inq[u] ? ((y >> 1) - cwy0) * J2_CX + (x >> 1) - cwx0 : J2_CX + 1;
    }
    auto fetch = [&](int z, Pj2Set &S) {
        const int zc = min(max(z, 0), a.nz - 1);
        const double *fz = a.f + (int64_t)zc * fpl;
        const uint8_t *cz = a.cls + (int64_t)zc * fpl;
#pragma unroll
        for (int u = 0; u < J2_PU; u++) {
            S.F[u] = *reinterpret_cast<const dbl2_t *>(fz + off[u]);
            S.C[u] = (int)*reinterpret_cast<const uint16_t *>(cz + off[u]);
        }
    };
    auto cfetch = [&](int Z, double (&v)[J2_CPF]) {
        const int64_t cpl = (int64_t)a.cx * a.cy;
#pragma unroll
        for (int u = 0; u < J2_CPF; u++) {
            const int p = tid + J2_NT * u;
            const int X = cwx0 + p % J2_CX, Y = cwy0 + p / J2_CX;
            const bool in = p < J2_CPL && (unsigned)X < (unsigned)a.cx && (unsigned)Y < (unsigned)a.cy &&
                            (unsigned)Z < (unsigned)a.cz;
            v[u] = a.vc[in ? (int64_t)Z * cpl + (int64_t)Y * a.cx + X : 0];
        }
    };
    auto cstore = [&](int Z, const double (&v)[J2_CPF]) {
#pragma unroll
        for (int u = 0; u < J2_CPF; u++) {
            const int p = tid + J2_NT * u;
            const int X = cwx0 + p % J2_CX, Y = cwy0 + p / J2_CX;
            const bool in = (unsigned)X < (unsigned)a.cx && (unsigned)Y < (unsigned)a.cy && (unsigned)Z < (unsigned)a.cz;
            if (p < J2_CPL) cring[(Z & 3) * J2_CPL + p] = in ? v[u] : 0.0;
        }
    };
    // v = d f + P v_c of plane z at the lane's units (0.0 outside the grid)
    auto interp = [&](int z, Pj2Set &S) {
        const bool zin = (unsigned)z < (unsigned)a.nz;
        const int16_t *pz = po + ((z >> 1) & 3) * 4 * a.nclass;
#pragma unroll
        for (int u = 0; u < J2_PU; u++) {
            double vv[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int c = (S.C[u] >> (8 * h)) & 255;
                const dbl2_t w01 = *reinterpret_cast<const dbl2_t *>(pw + 4 * c);
                const dbl2_t w23 = *reinterpret_cast<const dbl2_t *>(pw + 4 * c + 2);
                const uint2 oo = *reinterpret_cast<const uint2 *>(pz + 4 * c);
                const int o0 = (int)(int16_t)(oo.x & 0xffffu), o1 = (int)(int16_t)(oo.x >> 16);
                const int o2 = (int)(int16_t)(oo.y & 0xffffu), o3 = (int)(int16_t)(oo.y >> 16);
                double acc = 0.0;
                if (!(a.dbg & 2)) {
                    acc = fma(w01.x, cring[cb[u] + o0], acc);
                    acc = fma(w01.y, cring[cb[u] + o1], acc);
                    acc = fma(w23.x, cring[cb[u] + o2], acc);
                    acc = fma(w23.y, cring[cb[u] + o3], acc);
                }
                const double fv = h ? S.F[u].y : S.F[u].x;
                vv[h] = (zin && inq[u]) ? a.dk * fv + acc : 0.0;  // d*b (vec_mul's product) + P v_c
            }
            S.V[u] = dbl2_t{vv[0], vv[1]};
        }
    };
    auto publish = [&](int z, const Pj2Set &S) {
        double *g = vr + (z & 1) * 2 * J2_NU;
#pragma unroll
        for (int u = 0; u < J2_PU; u++) {
            const int q = tid + J2_NT * u;
            if (q < J2_NU) *reinterpret_cast<dbl2_t *>(g + 2 * q) = S.V[u];
        }
    };
    // coarse planes zb/2 - 2 .. zb/2 + 1 (those of v(zb - 1) .. v(zb + 1); zb is even)
    const int Zb = zb >> 1;
    {
        double cv[J2_CPF];
        for (int Z = Zb - 2; Z <= Zb + 1; Z++) {
            cfetch(Z, cv);
            cstore(Z, cv);
        }
    }
    Pj2Set S0, S1, S2, S3;  // plane zb + k in set k mod 4
    fetch(zb - 1, S3);
    fetch(zb, S0);
    fetch(zb + 1, S1);
    __syncthreads();
    interp(zb - 1, S3);
    interp(zb, S0);
    publish(zb, S0);
    int cmax = Zb + 2;
    double cp[J2_CPF];
    cfetch(cmax, cp);
    fetch(zb + 2, S2);
    __syncthreads();

    // step z: Sm = z - 1 (its V), Sz = z, S1 = z + 1 (f arrived: its v now), S3 = z + 3 (issued; the set of z - 1)
    auto step = [&](int z, Pj2Set &Sm, Pj2Set &Sz, Pj2Set &S1, Pj2Set &S3) {
        interp(z + 1, S1);
        publish(z + 1, S1);  // the slot of z - 1: its in-plane reads ended before the last barrier
        // z(z) = v + d (f - A v): spmv_dia_kernel's constant 7-point JACOBI sum
        const double *v0 = vr + (z & 1) * 2 * J2_NU;
        const bool zon = z < ze;
        double *oz = a.out + (int64_t)min(z, a.nz - 1) * fpl;
#pragma unroll
        for (int u = 0; u < J2_PU; u++) {
            if (!jac[u] || !zon || (a.dbg & 1)) continue;
            const int q = tid + J2_NT * u;
            if (a.dbg & 4) {
                *reinterpret_cast<dbl2_t *>(oz + off[u]) = Sz.V[u];
                continue;
            }
            const dbl2_t ym = *reinterpret_cast<const dbl2_t *>(v0 + 2 * (q - J2_UX));
            const dbl2_t yp = *reinterpret_cast<const dbl2_t *>(v0 + 2 * (q + J2_UX));
            const double xl = v0[2 * q - 1], xr = v0[2 * q + 2];
            const dbl2_t vm = Sm.V[u], vc = Sz.V[u], vp = S1.V[u];
            const double y0[7] = {vm.x, ym.x, xl, vc.x, vc.y, yp.x, vp.x};
            const double y1[7] = {vm.y, ym.y, vc.x, vc.y, xr, yp.y, vp.y};
            double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                acc0 = fma(a.cst[k], y0[k], acc0);
                acc1 = fma(a.cst[k], y1[k], acc1);
            }
            const dbl2_t fz = Sz.F[u];
            // streamed out (nontemporal: z is read by the next solve step, not by this cycle)
            __builtin_nontemporal_store(dbl2_t{vc.x + a.dk * (fz.x - acc0), vc.y + a.dk * (fz.y - acc1)},
                                        reinterpret_cast<dbl2_t *>(oz + off[u]));
        }
        cstore(cmax, cp);  // the coarse plane v(z + 2) adds (slot of cmax - 4: unread)
        cmax = ((z + 3) >> 1) + 1;
        cfetch(cmax, cp);
        fetch(min(z + 3, ze), S3);
        lds_barrier();
    };
    for (int z = zb; z < ze; z += 4) {
        step(z, S3, S0, S1, S3);
        step(z + 1, S0, S1, S2, S0);
        step(z + 2, S1, S2, S3, S1);
        step(z + 3, S2, S3, S0, S2);
    }
}

// ------------------------------------------------------------ host side

// workgroups of k_fine_interp_jacobi per CU (cached)
static int fine_pj_occupancy() {
    static std::once_flag once;
    static int n = 1;
    std::call_once(once, [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k_fine_interp_jacobi<4>, 256, 16 * 512) == hipSuccess &&
            v >= 1)
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
    // the coarse level's d coded (8-bit) or one value: no global load in the plane loop
    if (!epic.y2 || !epic.dc) return false;
    for (int q = 0; q < 3; q++)
        if (R.gtc_fg[q] != A.dia_cst_n[q] || R.gtc_cg[q] != (R.gtc_fg[q] + 1) / 2) return false;
    // even nx: the 16-B units of a window row never straddle the end of a grid row
    // except where the kernels shift them (an odd nx runs the unfused launches)
    if (R.gtc_fg[0] % 2 != 0) return false;
    return A.nrows == R.ncols && R.nrows == R.gtc_cg[0] * R.gtc_cg[1] * R.gtc_cg[2];
}

// workgroups of k_fine_rr per CU (cached)
static int fine_rr2_occupancy(size_t dyn) {
    static std::mutex mu;
    static std::unordered_map<size_t, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dyn);
    if (it != cache.end()) return it->second;
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k_fine_rr, 256, dyn) != hipSuccess || v < 1) {
        (void)hipGetLastError();
        v = 1;
    }
    cache[dyn] = v;
    return v;
}

// FAMG_FINE_RR=1: the round-5 resid+restrict kernel (A/B timing)
static bool fine_rr_v1() {
    static const bool on = [] {
        const char *e = getenv("FAMG_FINE_RR");
        return e && e[0] == '1';
    }();
    return on;
}

static void fine_rr2(const GpuCsr &A, const GpuCsr &R, const double *f, double dk, double *fc, const SpmvEpi &epic,
                     hipStream_t s) {
    FineRr2Args a{};
    a.cls = R.gtc_cls.get();
    a.wt = R.gtc_wt.get();
    a.nclass = R.gtc_nclass;
    a.nx = (int)R.gtc_fg[0]; a.ny = (int)R.gtc_fg[1]; a.nz = (int)R.gtc_fg[2];
    a.cx = (int)R.gtc_cg[0]; a.cy = (int)R.gtc_cg[1]; a.cz = (int)R.gtc_cg[2];
    a.ntx = (int)ceil_div(a.cx, R2_TX);
    a.nty = (int)ceil_div(a.cy, R2_TY);
    a.f = f;
    a.fc = fc;
    a.dfc = epic.y2;
    if (epic.dc && epic.dk != 0.0 && flag(FLAG_DIA_DK) != 0) {
        a.dmode = 0;
        a.dkc = epic.dk;
    } else {
        a.dmode = 1;
        a.dcc = epic.dc;
        a.dtc = epic.dt;
    }
    a.dk = dk;
    for (int k = 0; k < 7; k++) a.cst[k] = A.dia_cst_v[k];
    {
        const char *e = getenv("FAMG_FINE_DBG");  // timing experiments only (results wrong)
        a.dbg = e ? atoi(e) : 0;
    }
    const int64_t ntxy = (int64_t)a.ntx * a.nty;
    // occupancy at a typical run length, then the run length for one round of workgroups
    const size_t dyn = (size_t)8 * R2_WS * a.nclass;
    const int64_t want = (int64_t)fine_rr2_occupancy(dyn) * std::max(A.ctx ? A.ctx->num_cus : 256, 1);
    a.jper = (int)std::max<int64_t>(1, ceil_div((int64_t)a.cz * ntxy, want));
    if (flag(FLAG_FINE_FUSE) > 1) a.jper = (int)std::max<int64_t>(1, flag(FLAG_FINE_FUSE) / 2);
    const dim3 grid((unsigned)(ntxy * ceil_div(a.cz, a.jper)));
    k_fine_rr<<<grid, dim3(256), dyn, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
}

void fine_resid_restrict(const GpuCsr &A, const GpuCsr &R, const double *f, double dk, double *fc,
                         const SpmvEpi &epic, hipStream_t s) {
    if (!fine_rr_v1() && R.gtc_wt.get() && R.gtc_nclass <= R2_CMAX && R.gtc_fg[0] * R.gtc_fg[1] < (int64_t(1) << 31)) {
        fine_rr2(A, R, f, dk, fc, epic, s);
        const int64_t n = A.nrows, nc = R.nrows;
        log_launch("fine-rr", SPMV_KERNEL_DIA, -1, n, 8 * n + 16 * nc + nc + (epic.dc && !(epic.dk != 0.0 && flag(FLAG_DIA_DK) != 0) ? nc : 0),
                   (12 * A.nnz + 4 * (n + 1) + 32 * n) + (12 * R.nnz + 4 * (nc + 1) + 8 * n + 16 * nc));
        return;
    }
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
    } else {
        a.dmode = 1;
        a.dcc = epic.dc;
        a.dtc = epic.dt;
    }
    a.dk = dk;
    for (int k = 0; k < 7; k++) a.cst[k] = A.dia_cst_v[k];
    {
        const char *e = getenv("FAMG_FINE_DBG");  // timing experiments only (results wrong)
        a.dbg = e ? atoi(e) : 0;
    }
    const int64_t ntxy = (int64_t)a.ntx * a.nty;
    // occupancy with the dictionary part of the dynamic LDS (the per-plane class
    // bytes are small), then the run length, then the exact dynamic size
    const size_t dyn0 = (size_t)((5 * a.nclass + 15) & ~15) + 72 * (size_t)a.nclass;
    const int64_t want = (int64_t)fine_rr_occupancy(dyn0 + 2 * 256 * 16) * std::max(A.ctx ? A.ctx->num_cus : 256, 1);
    a.jper = (int)std::max<int64_t>(1, ceil_div((int64_t)a.cz * ntxy, want));
    if (flag(FLAG_FINE_FUSE) > 1) a.jper = (int)std::max<int64_t>(1, flag(FLAG_FINE_FUSE) / 2);
    a.jper = std::min(a.jper, 64);  // (the class bytes of a run: 512 per plane)
    const size_t dyn = dyn0 + (size_t)2 * 256 * a.jper;
    const dim3 grid((unsigned)(ntxy * ceil_div(a.cz, a.jper)));
    k_fine_resid_restrict<<<grid, dim3(256), dyn, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
    const int64_t n = A.nrows, nc = R.nrows;
    // f in once, f_c and d_c f_c out, R's class ids (1 B per coarse row; a coded d_c: 1 B more);
    // CSR-equivalent: A's RESID0 (x, b = f; r out; d gathered) + R's SETDF
    log_launch("fine-rr", SPMV_KERNEL_DIA, -1, n, 8 * n + 16 * nc + nc + (a.dmode == 1 ? nc : 0),
               (12 * A.nnz + 4 * (n + 1) + 32 * n) + (12 * R.nnz + 4 * (nc + 1) + 8 * n + 16 * nc));
}

bool fine_interp_jacobi_ok(const GpuCsr &A, const GpuCsr &P, const SpmvEpi &epi) {
    if (flag(FLAG_FINE_FUSE) == 0 || !dia7_cst_dk(A, epi)) return false;
    if (!P.gtc_on || P.gtc_r || P.rframe.on() || P.cframe.on() || P.gtc_nce > 512 ||
        (P.gtc_ke != 4 && P.gtc_ke != 8) ||
        P.gtc_ntab > 256)
        return false;
    for (int q = 0; q < 3; q++)
        if (P.gtc_fg[q] != A.dia_cst_n[q] || P.gtc_cg[q] != (P.gtc_fg[q] + 1) / 2) return false;
    if (P.gtc_fg[0] % 2 != 0) return false;  // even nx (16-B units of two points in one box)
    return A.nrows == P.nrows && P.ncols == P.gtc_cg[0] * P.gtc_cg[1] * P.gtc_cg[2];
}

// workgroups of k_fine_pj per CU (cached)
static int fine_pj2_occupancy() {
    static std::once_flag once;
    static int n = 1;
    std::call_once(once, [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k_fine_pj, J2_NT, 0) == hipSuccess && v >= 1)
            n = v;
        else
            (void)hipGetLastError();
    });
    return n;
}

// FAMG_FINE_PJ=1: the round-5 interp+Jacobi kernel (A/B timing)
static bool fine_pj_v1() {
    static const bool on = [] {
        const char *e = getenv("FAMG_FINE_PJ");
        return e && e[0] == '1';
    }();
    return on;
}

static void fine_pj2(const GpuCsr &A, const GpuCsr &P, const double *vc, const double *f, double dk, double *out,
                     hipStream_t s) {
    FinePj2Args a{};
    a.cls = P.gtc_cls.get();
    a.dict = P.gtc_dict.get();
    a.vtab = P.gtc_vtab.get();
    a.nclass = P.gtc_nclass;
    a.nx = (int)P.gtc_fg[0]; a.ny = (int)P.gtc_fg[1]; a.nz = (int)P.gtc_fg[2];
    a.cx = (int)P.gtc_cg[0]; a.cy = (int)P.gtc_cg[1]; a.cz = (int)P.gtc_cg[2];
    a.ntx = (int)ceil_div(a.nx, J2_TX);
    a.nty = (int)ceil_div(a.ny, J2_TY);
    a.vc = vc;
    a.f = f;
    a.out = out;
    a.dk = dk;
    for (int k = 0; k < 7; k++) a.cst[k] = A.dia_cst_v[k];
    {
        const char *e = getenv("FAMG_FINE_DBG");  // timing experiments only (results wrong)
        a.dbg = e ? atoi(e) : 0;
    }
    const int64_t ntxy = (int64_t)a.ntx * a.nty;
    const int64_t want = (int64_t)fine_pj2_occupancy() * std::max(A.ctx ? A.ctx->num_cus : 256, 1);
    int jper = (int)std::max<int64_t>(2, ceil_div((int64_t)a.nz * ntxy, want));
    if (flag(FLAG_FINE_FUSE) > 1) jper = (int)flag(FLAG_FINE_FUSE);
    a.jper = jper + (jper & 1);
    const dim3 grid((unsigned)(ntxy * ceil_div(a.nz, a.jper)));
    k_fine_pj<<<grid, dim3(J2_NT), 0, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
}

void fine_interp_jacobi(const GpuCsr &A, const GpuCsr &P, const double *vc, const double *f, double dk, double *out,
                        hipStream_t s) {
    if (!fine_pj_v1() && P.gtc_ke == 4 && P.gtc_nclass <= J2_CMAX && P.gtc_fg[0] * P.gtc_fg[1] < (int64_t(1) << 31)) {
        fine_pj2(A, P, vc, f, dk, out, s);
        const int64_t n = A.nrows;
        log_launch("fine-pj", SPMV_KERNEL_DIA, -1, n, 8 * n + 8 * P.ncols + 8 * n + n,
                   (12 * P.nnz + 4 * (n + 1) + 8 * P.ncols + 16 * n) + (12 * A.nnz + 4 * (n + 1) + 32 * n));
        return;
    }
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
    const size_t dyn = (size_t)16 * a.nce;  // the decoded dictionary, four ring phases
    if (a.ke == 4) k_fine_interp_jacobi<4><<<grid, dim3(256), dyn, s>>>(a);
    else k_fine_interp_jacobi<8><<<grid, dim3(256), dyn, s>>>(a);
    FAMG_CHECK_HIP(hipGetLastError());
    const int64_t n = A.nrows;
    // f and z once, v_c once, the class ids (1 B per row); CSR-equivalent: P's ADD0 + A's JACOBI
    log_launch("fine-pj", SPMV_KERNEL_DIA, -1, n, 8 * n + 8 * P.ncols + 8 * n + n,
               (12 * P.nnz + 4 * (n + 1) + 8 * P.ncols + 16 * n) + (12 * A.nnz + 4 * (n + 1) + 32 * n));
}

}  // namespace famg
