// sgs27.hip -- multicolor SGS sweeps on a 3-D 27-point grid operator, fused
// into plane-parity phases.
//
// The colour sweeps of SgsOp (ops.hip) update one colour per launch; each
// launch updates 1/8 of the rows but gathers from the whole x, so an SGS step
// (15 launches) streams x about 15 times.  On a structured nx x ny x nz grid
// whose greedy colouring is the parity colouring c = (x&1) + 2 (y&1) + 4 (z&1)
// (what greedy first-fit in row order gives for the 27-point stencil) the
// sweep has plane structure:
//   forward  colours 0..3 touch even planes only and read the odd planes'
//            old values; colours 4..7 touch odd planes and read the even
//            planes' new values;
//   backward colours 6,5,4 (odd planes), then 3,2,1,0 (even planes).
// So an SGS step is four phases (even fwd, odd fwd, odd bwd, even bwd); in a
// phase every plane of one parity runs its 3-4 in-plane colours in order while
// the other parity is read-only.  One workgroup owns TY rows of one plane: it
// loads those rows plus nst rows of halo on each side into LDS, runs the
// colours on shrinking halos (colour s is recomputed up to nst-1-s rows out,
// so its neighbours are final when the next colour reads them), and writes its
// TY rows to the phase's target buffer.  Each phase reads its planes from one
// buffer and writes them to another (no workgroup reads what another writes
// in the same launch); the other parity is read from where it currently lives.
//
// Arithmetic is the colour launches' exactly: row i of colour c sums
// fma(a_ik, x_k, acc) over its 27 diagonals in ascending column order with
// the latest values of lower colours and the old values of higher ones, then
// x_i + (1/a_ii) (b_i - acc) -- bitwise equal to spmv_dia_sgs_kernel.  The
// coefficients are the operator's own DIA codes (A's storage, original row
// order); positions outside the grid carry the +0.0 code and read 0.0.
#include <algorithm>
#include <cstring>

#include "famg.hpp"

namespace famg {

struct Sgs27Args {
    const uint32_t *codes;  // A's DIA codes (original rows), CW words per row
    const double *vtab;
    int ntab;
    int nx, ny, nz;
    int pz;     // plane parity of this phase
    int nst;    // in-plane colours applied, in order (<= 8)
    int px[8], py[8];
    const double *S;  // this parity's values before the phase
    const double *O;  // the other parity's values (read-only in the phase)
    double *T;        // this parity's values after the phase
    const double *b;
    int own_zero, other_zero;  // values known to be zero (sweep from e = 0): not read
    int ntiles;
    int ty;
    uint32_t icode[8];     // code group of an interior row (all 27 entries present)
    uint32_t fmask[6][8];  // code bits of the 9 entries leaving the grid at each face (x-,x+,y-,y+,z-,z+)
    double icoef[27];      // the interior row's coefficients (table values of icode)
    double idinv;          // 1 / icoef[13]
    const double *zero;    // >= nx zeros (rows outside the grid)
    const double *cpy_src; // optional: the tile's rows of plane z + 1 copied from cpy_src to cpy_dst
    double *cpy_dst;
    int jper;    // march: planes of the parity per workgroup
    int ext[8];  // march: colour s is computed on rows [y0 - ext[s], y1 + ext[s]) of its parity
    int halo;    // march: own rows staged from y0 - halo (max ext + 1)
    float rnx2;  // march: 1 / (nx / 2), rounded (q / (nx / 2) as (q + 0.5) * rnx2: exact for q < 2^14)
};


typedef double sgs_dbl2_t __attribute__((ext_vector_type(2)));
typedef uint32_t sgs_u32x4_t __attribute__((ext_vector_type(4)));

// One colour stage of a workgroup.  Work is split into wave tasks: a task is
// 64 consecutive points of the colour in one grid row y (x = PX + 2k, k =
// 64 seg + lane), so y -- and with it every row address the 27-point stencil
// needs (3 LDS rows of the own plane, 6 rows of the other parity's planes
// z +- 1, or a zero row where the row leaves the grid) -- is wave-uniform and
// lives in scalar registers; a lane only adds its x offset.  The three values
// x-1, x, x+1 of a row come from two aligned 16-B pair loads; the only lanes
// whose window leaves the row are x = 0 (PX = 0, k = 0) and x = nx-1 (PX = 1,
// k = nk-1), which clamp the pair address and select 0.0.  U tasks per trip
// with all loads issued before the sums.  (Sharing one pair load per lane
// through DPP wave shifts measured slower: each shift waits for its load.)
//
// A lane whose row carries the interior code group -- with the entries that
// leave the grid at its faces cleared to the +0.0 code, i.e. a constant
// stencil truncated at the boundary -- may use the interior coefficients from
// the kernel arguments instead of decoding 27 codes through the LDS table;
// when all lanes of the wave can, the wave does.  A replaced entry multiplies
// an x operand of 0.0 on both paths; the product (+-0.0) added to an
// accumulator that starts at +0.0 and can never become -0.0 leaves it
// unchanged, so the sums are bitwise the same.
// CST: every row is the interior stencil truncated at the grid faces (checked
// at setup), so no row's codes are loaded: the interior coefficients always.
// OL: the other parity's rows z -+ 1 come from an LDS copy (olds: orw rows per
// plane from grid row r0 - 1) instead of global memory.
template <int VB, int CW, int PX, int U, int NW, bool CST, bool OL>
__device__ __forceinline__ void sgs27_stage(const Sgs27Args &a, double *lds, const double *stab, const double *scoef,
                                            int z, int r0, int ys0, int ys1, int py, bool first_zero,
                                            const double *olds, int orw) {
    constexpr uint32_t MASK = (1u << VB) - 1;
    const int nx = a.nx, ny = a.ny, nz = a.nz;
    const int64_t plane = (int64_t)nx * ny;
    const int yfirst = ys0 + ((ys0 & 1) != py ? 1 : 0);
    const int nrow = yfirst < ys1 ? (ys1 - yfirst + 1) / 2 : 0;
    const int nk = nx / 2;  // points of each x parity per row (nx even)
    const int nseg = (nk + 63) >> 6;
    const int ntask = nrow * nseg;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const bool zlo = z == 0, zhi = z == nz - 1;
    for (int t0 = wave; t0 < ntask; t0 += NW * U) {
        double w[U][9][3];
        uint32_t cw[U][CW];
        double br[U];
        int li[U];
        bool live[U], inter = true;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = min(t0 + NW * u, ntask - 1);  // wave-uniform
            const int yr = t / nseg, sg = t - yr * nseg;
            const int y = yfirst + 2 * yr;
            const int k = (sg << 6) + lane;
            live[u] = t0 + NW * u < ntask && k < nk;
            const int x = PX + 2 * min(k, nk - 1);
            const bool lo = PX == 0 && x == 0, hi = PX == 1 && x == nx - 1;
            // pair offsets: A = [x-2+PX, x-1+PX], B = A + 2 (clamped into the row at the edges)
            const int offA = max(x - 2 + PX, 0), offB = min(x + PX, nx - 2);
            const int64_t rowg = (int64_t)z * plane + (int64_t)y * nx;
            const int64_t gi = rowg + x;
            li[u] = (y - r0 + 1) * nx + x;
#pragma unroll
            for (int q = 0; q < (CST ? 0 : CW / 4); q++) {
                const sgs_u32x4_t c =
                    __builtin_nontemporal_load(reinterpret_cast<const sgs_u32x4_t *>(a.codes + gi * CW) + q);
#pragma unroll
                for (int e = 0; e < 4; e++) cw[u][4 * q + e] = c[e];
            }
            br[u] = a.b[gi];
#pragma unroll
            for (int j = 0; j < 9; j++) {
                const int dz = j / 3 - 1, dy = j % 3 - 1;
                const int yy = y + dy, zz = z + dz;
                const bool rowok = yy >= 0 && yy < ny && zz >= 0 && zz < nz;  // wave-uniform
                const double *row;
                if (dz == 0) row = lds + (rowok ? (yy - r0 + 1) * nx : 0);  // LDS row 0: zeros
                else if (a.other_zero || !rowok) row = OL ? lds : a.zero;
                else if (OL) row = olds + ((dz > 0 ? orw : 0) + (yy - r0 + 1)) * nx;
                else row = a.O + rowg + (int64_t)dz * plane + (int64_t)dy * nx;
                const sgs_dbl2_t pa = *reinterpret_cast<const sgs_dbl2_t *>(row + offA);
                const sgs_dbl2_t pb = *reinterpret_cast<const sgs_dbl2_t *>(row + offB);
                if (PX == 0) {
                    w[u][j][0] = lo ? 0.0 : pa.y;
                    w[u][j][1] = pb.x;
                    w[u][j][2] = pb.y;
                } else {
                    w[u][j][0] = pa.x;
                    w[u][j][1] = pa.y;
                    w[u][j][2] = hi ? 0.0 : pb.x;
                }
            }
            // the interior group with the entries leaving the grid cleared
            const bool ylo = y == 0, yhi = y == ny - 1;
#pragma unroll
            for (int q = 0; q < (CST ? 0 : CW); q++) {
                const uint32_t clr = (lo ? a.fmask[0][q] : 0u) | (hi ? a.fmask[1][q] : 0u) |
                                     (ylo ? a.fmask[2][q] : 0u) | (yhi ? a.fmask[3][q] : 0u) |
                                     (zlo ? a.fmask[4][q] : 0u) | (zhi ? a.fmask[5][q] : 0u);
                inter = inter && cw[u][q] == (a.icode[q] & ~clr);
            }
        }
        double acc[U], dr[U];
        if (CST || __all(inter)) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                acc[u] = 0.0;
#pragma unroll
                for (int k = 0; k < 27; k++) acc[u] = fma(a.icoef[k], w[u][k / 3][k % 3], acc[u]);  // LDS broadcast
                dr[u] = a.idinv;
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                acc[u] = 0.0;
#pragma unroll
                for (int k = 0; k < 27; k++)
                    acc[u] = fma(stab[(cw[u][(k * VB) >> 5] >> ((k * VB) & 31)) & MASK], w[u][k / 3][k % 3], acc[u]);
                dr[u] = 1.0 / stab[(cw[u][(13 * VB) >> 5] >> ((13 * VB) & 31)) & MASK];
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const double xr = w[u][4][1];  // the point's own old value
            if (live[u]) lds[li[u]] = first_zero ? dr[u] * br[u] : xr + dr[u] * (br[u] - acc[u]);
        }
    }
}

template <int VB, int CW, int U, int NW, bool CST, bool OL>
__global__ __launch_bounds__(64 * NW) void k_sgs27_phase(Sgs27Args a) {
    constexpr int NT = 64 * NW;
    extern __shared__ sgs_dbl2_t lds_pairs[];  // 16-B aligned: rows are read as pairs
    double *lds = reinterpret_cast<double *>(lds_pairs);  // row 0: zeros; row 1 + (y - r0): grid row y
    __shared__ double stab[VB == 4 ? 16 : 256];
    __shared__ double scoef[28];  // interior coefficients + 1/a_ii (uniform reads: LDS broadcast, no SGPR pressure)
    const int tid = threadIdx.x;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    if (tid < 27) scoef[tid] = a.icoef[tid];
    if (tid == 27) scoef[27] = a.idinv;
    const int zp = w / a.ntiles, tile = w - zp * a.ntiles;
    const int z = 2 * zp + a.pz;
    const int nx = a.nx, ny = a.ny;
    const int y0 = tile * a.ty, y1 = min(y0 + a.ty, ny);
    const int r0 = max(y0 - a.nst, 0), r1 = min(y1 + a.nst, ny);
    const int64_t zoff = (int64_t)z * nx * ny;
    for (int q = tid; q < a.ntab; q += NT) stab[q] = a.vtab[q];
    const int nx2 = nx / 2;
    const int nload2 = (r1 - r0) * nx2;  // nx even: whole rows of 16-B pairs
    sgs_dbl2_t *l2 = reinterpret_cast<sgs_dbl2_t *>(lds);
    for (int q = tid; q < nx2; q += NT) l2[q] = sgs_dbl2_t{0.0, 0.0};
    if (a.own_zero) {
        for (int q = tid; q < nload2; q += NT) l2[nx2 + q] = sgs_dbl2_t{0.0, 0.0};
    } else {
        // all of a lane's loads issued before its LDS writes (a load-wait-write
        // loop serialises ~13 memory latencies per workgroup)
        const sgs_dbl2_t *src = reinterpret_cast<const sgs_dbl2_t *>(a.S + zoff + (int64_t)r0 * nx);
        constexpr int PF = 8;
        for (int q0 = tid; q0 < nload2; q0 += NT * PF) {
            sgs_dbl2_t v[PF];
#pragma unroll
            for (int u = 0; u < PF; u++) v[u] = src[min(q0 + NT * u, nload2 - 1)];
#pragma unroll
            for (int u = 0; u < PF; u++)
                if (q0 + NT * u < nload2) l2[nx2 + q0 + NT * u] = v[u];
        }
    }
    // OL: rows r0-1 .. r1 of planes z-1 and z+1 (zeros outside the grid)
    const int orw = a.ty + 2 * a.nst + 2;
    double *olds = lds + (int64_t)(1 + a.ty + 2 * a.nst) * nx;
    if (OL && !a.other_zero) {
        const int nrow_o = r1 - r0 + 2;
        const int nload_o = 2 * nrow_o * nx2;
        sgs_dbl2_t *o2 = reinterpret_cast<sgs_dbl2_t *>(olds);
        constexpr int PF = 4;
        for (int q0 = tid; q0 < nload_o; q0 += NT * PF) {
            sgs_dbl2_t v[PF];
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int q = q0 + NT * u;
                const int pr = q / nx2, c = q - pr * nx2;      // pr: plane-row index
                const int pi = pr >= nrow_o ? 1 : 0, j = pr - pi * nrow_o;
                const int yy = r0 - 1 + j, zz = z + (pi ? 1 : -1);
                const bool ok = q < nload_o && yy >= 0 && yy < ny && zz >= 0 && zz < a.nz;
                v[u] = ok ? reinterpret_cast<const sgs_dbl2_t *>(a.O + (int64_t)zz * nx * ny + (int64_t)yy * nx)[c]
                          : sgs_dbl2_t{0.0, 0.0};
            }
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int q = q0 + NT * u;
                if (q < nload_o) {
                    const int pr = q / nx2, c = q - pr * nx2;
                    const int pi = pr >= nrow_o ? 1 : 0, j = pr - pi * nrow_o;
                    o2[(pi * orw + j) * nx2 + c] = v[u];
                }
            }
        }
    }
    __syncthreads();
    for (int s = 0; s < a.nst; s++) {
        const int h = a.nst - 1 - s;
        const int ys0 = max(y0 - h, 0), ys1 = min(y1 + h, ny);
        const bool first_zero = a.own_zero && a.other_zero && s == 0;
        if (a.px[s] == 0) sgs27_stage<VB, CW, 0, U, NW, CST, OL>(a, lds, stab, scoef, z, r0, ys0, ys1, a.py[s], first_zero, olds, orw);
        else sgs27_stage<VB, CW, 1, U, NW, CST, OL>(a, lds, stab, scoef, z, r0, ys0, ys1, a.py[s], first_zero, olds, orw);
        __syncthreads();
    }
    sgs_dbl2_t *dst = reinterpret_cast<sgs_dbl2_t *>(a.T + zoff + (int64_t)y0 * nx);
    const sgs_dbl2_t *srcl = reinterpret_cast<const sgs_dbl2_t *>(lds + (y0 - r0 + 1) * nx);
    for (int q = tid; q < (y1 - y0) * nx2; q += NT) dst[q] = srcl[q];
    if (a.cpy_src && z + 1 < a.nz) {  // plane z + 1 (the other parity) carried to the next phase's source
        const int64_t o = zoff + (int64_t)nx * ny + (int64_t)y0 * nx;
        const sgs_dbl2_t *cs = reinterpret_cast<const sgs_dbl2_t *>(a.cpy_src + o);
        sgs_dbl2_t *cd = reinterpret_cast<sgs_dbl2_t *>(a.cpy_dst + o);
        for (int q = tid; q < (y1 - y0) * nx2; q += NT) cd[q] = cs[q];
    }
}


// Marching phase (CST, nx <= 256): one workgroup per (grid-row tile, run of
// jper planes of the parity).  Three LDS slots of rows r0 - 1 .. r1 (zero rows
// outside the grid, so no row needs a range test): the own plane and the other
// parity's planes z - 1 and z + 1.  While plane z runs its colours, registers
// fetch plane z + 2's own rows and plane z + 3's rows; after z's rows are
// written they go to the own slot and to the slot that held plane z - 1.  Each
// plane of the other parity is staged once per tile column instead of twice,
// and the staging overlaps the colour stages.  Per point the arithmetic is
// sgs27_stage's (bitwise the colour launches).
template <int NW, int PFS, int PFO>
__device__ __forceinline__ void sgs27m_fetch(const Sgs27Args &a, int z, int zz, int r0, int nown2, int npl2,
                                             bool own, sgs_dbl2_t (&vo)[PFS], sgs_dbl2_t (&vp)[PFO]) {
    constexpr int NT = 64 * NW;
    const int nx = a.nx, ny = a.ny, nx2 = nx / 2;
    const int tid = threadIdx.x;
    if (own) {
        const sgs_dbl2_t *src = reinterpret_cast<const sgs_dbl2_t *>(a.S + ((int64_t)z * ny + r0) * nx);
#pragma unroll
        for (int u = 0; u < PFS; u++) vo[u] = src[min(tid + NT * u, nown2 - 1)];
    }
    const bool pok = !a.other_zero && zz >= 0 && zz < a.nz;
    const sgs_dbl2_t *o2 = reinterpret_cast<const sgs_dbl2_t *>(a.O + (int64_t)zz * nx * ny);
#pragma unroll
    for (int u = 0; u < PFO; u++) {
        const int q = min(tid + NT * u, npl2 - 1);
        const int pr = (int)(((float)q + 0.5f) * a.rnx2), c = q - pr * nx2;
        const int yy = r0 - 1 + pr;
        vp[u] = pok && yy >= 0 && yy < ny ? o2[(int64_t)yy * nx2 + c] : sgs_dbl2_t{0.0, 0.0};
    }
}

// One colour of a marching phase.  Slot rows have a stride of nx + 4 doubles,
// x at 2 + x, two zero columns on each side (never written), so the window
// x - 1 .. x + 1 needs neither clamps nor selects: one 8-B and one 16-B read
// per row.  Waves are split over the row's 64-point segments without a
// division: wave w takes segment w % nseg of rows w / nseg, w / nseg + NW / nseg, ...
template <int PX, int NW>
__device__ __forceinline__ void sgs27m_stage(const Sgs27Args &a, double *own, const double *lo, const double *hi,
                                             int z, int r0, int ys0, int ys1, int py, bool first_zero) {
    const int nx = a.nx, ny = a.ny, rs = nx + 4;
    const int yfirst = ys0 + ((ys0 & 1) != py ? 1 : 0);
    const int nrow = yfirst < ys1 ? (ys1 - yfirst + 1) / 2 : 0;
    const int nk = nx / 2;
    const int nseg = (nk + 63) >> 6;  // 1 or 2 (nx <= 256): divides NW
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int sg = wave & (nseg - 1), wstep = NW / nseg;
    const int k = (sg << 6) + lane;
    const bool live = k < nk;
    const int x = PX + 2 * min(k, nk - 1);
    const int o16 = 2 + x - PX, o8 = PX == 0 ? 1 + x : 3 + x;  // [x - PX, x - PX + 1] and the third value
    const double *planes[3] = {lo, own, hi};
    for (int yr = wave / nseg; yr < nrow; yr += wstep) {
        const int y = yfirst + 2 * yr;
        const double br = a.b[((int64_t)z * ny + y) * nx + x];
        double w[9][3];
#pragma unroll
        for (int j = 0; j < 9; j++) {
            const double *row = planes[j / 3] + (y + j % 3 - r0) * rs;
            const sgs_dbl2_t p = *reinterpret_cast<const sgs_dbl2_t *>(row + o16);
            const double v = row[o8];
            w[j][0] = PX == 0 ? v : p.x;
            w[j][1] = PX == 0 ? p.x : p.y;
            w[j][2] = PX == 0 ? p.y : v;
        }
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 27; q++) acc = fma(a.icoef[q], w[q / 3][q % 3], acc);  // coefficients in SGPRs
        const double xr = w[4][1];
        if (live) own[(y - r0 + 1) * rs + 2 + x] = first_zero ? a.idinv * br : xr + a.idinv * (br - acc);
    }
}

// pairs q of a row set (nx / 2 per row) -> LDS pair index in slot rows of nx + 4
__device__ __forceinline__ int sgs27m_lpair(int q, int nx2, float rnx2) {
    const int pr = (int)(((float)q + 0.5f) * rnx2);
    return pr * (nx2 + 2) + 1 + (q - pr * nx2);
}

template <int NW, int PFS, int PFO>
__global__ __launch_bounds__(64 * NW) void k_sgs27_march(Sgs27Args a) {
    constexpr int NT = 64 * NW;
    extern __shared__ sgs_dbl2_t lds_pairs[];
    double *lds = reinterpret_cast<double *>(lds_pairs);
    const int tid = threadIdx.x;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = w / a.ntiles, tile = w - chunk * a.ntiles;
    const int nplanes = (a.nz - a.pz + 1) / 2;
    const int j0 = chunk * a.jper, j1 = min(j0 + a.jper, nplanes);
    const int nx = a.nx, ny = a.ny, nx2 = nx / 2, rs = nx + 4;
    const int y0 = tile * a.ty, y1 = min(y0 + a.ty, ny);
    const int r0 = max(y0 - a.halo, 0), r1 = min(y1 + a.halo, ny);
    const int nown2 = (r1 - r0) * nx2, npl2 = (r1 - r0 + 2) * nx2;
    const int srw = a.ty + 2 * a.halo + 2;  // rows per slot
    double *own = lds, *lo = lds + (int64_t)srw * rs, *hi = lo + (int64_t)srw * rs;
    sgs_dbl2_t *ow2 = reinterpret_cast<sgs_dbl2_t *>(own);
    // everything zero first: the pad columns and the own slot's rows r0 - 1 and r1
    // are read where they leave the grid and never written
    for (int q = tid; q < 3 * srw * (nx2 + 2); q += NT) lds_pairs[q] = sgs_dbl2_t{0.0, 0.0};
    __syncthreads();
    int z = 2 * j0 + a.pz;
    {
        sgs_dbl2_t vo[PFS], vp[PFO], vq[PFO];
        sgs27m_fetch<NW, PFS, PFO>(a, z, z - 1, r0, nown2, npl2, !a.own_zero, vo, vp);
        sgs_dbl2_t dummy[PFS];
        sgs27m_fetch<NW, PFS, PFO>(a, z, z + 1, r0, nown2, npl2, false, dummy, vq);
        if (!a.own_zero) {
#pragma unroll
            for (int u = 0; u < PFS; u++)
                if (tid + NT * u < nown2) ow2[(nx2 + 2) + sgs27m_lpair(tid + NT * u, nx2, a.rnx2)] = vo[u];
        }
        sgs_dbl2_t *s0 = reinterpret_cast<sgs_dbl2_t *>(lo), *s1 = reinterpret_cast<sgs_dbl2_t *>(hi);
#pragma unroll
        for (int u = 0; u < PFO; u++)
            if (tid + NT * u < npl2) {
                const int l = sgs27m_lpair(tid + NT * u, nx2, a.rnx2);
                s0[l] = vp[u];
                s1[l] = vq[u];
            }
    }
    __syncthreads();
    for (int j = j0; j < j1; j++, z += 2) {
        const bool more = j + 1 < j1;
        sgs_dbl2_t vo[PFS], vp[PFO];
        if (more) sgs27m_fetch<NW, PFS, PFO>(a, z + 2, z + 3, r0, nown2, npl2, !a.own_zero, vo, vp);
        for (int s = 0; s < a.nst; s++) {
            const int h = a.ext[s];
            const int ys0 = max(y0 - h, 0), ys1 = min(y1 + h, ny);
            const bool first_zero = a.own_zero && a.other_zero && s == 0;
            if (a.px[s] == 0) sgs27m_stage<0, NW>(a, own, lo, hi, z, r0, ys0, ys1, a.py[s], first_zero);
            else sgs27m_stage<1, NW>(a, own, lo, hi, z, r0, ys0, ys1, a.py[s], first_zero);
            __syncthreads();
        }
        sgs_dbl2_t *dst = reinterpret_cast<sgs_dbl2_t *>(a.T + ((int64_t)z * ny + y0) * nx);
        const sgs_dbl2_t *srcl = ow2 + (y0 - r0 + 1) * (nx2 + 2);
        for (int q = tid; q < (y1 - y0) * nx2; q += NT) dst[q] = srcl[sgs27m_lpair(q, nx2, a.rnx2)];
        if (more) {
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PFS; u++)
                if (tid + NT * u < nown2)
                    ow2[(nx2 + 2) + sgs27m_lpair(tid + NT * u, nx2, a.rnx2)] = a.own_zero ? sgs_dbl2_t{0.0, 0.0} : vo[u];
            sgs_dbl2_t *sl = reinterpret_cast<sgs_dbl2_t *>(lo);
#pragma unroll
            for (int u = 0; u < PFO; u++)
                if (tid + NT * u < npl2) sl[sgs27m_lpair(tid + NT * u, nx2, a.rnx2)] = vp[u];
            double *t = lo;
            lo = hi;
            hi = t;
            __syncthreads();
        }
    }
}

// FAMG_SGS_FUSED=0 (or amg_set_sgs_fused(0)): colour launches instead of the
// fused phases; 2: four phases per step instead of three (A/B, tests)
int g_sgs_fused = [] {
    const char *e = getenv("FAMG_SGS_FUSED");
    return (e && e[0] == '0') ? 0 : (e && e[0] == '2') ? 2 : 1;
}();
static bool sgs_fused_enabled() { return g_sgs_fused != 0; }

// rows per workgroup and independent points per lane (A/B switches
// FAMG_SGS27_TY, FAMG_SGS27_U)
static int sgs27_ty() {
    static const int v = [] {
        const char *e = getenv("FAMG_SGS27_TY");
        const int t = e ? atoi(e) : 0;
        return t >= 2 && t <= 64 ? t : 16;
    }();
    return v;
}
static int sgs27_u() {
    static const int v = [] {
        const char *e = getenv("FAMG_SGS27_U");
        return (e && e[0] == '2') ? 2 : 1;
    }();
    return v;
}
// waves per workgroup (FAMG_SGS27_NW: 4 or 8)
static int sgs27_nw() {
    static const int v = [] {
        const char *e = getenv("FAMG_SGS27_NW");
        return (e && e[0] == '8') ? 8 : 4;
    }();
    return v;
}
// FAMG_SGS27_CST=0: load every row's codes even for a constant stencil (A/B)
static bool sgs27_cst() {
    static const bool on = [] {
        const char *e = getenv("FAMG_SGS27_CST");
        return !(e && e[0] == '0');
    }();
    return on;
}
// The other parity's rows in LDS too (1024-thread workgroups, one per CU):
// rows of TY + 2 nst (own) + 2 (TY + 2 nst + 2) (planes z -+ 1) doubles of nx
// within 160 KB.  Returns the TY used, 0 if it does not fit or FAMG_SGS27_OL=0.
static int sgs27_ol_ty(int nx, int nst) {
    static const bool on = [] {
        const char *e = getenv("FAMG_SGS27_OL");
        return !(e && e[0] == '0');
    }();
    if (!on) return 0;
    for (int ty : {16, 12, 8, 4})
        if ((size_t)(ty + 2 * nst + 1 + 2 * (ty + 2 * nst + 2)) * nx * sizeof(double) <= 160 * 1024) return ty;
    return 0;
}
// odd planes' forward and backward colours in one phase (g_sgs_fused == 2: two)
static int sgs27_p23() { return g_sgs_fused != 2; }
constexpr int SGS27_MAX_NX = 512;  // LDS: (TY + 8) rows of nx doubles (TY = 16: 96 KB at nx = 512)

__global__ void k_sgs27_check(const uint32_t *codes, int cw, int vb, int zcode, int nx, int ny, int nz,
                              int *bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = (int64_t)nx * ny * nz;
    if (i >= n) return;
    const int x = (int)(i % nx), y = (int)((i / nx) % ny), z = (int)(i / ((int64_t)nx * ny));
    const uint32_t mask = (1u << vb) - 1;
    for (int k = 0; k < 27; k++) {
        const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
        const bool in = x + dx >= 0 && x + dx < nx && y + dy >= 0 && y + dy < ny && z + dz >= 0 && z + dz < nz;
        const uint32_t c = (codes[i * cw + ((k * vb) >> 5)] >> ((k * vb) & 31)) & mask;
        if (!in && (int)c != zcode) bad[0] = 1;
    }
}

struct Sgs27Const {
    uint32_t icode[8], fmask[6][8];
};
// every row equals the interior code group with the entries leaving the grid cleared
__global__ void k_sgs27_const(const uint32_t *codes, int cw, Sgs27Const c, int nx, int ny, int nz, int *bad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = (int64_t)nx * ny * nz;
    if (i >= n) return;
    const int x = (int)(i % nx), y = (int)((i / nx) % ny), z = (int)(i / ((int64_t)nx * ny));
    for (int q = 0; q < cw; q++) {
        const uint32_t clr = (x == 0 ? c.fmask[0][q] : 0u) | (x == nx - 1 ? c.fmask[1][q] : 0u) |
                             (y == 0 ? c.fmask[2][q] : 0u) | (y == ny - 1 ? c.fmask[3][q] : 0u) |
                             (z == 0 ? c.fmask[4][q] : 0u) | (z == nz - 1 ? c.fmask[5][q] : 0u);
        if (codes[i * cw + q] != (c.icode[q] & ~clr)) bad[0] = 1;
    }
}

// A 7- or 27-point DIA operator (whole matrix, offsets of an nx x ny x nz grid,
// nx even) whose every row is the interior row's code group with the entries
// leaving the grid cleared to the +0.0 code (code 0): the SpMV can use the
// interior coefficients and zero the x operands that leave the grid instead of
// decoding each row's codes (the CST DIA kernels: the same products, the
// cleared ones +-0.0 added to an accumulator that is never -0.0).
bool dia_constant(GpuCsr &m) {
    m.dia_cst = false;
    const int K = m.dia_k;
    if (!m.has_dia() || m.dia_rowid || m.dia_r0 != 0 || m.dia_r1 != m.nrows || (K != 27 && K != 7) ||
        m.nrows != m.ncols || m.dia_pat)
        return false;
    if (K == 27 && !((m.dia_vbits == 4 && m.dia_cw == 4) || (m.dia_vbits == 8 && m.dia_cw == 8))) return false;
    if (K * m.dia_vbits > 32 * m.dia_cw || m.dia_cw > 8) return false;
    // the grid steps of diagonal k
    int st[27][3];
    for (int k = 0; k < K; k++) {
        if (K == 27) {
            st[k][0] = k % 3 - 1; st[k][1] = (k / 3) % 3 - 1; st[k][2] = k / 9 - 1;
        } else {
            static const int s7[7][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
            for (int q = 0; q < 3; q++) st[k][q] = s7[k][q];
        }
    }
    const std::vector<int> &off = m.dia_off;
    const int64_t nx = K == 27 ? off[16] : off[5], pl = K == 27 ? off[22] : off[6];
    if (nx < 2 || (nx & 1) || pl <= 0 || pl % nx != 0 || m.nrows % pl != 0) return false;
    const int64_t ny = pl / nx, nz = m.nrows / pl;
    for (int k = 0; k < K; k++)
        if (off[k] != st[k][2] * pl + st[k][1] * nx + st[k][0]) return false;
    hipStream_t s = m.ctx->stream;
    std::vector<double> tab(m.dia_ntab);
    FAMG_CHECK_HIP(hipMemcpyAsync(tab.data(), m.dia_vtab.get(), tab.size() * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    uint64_t bits0 = 1;
    if (!tab.empty()) std::memcpy(&bits0, &tab[0], 8);
    if (bits0 != 0) return false;  // code 0 must be +0.0
    const int64_t ic = ((nz / 2) * ny + ny / 2) * nx + nx / 2;
    std::vector<uint32_t> w(m.dia_cw);
    FAMG_CHECK_HIP(hipMemcpyAsync(w.data(), m.dia_codes.get() + ic * m.dia_cw, m.dia_cw * 4, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    const uint32_t mask = (1u << m.dia_vbits) - 1;
    Sgs27Const c;
    for (int q = 0; q < 8; q++) c.icode[q] = q < m.dia_cw ? w[q] : 0xffffffffu;
    for (int f = 0; f < 6; f++)
        for (int q = 0; q < 8; q++) c.fmask[f][q] = 0;
    for (int k = 0; k < K; k++) {
        const int dx = st[k][0], dy = st[k][1], dz = st[k][2];
        const uint32_t b = mask << ((k * m.dia_vbits) & 31);
        const int q = (k * m.dia_vbits) >> 5;
        if (dx < 0) c.fmask[0][q] |= b;
        if (dx > 0) c.fmask[1][q] |= b;
        if (dy < 0) c.fmask[2][q] |= b;
        if (dy > 0) c.fmask[3][q] |= b;
        if (dz < 0) c.fmask[4][q] |= b;
        if (dz > 0) c.fmask[5][q] |= b;
    }
    // code bits past the K diagonals must match too (they are the +0.0 padding)
    DevBuf<int> bad(1);
    FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
    hipLaunchKernelGGL(k_sgs27_const, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s, m.dia_codes.get(),
                       m.dia_cw, c, (int)nx, (int)ny, (int)nz, bad.get());
    FAMG_CHECK_HIP(hipGetLastError());
    int hb = 1;
    FAMG_CHECK_HIP(hipMemcpyAsync(&hb, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (hb) return false;
    for (int k = 0; k < K; k++) m.dia_cst_v[k] = tab[(w[(k * m.dia_vbits) >> 5] >> ((k * m.dia_vbits) & 31)) & mask];
    m.dia_cst_n[0] = (int)nx;
    m.dia_cst_n[1] = (int)ny;
    m.dia_cst_n[2] = (int)nz;
    m.dia_cst = true;
    return true;
}

// Decide whether S's sweeps can run as fused plane-parity phases: A is stored
// as DIA codes (whole matrix) with the 27 offsets of an nx x ny x nz grid, the
// colouring is the parity colouring, and every entry that would leave the grid
// carries the +0.0 code.
void sgs27_setup(SgsOp &S) {
    S.fused27 = false;
    if (!sgs_fused_enabled() || !S.A) return;
    const GpuCsr &m = S.A->m;
    if (m.kernel != SPMV_KERNEL_DIA || !m.has_dia() || m.dia_rowid || m.dia_r0 != 0 || m.dia_r1 != m.nrows ||
        m.dia_k != 27 || m.nrows != m.ncols)
        return;
    if (!((m.dia_vbits == 4 && m.dia_cw == 4) || (m.dia_vbits == 8 && m.dia_cw == 8))) return;
    const std::vector<int> &off = m.dia_off;
    const int nx = off[16];       // diagonal (dz, dy, dx) = (0, +1, 0)
    if (nx < 2 || nx > SGS27_MAX_NX || (nx & 1)) return;  // even rows: aligned 16-B pairs
    const int64_t pl = off[22];   // diagonal (+1, 0, 0): nx * ny
    if (pl <= 0 || pl % nx != 0 || m.nrows % pl != 0) return;
    const int ny = (int)(pl / nx), nz = (int)(m.nrows / pl);
    for (int k = 0; k < 27; k++) {
        const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
        if (off[k] != (int64_t)dz * pl + (int64_t)dy * nx + dx) return;
    }
    if ((int64_t)S.host_colors.size() != m.nrows) return;
    for (int64_t i = 0; i < m.nrows; i++) {
        const int x = (int)(i % nx), y = (int)((i / nx) % ny), z = (int)(i / pl);
        if (S.host_colors[i] != (x & 1) + 2 * (y & 1) + 4 * (z & 1)) return;
    }
    // the +0.0 code: the table is sorted by bit pattern and holds +0.0
    std::vector<double> tab(m.dia_ntab);
    hipStream_t s = S.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(tab.data(), m.dia_vtab.get(), tab.size() * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    int zcode = -1;
    for (size_t q = 0; q < tab.size(); q++) {
        uint64_t bits;
        std::memcpy(&bits, &tab[q], 8);
        if (bits == 0) zcode = (int)q;
    }
    if (zcode < 0) return;
    DevBuf<int> bad(1);
    FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
    hipLaunchKernelGGL(k_sgs27_check, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s, m.dia_codes.get(),
                       m.dia_cw, m.dia_vbits, zcode, nx, ny, nz, bad.get());
    FAMG_CHECK_HIP(hipGetLastError());
    int hbad = 1;
    FAMG_CHECK_HIP(hipMemcpyAsync(&hbad, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (hbad) return;
    // code group of an interior row (the grid centre) and its coefficients
    {
        const int64_t ic = ((int64_t)(nz / 2) * ny + ny / 2) * nx + nx / 2;
        std::vector<uint32_t> w(m.dia_cw);
        FAMG_CHECK_HIP(hipMemcpyAsync(w.data(), m.dia_codes.get() + ic * m.dia_cw, m.dia_cw * 4,
                                      hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        S.icode27.assign(8, 0xffffffffu);
        for (int q = 0; q < m.dia_cw; q++) S.icode27[q] = w[q];
        S.icoef27.assign(27, 0.0);
        const uint32_t mask = (1u << m.dia_vbits) - 1;
        for (int k = 0; k < 27; k++)
            S.icoef27[k] = tab[(w[(k * m.dia_vbits) >> 5] >> ((k * m.dia_vbits) & 31)) & mask];
        // face masks: code bits of the entries with dx = -1 / +1, dy = -1 / +1, dz = -1 / +1
        S.fmask27.assign(6 * 8, 0u);
        for (int k = 0; k < 27; k++) {
            const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
            const uint32_t bits = mask << ((k * m.dia_vbits) & 31);
            const int q = (k * m.dia_vbits) >> 5;
            if (dx < 0) S.fmask27[0 * 8 + q] |= bits;
            if (dx > 0) S.fmask27[1 * 8 + q] |= bits;
            if (dy < 0) S.fmask27[2 * 8 + q] |= bits;
            if (dy > 0) S.fmask27[3 * 8 + q] |= bits;
            if (dz < 0) S.fmask27[4 * 8 + q] |= bits;
            if (dz > 0) S.fmask27[5 * 8 + q] |= bits;
        }
        if (zcode != 0) S.icode27.assign(8, 0xffffffffu);  // cleared entries would not read code 0: no fast path
    }
    // a constant stencil truncated at the faces: the phases load no codes
    S.const27 = false;
    if (zcode == 0) {
        Sgs27Const c;
        for (int q = 0; q < 8; q++) c.icode[q] = S.icode27[q];
        for (int f = 0; f < 6; f++)
            for (int q = 0; q < 8; q++) c.fmask[f][q] = S.fmask27[f * 8 + q];
        FAMG_CHECK_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int), s));
        hipLaunchKernelGGL(k_sgs27_const, dim3((unsigned)ceil_div(m.nrows, 256)), dim3(256), 0, s,
                           m.dia_codes.get(), m.dia_cw, c, nx, ny, nz, bad.get());
        FAMG_CHECK_HIP(hipGetLastError());
        int hb = 1;
        FAMG_CHECK_HIP(hipMemcpyAsync(&hb, bad.get(), sizeof(int), hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        S.const27 = hb == 0 && sgs27_cst();
    }
    S.nx27 = nx;
    S.ny27 = ny;
    S.nz27 = nz;
    S.fused_tmp.resize(m.nrows);
    S.fused_zero.resize(nx + 8);
    FAMG_CHECK_HIP(hipMemsetAsync(S.fused_zero.get(), 0, (nx + 8) * sizeof(double), s));
    S.fused27 = true;
}

// One phase: the planes of parity pz run the in-plane colours (px, py)[0..nst);
// cpy_src/cpy_dst (optional): each workgroup also copies its rows of plane z + 1.
static void sgs27_phase(const SgsOp &S, int pz, int nst, const int *px, const int *py, const double *src,
                        const double *other, double *dst, const double *b, bool own_zero, bool other_zero,
                        hipStream_t s, const double *cpy_src = nullptr, double *cpy_dst = nullptr) {
    const GpuCsr &m = S.A->m;
    const int nplanes = (S.nz27 - pz + 1) / 2;
    if (nplanes <= 0) return;
    Sgs27Args a{};
    a.codes = m.dia_codes.get();
    a.vtab = m.dia_vtab.get();
    a.ntab = (int)m.dia_ntab;
    a.nx = S.nx27;
    a.ny = S.ny27;
    a.nz = S.nz27;
    a.pz = pz;
    a.nst = nst;
    for (int q = 0; q < nst; q++) {
        a.px[q] = px[q];
        a.py[q] = py[q];
    }
    a.S = src;
    a.O = other;
    a.T = dst;
    a.b = b;
    a.own_zero = own_zero;
    a.other_zero = other_zero;
    a.cpy_src = cpy_src;
    a.cpy_dst = cpy_dst;
    const bool ol = sgs27_ol_ty(S.nx27, nst) > 0;
    a.ty = ol ? sgs27_ol_ty(S.nx27, nst) : sgs27_ty();
    for (int q = 0; q < 8; q++) a.icode[q] = S.icode27[q];
    for (int f = 0; f < 6; f++)
        for (int q = 0; q < 8; q++) a.fmask[f][q] = S.fmask27[f * 8 + q];
    for (int k = 0; k < 27; k++) a.icoef[k] = S.icoef27[k];
    a.idinv = 1.0 / S.icoef27[13];
    a.zero = S.fused_zero.get();
    a.ntiles = (int)ceil_div(S.ny27, a.ty);
    const int64_t rows = (int64_t)nplanes * S.ny27 * S.nx27;
    // algorithmic bytes: the parity's x read (unless zero) + written, its codes
    // and b, the other parity's x read once (unless zero), the copied planes
    if (g_launch_log)
        log_launch("sgs27_phase", SPMV_KERNEL_DIA, SPMV_SGS, rows,
                   rows * (8 + (S.const27 ? 0 : 4 * (int64_t)m.dia_cw) + 8) + (own_zero ? 0 : rows * 8) +
                       (other_zero ? 0 : (int64_t)(m.nrows - rows) * 8) +
                       (cpy_src ? (int64_t)(m.nrows - rows) * 16 : 0));
    constexpr int MPFS = 3, MPFO = 4;  // march: pairs per thread of a tile's own rows / a plane's rows
    // Exact halos: colour t at row y reads colour s < t at rows y +- 1 when their row
    // parities differ and only at row y (the x neighbours) when they agree, so colour
    // s is needed on ext[s] = max over t > s of ext[t] + (py[t] != py[s]) rows beyond the
    // tile (forward: 1, 1, 0, 0) -- not nst - 1 - s (256^3 SGS step 285.8 -> 281.9 us).
    // Tile height 16 where it fits: the per-plane step's fixed costs favour tall
    // tiles over single-round colours (ty 12 / 14 / 16 / 20: 593 / 316 / 282 / 293 us).
    int ext[8] = {0}, emax = 0;
    for (int q = nst - 2; q >= 0; q--)
        for (int t = q + 1; t < nst; t++) ext[q] = std::max(ext[q], ext[t] + (py[t] != py[q] ? 1 : 0));
    for (int q = 0; q < nst; q++) emax = std::max(emax, ext[q]);
    const int halo = emax + 1;
    int tym = 0;
    for (int ty = 16; ty >= 4 && !tym; ty--) {
        if ((int64_t)(ty + 2 * halo) * (S.nx27 / 2) <= MPFS * 1024 &&
            (int64_t)(ty + 2 * halo + 2) * (S.nx27 / 2) <= MPFO * 1024 &&
            (size_t)3 * (ty + 2 * halo + 2) * (S.nx27 + 4) * sizeof(double) <= 160 * 1024)
            tym = std::min(ty, S.ny27);
    }

    if (ol && S.const27 && S.nx27 <= 256 && nst <= 4 && flag(FLAG_SGS27_MARCH) > 0 && !cpy_src && tym > 0) {
        for (int q = 0; q < 8; q++) a.ext[q] = ext[q];
        a.halo = halo;
        a.ty = tym;
        a.ntiles = (int)ceil_div(S.ny27, a.ty);
        const int cus = std::max(S.ctx->num_cus, 1);
        a.rnx2 = 1.0f / (float)(S.nx27 / 2);
        FAMG_REQUIRE(fdiv_exact((a.ty + 2 * halo + 2) * (S.nx27 / 2) + 1024, S.nx27 / 2, a.rnx2), AMG_ERR_UNSUPPORTED,
                     "sgs27 march: float reciprocal division not exact for this plane width");
        a.jper = flag(FLAG_SGS27_MARCH) > 1 ? (int)flag(FLAG_SGS27_MARCH) : (int)std::max<int64_t>(1, ceil_div((int64_t)nplanes * a.ntiles, cus));
        const int64_t nchunks = ceil_div(nplanes, a.jper);
        const size_t lds_m = (size_t)3 * (a.ty + 2 * halo + 2) * (S.nx27 + 4) * sizeof(double);
        k_sgs27_march<16, MPFS, MPFO><<<dim3((unsigned)(nchunks * a.ntiles)), dim3(1024), lds_m, s>>>(a);
        FAMG_CHECK_HIP(hipGetLastError());
        return;
    }
    const dim3 grid((unsigned)(nplanes * a.ntiles));
    const size_t lds = (size_t)(a.ty + 2 * nst + 1 + (ol ? 2 * (a.ty + 2 * nst + 2) : 0)) * S.nx27 * sizeof(double);
    const bool u2 = sgs27_u() == 2;
    const int nw = sgs27_nw();
#define FAMG_SGS27_LAUNCH(VB, CW, U, NW)                                                           \
    if (S.const27) k_sgs27_phase<VB, CW, U, NW, true, false><<<grid, dim3(64 * NW), lds, s>>>(a);   \
    else k_sgs27_phase<VB, CW, U, NW, false, false><<<grid, dim3(64 * NW), lds, s>>>(a)
    if (ol) {
        if (m.dia_vbits == 4) {
            if (S.const27) k_sgs27_phase<4, 4, 1, 16, true, true><<<grid, dim3(1024), lds, s>>>(a);
            else k_sgs27_phase<4, 4, 1, 16, false, true><<<grid, dim3(1024), lds, s>>>(a);
        } else {
            if (S.const27) k_sgs27_phase<8, 8, 1, 16, true, true><<<grid, dim3(1024), lds, s>>>(a);
            else k_sgs27_phase<8, 8, 1, 16, false, true><<<grid, dim3(1024), lds, s>>>(a);
        }
    } else if (m.dia_vbits == 4) {
        if (nw == 8) { if (u2) FAMG_SGS27_LAUNCH(4, 4, 2, 8); else FAMG_SGS27_LAUNCH(4, 4, 1, 8); }
        else { if (u2) FAMG_SGS27_LAUNCH(4, 4, 2, 4); else FAMG_SGS27_LAUNCH(4, 4, 1, 4); }
    } else {
        if (nw == 8) { if (u2) FAMG_SGS27_LAUNCH(8, 8, 2, 8); else FAMG_SGS27_LAUNCH(8, 8, 1, 8); }
        else { if (u2) FAMG_SGS27_LAUNCH(8, 8, 2, 4); else FAMG_SGS27_LAUNCH(8, 8, 1, 4); }
    }
#undef FAMG_SGS27_LAUNCH
    FAMG_CHECK_HIP(hipGetLastError());
}

// x <- SGS step (forward colours 0..7, backward 6..0) as plane-parity phases;
// zero: x starts at 0 (sweep from e = 0: nothing of x is read).
bool sgs27_applies(const SgsOp &S, const double *x, const double *b) {
    return S.fused27 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
}

void sgs27_sweep(SgsOp &S, double *x, const double *b, bool zero) {
    hipStream_t s = S.ctx->stream;
    double *t1 = S.fused_tmp.get();
    static const int fpx[4] = {0, 1, 0, 1}, fpy[4] = {0, 0, 1, 1};  // colours 0,1,2,3 / 4,5,6,7
    static const int bopx[3] = {0, 1, 0}, bopy[3] = {1, 0, 0};       // colours 6,5,4
    static const int bepx[4] = {1, 0, 1, 0}, bepy[4] = {1, 1, 0, 0}; // colours 3,2,1,0
    static const int opx[7] = {0, 1, 0, 1, 0, 1, 0}, opy[7] = {0, 0, 1, 1, 1, 0, 0};  // 4,5,6,7,6,5,4
    if (sgs27_p23() && sgs27_ol_ty(S.nx27, 4) == 0 && (size_t)(sgs27_ty() + 15) * S.nx27 * sizeof(double) <= 150 * 1024) {
        // three phases: the odd planes run forward and backward colours in one
        // launch; reading its source from t1 and writing x, it needs the odd
        // planes' old values in t1 -- the even phase copies them (none when zero)
        sgs27_phase(S, 0, 4, fpx, fpy, x, x, t1, b, zero, zero, s, zero ? nullptr : x, zero ? nullptr : t1);
        sgs27_phase(S, 1, 7, opx, opy, t1, t1, x, b, zero, false, s);   // odd planes -> x
        sgs27_phase(S, 0, 4, bepx, bepy, t1, x, x, b, false, false, s); // even planes -> x
        return;
    }
    sgs27_phase(S, 0, 4, fpx, fpy, x, x, t1, b, zero, zero, s);      // even planes -> t1
    sgs27_phase(S, 1, 4, fpx, fpy, x, t1, t1, b, zero, false, s);    // odd planes -> t1
    sgs27_phase(S, 1, 3, bopx, bopy, t1, t1, x, b, false, false, s); // odd planes -> x
    sgs27_phase(S, 0, 4, bepx, bepy, t1, x, x, b, false, false, s);  // even planes -> x
}

}  // namespace famg
