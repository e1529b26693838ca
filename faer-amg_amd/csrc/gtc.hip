// gtc.hip -- grid-transfer classes: SpMV storage for the transfer operators of
// a 2 x 2 x 2 box-aggregation hierarchy on a structured grid.
//
// P (fine rows, coarse columns; interpolation/mod.rs:716-720 smoothed) and
// R = P^T (coarse rows, fine columns) have rows whose entries sit at a few
// fixed grid steps from an anchor: P's row (x, y, z) reads coarse points
// (x/2, y/2, z/2) + {-1,0,1}^3, R's row (X, Y, Z) reads fine points
// (2X, 2Y, 2Z) + {-1,..,2}^3.  Away from the boundary the rows repeat with the
// parity of (x, y, z) (P) or not at all (R), so a row is one 8-bit class id
// into a dictionary of (step, value) lists.  P_0 of the 256^3 7-point
// hierarchy: 1 B per row instead of 12.5 B of value-code SELL; 27-point: 1 B
// instead of ~25 B.  Dictionary entries are 16 bits: the value's index in a
// table of the operator's distinct values (<= 256) and the step's slot.
//
// Kernels: one workgroup per grid tile stages the tile's column-grid window
// (the coarse v_c for P, the fine vector for R; 0.0 outside the grid) in LDS,
// then each lane sums its rows' entries in stored (ascending column) order
// with fma from the window -- bitwise the oracle's CSR row sums; epilogues
// SET, ADD (y += P v_c), ADD0 (y = d*b + P v_c, the folded zero-guess step).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "famg.hpp"

namespace famg {

// ------------------------------------------------------------ host classes

bool gtc_classes(const GpuCsr &M, bool is_r, const int64_t *fg, const int64_t *cg, std::vector<uint8_t> &cls,
                 std::vector<std::vector<std::pair<uint8_t, double>>> &dict) {
    const int64_t n = M.nrows, nnz = M.nnz;
    if (n <= 0 || nnz <= 0) return false;
    const int64_t rx = is_r ? cg[0] : fg[0], ry = is_r ? cg[1] : fg[1], rz = is_r ? cg[2] : fg[2];  // row grid
    const int64_t kx = is_r ? fg[0] : cg[0], ky = is_r ? fg[1] : cg[1], kz = is_r ? fg[2] : cg[2];  // column grid
    if (cg[0] != (fg[0] + 1) / 2 || cg[1] != (fg[1] + 1) / 2 || cg[2] != (fg[2] + 1) / 2) return false;
    // rows / columns: the whole grids, or (a rank-local matrix of a distributed
    // level) the owned planes of rframe over the [owned | ghost planes] vector of
    // cframe; classes and steps are taken in global grid coordinates, so a
    // local row gets its global row's class
    const SlabFrame &RF = M.rframe, &CF = M.cframe;
    if (RF.on() != CF.on()) return false;
    if (RF.on()) {
        if (RF.nx != rx || RF.ny != ry || RF.gz != rz || CF.nx != kx || CF.ny != ky || CF.gz != kz) return false;
        if (RF.n_own() != n || CF.n_own() + (CF.gl + CF.gh) * CF.pl() != M.ncols) return false;
    } else if (rx * ry * rz != n || kx * ky * kz != M.ncols) {
        return false;
    }
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    hipStream_t s = M.ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(rp.data(), M.rp64.get(), (n + 1) * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), M.col.get(), nnz * 4, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(val.data(), M.val.get(), nnz * 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    const int KEMAX = is_r ? 64 : 27;
    std::vector<uint8_t> slots(nnz);
    std::vector<uint64_t> h(n);
    bool ok = true;
#pragma omp parallel for schedule(static) reduction(&& : ok)
    for (int64_t i = 0; i < n; i++) {
        const int64_t x = i % rx, y = (i / rx) % ry, z = i / (rx * ry) + (RF.on() ? RF.z0 : 0);
        const int64_t ax = is_r ? 2 * x : x / 2, ay = is_r ? 2 * y : y / 2, az = is_r ? 2 * z : z / 2;  // anchor
        uint64_t hh = 0x9E3779B97F4A7C15ull ^ (uint64_t)(rp[i + 1] - rp[i]);
        int prev = -1;
        if (rp[i + 1] - rp[i] > KEMAX) ok = false;
        for (int64_t e = rp[i]; e < rp[i + 1]; e++) {
            const int64_t j = col[e];
            const int64_t jp = CF.on() ? CF.in_plane(j) : j % (kx * ky);
            const int64_t jz = CF.on() ? CF.plane_of(j) : j / (kx * ky);
            const int64_t dx = jp % kx - ax, dy = jp / kx - ay, dz = jz - az;
            int sl = 0;
            if (is_r) {
                if (dx < -1 || dx > 2 || dy < -1 || dy > 2 || dz < -1 || dz > 2) ok = false;
                else sl = (int)((dz + 1) * 16 + (dy + 1) * 4 + dx + 1);
            } else {
                if (dx < -1 || dx > 1 || dy < -1 || dy > 1 || dz < -1 || dz > 1) ok = false;
                else sl = (int)((dz + 1) * 9 + (dy + 1) * 3 + dx + 1);
            }
            if (sl <= prev) ok = false;  // ascending columns = ascending slots
            prev = sl;
            slots[e] = (uint8_t)sl;
            uint64_t bits;
            std::memcpy(&bits, &val[e], 8);
            hh = (hh ^ (uint64_t)sl) * 0x100000001B3ull;
            hh = (hh ^ bits) * 0xFF51AFD7ED558CCDull;
            hh ^= hh >> 29;
        }
        h[i] = hh;
    }
    if (!ok) return false;
    auto same = [&](int64_t i, int64_t j) {
        if (rp[i + 1] - rp[i] != rp[j + 1] - rp[j]) return false;
        for (int64_t a = rp[i], b = rp[j]; a < rp[i + 1]; a++, b++)
            if (slots[a] != slots[b] || std::memcmp(&val[a], &val[b], 8) != 0) return false;
        return true;
    };
    std::unordered_map<uint64_t, std::vector<int>> by_hash;
    std::vector<int64_t> rep;
    cls.assign(n, 0);
    int64_t last_i = -1;
    int last_c = -1;
    for (int64_t i = 0; i < n; i++) {
        int c = -1;
        if (last_c >= 0 && h[i] == h[last_i] && same(last_i, i)) c = last_c;  // runs of equal rows
        if (c < 0) {
            auto &cands = by_hash[h[i]];
            for (int q : cands)
                if (same(rep[q], i)) { c = q; break; }
            if (c < 0) {
                c = (int)rep.size();
                if (c >= 256) return false;
                rep.push_back(i);
                cands.push_back(c);
            }
        }
        cls[i] = (uint8_t)c;
        last_i = i;
        last_c = c;
    }
    dict.assign(rep.size(), {});
    for (size_t c = 0; c < rep.size(); c++)
        for (int64_t e = rp[rep[c]]; e < rp[rep[c] + 1]; e++) dict[c].push_back({slots[e], val[e]});
    return true;
}

// ------------------------------------------------------------ kernels

constexpr int GP_TX = 32, GP_TY = 8;                             // P: fine tile (TZ rows per lane along z)
constexpr int GP_WX = GP_TX / 2 + 2, GP_WY = GP_TY / 2 + 2;      // coarse window 18 x 6 x (TZ/2 + 2)
constexpr int GR_TX = 16, GR_TY = 8;                             // R: coarse tile (TZ rows per lane along z)
constexpr int GR_WX = 2 * GR_TX + 2, GR_WY = 2 * GR_TY + 2;      // fine window 34 x 18 x (2 TZ + 2)
constexpr int G_DMAX = 2048;   // P: dictionary entries (nclass * ke) staged in LDS
constexpr int G_RMAX = 8192;   // R: more boundary classes of 64 entries (R_1 of a radius-2 A_1)

struct GtcArgs {
    const uint8_t *cls;
    const uint16_t *dict;  // nclass x ke entries: value index << 8 | slot
    const double *vtab;    // distinct values
    int ke, nce, ntab;
    int rx, ry, rz;        // row grid (rz: the owned row planes of a rank-local matrix)
    int kx, ky, kz;        // column grid (kz: owned column planes)
    int ntx, nty;
    int tile0;             // first tile of this launch (z-tile range of a segment)
    // column planes: local plane Z is loadable for kz_lo <= Z < kz_hi (else 0.0) and
    // starts at Z * plane + (Z < 0 ? add_lo : Z >= kz ? add_hi : 0); rz0 / kz0 =
    // the global grid plane of local row / column plane 0 (single GPU: 0, 0, kz, 0, 0)
    int kz_lo, kz_hi, rz0, kz0;
    int64_t add_lo, add_hi;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const uint8_t *dc;
    const double *dt;
    int dconst;  // ADD0 / SETDF with coded d of one value: d = dk, no codes read
    double dk;
    double *y2;  // restriction SETDF: y2 = d * y (the next level's first Jacobi step from zero)
    int mz0, mz1, jper;  // marching R: coarse planes [mz0, mz1) of the launch, planes per workgroup
};

// The class dictionary and value table into LDS: every load of a lane issued
// before its stores (a load-wait-store loop serialises one memory latency per
// trip: 4 trips cost P_0 of the 256^3 cycle ~20 us)
template <int DMAX>
__device__ __forceinline__ void gtc_stage_dict(const GtcArgs &a, uint16_t *sd, double *st) {
    constexpr int PF = 8;
    const double t = a.vtab[min((int)threadIdx.x, a.ntab - 1)];
    for (int b = 0; b < a.nce; b += 256 * PF) {  // one trip per 2048 entries
        uint16_t v[PF];
#pragma unroll
        for (int u = 0; u < PF; u++) v[u] = a.dict[min(b + (int)threadIdx.x + 256 * u, a.nce - 1)];
#pragma unroll
        for (int u = 0; u < PF; u++)
            if (b + (int)threadIdx.x + 256 * u < a.nce) sd[b + threadIdx.x + 256 * u] = v[u];
    }
    if ((int)threadIdx.x < a.ntab) st[threadIdx.x] = t;
}

// P v_c over a fine tile of 32 x 8 x 4 points: lane (x, y) of the tile takes
// its four points along z; the coarse window 18 x 6 x 4 around them in LDS.
// NT: the fine-vector streams (b / y read, y written) non-temporal
template <int MODE, int GP_TZ, bool NT>
__global__ __launch_bounds__(256) void k_gtc_interp(GtcArgs a) {
    constexpr int GP_WZ = GP_TZ / 2 + 2;
    __shared__ double win[GP_WX * GP_WY * GP_WZ];
    __shared__ uint16_t sd[G_DMAX];
    __shared__ double st[256];
    __shared__ int16_t lut[27];
    const int tid = threadIdx.x;
    const int t = a.tile0 + xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int x0 = tix * GP_TX, y0 = tiy * GP_TY, z0 = tiz * GP_TZ;
    // window origin (local coarse planes; rz0 is even, so the tile's four fine
    // planes map to two coarse planes)
    const int wx0 = x0 / 2 - 1, wy0 = y0 / 2 - 1, wz0 = ((a.rz0 + z0) >> 1) - 1 - a.kz0;
    const int64_t fplane = (int64_t)a.rx * a.ry, cplane = (int64_t)a.kx * a.ky;
    // the rows' class ids and epilogue operands first
    const int lx = tid % GP_TX, ly = tid / GP_TX, gx = x0 + lx, gy = y0 + ly;
    __shared__ double sdt[256];  // the coded Jacobi diagonal's table (ADD0)
    int cl[GP_TZ], dci[GP_TZ];
    double yb[GP_TZ];
    bool live[GP_TZ];
    if constexpr (MODE == SPMV_ADD0)
        if (a.dc && !a.dconst) sdt[tid] = a.dt[tid];
    double dk = 0.0;
    if constexpr (MODE == SPMV_ADD0)
        if (a.dconst) dk = a.dk;
#pragma unroll
    for (int j = 0; j < GP_TZ; j++) {
        const int gz = z0 + j;
        live[j] = gx < a.rx && gy < a.ry && gz < a.rz;
        const int64_t i = live[j] ? (int64_t)gz * fplane + (int64_t)gy * a.rx + gx : 0;
        cl[j] = a.cls[i];
        yb[j] = 0.0;
        if (live[j]) {
            if constexpr (MODE == SPMV_ADD) yb[j] = NT ? __builtin_nontemporal_load(a.y + i) : a.y[i];
            if constexpr (MODE == SPMV_ADD0) {
                yb[j] = NT ? __builtin_nontemporal_load(a.b + i) : a.b[i];
                if (a.dconst) yb[j] = dk * yb[j];  // d*b (vec_mul's product)
                else if (a.dc) dci[j] = a.dc[i];
                else yb[j] = a.d[i] * yb[j];
            }
        }
    }
    for (int q = tid; q < GP_WX * GP_WY * GP_WZ; q += 256) {
        const int X = wx0 + q % GP_WX, Y = wy0 + (q / GP_WX) % GP_WY, Z = wz0 + q / (GP_WX * GP_WY);
        const bool in = (unsigned)X < (unsigned)a.kx && (unsigned)Y < (unsigned)a.ky && Z >= a.kz_lo && Z < a.kz_hi;
        const int64_t zb = (int64_t)Z * cplane + (Z < 0 ? a.add_lo : Z >= a.kz ? a.add_hi : 0);
        win[q] = in ? a.x[zb + (int64_t)Y * a.kx + X] : 0.0;
    }
    gtc_stage_dict<G_DMAX>(a, sd, st);
    if (tid < 27) lut[tid] = (int16_t)(((tid / 9 - 1) * GP_WY + (tid / 3) % 3 - 1) * GP_WX + tid % 3 - 1);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < GP_TZ; j++) {
        if (!live[j]) continue;
        if constexpr (MODE == SPMV_ADD0)
            if (a.dc && !a.dconst) yb[j] = sdt[dci[j]] * yb[j];  // d*b, d decoded after the barrier
        const int gz = z0 + j;
        const int base = ((((a.rz0 + gz) >> 1) - a.kz0 - wz0) * GP_WY + (gy >> 1) - wy0) * GP_WX + (gx >> 1) - wx0;
        const uint16_t *e = sd + cl[j] * a.ke;
        double acc = 0.0;
        for (int k = 0; k < a.ke; k += 4) {
            double v[4], w[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint16_t c = e[k + u];
                v[u] = st[c >> 8];
                w[u] = win[base + lut[c & 255]];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) acc = fma(v[u], w[u], acc);
        }
        const int64_t i = (int64_t)gz * fplane + (int64_t)gy * a.rx + gx;
        const double out = MODE == SPMV_SET ? acc : yb[j] + acc;  // ADD, ADD0: y + P v
        if (NT) __builtin_nontemporal_store(out, a.y + i);
        else a.y[i] = out;
    }
}

// R r over a coarse tile of 16 x 8 x GR_TZ points (GR_TZ / 2 rows per lane,
// along z); the fine window 34 x 18 x (2 GR_TZ + 2) around their boxes in LDS,
// the dictionary in dynamic LDS (nce entries).  DF (SETDF): also y2 = d * y.
template <int GR_TZ, bool DF>
__global__ __launch_bounds__(256) void k_gtc_restrict(GtcArgs a) {
    constexpr int GR_WZ = 2 * GR_TZ + 2, RL = GR_TZ / 2;
    __shared__ double win[GR_WX * GR_WY * GR_WZ];
    extern __shared__ uint16_t sd[];
    __shared__ double st[256];
    __shared__ int16_t lut[64];
    __shared__ double sdt[DF ? 256 : 1];  // SETDF: the coded diagonal's table
    const int tid = threadIdx.x;
    const int t = a.tile0 + xcd_remap(blockIdx.x, gridDim.x);
    const int tix = t % a.ntx, tiy = (t / a.ntx) % a.nty, tiz = t / (a.ntx * a.nty);
    const int X0 = tix * GR_TX, Y0 = tiy * GR_TY, Z0 = tiz * GR_TZ;
    const int wx0 = 2 * X0 - 1, wy0 = 2 * Y0 - 1, wz0 = 2 * (a.rz0 + Z0) - 1 - a.kz0;  // window origin (local fine)
    const int64_t cplane = (int64_t)a.rx * a.ry, fplane = (int64_t)a.kx * a.ky;
    const int lx = tid % GR_TX, ly = (tid / GR_TX) % GR_TY, lz0 = tid / (GR_TX * GR_TY);  // lz0 in {0, 1}
    bool live[RL];
    int64_t J[RL];
    int c[RL];
#pragma unroll
    for (int j = 0; j < RL; j++) {
        const int X = X0 + lx, Y = Y0 + ly, Z = Z0 + lz0 + 2 * j;
        live[j] = X < a.rx && Y < a.ry && Z < a.rz;
        J[j] = live[j] ? (int64_t)Z * cplane + (int64_t)Y * a.rx + X : 0;
        c[j] = a.cls[J[j]];
    }
    int dci[RL];  // SETDF with coded d: the rows' codes loaded with the class ids
    if constexpr (DF) {
        if (a.dc && !a.dconst) {
            sdt[tid] = a.dt[tid];
#pragma unroll
            for (int j = 0; j < RL; j++) dci[j] = a.dc[J[j]];
        }
    }
    constexpr int W = GR_WX * GR_WY * GR_WZ, PF = (W + 255) / 256;
    double v[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) {  // all of a lane's window loads before its LDS stores
        const int q = tid + 256 * u;
        const int x = wx0 + q % GR_WX, y = wy0 + (q / GR_WX) % GR_WY, z = wz0 + q / (GR_WX * GR_WY);
        const bool in = q < W && (unsigned)x < (unsigned)a.kx && (unsigned)y < (unsigned)a.ky && z >= a.kz_lo &&
                        z < a.kz_hi;
        const int64_t zb = (int64_t)z * fplane + (z < 0 ? a.add_lo : z >= a.kz ? a.add_hi : 0);
        v[u] = in ? a.x[zb + (int64_t)y * a.kx + x] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < PF; u++)
        if (tid + 256 * u < W) win[tid + 256 * u] = v[u];
    gtc_stage_dict<G_RMAX>(a, sd, st);
    if (tid < 64) lut[tid] = (int16_t)(((tid / 16 - 1) * GR_WY + (tid / 4) % 4 - 1) * GR_WX + tid % 4 - 1);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RL; j++) {
        if (!live[j]) continue;
        const int lz = lz0 + 2 * j;
        const int base = ((2 * lz + 1) * GR_WY + 2 * ly + 1) * GR_WX + 2 * lx + 1;
        const uint16_t *e = sd + c[j] * a.ke;
        double acc = 0.0;
        for (int k = 0; k < a.ke; k += 8) {
            double cv[8], w[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint16_t q = e[k + u];
                cv[u] = st[q >> 8];
                w[u] = win[base + lut[q & 255]];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) acc = fma(cv[u], w[u], acc);
        }
        a.y[J[j]] = acc;
        if constexpr (DF) {
            const double dd = a.dconst ? a.dk : a.dc ? sdt[dci[j]] : a.d[J[j]];
            a.y2[J[j]] = dd * acc;  // vec_mul(_coded)'s product
        }
    }
}


// Marching R (k_gtc_restrict_march): a workgroup takes a 32 x 8 tile of coarse
// rows through a run of jper coarse planes.  Coarse plane Z reads fine planes
// 2Z - 1 .. 2Z + 2, so consecutive planes share two: a ring of four fine-plane
// windows (66 x 18 each) in LDS, ring slot = fine plane mod 4, and while plane Z
// is summed the registers fetch fine planes 2Z + 3 and 2Z + 4, which then
// replace 2Z - 1 and 2Z.  Each fine value is staged ~1.2 times (the x/y halo)
// instead of ~1.8 (tiles of two coarse planes with their z halo).  Same
// dictionary walk per row as k_gtc_restrict (bitwise the same sums).
constexpr int GM_TX = 32, GM_TY = 8;
constexpr int GM_WX = 2 * GM_TX + 2, GM_WY = 2 * GM_TY + 2, GM_PL = GM_WX * GM_WY;
constexpr int GM_PF = (2 * GM_PL + 255) / 256;  // registers per lane for two fine planes

__device__ __forceinline__ void gtc_march_fetch(const GtcArgs &a, int wx0, int wy0, int fz, double (&v)[GM_PF]) {
    // fine local planes fz, fz + 1 of the tile's window
    const int64_t fplane = (int64_t)a.kx * a.ky;
#pragma unroll
    for (int u = 0; u < GM_PF; u++) {
        const int q = threadIdx.x + 256 * u;
        const int pl = q >= GM_PL ? 1 : 0, qq = q - pl * GM_PL;
        const int y = wy0 + qq / GM_WX, x = wx0 + qq % GM_WX, z = fz + pl;
        const bool in = q < 2 * GM_PL && (unsigned)x < (unsigned)a.kx && (unsigned)y < (unsigned)a.ky &&
                        z >= a.kz_lo && z < a.kz_hi;
        const int64_t zb = (int64_t)z * fplane + (z < 0 ? a.add_lo : z >= a.kz ? a.add_hi : 0);
        v[u] = in ? a.x[zb + (int64_t)y * a.kx + x] : 0.0;
    }
}

// ring slot of fine plane 2 Z + dz: (2 Z + dz) & 3 (Z local coarse plane)
__device__ __forceinline__ void gtc_march_store(double *ring, int Z, const double (&v)[GM_PF], int dz) {
#pragma unroll
    for (int u = 0; u < GM_PF; u++) {
        const int q = threadIdx.x + 256 * u;
        if (q < 2 * GM_PL) {
            const int pl = q >= GM_PL ? 1 : 0, qq = q - pl * GM_PL;
            ring[((2 * Z + dz + pl) & 3) * GM_PL + qq] = v[u];
        }
    }
}

template <bool DF>
__global__ __launch_bounds__(256) void k_gtc_restrict_march(GtcArgs a) {
    __shared__ double ring[4 * GM_PL];
    extern __shared__ uint16_t sd[];
    __shared__ double st[256];
    __shared__ int16_t lut[2][64];  // [Z & 1][slot]: ring plane * GM_PL + dy * GM_WX + dx
    __shared__ double sdt[DF ? 256 : 1];
    const int tid = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int ntxy = a.ntx * a.nty;
    const int chunk = t / ntxy, txy = t - chunk * ntxy;
    const int X0 = (txy % a.ntx) * GM_TX, Y0 = (txy / a.ntx) * GM_TY;
    const int Zb = a.mz0 + chunk * a.jper, Ze = min(Zb + a.jper, a.mz1);
    const int wx0 = 2 * X0 - 1, wy0 = 2 * Y0 - 1;
    const int lx = tid % GM_TX, ly = tid / GM_TX;
    const int X = X0 + lx, Y = Y0 + ly;
    const bool live = X < a.rx && Y < a.ry;
    const int base = (2 * ly + 1) * GM_WX + 2 * lx + 1;
    const int64_t cplane = (int64_t)a.rx * a.ry;
    if (tid < 128) {
        const int par = tid >> 6, s = tid & 63;
        const int dz = s / 16 - 1, dy = (s / 4) % 4 - 1, dx = s % 4 - 1;
        lut[par][s] = (int16_t)(((2 * par + dz) & 3) * GM_PL + dy * GM_WX + dx);
    }
    if constexpr (DF)
        if (a.dc && !a.dconst) sdt[tid] = a.dt[tid];
    // fine local plane of coarse local plane Z, offset dz
    auto fzof = [&](int Z, int dz) { return 2 * (a.rz0 + Z) + dz - a.kz0; };
    {
        double v0[GM_PF], v1[GM_PF];
        gtc_march_fetch(a, wx0, wy0, fzof(Zb, -1), v0);
        gtc_march_fetch(a, wx0, wy0, fzof(Zb, 1), v1);
        gtc_march_store(ring, Zb, v0, -1);
        gtc_march_store(ring, Zb, v1, 1);
    }
    gtc_stage_dict<G_RMAX>(a, sd, st);
    __syncthreads();
    for (int Z = Zb; Z < Ze; Z++) {
        const bool more = Z + 1 < Ze;
        double v[GM_PF];
        if (more) gtc_march_fetch(a, wx0, wy0, fzof(Z, 3), v);
        const int64_t J = live ? (int64_t)Z * cplane + (int64_t)Y * a.rx + X : 0;
        const int c = a.cls[J];
        int dci = 0;
        if constexpr (DF)
            if (a.dc && !a.dconst) dci = a.dc[J];
        if (live) {
            const uint16_t *e = sd + c * a.ke;
            const int16_t *lz = lut[Z & 1];
            double acc = 0.0;
            for (int k = 0; k < a.ke; k += 8) {
                double cv[8], w[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const uint16_t q = e[k + u];
                    cv[u] = st[q >> 8];
                    w[u] = ring[base + lz[q & 255]];
                }
#pragma unroll
                for (int u = 0; u < 8; u++) acc = fma(cv[u], w[u], acc);
            }
            a.y[J] = acc;
            if constexpr (DF) {
                const double dd = a.dconst ? a.dk : a.dc ? sdt[dci] : a.d[J];
                a.y2[J] = dd * acc;  // vec_mul(_coded)'s product
            }
        }
        if (more) {
            __syncthreads();                  // plane Z's reads of 2Z - 1 and 2Z done
            gtc_march_store(ring, Z, v, 3);   // 2Z + 3 -> slot of 2Z - 1, 2Z + 4 -> slot of 2Z
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------ build / dispatch

void gtc_release(GpuCsr &m) {
    m.gtc_cls.release();
    m.gtc_dict.release();
    m.gtc_vtab.release();
    m.gtc_kdz.release();
    m.gtc_wt.release();
    m.gtc_ke = m.gtc_nce = m.gtc_ntab = m.gtc_nclass = 0;
    m.gtc_r = m.gtc_on = false;
}

// FAMG_GTC=0: keep the finalize-time storage for R and P
static bool gtc_enabled() {
    static const bool on = [] {
        const char *e = getenv("FAMG_GTC");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool gtc_attach(GpuCsr &m, const int64_t *fg, const int64_t *cg, int which) {
    gtc_release(m);
    m.gtc_tried = true;
    if (!gtc_enabled() || m.nnz >= (int64_t(1) << 31)) return false;
    const bool is_r = which < 0 ? m.nrows < m.ncols : which == 1;
    // a rank-local P starts at an even fine plane (its tiles' four fine planes
    // then map onto two coarse planes of the staged window)
    if (!is_r && m.rframe.on() && (m.rframe.z0 & 1)) return false;
    std::vector<uint8_t> cls;
    std::vector<std::vector<std::pair<uint8_t, double>>> dict;
    if (!gtc_classes(m, is_r, fg, cg, cls, dict)) return false;
    // distinct values (bit patterns), <= 256
    std::vector<uint64_t> vals;
    for (const auto &d : dict)
        for (const auto &e : d) {
            uint64_t b;
            std::memcpy(&b, &e.second, 8);
            vals.push_back(b);
        }
    vals.push_back(0);  // +0.0 for the padding entries
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    if (vals.size() > 256) return false;
    const int gran = is_r ? 8 : 4;
    size_t ke = 1;
    for (const auto &d : dict) ke = std::max(ke, d.size());
    ke = (ke + gran - 1) / gran * gran;
    if (dict.size() * ke > (size_t)(is_r ? G_RMAX : G_DMAX)) return false;
    const uint16_t zero_idx = (uint16_t)(std::lower_bound(vals.begin(), vals.end(), 0ull) - vals.begin());
    const uint16_t centre = is_r ? (uint16_t)(16 + 4 + 1) : (uint16_t)(9 + 3 + 1);
    // padding: +0.0 at the anchor (after the row's entries: a +0.0 term leaves
    // the accumulator unchanged)
    std::vector<uint16_t> hd(dict.size() * ke, (uint16_t)(zero_idx << 8 | centre));
    for (size_t c = 0; c < dict.size(); c++)
        for (size_t k = 0; k < dict[c].size(); k++) {
            uint64_t b;
            std::memcpy(&b, &dict[c][k].second, 8);
            const uint16_t vi = (uint16_t)(std::lower_bound(vals.begin(), vals.end(), b) - vals.begin());
            hd[c * ke + k] = (uint16_t)(vi << 8 | dict[c][k].first);
        }
    std::vector<double> vt(vals.size());
    for (size_t q = 0; q < vals.size(); q++) std::memcpy(&vt[q], &vals[q], 8);
    hipStream_t s = m.ctx->stream;
    m.gtc_cls.resize(cls.size());
    m.gtc_dict.resize(hd.size());
    m.gtc_vtab.resize(vt.size());
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtc_cls.get(), cls.data(), cls.size(), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtc_dict.get(), hd.data(), hd.size() * 2, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(m.gtc_vtab.get(), vt.data(), vt.size() * 8, hipMemcpyHostToDevice, s));
    if (is_r && ke <= 255) {  // per class: where each fine plane's entries start (slots ascend in dz)
        std::vector<uint8_t> kdz(dict.size() * 5);
        for (size_t c = 0; c < dict.size(); c++) {
            int k = 0;
            for (int g = 0; g < 4; g++) {
                kdz[c * 5 + g] = (uint8_t)k;
                while (k < (int)dict[c].size() && dict[c][k].first / 16 == g) k++;
            }
            kdz[c * 5 + 4] = (uint8_t)dict[c].size();
        }
        m.gtc_kdz.resize(kdz.size());
        FAMG_CHECK_HIP(hipMemcpyAsync(m.gtc_kdz.get(), kdz.data(), kdz.size(), hipMemcpyHostToDevice, s));
        // the 32-slot weights (fine.hip k_fine_rr): every entry in the slots a
        // 2 x 2 x 2 box smoothed by the 7-point stencil reaches, else none
        static const int8_t pat[64] = {
            // dz = -1: (dy, dx) in {1, 2}^2
            -1, -1, -1, -1, -1, 0, 1, -1, -1, 2, 3, -1, -1, -1, -1, -1,
            // dz = 0: the 2 x 2 centre and its x / y face neighbours
            -1, 4, 5, -1, 6, 7, 8, 9, 10, 11, 12, 13, -1, 14, 15, -1,
            // dz = 1
            -1, 16, 17, -1, 18, 19, 20, 21, 22, 23, 24, 25, -1, 26, 27, -1,
            // dz = 2
            -1, -1, -1, -1, -1, 28, 29, -1, -1, 30, 31, -1, -1, -1, -1, -1};
        std::vector<double> wt(dict.size() * 32, 0.0);
        bool fits = true;
        for (size_t c = 0; c < dict.size() && fits; c++)
            for (const auto &e : dict[c]) {
                if (e.first >= 64 || pat[e.first] < 0) {
                    fits = false;
                    break;
                }
                wt[c * 32 + pat[e.first]] = e.second;
            }
        if (fits) {
            m.gtc_wt.resize(wt.size());
            FAMG_CHECK_HIP(hipMemcpyAsync(m.gtc_wt.get(), wt.data(), wt.size() * 8, hipMemcpyHostToDevice, s));
        }
    }
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    m.gtc_nclass = (int)dict.size();
    m.gtc_ke = (int)ke;
    m.gtc_nce = (int)(dict.size() * ke);
    m.gtc_ntab = (int)vt.size();
    m.gtc_r = is_r;
    for (int q = 0; q < 3; q++) {
        m.gtc_fg[q] = fg[q];
        m.gtc_cg[q] = cg[q];
    }
    m.gtc_on = true;
    return true;
}

void attach_box_transfers(const GpuCsr &Af, const GpuCsr &Ac, GpuCsr &R, GpuCsr &P) {
    const int64_t *fg = Af.grid, *cg = Ac.grid;
    for (int q = 0; q < 3; q++)
        if (fg[q] <= 0 || cg[q] != (fg[q] + 1) / 2) return;
    if (fg[0] * fg[1] * fg[2] != Af.nrows || cg[0] * cg[1] * cg[2] != Ac.nrows) return;
    if (P.nrows != Af.nrows || P.ncols != Ac.nrows || R.nrows != Ac.nrows || R.ncols != Af.nrows) return;
    if (!P.gtc_on && !P.gtc_tried) gtc_attach(P, fg, cg, 0);
    if (!R.gtc_on && !R.gtc_tried) gtc_attach(R, fg, cg, 1);
    if ((!P.gtc_on || gtx_mode() == 2) && !P.gtx_on && !P.gtx_tried) gtx_attach(P, fg, cg, 0);
    if ((!R.gtc_on || gtx_mode() == 2) && !R.gtx_on && !R.gtx_tried) gtx_attach(R, fg, cg, 1);
}

// fine points per lane along z in the P kernel (FAMG_GTC_TZ=8: eight)
static int gtc_tz() {
    static const int v = [] {
        const char *e = getenv("FAMG_GTC_TZ");
        return (e && e[0] == '8') ? 8 : 4;
    }();
    return v;
}

// coarse planes per R tile (FAMG_GTC_RTZ=4: four, two rows per lane)
static int gtc_rtz() {
    static const int v = [] {
        const char *e = getenv("FAMG_GTC_RTZ");
        return (e && e[0] == '4') ? 4 : 2;
    }();
    return v;
}

// workgroups of the marching R per CU with dyn bytes of dictionary (cached)
static int gtc_march_occupancy(bool df, size_t dyn) {
    static std::mutex mu;
    static std::unordered_map<size_t, int> cache;
    const size_t key = dyn * 2 + (df ? 1 : 0);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    const hipError_t e = df ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gtc_restrict_march<true>, 256, dyn)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gtc_restrict_march<false>, 256, dyn);
    if (e != hipSuccess || n < 1) {
        (void)hipGetLastError();
        n = 1;
    }
    cache[key] = n;
    return n;
}

// FAMG_GTC_MARCH=0: R in tiles of two coarse planes instead of marching workgroups
static bool gtc_march_r() {
    static const bool on = [] {
        const char *e = getenv("FAMG_GTC_MARCH");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool gtc_supports(const GpuCsr &m, SpmvMode mode) {
    return m.gtc_r ? (mode == SPMV_SET || mode == SPMV_SETDF) : (mode == SPMV_SET || mode == SPMV_ADD || mode == SPMV_ADD0);
}

// A/B switch FAMG_DIA_DK=0 (shared with the DIA kernels): a constant coded d is read per row
static bool gtc_dk_enabled() { return flag(FLAG_DIA_DK) != 0; }

// The z-tiles [ta, tb) of a launch whose column windows [w0(t), w0(t) + wz) read
// no ghost plane (planes [kz_lo, 0) and [kz_own, kz_hi)): they can run while the
// halo is in flight.
template <typename F>
static void interior_tiles(int ntz, int wz, int kz_own, int kz_lo, int kz_hi, F w0, int &ta, int &tb) {
    ta = 0;
    while (ta < ntz && w0(ta) < 0 && kz_lo < 0) ta++;
    tb = ta;
    while (tb < ntz && !(w0(tb) + wz > kz_own && kz_hi > kz_own)) tb++;
}

void spmv_gtc(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi, hipStream_t s,
              int64_t seg) {
    GtcArgs a{};
    a.cls = m.gtc_cls.get();
    a.dict = m.gtc_dict.get();
    a.vtab = m.gtc_vtab.get();
    a.ke = m.gtc_ke;
    a.nce = m.gtc_nce;
    a.ntab = m.gtc_ntab;
    const int64_t *rg = m.gtc_r ? m.gtc_cg : m.gtc_fg, *kg = m.gtc_r ? m.gtc_fg : m.gtc_cg;
    a.rx = (int)rg[0]; a.ry = (int)rg[1]; a.rz = (int)rg[2];
    a.kx = (int)kg[0]; a.ky = (int)kg[1]; a.kz = (int)kg[2];
    a.kz_lo = 0; a.kz_hi = a.kz; a.rz0 = 0; a.kz0 = 0; a.add_lo = a.add_hi = 0;
    if (m.rframe.on()) {  // rank-local: owned row planes, [owned | ghost planes] columns
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
    a.dconst = epi.dc && epi.dk != 0.0 && gtc_dk_enabled();
    a.dk = epi.dk;
    a.y2 = epi.y2;
    // the launch's z-tile range: all tiles, or (segments of a rank-local matrix)
    // 1 = the tiles that read owned columns only, 0 / 2 = those before / after
    auto range = [&](int ntz, int ta, int tb, int &z0, int &z1) {
        z0 = seg < 0 || seg == 0 ? 0 : seg == 1 ? ta : tb;
        z1 = seg < 0 || seg == 2 ? ntz : seg == 1 ? tb : ta;
    };
    if (m.gtc_r) {
        FAMG_REQUIRE(mode == SPMV_SET || mode == SPMV_SETDF, AMG_ERR_UNSUPPORTED, "grid-transfer R: SET / SETDF only");
        FAMG_REQUIRE(mode != SPMV_SETDF || (epi.y2 && (epi.d || epi.dc || epi.dk != 0.0)), AMG_ERR_INVALID,
                     "SETDF needs y2 and d");
        a.ntx = (int)ceil_div(a.rx, GR_TX);
        a.nty = (int)ceil_div(a.ry, GR_TY);
        if (gtc_march_r() && m.ctx) {
            // marching R: z segments in single coarse planes
            int ta = 0, tb = a.rz, z0, z1;
            if (seg >= 0)
                interior_tiles(a.rz, 4, a.kz, a.kz_lo, a.kz_hi, [&](int t) { return 2 * (a.rz0 + t) - 1 - a.kz0; }, ta, tb);
            range(a.rz, ta, tb, z0, z1);
            if (z1 <= z0) return;
            a.ntx = (int)ceil_div(a.rx, GM_TX);
            a.nty = (int)ceil_div(a.ry, GM_TY);
            const int64_t ntxy = (int64_t)a.ntx * a.nty;
            // exactly one round of workgroups: as many as fit the chip at once (a
            // second, partial round left most CUs idle: 512 / 768 / 1024 / 1408
            // workgroups on R_0 of the 256^3 cycle ran 68 / 54 / 70 / 63 us)
            const size_t dyn = (size_t)a.nce * sizeof(uint16_t);
            const int per_cu = gtc_march_occupancy(mode == SPMV_SETDF, dyn);
            const int64_t want = (int64_t)per_cu * std::max(m.ctx->num_cus, 1);
            a.jper = (int)std::max<int64_t>(1, ceil_div((int64_t)(z1 - z0) * ntxy, want));
            a.mz0 = z0;
            a.mz1 = z1;
            const dim3 grid((unsigned)(ntxy * ceil_div(z1 - z0, a.jper)));
            if (mode == SPMV_SETDF) k_gtc_restrict_march<true><<<grid, dim3(256), dyn, s>>>(a);
            else k_gtc_restrict_march<false><<<grid, dim3(256), dyn, s>>>(a);
            FAMG_CHECK_HIP(hipGetLastError());
            return;
        }
        const int rtz = gtc_rtz();  // coarse planes per tile
        const int ntz = (int)ceil_div(a.rz, rtz);
        int ta = 0, tb = ntz, z0, z1;
        if (seg >= 0)
            interior_tiles(ntz, 2 * rtz + 2, a.kz, a.kz_lo, a.kz_hi, [&](int t) { return 2 * (a.rz0 + t * rtz) - 1 - a.kz0; }, ta, tb);
        range(ntz, ta, tb, z0, z1);
        if (z1 <= z0) return;
        a.tile0 = a.ntx * a.nty * z0;
        const size_t dyn = (size_t)a.nce * sizeof(uint16_t);
        const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * (z1 - z0)));
        const bool df = mode == SPMV_SETDF;
        if (rtz == 4) {
            if (df) k_gtc_restrict<4, true><<<grid, dim3(256), dyn, s>>>(a);
            else k_gtc_restrict<4, false><<<grid, dim3(256), dyn, s>>>(a);
        } else {
            if (df) k_gtc_restrict<2, true><<<grid, dim3(256), dyn, s>>>(a);
            else k_gtc_restrict<2, false><<<grid, dim3(256), dyn, s>>>(a);
        }
    } else {
        a.ntx = (int)ceil_div(a.rx, GP_TX);
        a.nty = (int)ceil_div(a.ry, GP_TY);
        const int tz = gtc_tz();
        const int ntz = (int)ceil_div(a.rz, tz);
        int ta = 0, tb = ntz, z0, z1;
        if (seg >= 0)
            interior_tiles(ntz, tz / 2 + 2, a.kz, a.kz_lo, a.kz_hi, [&](int t) { return ((a.rz0 + t * tz) >> 1) - 1 - a.kz0; }, ta, tb);
        range(ntz, ta, tb, z0, z1);
        if (z1 <= z0) return;
        a.tile0 = a.ntx * a.nty * z0;
        const dim3 grid((unsigned)((int64_t)a.ntx * a.nty * (z1 - z0))), block(256);
#define FAMG_GTCI(TZ, NT)                                                                            \
    switch (mode) {                                                                                \
    case SPMV_SET: k_gtc_interp<SPMV_SET, TZ, NT><<<grid, block, 0, s>>>(a); break;                \
    case SPMV_ADD: k_gtc_interp<SPMV_ADD, TZ, NT><<<grid, block, 0, s>>>(a); break;                \
    case SPMV_ADD0: k_gtc_interp<SPMV_ADD0, TZ, NT><<<grid, block, 0, s>>>(a); break;              \
    default: fail(AMG_ERR_UNSUPPORTED, "grid-transfer P: unsupported SpMV epilogue");              \
    }
        // FAMG_GTC_NT=0: cached fine-vector streams (non-temporal: P_0 ADD0 75.3 -> 72.8 us)
        static const bool nt = !(getenv("FAMG_GTC_NT") && getenv("FAMG_GTC_NT")[0] == '0');
        if (nt) {
            if (tz == 8) { FAMG_GTCI(8, true) }
            else { FAMG_GTCI(4, true) }
        } else {
            if (tz == 8) { FAMG_GTCI(8, false) }
            else { FAMG_GTCI(4, false) }
        }
#undef FAMG_GTCI
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

}  // namespace famg
