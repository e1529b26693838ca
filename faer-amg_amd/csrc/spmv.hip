// spmv.hip -- fp64 CSR SpMV for gfx950 with fused V-cycle epilogues.
//
// Replaces the reference's CPU SpMV (ParSpmmOp, par_spmm.rs:98-133, and faer's
// SparseRowMat LinOp used at multigrid.rs:137-158) and fuses the vector work of
// Multigrid::cycle / smooth (multigrid.rs:341-350, 407-424) into its epilogue.
//
// Design ("CSR-stream", MI355X-first):
//  * The row space is cut on the host into blocks of <= 256 rows holding
//    <= SPMV_CAP nonzeros (GpuCsr::sched).  A 256-thread workgroup streams its
//    block's values and column indices HBM -> LDS with 16-byte, fully coalesced,
//    non-temporal loads (they are read exactly once), then computes rows out of
//    LDS.  x is gathered through L1/L2 (it is re-read by neighbouring rows).
//  * Rows per block decide the lanes per row L (a power of two, L*rows <= 256):
//    short rows (7-pt: 256 rows, L = 1) are summed by one lane sequentially in
//    ascending column order with fma -- bit-identical to the oracle -- while long
//    rows (Galerkin 125-pt, R) spread over L lanes and finish with a shuffle tree.
//    A single row longer than SPMV_CAP gets a whole workgroup.
//  * Workgroups are remapped so that each XCD (blocks b and b+8 share one) walks
//    a contiguous slab of rows: the x window of a slab (3 planes of a 7-pt
//    operator, ~1.5 MB at 256^3) then stays in that XCD's 4 MB L2.
#include "famg.hpp"

namespace famg {

typedef double dbl2_t __attribute__((ext_vector_type(2)));
typedef int32_t i32x4_t __attribute__((ext_vector_type(4)));

constexpr int SPMV_BS = 256;
constexpr int SPMV_CAP = 2048;

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, idx = b >> 3;
    return x * q + min(x, r) + idx;
}

struct SpmvArgs {
    const int32_t *rowptr;
    const int32_t *col;
    const double *val;
    const int32_t *sched;
    int32_t nblocks;
    const double *x;
    double *y;
    const double *b;
    const double *d;
    const int32_t *perm;
};

template <int MODE>
__device__ __forceinline__ void spmv_epilogue(const SpmvArgs &a, int row, double acc) {
    if constexpr (MODE == SPMV_SET) {
        a.y[row] = acc;
    } else if constexpr (MODE == SPMV_ADD) {
        a.y[row] = a.y[row] + acc;
    } else if constexpr (MODE == SPMV_RESID) {
        a.y[row] = a.b[row] - acc;
    } else if constexpr (MODE == SPMV_JACOBI) {
        a.y[row] = a.x[row] + a.d[row] * (a.b[row] - acc);
    } else {  // SPMV_SGS: row is the permuted index
        const int i = a.perm[row];
        a.y[i] = a.x[i] + a.d[row] * (a.b[i] - acc);
    }
}

template <int MODE>
__global__ __launch_bounds__(SPMV_BS) void spmv_stream_kernel(SpmvArgs a) {
    __shared__ __attribute__((aligned(16))) double sval[SPMV_CAP + 2];
    __shared__ __attribute__((aligned(16))) int32_t scol[SPMV_CAP + 4];
    __shared__ double sred[SPMV_BS / 64];

    const int blk = xcd_remap(blockIdx.x, a.nblocks);
    const int r0 = a.sched[blk], r1 = a.sched[blk + 1];
    const int e0 = a.rowptr[r0], e1 = a.rowptr[r1];
    const int tid = threadIdx.x;
    const int nnz = e1 - e0;

    if (nnz > SPMV_CAP) {
        // one long row (r1 == r0 + 1): the whole workgroup reduces it
        double acc = 0.0;
        for (int k = e0 + tid; k < e1; k += SPMV_BS) acc = fma(a.val[k], a.x[a.col[k]], acc);
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if ((tid & 63) == 0) sred[tid >> 6] = acc;
        __syncthreads();
        if (tid == 0) {
            double s = sred[0];
            for (int w = 1; w < SPMV_BS / 64; w++) s += sred[w];
            spmv_epilogue<MODE>(a, r0, s);
        }
        return;
    }

    // ---- stage values and column indices (16-byte coalesced, non-temporal)
    const int bv = e0 & ~1;
    const int nv = (e1 - bv + 1) >> 1;
    const dbl2_t *gv = reinterpret_cast<const dbl2_t *>(a.val + bv);
    dbl2_t *sv2 = reinterpret_cast<dbl2_t *>(sval);
    for (int k = tid; k < nv; k += SPMV_BS) sv2[k] = __builtin_nontemporal_load(gv + k);
    const int bc = e0 & ~3;
    const int nc = (e1 - bc + 3) >> 2;
    const i32x4_t *gc = reinterpret_cast<const i32x4_t *>(a.col + bc);
    i32x4_t *sc4 = reinterpret_cast<i32x4_t *>(scol);
    for (int k = tid; k < nc; k += SPMV_BS) sc4[k] = __builtin_nontemporal_load(gc + k);
    __syncthreads();

    const int nrows = r1 - r0;
    int L = 1;
    while (L < 64 && 2 * L * nrows <= SPMV_BS) L <<= 1;
    const int rl = tid / L;
    const int sub = tid & (L - 1);
    const int vo = e0 - bv, co = e0 - bc;

    double acc = 0.0;
    if (rl < nrows) {
        const int rs = a.rowptr[r0 + rl] - e0;
        const int re = a.rowptr[r0 + rl + 1] - e0;
        for (int k = rs + sub; k < re; k += L) acc = fma(sval[vo + k], a.x[scol[co + k]], acc);
    }
    for (int off = L >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (rl < nrows && sub == 0) spmv_epilogue<MODE>(a, r0 + rl, acc);
}

void spmv(const GpuCsr &m, const double *x, double *y, SpmvMode mode, const SpmvEpi &epi,
          hipStream_t s, int64_t blk_begin, int64_t blk_end, const int32_t *sched_override) {
    FAMG_REQUIRE(m.spmv_ready(), AMG_ERR_UNSUPPORTED,
                 "SpMV needs nnz < 2^31 (32-bit row pointers)");
    if (blk_end < 0) blk_end = m.nblocks;
    const int64_t nb = blk_end - blk_begin;
    if (nb <= 0) return;
    SpmvArgs a;
    a.rowptr = m.rp32.get();
    a.col = m.col.get();
    a.val = m.val.get();
    a.sched = (sched_override ? sched_override : m.sched.get()) + blk_begin;
    a.nblocks = static_cast<int32_t>(nb);
    a.x = x;
    a.y = y;
    a.b = epi.b;
    a.d = epi.d;
    a.perm = epi.perm;
    dim3 grid(static_cast<unsigned>(nb)), block(SPMV_BS);
    switch (mode) {
    case SPMV_SET: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_SET>, grid, block, 0, s, a); break;
    case SPMV_ADD: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_ADD>, grid, block, 0, s, a); break;
    case SPMV_RESID: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_RESID>, grid, block, 0, s, a); break;
    case SPMV_JACOBI: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_JACOBI>, grid, block, 0, s, a); break;
    case SPMV_SGS: hipLaunchKernelGGL(spmv_stream_kernel<SPMV_SGS>, grid, block, 0, s, a); break;
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

// Host-side schedule: greedy blocks of <= SPMV_BS rows and <= SPMV_CAP nonzeros;
// a row longer than SPMV_CAP is a block of its own.  Blocks never cross the
// given segment boundaries (SGS colors).
void build_schedule(const std::vector<int64_t> &rp, const std::vector<int64_t> &seg_bounds,
                    std::vector<int32_t> &sched, std::vector<int64_t> &seg_blocks) {
    sched.clear();
    seg_blocks.clear();
    sched.push_back(static_cast<int32_t>(seg_bounds.empty() ? 0 : seg_bounds[0]));
    seg_blocks.push_back(0);
    for (size_t s = 0; s + 1 < seg_bounds.size(); s++) {
        int64_t r0 = seg_bounds[s];
        const int64_t end = seg_bounds[s + 1];
        while (r0 < end) {
            int64_t r1;
            if (rp[r0 + 1] - rp[r0] > SPMV_CAP) {
                r1 = r0 + 1;
            } else {
                r1 = r0;
                while (r1 < end && r1 - r0 < SPMV_BS && rp[r1 + 1] - rp[r0] <= SPMV_CAP) r1++;
            }
            sched.push_back(static_cast<int32_t>(r1));
            r0 = r1;
        }
        seg_blocks.push_back(static_cast<int64_t>(sched.size()) - 1);
    }
}

}  // namespace famg
