// dist.hip -- multi-GPU V-cycle: row-block partition of every level, halo
// exchange before each SpMV, agglomeration of the coarse levels.
//
// The reference is shared-memory only (rayon), so this
// layer is new.  One process per GPU; rank p owns a contiguous row range of
// every level.  Per level the rank's vector space is laid out [owned | ghost]
// with the ghosts sorted by global index (so grouped by owner rank): a local
// matrix row keeps its global column order, which keeps every row sum in the
// same order as the single-GPU path (bitwise equal for short rows).
// The ghost set of level l is the union of the columns referenced by A_l, R_l
// (fine columns) and P_{l-1} (coarse columns) rows owned here, so one halo
// exchange per vector refresh serves all three.  The exchange packs the
// requested owned entries into a send buffer and runs grouped point-to-point
// sends/receives straight into the ghost region of the peer's vector.
// Levels below `agglomerate_rows` are all-gathered and cycled redundantly by
// every rank with the single-GPU MultigridOp (the global coarse operators).
//
// Transports: RCCL (ncclSend/ncclRecv/ncclAllGather/ncclAllReduce on the
// context stream, over xGMI) and a loopback hub (virtual ranks as host threads
// of one process sharing one GPU) that validates the whole algorithm on a
// single device.
#include <dlfcn.h>
#include <link.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "handles.hpp"
#include "plan.hpp"
#include "solve.hpp"

using namespace famg;

namespace famg {

// ------------------------------------------------------------- RCCL binding
//
// One RCCL per process: the library is not linked against librccl; the entry
// points are resolved at first use from the librccl the process has already
// mapped (torch's bundled one when torch is imported), else from
// $FAMG_RCCL_PATH, librccl.so.1 on the loader path, /opt/rocm/lib/librccl.so.1.
// Two RCCL builds in one process (the linked one and torch's) would share
// symbol names and interpose on each other.
struct RcclApi {
    void *h = nullptr;
    std::string path, error;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
};

// The mapped object whose basename is librccl.so or librccl.so.<version> (not a
// plugin such as librccl-net.so).
static int find_mapped_rccl(struct dl_phdr_info *info, size_t, void *data) {
    if (!info->dlpi_name) return 0;
    const char *base = std::strrchr(info->dlpi_name, '/');
    base = base ? base + 1 : info->dlpi_name;
    if (std::strncmp(base, "librccl.so", 10) == 0 && (base[10] == '\0' || base[10] == '.')) {
        *static_cast<std::string *>(data) = info->dlpi_name;
        return 1;
    }
    return 0;
}

static const char *const RCCL_SYMS[] = {"ncclGetErrorString", "ncclGetUniqueId", "ncclCommInitRank",
                                        "ncclCommDestroy",    "ncclGroupStart",  "ncclGroupEnd",
                                        "ncclSend",           "ncclRecv",        "ncclAllGather",
                                        "ncclAllReduce"};

static RcclApi load_rccl() {
    RcclApi a;
    std::string mapped;
    dl_iterate_phdr(find_mapped_rccl, &mapped);
    std::vector<std::pair<std::string, int>> cands;
    if (!mapped.empty()) cands.push_back({mapped, RTLD_NOW | RTLD_NOLOAD});
    if (const char *e = getenv("FAMG_RCCL_PATH")) cands.push_back({e, RTLD_NOW});
    cands.push_back({"librccl.so.1", RTLD_NOW});
    cands.push_back({"/opt/rocm/lib/librccl.so.1", RTLD_NOW});
    // first candidate that loads and exports every entry point; a candidate
    // lacking one is closed and the next one tried
    std::string tried;
    for (auto &c : cands) {
        void *h = dlopen(c.first.c_str(), c.second);
        if (!h) {
            tried += " " + c.first + " (not loadable)";
            continue;
        }
        const char *missing = nullptr;
        for (const char *name : RCCL_SYMS)
            if (!dlsym(h, name)) { missing = name; break; }
        if (missing) {
            tried += " " + c.first + " (lacks " + missing + ")";
            dlclose(h);
            continue;
        }
        a.h = h;
        a.path = c.first;
        break;
    }
    if (!a.h) {
        a.error = "cannot load librccl:" + tried;
        return a;
    }
    auto sym = [&](const char *name) {
        void *f = dlsym(a.h, name);
        if (!f && a.error.empty()) a.error = std::string("librccl lacks ") + name;
        return f;
    };
    a.GetErrorString = reinterpret_cast<decltype(a.GetErrorString)>(sym("ncclGetErrorString"));
    a.GetUniqueId = reinterpret_cast<decltype(a.GetUniqueId)>(sym("ncclGetUniqueId"));
    a.CommInitRank = reinterpret_cast<decltype(a.CommInitRank)>(sym("ncclCommInitRank"));
    a.CommDestroy = reinterpret_cast<decltype(a.CommDestroy)>(sym("ncclCommDestroy"));
    a.GroupStart = reinterpret_cast<decltype(a.GroupStart)>(sym("ncclGroupStart"));
    a.GroupEnd = reinterpret_cast<decltype(a.GroupEnd)>(sym("ncclGroupEnd"));
    a.Send = reinterpret_cast<decltype(a.Send)>(sym("ncclSend"));
    a.Recv = reinterpret_cast<decltype(a.Recv)>(sym("ncclRecv"));
    a.AllGather = reinterpret_cast<decltype(a.AllGather)>(sym("ncclAllGather"));
    a.AllReduce = reinterpret_cast<decltype(a.AllReduce)>(sym("ncclAllReduce"));
    return a;
}

static const RcclApi &rccl() {
    static const RcclApi api = load_rccl();
    FAMG_REQUIRE(api.error.empty(), AMG_ERR_RCCL, api.error);
    return api;
}

// ------------------------------------------------------------- transports

struct Peer {
    int rank;
    const void *sbuf;
    int64_t sbytes;
    void *rbuf;
    int64_t rbytes;
};

struct Transport {
    int nranks = 1, rank = 0;
    virtual ~Transport() = default;
    virtual void exchange(const std::vector<Peer> &peers, hipStream_t s) = 0;
    virtual void allgather(const void *sbuf, void *rbuf, int64_t bytes, hipStream_t s) = 0;
    virtual void allreduce(double *buf, int64_t count, bool is_max, hipStream_t s) = 0;
    virtual void barrier(hipStream_t s) = 0;
};

#define FAMG_CHECK_NCCL(expr)                                                              \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess)                                                             \
            ::famg::fail(AMG_ERR_RCCL, std::string(#expr) + ": " + rccl().GetErrorString(r_)); \
    } while (0)

struct RcclTransport : Transport {
    ncclComm_t comm = nullptr;
    DevBuf<double> one;
    ~RcclTransport() override {
        if (comm) rccl().CommDestroy(comm);
    }
    void exchange(const std::vector<Peer> &peers, hipStream_t s) override {
        if (peers.empty()) return;
        FAMG_CHECK_NCCL(rccl().GroupStart());
        for (const Peer &p : peers) {
            if (p.sbytes) FAMG_CHECK_NCCL(rccl().Send(p.sbuf, p.sbytes, ncclUint8, p.rank, comm, s));
            if (p.rbytes) FAMG_CHECK_NCCL(rccl().Recv(p.rbuf, p.rbytes, ncclUint8, p.rank, comm, s));
        }
        FAMG_CHECK_NCCL(rccl().GroupEnd());
    }
    void allgather(const void *sbuf, void *rbuf, int64_t bytes, hipStream_t s) override {
        FAMG_CHECK_NCCL(rccl().AllGather(sbuf, rbuf, bytes, ncclUint8, comm, s));
    }
    void allreduce(double *buf, int64_t count, bool is_max, hipStream_t s) override {
        FAMG_CHECK_NCCL(rccl().AllReduce(buf, buf, count, ncclDouble, is_max ? ncclMax : ncclSum, comm, s));
    }
    void barrier(hipStream_t s) override {
        if (one.size() < 1) one.resize(1);
        FAMG_CHECK_NCCL(rccl().AllReduce(one.get(), one.get(), 1, ncclDouble, ncclSum, comm, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
    }
};

// Virtual ranks in one process: every collective is a rendezvous of the rank
// threads; data moves with device-to-device copies issued by the receiver.
struct LoopbackHub {
    int nranks;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const std::vector<Peer> *> posted;
    std::vector<const void *> gptr;
    explicit LoopbackHub(int n) : nranks(n), posted(n), gptr(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = generation;
        if (++arrived == nranks) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != g; });
        }
    }
};

struct LoopbackTransport : Transport {
    std::shared_ptr<LoopbackHub> hub;
    void exchange(const std::vector<Peer> &peers, hipStream_t s) override {
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->posted[rank] = &peers;
        hub->wait();
        for (const Peer &p : peers) {
            if (!p.rbytes) continue;
            const Peer *src = nullptr;
            for (const Peer &q : *hub->posted[p.rank])
                if (q.rank == rank) src = &q;
            FAMG_REQUIRE(src && src->sbytes == p.rbytes, AMG_ERR_INVALID, "loopback: unmatched exchange");
            FAMG_CHECK_HIP(hipMemcpyAsync(p.rbuf, src->sbuf, p.rbytes, hipMemcpyDeviceToDevice, s));
        }
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->wait();
    }
    void allgather(const void *sbuf, void *rbuf, int64_t bytes, hipStream_t s) override {
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->gptr[rank] = sbuf;
        hub->wait();
        for (int q = 0; q < nranks; q++)
            FAMG_CHECK_HIP(hipMemcpyAsync(static_cast<char *>(rbuf) + q * bytes, hub->gptr[q], bytes,
                                          hipMemcpyDeviceToDevice, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->wait();
    }
    void allreduce(double *buf, int64_t count, bool is_max, hipStream_t s) override {
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->gptr[rank] = buf;
        hub->wait();
        std::vector<double> acc(count), tmp(count);
        for (int q = 0; q < nranks; q++) {
            FAMG_CHECK_HIP(hipMemcpy(tmp.data(), hub->gptr[q], count * sizeof(double), hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < count; i++)
                acc[i] = q == 0 ? tmp[i] : (is_max ? std::max(acc[i], tmp[i]) : acc[i] + tmp[i]);
        }
        hub->wait();  // everyone has read before anyone writes
        FAMG_CHECK_HIP(hipMemcpy(buf, acc.data(), count * sizeof(double), hipMemcpyHostToDevice));
        hub->wait();
    }
    void barrier(hipStream_t s) override {
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        hub->wait();
    }
};

}  // namespace famg

struct amg_loopback_hub {
    std::shared_ptr<LoopbackHub> hub;
};

struct amg_comm {
    Ctx *ctx;
    std::shared_ptr<Transport> tr;
};

namespace famg {

// --------------------------------------------------------------- kernels

__global__ void k_extract_rp(const int64_t *rp, int64_t r0, int64_t n, int64_t *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i <= n) out[i] = rp[r0 + i] - rp[r0];
}

// mark[c] = 1 for every referenced column outside [c0, c1)
__global__ void k_mark_ghost(const int32_t *col, int64_t nnz, int64_t c0, int64_t c1, int64_t *mark) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < nnz) {
        const int64_t c = col[e];
        if (c < c0 || c >= c1) mark[c] = 1;
    }
}

__global__ void k_compact_ghost(const int64_t *mark, const int64_t *scan, int64_t n, int64_t *ids) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n && mark[j]) ids[scan[j]] = j;
}

__global__ void k_remap_cols(int32_t *col, int64_t nnz, int64_t c0, int64_t c1, int64_t n_own,
                             const int64_t *scan) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < nnz) {
        const int64_t c = col[e];
        col[e] = (c >= c0 && c < c1) ? (int32_t)(c - c0) : (int32_t)(n_own + scan[c]);
    }
}

// the lowest marked column below r0 and the highest at or above r1
__global__ void k_ghost_extent(const int64_t *mark, int64_t n, int64_t r0, int64_t r1, unsigned long long *ext) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= n || !mark[c]) return;
    if (c < r0) atomicMin(&ext[0], (unsigned long long)c);
    else if (c >= r1) atomicMax(&ext[1], (unsigned long long)c);
}

__global__ void k_mark_range(int64_t *mark, int64_t c0, int64_t c1) {
    const int64_t c = c0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c < c1) mark[c] = 1;
}

__global__ void k_gather_idx(const double *x, const int32_t *idx, int64_t n, double *out) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) out[k] = x[idx[k]];
}

static unsigned g1(int64_t n) { return (unsigned)std::max<int64_t>(1, ceil_div(n, 256)); }

// -------------------------------------------------------- vector spaces

// A level's vector space on this rank: the host plan (plan.hpp: ghost set,
// requests, send lists, neighbours) plus its device buffers.
struct Space {
    bool redundant = false;
    HaloPlan plan;
    int64_t n_glob = 0, r0 = 0, r1 = 0, n_own = 0, n_ghost = 0;
    // a grid level split into whole planes: the ghost set is made of whole
    // planes (below, then above the owned ones), so the local vector has the
    // SlabFrame layout and the grid kernels run on the rank-local matrices
    SlabFrame frame;
    DevBuf<int64_t> mark, scan;           // setup only (global length)
    // halo plan (copied from `plan`)
    std::vector<int> nbr;
    std::vector<int64_t> soff, scnt, roff, rcnt;
    DevBuf<int32_t> send_idx;
    DevBuf<double> sendbuf;
    std::vector<Peer> peers;              // rebuilt per vector (rbuf differs)
    int64_t nsend = 0;
    // Sweep-position halo lists of a level smoothed by multicolor SGS (sgs_sweep;
    // ADVICE r03 / verdict r04 item 7).  An SGS step sweeps the colours in the
    // order seq = 0, 1, ..., C-1, C-2, ..., 0 (positions 0 .. 2C-2); the exchange
    // before position p >= 1 carries the ghost entries of colour seq[p-1] -- just
    // updated -- that a row of the reading rank reads at a later position before
    // that colour is updated again, and the exchange before position 0 (x not
    // zero: after an interpolation) the entries read before their first update.
    // Which rows read an entry is known on both sides (the reader's colours per
    // ghost entry, sent to the owner once at setup), so sender and receiver build
    // the same lists.  Slots ordered (position, peer, global id).
    int64_t ncol = 0;
    std::vector<int64_t> cs_off, cr_off;  // [p * npeer + k] .. +1: slot ranges, ((2C-1) * npeer + 1) entries
    DevBuf<int32_t> cs_idx, cr_idx;       // owned local index to send / ghost local index to fill
    DevBuf<double> cs_buf, cr_buf;
};

// x[idx[k]] = in[k]: a colour's received ghost entries into their slots
__global__ void k_scatter_idx(double *x, const int32_t *idx, int64_t n, const double *in) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) x[idx[k]] = in[k];
}

// Local copy of rows [r0, r1) of M with global column ids.
static void extract_rows(const GpuCsr &M, int64_t r0, int64_t r1, GpuCsr &out, Ctx *ctx) {
    hipStream_t s = ctx->stream;
    const int64_t n = r1 - r0;
    int64_t e0 = 0, e1 = 0;
    FAMG_CHECK_HIP(hipMemcpyAsync(&e0, M.rp64.get() + r0, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipMemcpyAsync(&e1, M.rp64.get() + r1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    csr_alloc(out, ctx, n, M.ncols, e1 - e0);
    hipLaunchKernelGGL(k_extract_rp, dim3(g1(n + 1)), dim3(256), 0, s, M.rp64.get(), r0, n, out.rp64.get());
    if (e1 > e0) {
        FAMG_CHECK_HIP(hipMemcpyAsync(out.col.get(), M.col.get() + e0, (e1 - e0) * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        FAMG_CHECK_HIP(hipMemcpyAsync(out.val.get(), M.val.get() + e0, (e1 - e0) * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

static void space_mark(Space &sp, const GpuCsr &local, Ctx *ctx) {
    if (local.nnz)
        hipLaunchKernelGGL(k_mark_ghost, dim3(g1(local.nnz)), dim3(256), 0, ctx->stream, local.col.get(),
                           local.nnz, sp.r0, sp.r1, sp.mark.get());
    FAMG_CHECK_HIP(hipGetLastError());
}

// After all matrices of the space are marked: the ghost list (device compaction
// of the marks, the same set plan_add_columns computes on the host), then the
// host plan (plan.hpp) with its two request exchanges over the transport.
// Slab levels: extend the marked ghost columns to whole planes (the planes the
// level's stencils reach below and above the owned ones), so the ghost region
// is the frame's ghost planes.  Costs extra halo entries only where a plane was
// referenced partly.
static void space_mark_planes(Space &sp, Ctx *ctx) {
    if (!sp.frame.on()) return;
    hipStream_t s = ctx->stream;
    const int64_t pl = sp.frame.pl();
    DevBuf<unsigned long long> ext(2);
    const unsigned long long init[2] = {~0ull, 0ull};
    FAMG_CHECK_HIP(hipMemcpyAsync(ext.get(), init, sizeof(init), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ghost_extent, dim3(g1(sp.n_glob)), dim3(256), 0, s, sp.mark.get(), sp.n_glob, sp.r0, sp.r1,
                       ext.get());
    unsigned long long h[2];
    FAMG_CHECK_HIP(hipMemcpyAsync(h, ext.get(), sizeof(h), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (h[0] != ~0ull) {
        const int64_t c0 = (int64_t)h[0] / pl * pl;
        hipLaunchKernelGGL(k_mark_range, dim3(g1(sp.r0 - c0)), dim3(256), 0, s, sp.mark.get(), c0, sp.r0);
    }
    if (h[1] >= (unsigned long long)sp.r1) {
        const int64_t c1 = std::min<int64_t>(sp.n_glob, ((int64_t)h[1] / pl + 1) * pl);
        hipLaunchKernelGGL(k_mark_range, dim3(g1(c1 - sp.r1)), dim3(256), 0, s, sp.mark.get(), sp.r1, c1);
    }
    FAMG_CHECK_HIP(hipGetLastError());
}

static void space_plan(Space &sp, Transport &tr, Ctx *ctx) {
    hipStream_t s = ctx->stream;
    sp.scan.resize(sp.n_glob + 1);
    const int64_t ng = scan_counts(sp.mark.get(), sp.scan.get(), sp.n_glob, *ctx);
    DevBuf<int64_t> ids(ng);
    hipLaunchKernelGGL(k_compact_ghost, dim3(g1(sp.n_glob)), dim3(256), 0, s, sp.mark.get(), sp.scan.get(),
                       sp.n_glob, ids.get());
    std::vector<int64_t> ghost_ids(ng);
    if (ng) FAMG_CHECK_HIP(hipMemcpyAsync(ghost_ids.data(), ids.get(), ng * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    if (sp.frame.on()) {  // ghost planes below / above (whole planes: space_mark_planes)
        const int64_t P = sp.frame.pl();
        int64_t below = 0;
        while (below < ng && ghost_ids[below] < sp.r0) below++;
        sp.frame.gl = below / P;
        sp.frame.gh = (ng - below) / P;
        const bool whole = below % P == 0 && (ng - below) % P == 0 &&
                           (below == 0 || ghost_ids[0] == sp.r0 - below) &&
                           (ng == below || ghost_ids[ng - 1] == sp.r1 + (ng - below) - 1);
        if (!whole) sp.frame = SlabFrame{};
    }
    HaloPlan &pl = sp.plan;
    plan_set_ghosts(pl, std::move(ghost_ids));
    sp.n_ghost = pl.n_ghost();
    const int P = tr.nranks;
    // all-to-all request counts
    DevBuf<int64_t> dsend(P), drecv(P);
    FAMG_CHECK_HIP(hipMemcpyAsync(dsend.get(), pl.req_cnt.data(), P * sizeof(int64_t), hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipMemsetAsync(drecv.get(), 0, P * sizeof(int64_t), s));
    std::vector<Peer> cp;
    for (int q = 0; q < P; q++)
        if (q != tr.rank) cp.push_back({q, dsend.get() + q, 8, drecv.get() + q, 8});
    tr.exchange(cp, s);
    std::vector<int64_t> got(P);
    FAMG_CHECK_HIP(hipMemcpyAsync(got.data(), drecv.get(), P * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    got[tr.rank] = 0;
    std::vector<int64_t> got_off(P + 1, 0);
    for (int q = 0; q < P; q++) got_off[q + 1] = got_off[q] + got[q];
    // exchange the requested ids
    DevBuf<int64_t> req_ids(std::max<int64_t>(1, sp.n_ghost)), in_ids(std::max<int64_t>(1, got_off[P]));
    if (sp.n_ghost)
        FAMG_CHECK_HIP(hipMemcpyAsync(req_ids.get(), pl.ghost_ids.data(), sp.n_ghost * sizeof(int64_t),
                                      hipMemcpyHostToDevice, s));
    std::vector<Peer> ip;
    for (int q = 0; q < P; q++) {
        if (q == tr.rank || (pl.req_cnt[q] == 0 && got[q] == 0)) continue;
        ip.push_back({q, req_ids.get() + pl.req_off[q], pl.req_cnt[q] * 8, in_ids.get() + got_off[q], got[q] * 8});
    }
    tr.exchange(ip, s);
    std::vector<int64_t> inh(got_off[P]);
    if (got_off[P])
        FAMG_CHECK_HIP(hipMemcpyAsync(inh.data(), in_ids.get(), got_off[P] * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    plan_set_incoming(pl, got.data(), inh.data());
    sp.nsend = (int64_t)pl.send_idx.size();
    sp.send_idx.resize(std::max<int64_t>(1, sp.nsend));
    sp.sendbuf.resize(std::max<int64_t>(1, sp.nsend));
    if (sp.nsend)
        FAMG_CHECK_HIP(hipMemcpyAsync(sp.send_idx.get(), pl.send_idx.data(), sp.nsend * sizeof(int32_t),
                                      hipMemcpyHostToDevice, s));
    sp.nbr = pl.nbr;
    sp.soff = pl.soff;
    sp.scnt = pl.scnt;
    sp.roff = pl.roff;
    sp.rcnt = pl.rcnt;
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
}

// flag[i] = 1 when row i references a ghost column (local column >= n_own)
__global__ void k_row_ghost(const int64_t *rp, const int32_t *col, int64_t n, int64_t n_own, uint8_t *flag) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint8_t g = 0;
    for (int64_t e = rp[i]; e < rp[i + 1]; e++)
        if (col[e] >= n_own) { g = 1; break; }
    flag[i] = g;
}

// Remap a local matrix to the [owned | ghost] numbering and cut its rows into
// three segments [0, lo) [lo, hi) [hi, n): [lo, hi) is the longest run of rows
// that read owned entries only (the interior of a slab), which can run while
// the halo is in flight.
static void space_remap(const Space &sp, GpuCsr &local, Ctx *ctx) {
    hipStream_t s = ctx->stream;
    if (local.nnz)
        hipLaunchKernelGGL(k_remap_cols, dim3(g1(local.nnz)), dim3(256), 0, s, local.col.get(),
                           local.nnz, sp.r0, sp.r1, sp.n_own, sp.scan.get());
    FAMG_CHECK_HIP(hipGetLastError());
    local.ncols = sp.n_own + sp.n_ghost;
    const int64_t n = local.nrows;
    if (sp.n_ghost == 0 || n == 0) {
        csr_finalize(local);
        return;
    }
    DevBuf<uint8_t> dflag(n);
    hipLaunchKernelGGL(k_row_ghost, dim3(g1(n)), dim3(256), 0, s, local.rp64.get(), local.col.get(), n,
                       sp.n_own, dflag.get());
    std::vector<uint8_t> flag(n);
    FAMG_CHECK_HIP(hipMemcpyAsync(flag.data(), dflag.get(), n, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    int64_t lo = 0, hi = 0;
    interior_segment(flag.data(), n, lo, hi);
    const std::vector<int64_t> segs{0, lo, hi, n};
    csr_finalize(local, &segs);
}

static void halo_pack(Space &sp, const double *x, hipStream_t s) {
    if (sp.nsend)
        hipLaunchKernelGGL(k_gather_idx, dim3(g1(sp.nsend)), dim3(256), 0, s, x, sp.send_idx.get(), sp.nsend,
                           sp.sendbuf.get());
    FAMG_CHECK_HIP(hipGetLastError());
}

static void halo_exchange(Space &sp, double *x, Transport &tr, hipStream_t s) {
    sp.peers.clear();
    for (size_t k = 0; k < sp.nbr.size(); k++)
        sp.peers.push_back({sp.nbr[k], sp.sendbuf.get() + sp.soff[k], sp.scnt[k] * 8,
                            x + sp.n_own + sp.roff[k], sp.rcnt[k] * 8});
    tr.exchange(sp.peers, s);
}

// the plan record of a halo exchange (kernel -2: bytes this rank sends + receives)
static void log_halo(const char *name, int64_t entries_sent, int64_t entries_recv) {
    log_launch(name, -2, -1, entries_recv, 8 * (entries_sent + entries_recv));
}

// refresh the ghost region of x (x has n_own + n_ghost entries)
static void halo(Space &sp, double *x, Transport &tr, hipStream_t s) {
    if (sp.redundant || sp.nbr.empty()) return;
    halo_pack(sp, x, s);
    halo_exchange(sp, x, tr, s);
    log_halo("halo", sp.nsend, sp.n_ghost);
}

// the exchange before sweep position p of an SGS level (its position lists)
static void halo_position(Space &sp, double *x, int64_t p, Transport &tr, hipStream_t s) {
    if (sp.redundant || sp.nbr.empty()) return;
    const int64_t np = (int64_t)sp.nbr.size();
    const int64_t s0 = sp.cs_off[p * np], s1 = sp.cs_off[(p + 1) * np];
    const int64_t q0 = sp.cr_off[p * np], q1 = sp.cr_off[(p + 1) * np];
    if (s1 > s0)
        hipLaunchKernelGGL(k_gather_idx, dim3(g1(s1 - s0)), dim3(256), 0, s, x, sp.cs_idx.get() + s0, s1 - s0,
                           sp.cs_buf.get() + s0);
    FAMG_CHECK_HIP(hipGetLastError());
    sp.peers.clear();
    for (int64_t k = 0; k < np; k++) {
        const int64_t a = sp.cs_off[p * np + k], b = sp.cs_off[p * np + k + 1];
        const int64_t ra = sp.cr_off[p * np + k], rb = sp.cr_off[p * np + k + 1];
        if (b == a && rb == ra) continue;  // the peer's mirrored counts are zero too
        sp.peers.push_back({sp.nbr[k], sp.cs_buf.get() + a, (b - a) * 8, sp.cr_buf.get() + ra, (rb - ra) * 8});
    }
    tr.exchange(sp.peers, s);
    if (q1 > q0)
        hipLaunchKernelGGL(k_scatter_idx, dim3(g1(q1 - q0)), dim3(256), 0, s, x, sp.cr_idx.get() + q0, q1 - q0,
                           sp.cr_buf.get() + q0);
    FAMG_CHECK_HIP(hipGetLastError());
    log_halo("halo_sgs", s1 - s0, q1 - q0);
}

// Does the exchange before position p carry an entry of colour c whose reading
// rows (on the receiving rank) have the colours in `readers`?  (Space comment)
static bool sgs_needed(int64_t p, int64_t c, uint32_t readers, int64_t C) {
    auto first = [&](int64_t col) { return col; };                            // forward position
    auto second = [&](int64_t col) { return col <= C - 2 ? 2 * C - 2 - col : INT64_MAX; };  // backward
    int64_t lo, hi;  // a reader at a position in [lo, hi) needs the value this exchange carries
    if (p == 0) {
        lo = 0;
        hi = first(c);
    } else {
        const int64_t t = p - 1, ct = t < C ? t : 2 * C - 2 - t;  // colour swept at t
        if (ct != c) return false;
        lo = p;
        hi = t == first(c) ? second(c) : INT64_MAX;
    }
    for (int64_t r = 0; r < C; r++) {
        if (!((readers >> r) & 1u)) continue;
        const int64_t q1 = first(r), q2 = second(r);
        if ((q1 >= lo && q1 < hi) || (q2 != INT64_MAX && q2 >= lo && q2 < hi)) return true;
    }
    return false;
}

// Position lists of an SGS level from its plan, the local A (owned rows, columns
// [owned | ghost]) and the global colouring (every rank holds it).  The reading
// colours of every ghost entry go to its owner once (a reversed halo exchange).
static void space_sgs_lists(Space &sp, const GpuCsr &A, const std::vector<int32_t> &colors, int64_t C, Transport &tr,
                            Ctx *ctx) {
    const int64_t np = (int64_t)sp.nbr.size(), P = 2 * C - 1;
    sp.ncol = C;
    sp.cs_off.assign(P * np + 1, 0);
    sp.cr_off.assign(P * np + 1, 0);
    if (sp.redundant || np == 0 || C > 32) return;
    hipStream_t s = ctx->stream;
    const HaloPlan &pl = sp.plan;
    // the colours of my rows reading each ghost entry
    std::vector<int64_t> rp(A.nrows + 1);
    std::vector<int32_t> col(std::max<int64_t>(1, A.nnz));
    FAMG_CHECK_HIP(hipMemcpyAsync(rp.data(), A.rp64.get(), (A.nrows + 1) * 8, hipMemcpyDeviceToHost, s));
    if (A.nnz) FAMG_CHECK_HIP(hipMemcpyAsync(col.data(), A.col.get(), A.nnz * 4, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    std::vector<uint32_t> rmask(sp.n_ghost, 0);
    for (int64_t i = 0; i < A.nrows; i++)
        for (int64_t e = rp[i]; e < rp[i + 1]; e++)
            if (col[e] >= sp.n_own) rmask[col[e] - sp.n_own] |= 1u << colors[sp.r0 + i];
    // ... to the owners: my receive range of peer k -> its send range to me
    DevBuf<uint32_t> dr(std::max<int64_t>(1, sp.n_ghost)), ds(std::max<int64_t>(1, sp.nsend));
    if (sp.n_ghost) FAMG_CHECK_HIP(hipMemcpyAsync(dr.get(), rmask.data(), sp.n_ghost * 4, hipMemcpyHostToDevice, s));
    std::vector<Peer> rev;
    for (int64_t k = 0; k < np; k++)
        rev.push_back({sp.nbr[k], dr.get() + sp.roff[k], sp.rcnt[k] * 4, ds.get() + sp.soff[k], sp.scnt[k] * 4});
    tr.exchange(rev, s);
    std::vector<uint32_t> smask(sp.nsend, 0);
    if (sp.nsend) FAMG_CHECK_HIP(hipMemcpyAsync(smask.data(), ds.get(), sp.nsend * 4, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
    std::vector<int32_t> si, ri;
    for (int64_t p = 0; p < P; p++)
        for (int64_t k = 0; k < np; k++) {
            for (int64_t i = sp.soff[k]; i < sp.soff[k] + sp.scnt[k]; i++) {
                const int32_t li = pl.send_idx[i];
                if (sgs_needed(p, colors[sp.r0 + li], smask[i], C)) si.push_back(li);
            }
            for (int64_t j = sp.roff[k]; j < sp.roff[k] + sp.rcnt[k]; j++)
                if (sgs_needed(p, colors[pl.ghost_ids[j]], rmask[j], C)) ri.push_back((int32_t)(sp.n_own + j));
            sp.cs_off[p * np + k + 1] = (int64_t)si.size();
            sp.cr_off[p * np + k + 1] = (int64_t)ri.size();
        }
    sp.cs_idx.resize(std::max<size_t>(1, si.size()));
    sp.cr_idx.resize(std::max<size_t>(1, ri.size()));
    sp.cs_buf.resize(std::max<size_t>(1, si.size()));
    sp.cr_buf.resize(std::max<size_t>(1, ri.size()));
    if (!si.empty()) FAMG_CHECK_HIP(hipMemcpyAsync(sp.cs_idx.get(), si.data(), si.size() * 4, hipMemcpyHostToDevice, s));
    if (!ri.empty()) FAMG_CHECK_HIP(hipMemcpyAsync(sp.cr_idx.get(), ri.data(), ri.size() * 4, hipMemcpyHostToDevice, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------- multigrid

struct DLevel {
    Space sp;
    CsrPtr A, R, P;  // local: A rows own(l) cols space l; R rows own(l+1) cols space l;
                     // P rows own(l) cols space l+1 (global ids when l+1 is redundant)
    std::shared_ptr<DiagOp> S;  // diagonal smoother slice, or
    std::shared_ptr<SgsOp> G;   // SGS over the owned rows (global colors)
    DevBuf<double> v, t, f, r;
};

struct DistMultigridOp : LinOp {
    std::shared_ptr<Transport> tr;
    std::vector<DLevel> L;                 // distributed levels [0, La)
    std::shared_ptr<MultigridOp> tail;     // global levels [La, end)
    int64_t La = 0, nlevels = 0;
    int64_t mu = 1, steps = 1;
    std::vector<int64_t> tail_splits;      // row splits of level La
    int64_t tail_max = 0;
    DevBuf<double> fc_own, gather, fc_full, vc_full;
    std::mutex mtx;
    // halo/interior overlap: the exchange runs on comm_stream while the
    // interior rows run on the context stream
    bool overlap = true;
    // SGS levels exchange, before each colour, only what later colours read (option 2)
    bool per_colour_halo = true;
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_pack = nullptr, ev_halo = nullptr;
    // hipGraph replay of the cycle (option 1, off by default): RCCL transport only
    // -- its grouped send/recv and all-gather are stream-ordered and capturable,
    // the loopback transport synchronises on the host
    bool use_graph = false;
    struct Graph {
        double *out;
        const double *rhs;
        hipGraphExec_t exec;
    };
    std::vector<Graph> graphs_;
    uint64_t flags_gen_ = 0;
    void drop_graphs() {
        for (auto &g : graphs_) (void)hipGraphExecDestroy(g.exec);
        graphs_.clear();
    }
    Kind kind() const override { return Kind::DistMultigrid; }
    bool is_precond() const override { return true; }
    ~DistMultigridOp() override {
        drop_graphs();
        if (ev_pack) (void)hipEventDestroy(ev_pack);
        if (ev_halo) (void)hipEventDestroy(ev_halo);
        if (comm_stream) (void)hipStreamDestroy(comm_stream);
    }

    // y = m x (with epilogue) after refreshing x's ghosts.  For a matrix cut
    // into [boundary | interior | boundary] the interior rows run while the
    // exchange is in flight on comm_stream.
    void halo_spmv(Space &sp, double *x, const GpuCsr &m, double *y, SpmvMode mode, const SpmvEpi &epi) {
        hipStream_t s = ctx->stream;
        if (!overlap || sp.redundant || sp.nbr.empty() || m.seg_rows.size() != 4) {
            halo(sp, x, *tr, s);
            spmv(m, x, y, mode, epi, s);
            return;
        }
        halo_pack(sp, x, s);
        FAMG_CHECK_HIP(hipEventRecord(ev_pack, s));
        FAMG_CHECK_HIP(hipStreamWaitEvent(comm_stream, ev_pack, 0));
        halo_exchange(sp, x, *tr, comm_stream);
        FAMG_CHECK_HIP(hipEventRecord(ev_halo, comm_stream));
        spmv(m, x, y, mode, epi, s, 1);
        FAMG_CHECK_HIP(hipStreamWaitEvent(s, ev_halo, 0));
        spmv(m, x, y, mode, epi, s, 0);
        spmv(m, x, y, mode, epi, s, 2);
    }

    // Multicolor SGS on a distributed level: the global smoother's color sweeps
    // (SgsOp::sweep / sweep_x) with the ghosts refreshed before every color, so
    // each color reads the values the previous colors wrote on every rank.
    // zero: e = SGS(b) from e = 0 (ghosts of e filled with 0 first); otherwise
    // x <- x + SGS(b - A x) in place.  Rows of one color do not couple, and a
    // row's entries keep their stored order, so every rank's rows get exactly
    // the single-GPU sweep's values.
    void sgs_sweep(DLevel &D, double *x, const double *b, bool zero) {
        SgsOp &G = *D.G;
        hipStream_t s = ctx->stream;
        const int64_t C = G.ncolors;
        SpmvEpi epi;
        epi.b = b;
        epi.d = G.dinv.get();
        epi.perm = G.perm.get();
        int64_t c0 = 0;
        if (zero) {
            vec_fill(x, 0.0, D.sp.n_own + D.sp.n_ghost, s);
            if (D.sp.n_own) G.first_color(x, b);
            c0 = 1;
        }
        // ghosts before each colour: the position lists (only what a later colour
        // reads; none before colour 0 from zero: the ghosts are zero), else the
        // whole halo before every colour as in round 3
        const bool pl = per_colour_halo && D.sp.ncol == C && C <= 32;
        for (int64_t c = c0; c < C; c++) {
            if (!pl) halo(D.sp, x, *tr, s);
            else if (c > 0 || !zero) halo_position(D.sp, x, c, *tr, s);
            if (D.sp.n_own) spmv(G.Ap, x, x, SPMV_SGS, epi, s, c);
        }
        for (int64_t c = C - 2; c >= 0; c--) {
            if (pl) halo_position(D.sp, x, 2 * C - 2 - c, *tr, s);
            else halo(D.sp, x, *tr, s);
            if (D.sp.n_own) spmv(G.Ap, x, x, SPMV_SGS, epi, s, c);
        }
    }

    // last_out: the final step writes there (owned rows only) instead of t
    // pre_df: t = d*f (the first step from zero) was written by the restriction (SPMV_SETDF)
    void smooth(int64_t l, double *&v, double *&t, const double *f, bool zero, double *last_out = nullptr,
                bool pre_df = false) {
        DLevel &D = L[l];
        hipStream_t s = ctx->stream;
        log_at(l, AMG_ROLE_SMOOTH);
        if (D.G) {  // in place on v; the residual form as MultigridOp::smooth
            for (int64_t it = 0; it < steps; it++) {
                if (zero && it == 0) {
                    sgs_sweep(D, v, f, true);
                } else if (tail->sgs_residual_form) {
                    SpmvEpi epi;
                    epi.b = f;
                    halo_spmv(D.sp, v, D.A->m, D.r.get(), SPMV_RESID, epi);
                    sgs_sweep(D, t, D.r.get(), true);
                    vec_add_inplace(v, t, D.sp.n_own, s);
                } else {
                    sgs_sweep(D, v, f, false);
                }
            }
            return;
        }
        for (int64_t it = 0; it < steps; it++) {
            if (last_out && it + 1 == steps) t = last_out;
            if (zero && it == 0) {
                if (pre_df) {
                    // written by the restriction
                } else if (D.S->dcode.get()) {
                    vec_mul_coded(t, D.S->dcode.get(), D.S->dtab.get(), f, D.sp.n_own, s);
                } else {
                    vec_mul(t, D.S->d.get(), f, D.sp.n_own, s);
                }
            } else {
                SpmvEpi epi;
                epi.b = f;
                epi.d = D.S->d.get();
                epi.dc = D.S->dcode.get();
                epi.dt = D.S->dtab.get();
                epi.dk = D.S->dconst;
                halo_spmv(D.sp, v, D.A->m, t, SPMV_JACOBI, epi);
            }
            std::swap(v, t);
        }
    }

    // gather the owned part of level La into the full vector on every rank
    void gather_tail(const double *own) {
        hipStream_t s = ctx->stream;
        const int P = tr->nranks;
        const int64_t cnt = tail_splits[tr->rank + 1] - tail_splits[tr->rank];
        if (cnt) vec_copy(fc_own.get(), own, cnt, s);
        tr->allgather(fc_own.get(), gather.get(), tail_max * 8, s);
        for (int q = 0; q < P; q++) {
            const int64_t c = tail_splits[q + 1] - tail_splits[q];
            if (c) vec_copy(fc_full.get() + tail_splits[q], gather.get() + q * tail_max, c, s);
        }
    }

    // out (level 0 only, may be null): the post-smoothing's last Jacobi step
    // writes the owned rows there directly, saving the final n_own copy
    // the single-GPU cycle's zero-guess fold (fold_level) where the level's
    // residual needs no halo (a rank that owns the whole level): RESID0 reads
    // f and d at every column, which a ghost region of f would have to carry
    bool folds(const DLevel &D, bool zero) const {
        return zero && !D.G && D.sp.nbr.empty() && D.sp.n_ghost == 0 &&
               fold_level(D.A.get(), D.S.get(), D.P.get(), tail->fold_zero_guess, true, steps);
    }
    // the restriction out of distributed level l writes level l + 1's first
    // Jacobi step from zero (SPMV_SETDF), as MultigridOp::cycle does
    bool restrict_df(int64_t l) const {
        if (!tail->restrict_df || !setdf_enabled() || steps < 1 || !r_has_setdf(L[l].R.get())) return false;
        if (l + 1 < La) {
            const DLevel &C = L[l + 1];
            return C.S && !C.G && !folds(C, true);
        }
        // into the tail: one rank restricts straight into the tail's input
        if (tr->nranks != 1 || tail->levels.size() < 2) return false;
        const MgLevel &T = tail->levels[0];
        auto *Ac = dynamic_cast<const CsrOp *>(T.A.get());
        auto *Dc = dynamic_cast<const DiagOp *>(T.S.get());
        auto *Pc = dynamic_cast<const CsrOp *>(T.P.get());
        return Ac && Dc && !fold_level(Ac, Dc, Pc, tail->fold_zero_guess, true, steps);
    }
    static SpmvEpi df_epi(const DiagOp &S, double *y2) {
        SpmvEpi e;
        e.d = S.d.get();
        e.dc = S.dcode.get();
        e.dt = S.dtab.get();
        e.dk = S.dconst;
        e.y2 = y2;
        return e;
    }

    void cycle(int64_t l, double *v, const double *f, bool zero, double *out = nullptr, bool pre_df = false) {
        DLevel &D = L[l];
        hipStream_t s = ctx->stream;
        double *v0 = v;
        double *t = (v == D.t.get()) ? D.v.get() : D.t.get();
        const bool fold = folds(D, zero);
        SpmvEpi epi;
        epi.b = f;
        SpmvEpi epi0 = epi;  // the folded epilogues' d*f
        if (D.S) {
            epi0.d = D.S->d.get();
            epi0.dc = D.S->dcode.get();
            epi0.dt = D.S->dtab.get();
            epi0.dk = D.S->dconst;
        }
        if (fold) {
            log_at(l, AMG_ROLE_RESID);
            spmv(D.A->m, f, D.r.get(), SPMV_RESID0, epi0, s);  // f - A (d f)
        } else {
            smooth(l, v, t, f, zero, nullptr, pre_df);
            log_at(l, AMG_ROLE_RESID);
            halo_spmv(D.sp, v, D.A->m, D.r.get(), SPMV_RESID, epi);
        }
        const bool df = restrict_df(l);
        if (l + 1 < La) {
            DLevel &C = L[l + 1];
            log_at(l, AMG_ROLE_RESTRICT);
            if (df) halo_spmv(D.sp, D.r.get(), D.R->m, C.f.get(), SPMV_SETDF, df_epi(*C.S, C.t.get()));
            else halo_spmv(D.sp, D.r.get(), D.R->m, C.f.get(), SPMV_SET, SpmvEpi{});
            for (int64_t k = 0; k < mu; k++) cycle(l + 1, C.v.get(), C.f.get(), k == 0, nullptr, df && k == 0);
            log_at(l, AMG_ROLE_INTERP);
            if (fold) {
                halo_spmv(C.sp, C.v.get(), D.P->m, t, SPMV_ADD0, epi0);  // v = d f + P v_c
                std::swap(v, t);
            } else {
                halo_spmv(C.sp, C.v.get(), D.P->m, v, SPMV_ADD, SpmvEpi{});
            }
        } else {
            const int64_t cnt = tail_splits[tr->rank + 1] - tail_splits[tr->rank];
            log_at(l, AMG_ROLE_RESTRICT);
            if (tr->nranks == 1) {  // nothing to gather: restrict into the tail's input
                if (df)
                    halo_spmv(D.sp, D.r.get(), D.R->m, fc_full.get(), SPMV_SETDF,
                              df_epi(*dynamic_cast<const DiagOp *>(tail->levels[0].S.get()), tail->levels[0].t.get()));
                else
                    halo_spmv(D.sp, D.r.get(), D.R->m, fc_full.get(), SPMV_SET, SpmvEpi{});
            } else {
                if (cnt) halo_spmv(D.sp, D.r.get(), D.R->m, gather.get() + tr->rank * tail_max, SPMV_SET, SpmvEpi{});
                else halo(D.sp, D.r.get(), *tr, s);
                gather_tail(gather.get() + tr->rank * tail_max);
            }
            if (g_launch_log) g_launch_log->level_base = (int32_t)La;
            for (int64_t k = 0; k < mu; k++) tail->cycle(0, vc_full.get(), fc_full.get(), k == 0, nullptr, df && k == 0);
            if (g_launch_log) g_launch_log->level_base = 0;
            log_at(l, AMG_ROLE_INTERP);
            if (fold) {
                spmv(D.P->m, vc_full.get(), t, SPMV_ADD0, epi0, s);
                std::swap(v, t);
            } else {
                spmv(D.P->m, vc_full.get(), v, SPMV_ADD, SpmvEpi{}, s);
            }
        }
        const bool direct = out && steps >= 1 && D.S && !D.G;
        smooth(l, v, t, f, false, direct ? out : nullptr);
        if (direct) return;
        if (v != v0) vec_copy(v0, v, D.sp.n_own, s);
        if (out) vec_copy(out, v0, D.sp.n_own, s);  // SGS (in place on v) or no smoothing steps
    }

    // Allocation length of a level-0 vector that A_0 reads in place: the owned
    // rows, then room for the halo entries (the solve loops keep x and p so)
    int64_t n_alloc0() const { return La > 0 ? L[0].sp.n_own + L[0].sp.n_ghost : nrows; }

    // r_own = b_own - (A_0 x)_own for the finest level, distributed or not; x
    // has n_alloc0() entries and its halo region is overwritten (no copy)
    DevBuf<double> rfull_;
    void residual0(const double *b, double *x, double *r) {
        hipStream_t s = ctx->stream;
        SpmvEpi epi;
        epi.b = b;
        if (La > 0) {
            halo_spmv(L[0].sp, x, L[0].A->m, r, SPMV_RESID, epi);
            return;
        }
        // everything replicated: gather x, global SpMV, keep the owned rows
        auto *A = dynamic_cast<CsrOp *>(tail->levels[0].A.get());
        FAMG_REQUIRE(A, AMG_ERR_UNSUPPORTED, "finest operator is not CSR");
        const int64_t r0 = tail_splits[tr->rank], cnt = tail_splits[tr->rank + 1] - r0;
        if (rfull_.size() < (size_t)A->nrows) rfull_.resize(A->nrows);
        gather_tail(x);
        spmv(A->m, fc_full.get(), rfull_.get(), SPMV_SET, SpmvEpi{}, s);
        if (cnt) vec_sub(r, b, rfull_.get() + r0, cnt, s);
    }

    // out_own = (A_0 x)_own, distributed or not (x as in residual0)
    void apply0(double *out, double *x) {
        hipStream_t s = ctx->stream;
        if (La > 0) {
            halo_spmv(L[0].sp, x, L[0].A->m, out, SPMV_SET, SpmvEpi{});
            return;
        }
        auto *A = dynamic_cast<CsrOp *>(tail->levels[0].A.get());
        FAMG_REQUIRE(A, AMG_ERR_UNSUPPORTED, "finest operator is not CSR");
        const int64_t r0 = tail_splits[tr->rank], cnt = tail_splits[tr->rank + 1] - r0;
        if (rfull_.size() < (size_t)A->nrows) rfull_.resize(A->nrows);
        gather_tail(x);
        spmv(A->m, fc_full.get(), rfull_.get(), SPMV_SET, SpmvEpi{}, s);
        if (cnt) vec_copy(out, rfull_.get() + r0, cnt, s);
    }

    void apply(double *out, const double *rhs) override {
        std::lock_guard<std::mutex> lk(mtx);
        hipStream_t s = ctx->stream;
        tail->ensure_workspace();
        if (flags_gen_ != flags_generation()) {  // a switch changed: graphs recorded the old launches
            drop_graphs();
            flags_gen_ = flags_generation();
        }
        if (!use_graph || !dynamic_cast<RcclTransport *>(tr.get())) {
            apply_eager(out, rhs);
            return;
        }
        for (auto &g : graphs_)
            if (g.out == out && g.rhs == rhs) {
                FAMG_CHECK_HIP(hipGraphLaunch(g.exec, s));
                return;
            }
        hipGraph_t graph = nullptr;
        FAMG_CHECK_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
            apply_eager(out, rhs);
        } catch (...) {
            (void)hipStreamEndCapture(s, &graph);
            if (graph) (void)hipGraphDestroy(graph);
            throw;
        }
        FAMG_CHECK_HIP(hipStreamEndCapture(s, &graph));
        hipGraphExec_t exec = nullptr;
        FAMG_CHECK_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        (void)hipGraphDestroy(graph);
        if (graphs_.size() >= 8) {
            (void)hipGraphExecDestroy(graphs_.front().exec);
            graphs_.erase(graphs_.begin());
        }
        graphs_.push_back({out, rhs, exec});
        FAMG_CHECK_HIP(hipGraphLaunch(exec, s));
    }

    // launch records of one eager cycle on scratch vectors (amg_dist_cycle_plan)
    std::vector<LaunchRec> cycle_plan() {
        std::lock_guard<std::mutex> lk(mtx);
        tail->ensure_workspace();
        DevBuf<double> b(std::max<int64_t>(1, nrows)), z(std::max<int64_t>(1, nrows));
        vec_fill(b.get(), 1.0, nrows, ctx->stream);
        LaunchLog log;
        g_launch_log = &log;
        try {
            apply_eager(z.get(), b.get());
        } catch (...) {
            g_launch_log = nullptr;
            throw;
        }
        g_launch_log = nullptr;
        FAMG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
        return log.recs;
    }

    // one cycle issued on the stream (workspaces allocated beforehand)
    void apply_eager(double *out, const double *rhs) {
        hipStream_t s = ctx->stream;
        if (La == 0) {
            gather_tail(rhs);
            tail->cycle(0, vc_full.get(), fc_full.get(), true, nullptr);
            const int64_t r0 = tail_splits[tr->rank], cnt = tail_splits[tr->rank + 1] - r0;
            if (cnt) vec_copy(out, vc_full.get() + r0, cnt, s);
            return;
        }
        if (out != rhs) {
            cycle(0, L[0].v.get(), rhs, true, out);
        } else {  // in place: rhs is read by the last step's epilogue
            cycle(0, L[0].v.get(), rhs, true);
            vec_copy(out, L[0].v.get(), L[0].sp.n_own, s);
        }
    }
};

// Distributed A_l as a LinOp: out_own = A (x_own with halo)
struct DistLevelOp : LinOp {
    std::shared_ptr<DistMultigridOp> mg;
    int64_t level = 0;
    DevBuf<double> x;
    Kind kind() const override { return Kind::DistCsr; }
    // The caller's rhs holds the owned rows only (LinOp::apply hands over an
    // n_own vector), so it is staged into a buffer with room for the halo; the
    // V-cycle and the solve loops read their own padded vectors in place.
    void apply(double *out, const double *rhs) override {
        std::lock_guard<std::mutex> lk(mg->mtx);  // halo buffers/events are shared with the V-cycle
        ctx->set_device();
        DLevel &D = mg->L[level];
        hipStream_t s = ctx->stream;
        vec_copy(x.get(), rhs, D.sp.n_own, s);
        mg->halo_spmv(D.sp, x.get(), D.A->m, out, SPMV_SET, SpmvEpi{});
    }
};

// The owned planes [r0, r1) of a grid operator as a frame (no ghosts yet), or
// off when the operator has no grid hint or the split cuts a plane.
static SlabFrame owned_frame(const GpuCsr &A, int64_t r0, int64_t r1) {
    SlabFrame f;
    const int64_t *g = A.grid;
    if (g[0] <= 0 || g[1] <= 0 || g[2] <= 0 || g[0] * g[1] * g[2] != A.nrows || r1 <= r0) return f;
    const int64_t pl = g[0] * g[1];
    if (r0 % pl || r1 % pl) return f;
    f.nx = g[0]; f.ny = g[1]; f.gz = g[2];
    f.z0 = r0 / pl;
    f.nz = (r1 - r0) / pl;
    return f;
}

// A rank-local matrix with slab frames: its rows are rf's owned planes, its
// columns cf's vector (both must be on for the grid kernels to take it)
static void set_frames(GpuCsr &m, const SlabFrame &rf, const SlabFrame &cf, bool square) {
    auto whole = [](const SlabFrame &f) { return f.on() && f.z0 == 0 && f.nz == f.gz && f.gl == 0 && f.gh == 0; };
    if (whole(rf) && whole(cf)) {  // a rank that owns the whole level: the global matrix, unframed
        m.rframe = m.cframe = SlabFrame{};
        if (square) {
            m.grid[0] = rf.nx; m.grid[1] = rf.ny; m.grid[2] = rf.gz;
            m.grid_src = 1;
        }
        return;
    }
    m.rframe = rf;
    m.cframe = cf;
    if (square && rf.on() && cf.on()) {  // the owned grid: the x-staged classes' row grid
        m.grid[0] = rf.nx; m.grid[1] = rf.ny; m.grid[2] = rf.nz;
        m.grid_src = 1;
    }
}

static std::shared_ptr<DistMultigridOp> build_dist(amg_comm *comm, MultigridOp &g_in,
                                                   const int64_t *splits, int64_t agglo) {
    // the caller's operators (a multigrid that ran may hold renumbered copies of
    // some levels, reorder.hip): the splits refer to their rows
    const std::shared_ptr<MultigridOp> gview = g_in.original_view();
    const MultigridOp &g = *gview;
    Ctx *ctx = comm->ctx;
    Transport &tr = *comm->tr;
    const int P = tr.nranks, me = tr.rank;
    auto d = std::make_shared<DistMultigridOp>();
    d->ctx = ctx;
    d->tr = comm->tr;
    FAMG_CHECK_HIP(hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking));
    FAMG_CHECK_HIP(hipEventCreateWithFlags(&d->ev_pack, hipEventDisableTiming));
    FAMG_CHECK_HIP(hipEventCreateWithFlags(&d->ev_halo, hipEventDisableTiming));
    d->mu = g.mu;
    d->steps = g.steps;
    d->nlevels = (int64_t)g.levels.size();
    {
        std::vector<int64_t> rows(d->nlevels);
        for (int64_t l = 0; l < d->nlevels; l++) rows[l] = g.levels[l].A->nrows;
        d->La = first_redundant_level(rows.data(), d->nlevels, agglo);
    }
    auto sp_of = [&](int64_t l) {
        std::vector<int64_t> s(splits + l * (P + 1), splits + (l + 1) * (P + 1));
        FAMG_REQUIRE(s[0] == 0 && s[P] == g.levels[l].A->nrows, AMG_ERR_DIM, "level splits must cover the level");
        for (int q = 0; q < P; q++) FAMG_REQUIRE(s[q + 1] >= s[q], AMG_ERR_INVALID, "splits must be monotone");
        return s;
    };
    d->L.resize(d->La);
    for (int64_t l = 0; l < d->La; l++) {
        DLevel &D = d->L[l];
        auto *A = dynamic_cast<CsrOp *>(g.levels[l].A.get());
        auto *R = dynamic_cast<CsrOp *>(g.levels[l].R.get());
        auto *Pm = dynamic_cast<CsrOp *>(g.levels[l].P.get());
        auto *S = dynamic_cast<DiagOp *>(g.levels[l].S.get());
        auto *G = dynamic_cast<SgsOp *>(g.levels[l].S.get());
        FAMG_REQUIRE(A && R && Pm, AMG_ERR_UNSUPPORTED, "distributed levels need CSR operators");
        FAMG_REQUIRE(S || G, AMG_ERR_UNSUPPORTED,
                     "distributed levels need a diagonal (Jacobi/L1/L2) or multicolor SGS smoother");
        const std::vector<int64_t> spl = sp_of(l);
        plan_init(D.sp.plan, P, me, spl.data());
        D.sp.n_glob = A->nrows;
        D.sp.r0 = D.sp.plan.r0;
        D.sp.r1 = D.sp.plan.r1;
        D.sp.n_own = D.sp.plan.n_own;
        D.sp.frame = owned_frame(A->m, D.sp.r0, D.sp.r1);
    }
    int64_t tail_r0 = 0, tail_r1 = 0;  // this rank's rows of the first redundant level
    if (d->La < d->nlevels) {
        const std::vector<int64_t> ts = sp_of(d->La);
        tail_r0 = ts[me];
        tail_r1 = ts[me + 1];
    }
    // local matrices with global columns
    for (int64_t l = 0; l < d->La; l++) {
        DLevel &D = d->L[l];
        auto *A = dynamic_cast<CsrOp *>(g.levels[l].A.get());
        auto *R = dynamic_cast<CsrOp *>(g.levels[l].R.get());
        auto *Pm = dynamic_cast<CsrOp *>(g.levels[l].P.get());
        D.A = make_csr(ctx);
        extract_rows(A->m, D.sp.r0, D.sp.r1, D.A->m, ctx);
        D.P = make_csr(ctx);
        extract_rows(Pm->m, D.sp.r0, D.sp.r1, D.P->m, ctx);
        const std::vector<int64_t> cs = (l + 1 < d->La) ? std::vector<int64_t>() : sp_of(l + 1);
        const int64_t cr0 = (l + 1 < d->La) ? 0 : cs[me], cr1 = (l + 1 < d->La) ? 0 : cs[me + 1];
        D.R = make_csr(ctx);
        if (l + 1 < d->La) {
            // rows of R: coarse rows owned at level l+1 (its space is set up below)
            const std::vector<int64_t> c2 = sp_of(l + 1);
            extract_rows(R->m, c2[me], c2[me + 1], D.R->m, ctx);
        } else {
            extract_rows(R->m, cr0, cr1, D.R->m, ctx);
        }
        // smoother slice (SGS: built on the remapped local A below)
        auto *S = dynamic_cast<DiagOp *>(g.levels[l].S.get());
        if (!S) continue;
        D.S = std::make_shared<DiagOp>();
        D.S->ctx = ctx;
        D.S->nrows = D.S->ncols = D.sp.n_own;
        D.S->d.resize(D.sp.n_own);
        if (D.sp.n_own) vec_copy(D.S->d.get(), S->d.get() + D.sp.r0, D.sp.n_own, ctx->stream);
        array_codes_u8(D.S->d.get(), D.sp.n_own, *ctx, D.S->dcode, D.S->dtab, &D.S->dconst);  // 1 B per row when few values
        D.S->codes_tried = true;
    }
    // ghost sets: space l collects A_l, R_l (fine columns) and P_{l-1} (coarse columns)
    for (int64_t l = 0; l < d->La; l++) {
        Space &sp = d->L[l].sp;
        sp.mark.resize(sp.n_glob);
        FAMG_CHECK_HIP(hipMemsetAsync(sp.mark.get(), 0, sp.n_glob * sizeof(int64_t), ctx->stream));
        space_mark(sp, d->L[l].A->m, ctx);
        space_mark(sp, d->L[l].R->m, ctx);
        if (l > 0) space_mark(sp, d->L[l - 1].P->m, ctx);
        space_mark_planes(sp, ctx);
        space_plan(sp, tr, ctx);
        {  // slab frames of the local A_l, R_l (rows: level l+1) and P_{l-1} (columns: space l)
            const SlabFrame rows_next =
                owned_frame(dynamic_cast<CsrOp *>(g.levels[l + 1].A.get())->m, l + 1 < d->La ? d->L[l + 1].sp.r0 : tail_r0,
                            l + 1 < d->La ? d->L[l + 1].sp.r1 : tail_r1);
            set_frames(d->L[l].A->m, sp.frame, sp.frame, true);
            set_frames(d->L[l].R->m, rows_next, sp.frame, false);
            if (l > 0) set_frames(d->L[l - 1].P->m, d->L[l - 1].sp.frame, sp.frame, false);
        }
        space_remap(sp, d->L[l].A->m, ctx);
        space_remap(sp, d->L[l].R->m, ctx);
        if (l > 0) space_remap(sp, d->L[l - 1].P->m, ctx);
        sp.mark.release();
        sp.scan.release();
        // a wave-per-row local matrix splits its rows like the global one (same
        // waves per row: the same sums)
        {
            auto *Ag = dynamic_cast<CsrOp *>(g.levels[l].A.get());
            auto *Rg = dynamic_cast<CsrOp *>(g.levels[l].R.get());
            d->L[l].A->m.vec_wpr = Ag->m.vec_wpr;
            d->L[l].R->m.vec_wpr = Rg->m.vec_wpr;
            if (l > 0) d->L[l - 1].P->m.vec_wpr = dynamic_cast<CsrOp *>(g.levels[l - 1].P.get())->m.vec_wpr;
        }
        for (auto *op : {d->L[l].A.get(), d->L[l].R.get()}) {
            op->nrows = op->m.nrows;
            op->ncols = op->m.ncols;
        }
    }
    // SGS slices: the owned rows of the remapped local A (columns [owned | ghost],
    // owned row i = column i) under the global coloring
    for (int64_t l = 0; l < d->La; l++) {
        auto *G = dynamic_cast<SgsOp *>(g.levels[l].S.get());
        if (!G) continue;
        DLevel &D = d->L[l];
        FAMG_REQUIRE((int64_t)G->host_colors.size() == D.sp.n_glob, AMG_ERR_INVALID, "sgs: coloring size");
        auto *Ag = dynamic_cast<CsrOp *>(g.levels[l].A.get());
        D.G = make_sgs_slice(D.A, G->host_colors.data() + D.sp.r0, G->ncolors, Ag->diagonal() + D.sp.r0);
        space_sgs_lists(D.sp, D.A->m, G->host_colors, G->ncolors, *d->tr, ctx);
    }
    // the last distributed level's P references the replicated level La by global id
    if (d->La > 0) {
        DLevel &D = d->L[d->La - 1];
        const GpuCsr &Ag = dynamic_cast<CsrOp *>(g.levels[d->La].A.get())->m;
        set_frames(D.P->m, D.sp.frame, owned_frame(Ag, 0, Ag.nrows), false);
        csr_finalize(D.P->m);
        // the same waves per row as the global P (finalize chose from the local rows)
        D.P->m.vec_wpr = dynamic_cast<CsrOp *>(g.levels[d->La - 1].P.get())->m.vec_wpr;
    }
    // R_l / P_l of a 2x2x2-box level as grid-transfer classes through the slab
    // frames (the classes of their global rows; every entry checked)
    for (int64_t l = 0; l < d->La; l++) {
        const GpuCsr &Af = dynamic_cast<CsrOp *>(g.levels[l].A.get())->m;
        const GpuCsr &Ac = dynamic_cast<CsrOp *>(g.levels[l + 1].A.get())->m;
        bool box = true;
        for (int q = 0; q < 3; q++) box = box && Af.grid[q] > 0 && Ac.grid[q] == (Af.grid[q] + 1) / 2;
        if (!box) continue;
        GpuCsr &R = d->L[l].R->m, &Pm = d->L[l].P->m;
        if (R.nrows > 0) gtc_attach(R, Af.grid, Ac.grid, 1);  // gtc_classes checks the frames / grids first
        if (Pm.nrows > 0) gtc_attach(Pm, Af.grid, Ac.grid, 0);
        if (R.nrows > 0 && (!R.gtc_on || gtx_mode() == 2)) gtx_attach(R, Af.grid, Ac.grid, 1);
        if (Pm.nrows > 0 && (!Pm.gtc_on || gtx_mode() == 2)) gtx_attach(Pm, Af.grid, Ac.grid, 0);
    }
    for (int64_t l = 0; l < d->La; l++) {
        d->L[l].P->nrows = d->L[l].P->m.nrows;
        d->L[l].P->ncols = d->L[l].P->m.ncols;
    }
    // workspaces
    for (int64_t l = 0; l < d->La; l++) {
        DLevel &D = d->L[l];
        const int64_t nv = D.sp.n_own + D.sp.n_ghost;
        D.v.resize(std::max<int64_t>(1, nv));
        D.t.resize(std::max<int64_t>(1, nv));
        D.r.resize(std::max<int64_t>(1, nv));
        D.f.resize(std::max<int64_t>(1, D.sp.n_own));
        FAMG_CHECK_HIP(hipMemsetAsync(D.v.get(), 0, std::max<int64_t>(1, nv) * 8, ctx->stream));
        FAMG_CHECK_HIP(hipMemsetAsync(D.t.get(), 0, std::max<int64_t>(1, nv) * 8, ctx->stream));
        FAMG_CHECK_HIP(hipMemsetAsync(D.r.get(), 0, std::max<int64_t>(1, nv) * 8, ctx->stream));
    }
    // redundant tail
    d->tail = std::make_shared<MultigridOp>();
    d->tail->ctx = ctx;
    d->tail->mu = g.mu;
    d->tail->steps = g.steps;
    d->tail->fold_zero_guess = g.fold_zero_guess;
    d->tail->sgs_residual_form = g.sgs_residual_form;
    d->tail->restrict_df = g.restrict_df;  // DistMultigridOp::restrict_df reads it
    d->tail->reorder = 0;  // the distributed cycle drives the tail's levels directly, in their numbering
    for (int64_t l = d->La; l < d->nlevels; l++) d->tail->levels.push_back(MgLevel{g.levels[l].A, g.levels[l].S, g.levels[l].R, g.levels[l].P});
    d->tail->nrows = d->tail->ncols = g.levels[d->La].A->nrows;
    // the tail is cycled redundantly on every rank: under the auto policy,
    // CSR-stream matrices (e.g. from a global setup copy built CSR-only) get
    // the storage the policy picks now (SELL / wave-per-row).  That happens on
    // private copies: g's operators (and any hipGraph g captured over their
    // buffers) stay untouched.
    if (g_spmv_format_policy == 0)
        for (auto &lv : d->tail->levels)
            for (LinOpPtr *op : {&lv.A, &lv.R, &lv.P})
                if (auto *c = dynamic_cast<CsrOp *>(op->get()))
                    if (c->m.kernel == SPMV_KERNEL_STREAM) {
                        CsrPtr cp = make_csr(ctx);
                        csr_clone(c->m, cp->m);
                        csr_finalize(cp->m, nullptr);
                        cp->nrows = c->nrows;
                        cp->ncols = c->ncols;
                        if (cp->m.kernel != SPMV_KERNEL_STREAM) *op = cp;
                    }
    d->tail_splits = sp_of(d->La);
    for (int q = 0; q < P; q++) d->tail_max = std::max(d->tail_max, d->tail_splits[q + 1] - d->tail_splits[q]);
    const int64_t nt = g.levels[d->La].A->nrows;
    d->fc_own.resize(std::max<int64_t>(1, d->tail_max));
    d->gather.resize(std::max<int64_t>(1, d->tail_max * P));
    d->fc_full.resize(std::max<int64_t>(1, nt));
    d->vc_full.resize(std::max<int64_t>(1, nt));
    FAMG_CHECK_HIP(hipMemsetAsync(d->gather.get(), 0, std::max<int64_t>(1, d->tail_max * P) * 8, ctx->stream));
    d->nrows = d->ncols = d->La > 0 ? d->L[0].sp.n_own : (d->tail_splits[me + 1] - d->tail_splits[me]);
    FAMG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    tr.barrier(ctx->stream);
    return d;
}

}  // namespace famg

// ------------------------------------------------------------------ C ABI

#define dguard guard

static std::shared_ptr<DistMultigridOp> need_dist(const amg_linop *h) {
    FAMG_REQUIRE(h && h->op, AMG_ERR_INVALID, "null amg_linop handle");
    auto p = std::dynamic_pointer_cast<DistMultigridOp>(h->op);
    FAMG_REQUIRE(p, AMG_ERR_INVALID, "operator is not a distributed multigrid");
    return p;
}

extern "C" {

int32_t amg_comm_unique_id_size(void) { return (int32_t)sizeof(ncclUniqueId); }

const char *amg_rccl_library(void) {
    static std::string p;
    try {
        p = rccl().path;
    } catch (...) {
        p.clear();
    }
    return p.c_str();
}

amg_status amg_comm_get_unique_id(void *id) {
    return dguard([&] {
        FAMG_REQUIRE(id, AMG_ERR_INVALID, "null id buffer");
        ncclUniqueId u;
        FAMG_CHECK_NCCL(rccl().GetUniqueId(&u));
        std::memcpy(id, &u, sizeof(u));
    });
}

amg_status amg_comm_create(amg_ctx *ctx, int32_t nranks, int32_t rank, const void *id, amg_comm **out) {
    return dguard([&] {
        FAMG_REQUIRE(ctx && id && out && nranks > 0 && rank >= 0 && rank < nranks, AMG_ERR_INVALID, "bad argument");
        Ctx *c = reinterpret_cast<Ctx *>(ctx);
        c->set_device();
        auto t = std::make_shared<RcclTransport>();
        t->nranks = nranks;
        t->rank = rank;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        FAMG_CHECK_NCCL(rccl().CommInitRank(&t->comm, nranks, u, rank));
        // RCCL's device probing may leave a stale per-thread HIP error that the
        // next hipGetLastError() check would report as ours
        (void)hipGetLastError();
        *out = new amg_comm{c, t};
    });
}

amg_status amg_loopback_hub_create(int32_t nranks, amg_loopback_hub **out) {
    return dguard([&] {
        FAMG_REQUIRE(out && nranks > 0, AMG_ERR_INVALID, "bad argument");
        *out = new amg_loopback_hub{std::make_shared<LoopbackHub>(nranks)};
    });
}

amg_status amg_loopback_hub_destroy(amg_loopback_hub *hub) {
    return dguard([&] { delete hub; });
}

amg_status amg_comm_create_loopback(amg_ctx *ctx, amg_loopback_hub *hub, int32_t rank, amg_comm **out) {
    return dguard([&] {
        FAMG_REQUIRE(ctx && hub && out && rank >= 0 && rank < hub->hub->nranks, AMG_ERR_INVALID, "bad argument");
        auto t = std::make_shared<LoopbackTransport>();
        t->hub = hub->hub;
        t->nranks = hub->hub->nranks;
        t->rank = rank;
        *out = new amg_comm{reinterpret_cast<Ctx *>(ctx), t};
    });
}

amg_status amg_comm_destroy(amg_comm *comm) {
    return dguard([&] {
        if (comm) comm->ctx->set_device();
        delete comm;
    });
}

amg_status amg_comm_rank(const amg_comm *comm, int32_t *rank, int32_t *nranks) {
    return dguard([&] {
        FAMG_REQUIRE(comm, AMG_ERR_INVALID, "null comm");
        if (rank) *rank = comm->tr->rank;
        if (nranks) *nranks = comm->tr->nranks;
    });
}

amg_status amg_comm_barrier(amg_comm *comm) {
    return dguard([&] {
        FAMG_REQUIRE(comm, AMG_ERR_INVALID, "null comm");
        comm->ctx->set_device();
        comm->tr->barrier(comm->ctx->stream);
    });
}

static void reduce_host(amg_comm *comm, double *value, bool is_max) {
    FAMG_REQUIRE(comm && value, AMG_ERR_INVALID, "null argument");
    comm->ctx->set_device();
    DevBuf<double> b(1);
    hipStream_t s = comm->ctx->stream;
    FAMG_CHECK_HIP(hipMemcpyAsync(b.get(), value, 8, hipMemcpyHostToDevice, s));
    comm->tr->allreduce(b.get(), 1, is_max, s);
    FAMG_CHECK_HIP(hipMemcpyAsync(value, b.get(), 8, hipMemcpyDeviceToHost, s));
    FAMG_CHECK_HIP(hipStreamSynchronize(s));
}

amg_status amg_comm_allreduce_max(amg_comm *comm, double *value) {
    return dguard([&] { reduce_host(comm, value, true); });
}

amg_status amg_comm_allreduce_sum(amg_comm *comm, double *value) {
    return dguard([&] { reduce_host(comm, value, false); });
}

amg_status amg_dist_multigrid_create(amg_comm *comm, const amg_linop *mg_global, const int64_t *level_splits,
                                     int64_t agglomerate_rows, amg_linop **out) {
    return dguard([&] {
        FAMG_REQUIRE(comm && mg_global && mg_global->op && level_splits && out, AMG_ERR_INVALID, "null argument");
        auto g = std::dynamic_pointer_cast<MultigridOp>(mg_global->op);
        FAMG_REQUIRE(g, AMG_ERR_INVALID, "mg_global is not a multigrid");
        FAMG_REQUIRE(g->ctx == comm->ctx, AMG_ERR_INVALID, "multigrid and comm on different contexts");
        comm->ctx->set_device();
        *out = new amg_linop{build_dist(comm, *g, level_splits, agglomerate_rows)};
    });
}

amg_status amg_dist_local_rows(const amg_linop *dist, int64_t *begin, int64_t *end) {
    return dguard([&] {
        auto d = need_dist(dist);
        FAMG_REQUIRE(begin && end, AMG_ERR_INVALID, "null output");
        if (d->La > 0) {
            *begin = d->L[0].sp.r0;
            *end = d->L[0].sp.r1;
        } else {
            *begin = d->tail_splits[d->tr->rank];
            *end = d->tail_splits[d->tr->rank + 1];
        }
    });
}

amg_status amg_dist_level_info(const amg_linop *dist, int64_t level, int64_t *info) {
    return dguard([&] {
        auto d = need_dist(dist);
        FAMG_REQUIRE(info && level >= 0 && level < d->nlevels, AMG_ERR_INVALID, "bad level");
        if (level < d->La) {
            const Space &sp = d->L[level].sp;
            info[0] = sp.n_own;
            info[1] = sp.n_ghost;
            info[2] = (int64_t)sp.nbr.size();
            info[3] = 0;
            int64_t rc = 0;
            for (int64_t c : sp.rcnt) rc += c;
            info[4] = rc;
            info[5] = sp.n_glob;
        } else {
            const int64_t n = d->tail->levels[level - d->La].A->nrows;
            info[0] = n; info[1] = 0; info[2] = 0; info[3] = 1; info[4] = 0; info[5] = n;
        }
    });
}

amg_status amg_dist_level_operator(const amg_linop *dist, int64_t level, amg_linop **out) {
    return dguard([&] {
        auto d = need_dist(dist);
        FAMG_REQUIRE(out && level >= 0 && level < d->La, AMG_ERR_INVALID, "level must be distributed");
        auto op = std::make_shared<DistLevelOp>();
        op->ctx = d->ctx;
        op->mg = d;
        op->level = level;
        op->nrows = op->ncols = d->L[level].sp.n_own;
        op->x.resize(std::max<int64_t>(1, d->L[level].sp.n_own + d->L[level].sp.n_ghost));
        FAMG_CHECK_HIP(hipMemset(op->x.get(), 0, op->x.bytes()));
        *out = new amg_linop{op};
    });
}

amg_status amg_dist_level_matrix(const amg_linop *dist, int64_t level, int32_t which, amg_linop **out) {
    return dguard([&] {
        auto d = need_dist(dist);
        FAMG_REQUIRE(out && level >= 0 && level < d->La && which >= 0 && which <= 2, AMG_ERR_INVALID,
                     "level must be distributed, which in {0,1,2}");
        const DLevel &D = d->L[level];
        *out = new amg_linop{which == 0 ? D.A : which == 1 ? D.R : D.P};
    });
}

amg_status amg_dist_cycle_plan(amg_linop *dist, amg_launch_rec *recs, int64_t cap, int64_t *count) {
    return dguard([&] {
        auto d = need_dist(dist);
        FAMG_REQUIRE(count && cap >= 0, AMG_ERR_INVALID, "bad argument");
        d->ctx->set_device();
        export_plan(d->cycle_plan(), recs, cap, count);
    });
}

amg_status amg_dist_set_option(amg_linop *dist, int32_t option, int64_t value) {
    return dguard([&] {
        auto d = need_dist(dist);
        std::lock_guard<std::mutex> lk(d->mtx);
        switch (option) {
        case 0: d->overlap = value != 0; d->drop_graphs(); break;
        case 1: d->use_graph = value != 0; d->drop_graphs(); break;
        case 2: d->per_colour_halo = value != 0; d->drop_graphs(); break;
        default: fail(AMG_ERR_INVALID, "unknown distributed multigrid option");
        }
    });
}

static SolveOps dist_ops(const std::shared_ptr<DistMultigridOp> &d, bool precondition) {
    SolveOps o;
    o.ctx = d->ctx;
    o.n = d->nrows;
    o.n_alloc = d->n_alloc0();
    DistMultigridOp *dm = d.get();
    o.A = [dm](double *out, double *x) {
        std::lock_guard<std::mutex> lk(dm->mtx);
        dm->ctx->set_device();
        dm->apply0(out, x);
    };
    o.resid = [dm](double *r, const double *b, double *x) {
        std::lock_guard<std::mutex> lk(dm->mtx);
        dm->residual0(b, x, r);
    };
    if (precondition) o.M = [dm](double *out, const double *r) { dm->apply(out, r); };
    // the result and its partial sums in a buffer of this solve's own: loopback ranks
    // share one context, and the context's reduction scratch raced between them
    // (the bench's 8-rank rehearsal: rho_0 = 1.0000122)
    auto red = std::make_shared<DevBuf<double>>(1 + VEC_DOT_PARTIALS);
    o.dot = [dm, red](const double *u, const double *w) {
        Ctx &ctx = *dm->ctx;
        hipStream_t s = ctx.stream;
        vec_dot_dev(u, w, dm->nrows, red->get(), red->get() + 1, s);
        dm->tr->allreduce(red->get(), 1, false, s);
        double h = 0;
        FAMG_CHECK_HIP(hipMemcpyAsync(&h, red->get(), 8, hipMemcpyDeviceToHost, s));
        FAMG_CHECK_HIP(hipStreamSynchronize(s));
        return h;
    };
    return o;
}

amg_status amg_dist_stationary_solve(amg_linop *dist_mg, const double *b, double *x, int64_t max_iter,
                                     double rel_tol, double *hist, int64_t *iters) {
    return dguard([&] {
        auto d = need_dist(dist_mg);
        FAMG_REQUIRE(b && x && iters && max_iter > 0, AMG_ERR_INVALID, "bad argument");
        d->ctx->set_device();
        *iters = stationary_impl(dist_ops(d, true), b, x, max_iter, rel_tol, hist);
    });
}

amg_status amg_dist_pcg_solve(amg_linop *dist_mg, int32_t precondition, const double *b, double *x,
                              int64_t max_iter, double rel_tol, double abs_tol, double *hist, int64_t *iters) {
    return dguard([&] {
        auto d = need_dist(dist_mg);
        FAMG_REQUIRE(b && x && iters && max_iter >= 0, AMG_ERR_INVALID, "bad argument");
        d->ctx->set_device();
        *iters = pcg_impl(dist_ops(d, precondition != 0), b, x, max_iter, rel_tol, abs_tol, hist);
    });
}

}  // extern "C"
