// plan.cpp -- host-side distributed planning (plan.hpp) and its C ABI
// (amg_halo_plan_*, amg_dist_first_redundant_level).  No device calls.
#include "plan.hpp"

#include <algorithm>
#include <string>

#include "handles.hpp"

namespace famg {

int HaloPlan::owner(int64_t g) const {
    return int(std::upper_bound(splits.begin(), splits.end(), g) - splits.begin()) - 1;
}

void plan_init(HaloPlan &p, int nranks, int rank, const int64_t *splits) {
    FAMG_REQUIRE(nranks > 0 && rank >= 0 && rank < nranks && splits, AMG_ERR_INVALID, "plan: bad rank/splits");
    FAMG_REQUIRE(splits[0] == 0, AMG_ERR_DIM, "level splits must start at 0");
    for (int q = 0; q < nranks; q++)
        FAMG_REQUIRE(splits[q + 1] >= splits[q], AMG_ERR_INVALID, "splits must be monotone");
    p = HaloPlan{};
    p.nranks = nranks;
    p.rank = rank;
    p.splits.assign(splits, splits + nranks + 1);
    p.n_glob = splits[nranks];
    p.r0 = splits[rank];
    p.r1 = splits[rank + 1];
    p.n_own = p.r1 - p.r0;
}

void plan_add_columns(HaloPlan &p, const int64_t *cols, int64_t nnz) {
    FAMG_REQUIRE(!p.ghosts_final, AMG_ERR_INVALID, "plan: ghost set already final");
    for (int64_t e = 0; e < nnz; e++) {
        const int64_t c = cols[e];
        FAMG_REQUIRE(c >= 0 && c < p.n_glob, AMG_ERR_DIM, "plan: column outside the level");
        if (c < p.r0 || c >= p.r1) p.pending.push_back(c);
    }
}

static void split_requests(HaloPlan &p) {
    const int P = p.nranks;
    p.req_cnt.assign(P, 0);
    p.req_off.assign(P + 1, 0);
    for (int64_t g : p.ghost_ids) p.req_cnt[p.owner(g)]++;
    for (int q = 0; q < P; q++) p.req_off[q + 1] = p.req_off[q] + p.req_cnt[q];
    p.ghosts_final = true;
}

void plan_set_ghosts(HaloPlan &p, std::vector<int64_t> ghost_ids) {
    FAMG_REQUIRE(!p.ghosts_final, AMG_ERR_INVALID, "plan: ghost set already final");
    for (size_t k = 0; k < ghost_ids.size(); k++) {
        const int64_t g = ghost_ids[k];
        FAMG_REQUIRE(g >= 0 && g < p.n_glob && (g < p.r0 || g >= p.r1), AMG_ERR_INVALID, "plan: bad ghost id");
        FAMG_REQUIRE(k == 0 || g > ghost_ids[k - 1], AMG_ERR_INVALID, "plan: ghost ids must be sorted and unique");
    }
    p.ghost_ids = std::move(ghost_ids);
    split_requests(p);
}

void plan_finalize_ghosts(HaloPlan &p) {
    if (p.ghosts_final) return;
    std::sort(p.pending.begin(), p.pending.end());
    p.pending.erase(std::unique(p.pending.begin(), p.pending.end()), p.pending.end());
    p.ghost_ids.swap(p.pending);
    p.pending.clear();
    split_requests(p);
}

void plan_set_incoming(HaloPlan &p, const int64_t *in_cnt, const int64_t *in_ids) {
    FAMG_REQUIRE(p.ghosts_final, AMG_ERR_INVALID, "plan: finalize the ghost set first");
    const int P = p.nranks;
    p.in_cnt.assign(in_cnt, in_cnt + P);
    p.in_cnt[p.rank] = 0;
    FAMG_REQUIRE(in_cnt[p.rank] == 0, AMG_ERR_INVALID, "plan: a rank cannot request from itself");
    p.in_off.assign(P + 1, 0);
    for (int q = 0; q < P; q++) {
        FAMG_REQUIRE(p.in_cnt[q] >= 0, AMG_ERR_INVALID, "plan: negative request count");
        p.in_off[q + 1] = p.in_off[q] + p.in_cnt[q];
    }
    const int64_t nsend = p.in_off[P];
    p.send_idx.resize(nsend);
    for (int64_t k = 0; k < nsend; k++) {
        const int64_t g = in_ids[k];
        FAMG_REQUIRE(g >= p.r0 && g < p.r1, AMG_ERR_INVALID, "halo request for a row not owned");
        p.send_idx[k] = (int32_t)(g - p.r0);
    }
    p.nbr.clear(); p.soff.clear(); p.scnt.clear(); p.roff.clear(); p.rcnt.clear();
    for (int q = 0; q < P; q++) {
        if (q == p.rank || (p.req_cnt[q] == 0 && p.in_cnt[q] == 0)) continue;
        p.nbr.push_back(q);
        p.soff.push_back(p.in_off[q]);
        p.scnt.push_back(p.in_cnt[q]);
        p.roff.push_back(p.req_off[q]);
        p.rcnt.push_back(p.req_cnt[q]);
    }
    p.complete = true;
}

int64_t plan_local_col(const HaloPlan &p, int64_t g) {
    if (g >= p.r0 && g < p.r1) return g - p.r0;
    auto it = std::lower_bound(p.ghost_ids.begin(), p.ghost_ids.end(), g);
    FAMG_REQUIRE(it != p.ghost_ids.end() && *it == g, AMG_ERR_INVALID, "plan: column not in the ghost set");
    return p.n_own + (it - p.ghost_ids.begin());
}

void interior_segment(const uint8_t *flag, int64_t n, int64_t &lo, int64_t &hi) {
    lo = hi = 0;
    for (int64_t i = 0; i < n;) {
        if (flag[i]) { i++; continue; }
        int64_t j = i;
        while (j < n && !flag[j]) j++;
        if (j - i > hi - lo) { lo = i; hi = j; }
        i = j;
    }
    if (hi == lo) lo = hi = n;
}

int64_t first_redundant_level(const int64_t *level_rows, int64_t nlevels, int64_t agglomerate_rows) {
    FAMG_REQUIRE(nlevels > 0, AMG_ERR_INVALID, "no levels");
    for (int64_t l = 0; l < nlevels - 1; l++)
        if (level_rows[l] < agglomerate_rows) return l;
    return nlevels - 1;  // the coarsest level is always redundant
}

}  // namespace famg

using namespace famg;

struct amg_halo_plan {
    HaloPlan p;
};

extern "C" {

amg_status amg_halo_plan_create(int32_t nranks, int32_t rank, const int64_t *splits, amg_halo_plan **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        auto *h = new amg_halo_plan();
        try {
            plan_init(h->p, nranks, rank, splits);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

amg_status amg_halo_plan_destroy(amg_halo_plan *plan) {
    return guard([&] { delete plan; });
}

amg_status amg_halo_plan_add_columns(amg_halo_plan *plan, int64_t nnz, const int64_t *cols) {
    return guard([&] {
        FAMG_REQUIRE(plan && nnz >= 0 && (nnz == 0 || cols), AMG_ERR_INVALID, "bad argument");
        plan_add_columns(plan->p, cols, nnz);
    });
}

amg_status amg_halo_plan_requests(amg_halo_plan *plan, int64_t *req_counts, int64_t *n_ghost) {
    return guard([&] {
        FAMG_REQUIRE(plan, AMG_ERR_INVALID, "null plan");
        plan_finalize_ghosts(plan->p);
        if (req_counts)
            for (int q = 0; q < plan->p.nranks; q++) req_counts[q] = plan->p.req_cnt[q];
        if (n_ghost) *n_ghost = plan->p.n_ghost();
    });
}

amg_status amg_halo_plan_ghost_ids(const amg_halo_plan *plan, int64_t *ids) {
    return guard([&] {
        FAMG_REQUIRE(plan && plan->p.ghosts_final, AMG_ERR_INVALID, "plan: call amg_halo_plan_requests first");
        std::copy(plan->p.ghost_ids.begin(), plan->p.ghost_ids.end(), ids);
    });
}

amg_status amg_halo_plan_set_incoming(amg_halo_plan *plan, const int64_t *in_counts, const int64_t *in_ids) {
    return guard([&] {
        FAMG_REQUIRE(plan && in_counts, AMG_ERR_INVALID, "bad argument");
        plan_set_incoming(plan->p, in_counts, in_ids);
    });
}

amg_status amg_halo_plan_info(const amg_halo_plan *plan, int64_t *info6) {
    return guard([&] {
        FAMG_REQUIRE(plan && info6 && plan->p.complete, AMG_ERR_INVALID, "plan not complete");
        const HaloPlan &p = plan->p;
        int64_t nrecv = 0;
        for (int64_t c : p.rcnt) nrecv += c;
        info6[0] = p.n_own;
        info6[1] = p.n_ghost();
        info6[2] = (int64_t)p.nbr.size();
        info6[3] = (int64_t)p.send_idx.size();
        info6[4] = nrecv;
        info6[5] = p.r0;
    });
}

amg_status amg_halo_plan_neighbors(const amg_halo_plan *plan, int32_t *nbr, int64_t *soff, int64_t *scnt,
                                   int64_t *roff, int64_t *rcnt) {
    return guard([&] {
        FAMG_REQUIRE(plan && plan->p.complete, AMG_ERR_INVALID, "plan not complete");
        const HaloPlan &p = plan->p;
        for (size_t k = 0; k < p.nbr.size(); k++) {
            if (nbr) nbr[k] = p.nbr[k];
            if (soff) soff[k] = p.soff[k];
            if (scnt) scnt[k] = p.scnt[k];
            if (roff) roff[k] = p.roff[k];
            if (rcnt) rcnt[k] = p.rcnt[k];
        }
    });
}

amg_status amg_halo_plan_send_indices(const amg_halo_plan *plan, int32_t *idx) {
    return guard([&] {
        FAMG_REQUIRE(plan && plan->p.complete, AMG_ERR_INVALID, "plan not complete");
        std::copy(plan->p.send_idx.begin(), plan->p.send_idx.end(), idx);
    });
}

amg_status amg_halo_plan_remap(const amg_halo_plan *plan, int64_t nrows, const int64_t *rowptr, const int64_t *cols,
                               int32_t *local_cols, int64_t *lo, int64_t *hi) {
    return guard([&] {
        FAMG_REQUIRE(plan && plan->p.ghosts_final && rowptr && nrows >= 0, AMG_ERR_INVALID, "bad argument");
        const HaloPlan &p = plan->p;
        std::vector<uint8_t> flag(nrows, 0);
        for (int64_t i = 0; i < nrows; i++)
            for (int64_t e = rowptr[i]; e < rowptr[i + 1]; e++) {
                const int64_t c = plan_local_col(p, cols[e]);
                local_cols[e] = (int32_t)c;
                if (c >= p.n_own) flag[i] = 1;
            }
        int64_t l = nrows, h = nrows;
        if (p.n_ghost() > 0) interior_segment(flag.data(), nrows, l, h);
        if (lo) *lo = l;
        if (hi) *hi = h;
    });
}

amg_status amg_dist_first_redundant_level(int64_t nlevels, const int64_t *level_rows, int64_t agglomerate_rows,
                                          int64_t *level) {
    return guard([&] {
        FAMG_REQUIRE(level_rows && level, AMG_ERR_INVALID, "null argument");
        *level = first_redundant_level(level_rows, nlevels, agglomerate_rows);
    });
}

}  // extern "C"
