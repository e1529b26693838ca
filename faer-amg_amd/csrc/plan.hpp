// plan.hpp -- host-side planning of the row-block distributed V-cycle.
//
// Everything here is plain C++ on host arrays: no device, no transport.  The
// distributed multigrid (dist.hip) builds its halo plans, interior segments and
// agglomeration level with these functions (the bulk ghost marking and column
// renumbering of large levels run as device kernels that follow the same
// rules), and the C ABI exports them (amg_halo_plan_*) so a multi-process CPU
// test can run the library's own planner over gloo (tests/test_dist_gloo.py).
//
// The reference has no distributed backend (rayon only);
// the rules below are this build's:
//  * rank p owns rows [splits[p], splits[p+1]) of a level;
//  * a level's vector space on rank p is [owned | ghost], ghosts sorted by
//    global id (hence grouped by owner rank), the ghost set being the union of
//    the off-rank columns referenced by the rank's rows of A_l, R_l (fine
//    columns) and P_{l-1} (coarse columns);
//  * each rank sends each owner the ids it needs once at setup; a refresh packs
//    the requested owned entries per requesting rank (send_idx) and receives
//    straight into the ghost region (offsets roff/rcnt);
//  * [lo, hi) is the longest run of local rows reading owned columns only (it
//    can run while the halo is in flight);
//  * levels from the first one with fewer than `agglomerate_rows` rows down
//    (and always the coarsest) are gathered and cycled redundantly.
#pragma once

#include <cstdint>
#include <vector>

namespace famg {

struct HaloPlan {
    int nranks = 1, rank = 0;
    std::vector<int64_t> splits;  // nranks + 1
    int64_t n_glob = 0, r0 = 0, r1 = 0, n_own = 0;
    std::vector<int64_t> pending;    // off-rank columns added, not yet deduplicated
    std::vector<int64_t> ghost_ids;  // sorted, unique
    bool ghosts_final = false, complete = false;
    std::vector<int64_t> req_cnt, req_off;  // ids requested from each owner: ghost_ids[req_off[q] + k]
    std::vector<int64_t> in_cnt, in_off;    // ids requested by each rank (its send list)
    std::vector<int32_t> send_idx;          // local owned indices, grouped by requesting rank
    // neighbours in rank order (a rank we send to or receive from)
    std::vector<int> nbr;
    std::vector<int64_t> soff, scnt, roff, rcnt;
    int owner(int64_t g) const;
    int64_t n_ghost() const { return (int64_t)ghost_ids.size(); }
};

// Validate splits (monotone, splits[0] = 0) and set the rank's range.
void plan_init(HaloPlan &p, int nranks, int rank, const int64_t *splits);
// Columns (global ids) referenced by a local matrix's rows; off-rank ones join the ghost set.
void plan_add_columns(HaloPlan &p, const int64_t *cols, int64_t nnz);
// The ghost set as computed elsewhere (the device path): sorted, unique, off-rank.
void plan_set_ghosts(HaloPlan &p, std::vector<int64_t> ghost_ids);
// Deduplicate the added columns (if not set directly) and split the requests by owner.
void plan_finalize_ghosts(HaloPlan &p);
// The requests every other rank sent us (counts per rank, ids concatenated in
// rank order): send lists and the neighbour table.
void plan_set_incoming(HaloPlan &p, const int64_t *in_cnt, const int64_t *in_ids);
// Local column of a global id: owned -> g - r0, ghost -> n_own + rank in ghost_ids.
int64_t plan_local_col(const HaloPlan &p, int64_t g);
// [lo, hi): the longest run of rows whose flag (reads a ghost entry) is 0;
// lo = hi = n when there is none.
void interior_segment(const uint8_t *flag, int64_t n, int64_t &lo, int64_t &hi);
// First level run redundantly: the first l < nlevels-1 with rows[l] < agglomerate_rows, else nlevels-1.
int64_t first_redundant_level(const int64_t *level_rows, int64_t nlevels, int64_t agglomerate_rows);

}  // namespace famg
