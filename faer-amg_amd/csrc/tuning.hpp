// tuning.hpp -- frozen setup-time decisions (tuning.cpp)
#pragma once
#include <cstdint>

namespace famg {

enum TuneSource : int { TUNE_NONE = 0, TUNE_TABLE = 1, TUNE_TIMED = 2, TUNE_ENV = 3, TUNE_RULE = 4 };

struct TileKey {
    int64_t nx, ny, nz;
    int rx, ry, rz, k;
    int64_t ncls;
    bool framed;
};
// the frozen tile of an x-staged stencil-class operator of this shape, if any
bool tune_tile_lookup(const TileKey &k, int *t);
// append the decision to $FAMG_TUNE_LOG (no-op without it)
void tune_tile_record(const TileKey &k, const int *t, int source);

}  // namespace famg
