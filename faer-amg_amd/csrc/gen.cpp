// gen.cpp -- host generator of the in-tree stand-in for config C5
// (SuiteSparse Flan_1565: 3-D steel flange, hexahedral elasticity, block size
// 3; the file cannot be fetched here).
//
// Trilinear (Q1) hexahedral linear elasticity on an ex x ey x ez element box,
// isotropic material with a per-element Young's modulus E_e = 10^(c (2u_e - 1))
// (u_e from splitmix64(seed, e), so the operator has as many distinct values as
// elements), Poisson ratio nu, the nodes of the x = 0 face clamped (their rows
// and columns removed), and the free nodes optionally renumbered by a seeded
// random permutation (permute = 1: over all nodes; permute = W >= 2: within
// consecutive windows of W nodes, the locality of a mesh numbering) so the
// sparsity pattern has no stencil structure.  Dofs
// are interleaved per node (3p + c), the reference's block_size = 3 layout.
// Element matrices: 2x2x2 Gauss quadrature of B^T D B on the unit cube;
// assembly sums element contributions in ascending element order.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "handles.hpp"

using namespace famg;

namespace {

uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double unit(uint64_t seed, uint64_t i) { return (double)(splitmix64(seed + i * 0x9E3779B97F4A7C15ull) >> 11) * 0x1.0p-53; }

// 24 x 24 Q1 stiffness of the unit cube for E = 1 (row-major)
void q1_reference_stiffness(double nu, double *K) {
    const double lam = nu / ((1.0 + nu) * (1.0 - 2.0 * nu)), mu = 1.0 / (2.0 * (1.0 + nu));
    double D[6][6] = {};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) D[i][j] = lam + (i == j ? 2.0 * mu : 0.0);
    for (int i = 3; i < 6; i++) D[i][i] = mu;
    std::memset(K, 0, 24 * 24 * sizeof(double));
    const double g = 1.0 / std::sqrt(3.0);
    const double detJ = 0.125;  // (h/2)^3, h = 1
    for (int gz = 0; gz < 2; gz++)
        for (int gy = 0; gy < 2; gy++)
            for (int gx = 0; gx < 2; gx++) {
                const double xi = gx ? g : -g, et = gy ? g : -g, ze = gz ? g : -g;
                double B[6][24] = {};
                for (int a = 0; a < 8; a++) {
                    const double sa = (a & 1) ? 1.0 : -1.0, ta = (a & 2) ? 1.0 : -1.0, ua = (a & 4) ? 1.0 : -1.0;
                    // dN/dx = dN/dxi * 2/h
                    const double dx = 0.125 * sa * (1 + et * ta) * (1 + ze * ua) * 2.0;
                    const double dy = 0.125 * ta * (1 + xi * sa) * (1 + ze * ua) * 2.0;
                    const double dz = 0.125 * ua * (1 + xi * sa) * (1 + et * ta) * 2.0;
                    B[0][3 * a] = dx;
                    B[1][3 * a + 1] = dy;
                    B[2][3 * a + 2] = dz;
                    B[3][3 * a] = dy; B[3][3 * a + 1] = dx;
                    B[4][3 * a + 1] = dz; B[4][3 * a + 2] = dy;
                    B[5][3 * a] = dz; B[5][3 * a + 2] = dx;
                }
                double DB[6][24];
                for (int p = 0; p < 6; p++)
                    for (int j = 0; j < 24; j++) {
                        double t = 0.0;
                        for (int q = 0; q < 6; q++) t += D[p][q] * B[q][j];
                        DB[p][j] = t;
                    }
                for (int i = 0; i < 24; i++)
                    for (int j = 0; j < 24; j++) {
                        double t = 0.0;
                        for (int p = 0; p < 6; p++) t += B[p][i] * DB[p][j];
                        K[i * 24 + j] += t * detJ;
                    }
            }
}

}  // namespace

extern "C" amg_status amg_gen_elasticity_q1(int64_t ex, int64_t ey, int64_t ez, double contrast, double nu,
                                            uint64_t seed, int32_t permute, amg_host_csr **out) {
    return guard([&] {
        FAMG_REQUIRE(out && ex >= 1 && ey >= 1 && ez >= 1, AMG_ERR_INVALID, "element counts must be positive");
        FAMG_REQUIRE(nu > -1.0 && nu < 0.5, AMG_ERR_INVALID, "Poisson ratio must lie in (-1, 0.5)");
        const int64_t nx = ex + 1, ny = ey + 1, nz = ez + 1;
        const int64_t nfree = (nx - 1) * ny * nz;
        FAMG_REQUIRE(3 * nfree < (int64_t(1) << 31), AMG_ERR_UNSUPPORTED, "too many dofs for 32-bit indices");
        // free node numbering: mesh node (x>0) -> id
        std::vector<int64_t> id(nx * ny * nz, -1);
        {
            int64_t k = 0;
            for (int64_t z = 0; z < nz; z++)
                for (int64_t y = 0; y < ny; y++)
                    for (int64_t x = 1; x < nx; x++) id[x + nx * (y + ny * z)] = k++;
            if (permute) {  // Fisher-Yates on the ids (within windows), splitmix64 stream
                const int64_t W = permute == 1 ? nfree : permute;
                std::vector<int64_t> perm(nfree);
                for (int64_t i = 0; i < nfree; i++) perm[i] = i;
                for (int64_t w0 = 0; w0 < nfree; w0 += W) {
                    const int64_t m = std::min<int64_t>(W, nfree - w0);
                    for (int64_t i = m - 1; i > 0; i--) {
                        const uint64_t r =
                            splitmix64(seed ^ 0xA5A5A5A5ull) ^ splitmix64(seed + 7 * (uint64_t)(w0 + i));
                        const int64_t j = (int64_t)(r % (uint64_t)(i + 1));
                        std::swap(perm[w0 + i], perm[w0 + j]);
                    }
                }
                for (auto &v : id)
                    if (v >= 0) v = perm[v];
            }
        }
        // node graph: free neighbours within +-1 in every index, sorted by id
        std::vector<int64_t> nrp(nfree + 1, 0);
        std::vector<int64_t> mesh_of(nfree);
        for (int64_t g = 0; g < nx * ny * nz; g++)
            if (id[g] >= 0) mesh_of[id[g]] = g;
#pragma omp parallel for schedule(static)
        for (int64_t p = 0; p < nfree; p++) {
            const int64_t g = mesh_of[p], x = g % nx, y = (g / nx) % ny, z = g / (nx * ny);
            int64_t c = 0;
            for (int64_t dz = -1; dz <= 1; dz++)
                for (int64_t dy = -1; dy <= 1; dy++)
                    for (int64_t dx = -1; dx <= 1; dx++) {
                        const int64_t xx = x + dx, yy = y + dy, zz = z + dz;
                        if (xx < 1 || yy < 0 || zz < 0 || xx >= nx || yy >= ny || zz >= nz) continue;
                        c++;
                    }
            nrp[p + 1] = c;
        }
        for (int64_t p = 0; p < nfree; p++) nrp[p + 1] += nrp[p];
        std::vector<int64_t> ncol(nrp[nfree]);
#pragma omp parallel for schedule(static)
        for (int64_t p = 0; p < nfree; p++) {
            const int64_t g = mesh_of[p], x = g % nx, y = (g / nx) % ny, z = g / (nx * ny);
            int64_t o = nrp[p];
            for (int64_t dz = -1; dz <= 1; dz++)
                for (int64_t dy = -1; dy <= 1; dy++)
                    for (int64_t dx = -1; dx <= 1; dx++) {
                        const int64_t xx = x + dx, yy = y + dy, zz = z + dz;
                        if (xx < 1 || yy < 0 || zz < 0 || xx >= nx || yy >= ny || zz >= nz) continue;
                        ncol[o++] = id[xx + nx * (yy + ny * zz)];
                    }
            std::sort(ncol.begin() + nrp[p], ncol.begin() + nrp[p + 1]);
        }
        const int64_t n = 3 * nfree, nnz = 9 * nrp[nfree];
        auto *h = new amg_host_csr;
        std::unique_ptr<amg_host_csr> hold(h);
        h->nrows = h->ncols = n;
        h->rp.resize(n + 1);
        h->ci.resize(nnz);
        h->va.assign(nnz, 0.0);
#pragma omp parallel for schedule(static)
        for (int64_t p = 0; p < nfree; p++) {
            const int64_t deg = nrp[p + 1] - nrp[p];
            for (int64_t c = 0; c < 3; c++) {
                const int64_t r = 3 * p + c, start = 9 * nrp[p] + c * 3 * deg;
                h->rp[r] = start;
                for (int64_t q = 0; q < deg; q++)
                    for (int64_t d = 0; d < 3; d++) h->ci[start + 3 * q + d] = 3 * ncol[nrp[p] + q] + d;
            }
        }
        h->rp[n] = nnz;
        double K[24 * 24];
        q1_reference_stiffness(nu, K);
        // elements in ascending order; each entry sums its contributions in that order
        for (int64_t z = 0; z < ez; z++)
            for (int64_t y = 0; y < ey; y++)
                for (int64_t x = 0; x < ex; x++) {
                    const int64_t e = x + ex * (y + ey * z);
                    const double E = std::pow(10.0, contrast * (2.0 * unit(seed, (uint64_t)e) - 1.0));
                    int64_t node[8];
                    for (int a = 0; a < 8; a++)
                        node[a] = id[(x + (a & 1)) + nx * ((y + ((a >> 1) & 1)) + ny * (z + ((a >> 2) & 1)))];
                    for (int a = 0; a < 8; a++) {
                        const int64_t pa = node[a];
                        if (pa < 0) continue;
                        const int64_t deg = nrp[pa + 1] - nrp[pa];
                        for (int b = 0; b < 8; b++) {
                            const int64_t pb = node[b];
                            if (pb < 0) continue;
                            const int64_t q = std::lower_bound(ncol.begin() + nrp[pa], ncol.begin() + nrp[pa + 1], pb) -
                                              (ncol.begin() + nrp[pa]);
                            for (int c = 0; c < 3; c++) {
                                double *row = h->va.data() + 9 * nrp[pa] + c * 3 * deg + 3 * q;
                                for (int d = 0; d < 3; d++) row[d] += E * K[(3 * a + c) * 24 + 3 * b + d];
                            }
                        }
                    }
                }
        *out = hold.release();
    });
}
