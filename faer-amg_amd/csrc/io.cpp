// io.cpp -- host-side loaders for real datasets: Matrix
// Market coordinate files and the MFEM linear-system bundle
// (name.mtx / .bdy / .coords / .rhs) of the reference's
// load_mfem_linear_system (utils.rs:269-350).
//
// Semantics restated from the reference:
//  * load_matrix_triplets (utils.rs:508-534; the parser itself is the
//    matrix-market-rs 0.1.3 crate, Cargo.lock:1425-1427, absent here): sparse
//    coordinate files only, 1-based indices, entries equal to 0.0 dropped,
//    `symmetric` files expanded with the mirrored off-diagonal entry;
//  * triplets -> CSR as faer's try_new_from_triplets: duplicates summed (in
//    file order), columns sorted;
//  * boundary deletion (utils.rs:446-480): rows and columns listed in .bdy
//    removed, survivors renumbered in order; .bdy starts with its count
//    (utils.rs:364-395); .coords one row per line (utils.rs:397-415); .rhs a
//    flat column-major list whose length is a multiple of n (utils.rs:300-315).
// The file is memory-mapped and parsed by line-aligned chunks in parallel.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <numeric>
#include <sstream>

#include "handles.hpp"

using namespace famg;

struct amg_mfem_system {
    amg_host_csr A;
    int64_t rhs_cols = 0, coord_dim = 0, original_dim = 0;
    std::vector<double> rhs, coords;      // column-major n x k, n x d
    std::vector<int64_t> boundary;        // sorted, unique (original numbering)
    std::vector<int64_t> selection;       // solution index -> original index
    std::vector<int64_t> mesh_to_solution;  // original index -> solution index or -1
};

namespace {

struct Triplet {
    int64_t r, c;
    double v;
};

struct MappedFile {
    const char *p = nullptr;
    size_t n = 0;
    int fd = -1;
    explicit MappedFile(const std::string &path) {
        fd = open(path.c_str(), O_RDONLY);
        FAMG_REQUIRE(fd >= 0, AMG_ERR_INVALID, "cannot open " + path);
        struct stat st;
        fstat(fd, &st);
        n = (size_t)st.st_size;
        if (n) {
            void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            FAMG_REQUIRE(m != MAP_FAILED, AMG_ERR_INVALID, "cannot map " + path);
            p = static_cast<const char *>(m);
        }
    }
    ~MappedFile() {
        if (p) munmap(const_cast<char *>(p), n);
        if (fd >= 0) close(fd);
    }
};

std::string lower(std::string s) {
    for (auto &ch : s) ch = (char)std::tolower((unsigned char)ch);
    return s;
}

// Parse "i j [v]" lines of [b, e) (b at a line start) into out; '%' lines skipped.
void parse_entries(const char *b, const char *e, bool pattern, std::vector<Triplet> &out, bool &bad) {
    const char *q = b;
    while (q < e) {
        const char *eol = static_cast<const char *>(memchr(q, '\n', e - q));
        if (!eol) eol = e;
        const char *s = q;
        while (s < eol && (*s == ' ' || *s == '\t' || *s == '\r')) s++;
        if (s < eol && *s != '%') {
            char *end = nullptr;
            const long long i = strtoll(s, &end, 10);
            if (end == s) bad = true;
            const char *t = end;
            const long long j = strtoll(t, &end, 10);
            double v = 1.0;
            if (end == t) bad = true;
            if (!pattern) {
                t = end;
                v = strtod(t, &end);
                if (end == t) bad = true;
            }
            out.push_back({(int64_t)i - 1, (int64_t)j - 1, v});
        }
        q = eol + 1;
    }
}

// Triplets -> sorted CSR with duplicates summed in input order.
void to_csr(int64_t nrows, int64_t ncols, std::vector<Triplet> &t, amg_host_csr &out) {
    for (const Triplet &x : t)
        FAMG_REQUIRE(x.r >= 0 && x.r < nrows && x.c >= 0 && x.c < ncols, AMG_ERR_INVALID,
                     "matrix entry index out of range");
    std::vector<int64_t> cnt(nrows + 1, 0);
    for (const Triplet &x : t) cnt[x.r + 1]++;
    for (int64_t r = 0; r < nrows; r++) cnt[r + 1] += cnt[r];
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    std::vector<int64_t> c(t.size());
    std::vector<double> v(t.size());
    for (const Triplet &x : t) {  // row bucket, file order kept
        c[pos[x.r]] = x.c;
        v[pos[x.r]] = x.v;
        pos[x.r]++;
    }
    std::vector<Triplet>().swap(t);
    out.nrows = nrows;
    out.ncols = ncols;
    out.rp.assign(nrows + 1, 0);
    std::vector<int64_t> rowlen(nrows, 0);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t r = 0; r < nrows; r++) {
        const int64_t b = cnt[r], e = cnt[r + 1];
        std::vector<int64_t> idx(e - b);
        std::iota(idx.begin(), idx.end(), b);
        std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return c[x] < c[y]; });
        // compact in place into [b, b + len)
        std::vector<int64_t> cc;
        std::vector<double> vv;
        cc.reserve(e - b);
        vv.reserve(e - b);
        for (int64_t k : idx) {
            if (!cc.empty() && cc.back() == c[k]) vv.back() += v[k];
            else { cc.push_back(c[k]); vv.push_back(v[k]); }
        }
        std::copy(cc.begin(), cc.end(), c.begin() + b);
        std::copy(vv.begin(), vv.end(), v.begin() + b);
        rowlen[r] = (int64_t)cc.size();
    }
    for (int64_t r = 0; r < nrows; r++) out.rp[r + 1] = out.rp[r] + rowlen[r];
    out.ci.resize(out.rp[nrows]);
    out.va.resize(out.rp[nrows]);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; r++) {
        std::copy(c.begin() + cnt[r], c.begin() + cnt[r] + rowlen[r], out.ci.begin() + out.rp[r]);
        std::copy(v.begin() + cnt[r], v.begin() + cnt[r] + rowlen[r], out.va.begin() + out.rp[r]);
    }
}

// utils.rs:508-534 (+ the crate's coordinate parser): triplets with zeros dropped
// and symmetric entries mirrored.
void read_mtx_triplets(const std::string &path, int64_t &nrows, int64_t &ncols, std::vector<Triplet> &out) {
    MappedFile f(path);
    const char *p = f.p, *end = f.p + f.n;
    FAMG_REQUIRE(p && f.n > 0, AMG_ERR_INVALID, "empty Matrix Market file " + path);
    const char *eol = static_cast<const char *>(memchr(p, '\n', end - p));
    if (!eol) eol = end;
    std::istringstream hs(lower(std::string(p, eol)));
    std::string banner, object, format, field, symmetry;
    hs >> banner >> object >> format >> field >> symmetry;
    FAMG_REQUIRE(banner == "%%matrixmarket" && object == "matrix", AMG_ERR_INVALID,
                 "not a Matrix Market matrix file: " + path);
    FAMG_REQUIRE(format == "coordinate", AMG_ERR_UNSUPPORTED, "only sparse (coordinate) Matrix Market files are supported");
    FAMG_REQUIRE(field == "real" || field == "integer" || field == "double" || field == "pattern", AMG_ERR_UNSUPPORTED,
                 "unsupported Matrix Market field '" + field + "'");
    FAMG_REQUIRE(symmetry == "general" || symmetry == "symmetric", AMG_ERR_UNSUPPORTED,
                 "unsupported Matrix Market symmetry '" + symmetry + "'");
    const bool pattern = field == "pattern", sym = symmetry == "symmetric";
    // comments, then the size line
    p = eol + 1;
    int64_t nnz = -1;
    while (p < end) {
        eol = static_cast<const char *>(memchr(p, '\n', end - p));
        if (!eol) eol = end;
        std::string line(p, eol);
        p = eol + 1;
        const size_t k = line.find_first_not_of(" \t\r");
        if (k == std::string::npos || line[k] == '%') continue;
        std::istringstream ls(line);
        long long m = -1, n = -1, z = -1;
        ls >> m >> n >> z;
        FAMG_REQUIRE(m >= 0 && n >= 0 && z >= 0, AMG_ERR_INVALID, "bad Matrix Market size line");
        nrows = m;
        ncols = n;
        nnz = z;
        break;
    }
    FAMG_REQUIRE(nnz >= 0, AMG_ERR_INVALID, "Matrix Market file has no size line");
    // entries: line-aligned chunks parsed in parallel
    const char *body = std::min(p, end);
    const size_t len = end - body;
    const int nch = (int)std::max<size_t>(1, std::min<size_t>(256, len >> 20));
    std::vector<const char *> cut(nch + 1);
    cut[0] = body;
    cut[nch] = end;
    for (int k = 1; k < nch; k++) {
        const char *c = body + len * k / nch;
        const char *nl = static_cast<const char *>(memchr(c, '\n', end - c));
        cut[k] = nl ? nl + 1 : end;
        if (cut[k] < cut[k - 1]) cut[k] = cut[k - 1];
    }
    std::vector<std::vector<Triplet>> parts(nch);
    std::vector<char> badp(nch, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int k = 0; k < nch; k++) {
        bool bad = false;
        parse_entries(cut[k], cut[k + 1], pattern, parts[k], bad);
        badp[k] = bad;
    }
    int64_t total = 0;
    for (int k = 0; k < nch; k++) {
        FAMG_REQUIRE(!badp[k], AMG_ERR_INVALID, "malformed Matrix Market entry line");
        total += (int64_t)parts[k].size();
    }
    FAMG_REQUIRE(total == nnz, AMG_ERR_INVALID,
                 "Matrix Market entry count " + std::to_string(total) + " != header " + std::to_string(nnz));
    out.clear();
    out.reserve(sym ? 2 * total : total);
    for (auto &part : parts) {
        for (const Triplet &x : part) {
            if (x.v == 0.0) continue;
            out.push_back(x);
            if (sym && x.r != x.c) out.push_back({x.c, x.r, x.v});
        }
        std::vector<Triplet>().swap(part);
    }
}

std::string path_with_ext(const std::string &dir, const std::string &name, const char *ext) {
    std::string base = dir.empty() ? name : (dir.back() == '/' ? dir + name : dir + "/" + name);
    std::ifstream f(base + "." + ext);
    FAMG_REQUIRE(f.good(), AMG_ERR_INVALID, "Expected file " + base + "." + ext);
    return base + "." + ext;
}

std::vector<std::vector<double>> read_dense_rows(const std::string &path) {
    std::ifstream f(path);
    std::vector<std::vector<double>> rows;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ls(line);
        std::vector<double> r;
        std::string tok;
        while (ls >> tok) {
            char *e = nullptr;
            const double v = strtod(tok.c_str(), &e);
            FAMG_REQUIRE(e && *e == 0, AMG_ERR_INVALID, "bad number '" + tok + "' in " + path);
            r.push_back(v);
        }
        if (!r.empty()) rows.push_back(std::move(r));
    }
    return rows;
}

amg_host_csr &need_host(const amg_host_csr *h) {
    FAMG_REQUIRE(h, AMG_ERR_INVALID, "null host CSR");
    return *const_cast<amg_host_csr *>(h);
}

amg_mfem_system &need_sys(const amg_mfem_system *s) {
    FAMG_REQUIRE(s, AMG_ERR_INVALID, "null MFEM system");
    return *const_cast<amg_mfem_system *>(s);
}

}  // namespace

extern "C" {

amg_status amg_mtx_read(const char *path, amg_host_csr **out) {
    return guard([&] {
        FAMG_REQUIRE(path && out, AMG_ERR_INVALID, "null argument");
        auto h = std::make_unique<amg_host_csr>();
        int64_t m = 0, n = 0;
        std::vector<Triplet> t;
        read_mtx_triplets(path, m, n, t);
        to_csr(m, n, t, *h);
        *out = h.release();
    });
}

amg_status amg_host_csr_create(int64_t nrows, int64_t ncols, const int64_t *rowptr, const int64_t *colidx,
                               const double *vals, amg_host_csr **out) {
    return guard([&] {
        FAMG_REQUIRE(out && rowptr && nrows >= 0 && ncols >= 0 && rowptr[0] == 0, AMG_ERR_INVALID, "bad argument");
        const int64_t nnz = rowptr[nrows];
        FAMG_REQUIRE(nnz == 0 || (colidx && vals), AMG_ERR_INVALID, "null column/value array");
        auto h = std::make_unique<amg_host_csr>();
        h->nrows = nrows;
        h->ncols = ncols;
        h->rp.assign(rowptr, rowptr + nrows + 1);
        h->ci.assign(colidx, colidx + nnz);
        h->va.assign(vals, vals + nnz);
        for (int64_t i = 0; i < nrows; i++) {
            FAMG_REQUIRE(h->rp[i + 1] >= h->rp[i], AMG_ERR_INVALID, "rowptr not monotone");
            for (int64_t e = h->rp[i]; e < h->rp[i + 1]; e++)
                FAMG_REQUIRE(h->ci[e] >= 0 && h->ci[e] < ncols, AMG_ERR_INVALID, "column index out of range");
        }
        *out = h.release();
    });
}

amg_status amg_host_csr_dims(const amg_host_csr *h, int64_t *nrows, int64_t *ncols, int64_t *nnz) {
    return guard([&] {
        const amg_host_csr &a = need_host(h);
        if (nrows) *nrows = a.nrows;
        if (ncols) *ncols = a.ncols;
        if (nnz) *nnz = (int64_t)a.ci.size();
    });
}

amg_status amg_host_csr_arrays(const amg_host_csr *h, int64_t *rowptr, int64_t *colidx, double *vals) {
    return guard([&] {
        const amg_host_csr &a = need_host(h);
        FAMG_REQUIRE(rowptr && (a.ci.empty() || (colidx && vals)), AMG_ERR_INVALID, "null array");
        std::copy(a.rp.begin(), a.rp.end(), rowptr);
        std::copy(a.ci.begin(), a.ci.end(), colidx);
        std::copy(a.va.begin(), a.va.end(), vals);
    });
}

amg_status amg_host_csr_upload(amg_ctx *ctx, const amg_host_csr *h, amg_linop **out) {
    if (!h) return set_last_error(AMG_ERR_INVALID, "null host CSR");
    return amg_csr_create(ctx, h->nrows, h->ncols, h->rp.data(), h->ci.data(), h->va.data(), out);
}

amg_status amg_host_csr_destroy(amg_host_csr *h) {
    return guard([&] { delete h; });
}

amg_status amg_mfem_load(const char *dir, const char *name, int32_t delete_boundary, amg_mfem_system **out) {
    return guard([&] {
        FAMG_REQUIRE(dir && name && out, AMG_ERR_INVALID, "null argument");
        const std::string mtx = path_with_ext(dir, name, "mtx"), bdy = path_with_ext(dir, name, "bdy"),
                          crd = path_with_ext(dir, name, "coords"), rhs = path_with_ext(dir, name, "rhs");
        auto s = std::make_unique<amg_mfem_system>();
        // boundary list: count line, then one index per non-empty line
        {
            std::ifstream f(bdy);
            std::string line;
            FAMG_REQUIRE((bool)std::getline(f, line), AMG_ERR_INVALID, "Boundary file " + bdy + " is empty");
            const long long expect = std::stoll(line);
            while (std::getline(f, line)) {
                const size_t k = line.find_first_not_of(" \t\r");
                if (k == std::string::npos) continue;
                s->boundary.push_back(std::stoll(line));
            }
            FAMG_REQUIRE((long long)s->boundary.size() == expect, AMG_ERR_INVALID,
                         "Boundary file " + bdy + " expected " + std::to_string(expect) + " entries but found " +
                             std::to_string(s->boundary.size()));
            std::sort(s->boundary.begin(), s->boundary.end());
            s->boundary.erase(std::unique(s->boundary.begin(), s->boundary.end()), s->boundary.end());
        }
        int64_t n = 0, nc = 0;
        std::vector<Triplet> t;
        read_mtx_triplets(mtx, n, nc, t);
        FAMG_REQUIRE(n == nc, AMG_ERR_DIM, "The MFEM loader currently supports only square matrices");
        auto crows = read_dense_rows(crd);
        FAMG_REQUIRE((int64_t)crows.size() == n, AMG_ERR_DIM,
                     "Coordinate rows (" + std::to_string(crows.size()) + ") must match matrix dimension (" +
                         std::to_string(n) + ")");
        std::vector<double> flat;
        {
            std::ifstream f(rhs);
            std::string tok;
            while (f >> tok) {
                char *e = nullptr;
                flat.push_back(strtod(tok.c_str(), &e));
                FAMG_REQUIRE(e && *e == 0, AMG_ERR_INVALID, "bad number '" + tok + "' in " + rhs);
            }
        }
        FAMG_REQUIRE(n > 0 && flat.size() % n == 0, AMG_ERR_DIM,
                     "RHS length (" + std::to_string(flat.size()) + ") must be a multiple of the matrix dimension (" +
                         std::to_string(n) + ")");
        s->original_dim = n;
        s->rhs_cols = (int64_t)flat.size() / n;
        // selection / renumbering (utils.rs:446-480)
        std::vector<char> is_b(n, 0);
        if (delete_boundary) {
            for (int64_t b : s->boundary) {
                FAMG_REQUIRE(b >= 0 && b < n, AMG_ERR_INVALID,
                             "Boundary index " + std::to_string(b) + " out of range for matrix of size " +
                                 std::to_string(n));
                is_b[b] = 1;
            }
        }
        s->mesh_to_solution.assign(n, -1);
        for (int64_t i = 0; i < n; i++)
            if (!is_b[i]) {
                s->mesh_to_solution[i] = (int64_t)s->selection.size();
                s->selection.push_back(i);
            }
        const int64_t m = (int64_t)s->selection.size();
        if (delete_boundary) {
            size_t w = 0;
            for (const Triplet &x : t) {
                const int64_t r = s->mesh_to_solution[x.r], c = s->mesh_to_solution[x.c];
                if (r >= 0 && c >= 0) t[w++] = {r, c, x.v};
            }
            t.resize(w);
        }
        to_csr(m, m, t, s->A);
        // dense rows of the selection (utils.rs:482-506)
        s->coord_dim = m ? (int64_t)crows[s->selection[0]].size() : 0;
        s->coords.resize(m * s->coord_dim);
        for (int64_t i = 0; i < m; i++) {
            const auto &r = crows[s->selection[i]];
            FAMG_REQUIRE((int64_t)r.size() == s->coord_dim, AMG_ERR_INVALID, "Inconsistent column counts in dense data");
            for (int64_t j = 0; j < s->coord_dim; j++) s->coords[j * m + i] = r[j];
        }
        s->rhs.resize(m * s->rhs_cols);
        for (int64_t j = 0; j < s->rhs_cols; j++)
            for (int64_t i = 0; i < m; i++) s->rhs[j * m + i] = flat[j * n + s->selection[i]];
        *out = s.release();
    });
}

amg_status amg_mfem_info(const amg_mfem_system *sys, int64_t *info5) {
    return guard([&] {
        const amg_mfem_system &s = need_sys(sys);
        FAMG_REQUIRE(info5, AMG_ERR_INVALID, "null output");
        info5[0] = s.A.nrows;
        info5[1] = s.rhs_cols;
        info5[2] = s.coord_dim;
        info5[3] = s.original_dim;
        info5[4] = (int64_t)s.boundary.size();
    });
}

amg_status amg_mfem_matrix(const amg_mfem_system *sys, const amg_host_csr **out) {
    return guard([&] {
        FAMG_REQUIRE(out, AMG_ERR_INVALID, "null output");
        *out = &need_sys(sys).A;
    });
}

amg_status amg_mfem_rhs(const amg_mfem_system *sys, double *out, int64_t ld) {
    return guard([&] {
        const amg_mfem_system &s = need_sys(sys);
        const int64_t m = s.A.nrows;
        FAMG_REQUIRE(out && ld >= m, AMG_ERR_INVALID, "bad output");
        for (int64_t j = 0; j < s.rhs_cols; j++) std::copy_n(s.rhs.data() + j * m, m, out + j * ld);
    });
}

amg_status amg_mfem_coords(const amg_mfem_system *sys, double *out, int64_t ld) {
    return guard([&] {
        const amg_mfem_system &s = need_sys(sys);
        const int64_t m = s.A.nrows;
        FAMG_REQUIRE(out && ld >= m, AMG_ERR_INVALID, "bad output");
        for (int64_t j = 0; j < s.coord_dim; j++) std::copy_n(s.coords.data() + j * m, m, out + j * ld);
    });
}

amg_status amg_mfem_boundary(const amg_mfem_system *sys, int64_t *out) {
    return guard([&] {
        const amg_mfem_system &s = need_sys(sys);
        FAMG_REQUIRE(out || s.boundary.empty(), AMG_ERR_INVALID, "null output");
        std::copy(s.boundary.begin(), s.boundary.end(), out);
    });
}

amg_status amg_mfem_index_maps(const amg_mfem_system *sys, int64_t *solution_to_mesh, int64_t *mesh_to_solution) {
    return guard([&] {
        const amg_mfem_system &s = need_sys(sys);
        if (solution_to_mesh) std::copy(s.selection.begin(), s.selection.end(), solution_to_mesh);
        if (mesh_to_solution) std::copy(s.mesh_to_solution.begin(), s.mesh_to_solution.end(), mesh_to_solution);
    });
}

amg_status amg_mfem_destroy(amg_mfem_system *sys) {
    return guard([&] { delete sys; });
}

}  // extern "C"
