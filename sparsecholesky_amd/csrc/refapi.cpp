// Host helpers that mirror the rest of the reference API surface:
//   triplet_to_csc_matrix   include/chol.hpp:308-369
//   load_matrix_market_to_csc include/mtx_reader.hpp:16-62 (banner honoured)
//   compute_supernodes / atree  src/chol.cpp:42-136
// plus the deterministic synthetic input of SURVEY.md Appendix B.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "symbolic.hpp"

namespace sc {

i64 triplet_to_csc(i64 n, i64 nt, const i32* ti, const i32* tj, const double* tx, i64* Ap, i32* Ai,
                   double* Ax) {
    struct E {
        i32 r, c;
        double v;
    };
    std::vector<E> e;
    e.reserve((size_t)nt);
    for (i64 k = 0; k < nt; ++k) {
        i32 i = ti[k], j = tj[k];
        if (i < 0 || j < 0 || i >= n || j >= n) return SC_ERR_ARG;
        if (j < i) std::swap(i, j);  // store the upper triangle (chol.hpp:321-322)
        e.push_back({i, j, tx ? tx[k] : 1.0});
    }
    std::stable_sort(e.begin(), e.end(), [](const E& a, const E& b) {
        return a.c != b.c ? a.c < b.c : a.r < b.r;
    });
    std::vector<E> merged;  // sum duplicates (chol.hpp:336-346)
    for (auto& x : e) {
        if (!merged.empty() && merged.back().r == x.r && merged.back().c == x.c)
            merged.back().v += x.v;
        else
            merged.push_back(x);
    }
    if (Ap) {
        std::fill(Ap, Ap + n + 1, 0);
        for (auto& x : merged) Ap[x.c + 1]++;
        for (i64 j = 0; j < n; ++j) Ap[j + 1] += Ap[j];
    }
    if (Ai || Ax) {
        i64 q = 0;
        for (auto& x : merged) {
            if (Ai) Ai[q] = x.r;
            if (Ax) Ax[q] = x.v;
            ++q;
        }
    }
    return (i64)merged.size();
}

// MatrixMarket coordinate reader.  The reference skips '%' lines, reads
// "m n nnz" and swaps every entry to the upper triangle (mtx_reader.hpp:26-52).
// Here the banner "%%MatrixMarket matrix <format> <field> <symmetry>" decides:
//   coordinate only (array: SC_ERR_NOTIMPL); field real / integer / pattern
//   (pattern: value 1; complex: SC_ERR_NOTIMPL);
//   symmetric, hermitian (real field), no symmetry token or no banner -> as the
//     reference (every entry swapped to the upper triangle);
//   general -> the file must hold both triangles of a symmetric matrix: after
//     summing duplicates, every off-diagonal (r, c) must equal (c, r) exactly,
//     else SC_ERR_NOTSYM; only the upper entries are kept (the reference's swap
//     would add each mirror onto its twin and double the off-diagonal);
//   skew-symmetric -> SC_ERR_NOTSYM (zero diagonal: never positive definite).
// Indices out of [1, n], a non-square size or a short file: SC_ERR_ARG; a file that
// cannot be opened: SC_ERR_IO.
i64 read_mtx(const char* path, i64* n_out, i64* Ap, i32* Ai, double* Ax) {
    std::ifstream f(path);
    if (!f) return SC_ERR_IO;
    std::string line;
    bool pattern = false, general = false;
    if (!std::getline(f, line)) return SC_ERR_ARG;
    {
        std::string low = line;
        for (auto& ch : low) ch = (char)std::tolower((unsigned char)ch);
        if (low.rfind("%%matrixmarket", 0) == 0) {
            std::istringstream hs(low);
            std::string tag, object, format, field, symmetry;
            hs >> tag >> object >> format >> field >> symmetry;
            if (object != "matrix") return SC_ERR_ARG;
            if (format == "array") return SC_ERR_NOTIMPL;
            if (format != "coordinate") return SC_ERR_ARG;
            if (field == "complex") return SC_ERR_NOTIMPL;
            if (field == "pattern")
                pattern = true;
            else if (field != "real" && field != "integer" && field != "double")
                return SC_ERR_ARG;
            if (symmetry == "general")
                general = true;
            else if (symmetry == "skew-symmetric")
                return SC_ERR_NOTSYM;
            else if (!symmetry.empty() && symmetry != "symmetric" && symmetry != "hermitian")
                return SC_ERR_ARG;
        } else {
            f.seekg(0);
        }
    }
    while (f.peek() == '%' || f.peek() == '\n') std::getline(f, line);
    i64 nr = 0, nc = 0, nl = 0;
    if (!(f >> nr >> nc >> nl)) return SC_ERR_ARG;
    if (nr != nc || nr < 0 || nl < 0 || nr > INT32_MAX) return SC_ERR_ARG;
    std::vector<i32> ti, tj;
    std::vector<double> tx;
    ti.reserve((size_t)nl);
    tj.reserve((size_t)nl);
    tx.reserve((size_t)nl);
    struct Off {  // general: one off-diagonal entry of the pair {lo, hi}, side = (r > c)
        i32 lo, hi;
        int side;
        double v;
    };
    std::vector<Off> off;
    for (i64 l = 0; l < nl; ++l) {
        i64 r, c;
        double v = 1.0;
        if (!(f >> r >> c)) return SC_ERR_ARG;
        if (!pattern && !(f >> v)) return SC_ERR_ARG;
        if (r < 1 || c < 1 || r > nr || c > nr) return SC_ERR_ARG;
        --r;
        --c;
        if (general && r != c) off.push_back({(i32)std::min(r, c), (i32)std::max(r, c), r > c ? 1 : 0, v});
        if (general && r > c) continue;
        ti.push_back((i32)r);
        tj.push_back((i32)c);
        tx.push_back(v);
    }
    if (general) {
        // per pair, the summed upper side must equal the summed lower side (in input
        // order per side, as triplet_to_csc sums duplicates)
        std::stable_sort(off.begin(), off.end(), [](const Off& a, const Off& b) {
            return a.hi != b.hi ? a.hi < b.hi : a.lo < b.lo;
        });
        for (size_t q = 0; q < off.size();) {
            size_t e = q;
            double sum[2] = {0.0, 0.0};
            bool seen[2] = {false, false};
            while (e < off.size() && off[e].lo == off[q].lo && off[e].hi == off[q].hi) {
                sum[off[e].side] += off[e].v;
                seen[off[e].side] = true;
                ++e;
            }
            if (!seen[0] || !seen[1] || sum[0] != sum[1]) return SC_ERR_NOTSYM;
            q = e;
        }
    }
    *n_out = nr;
    return triplet_to_csc(nr, (i64)ti.size(), ti.data(), tj.data(), tx.data(), Ap, Ai, Ax);
}

// compute_supernodes on the reference pattern, natural order (src/chol.cpp:42-100).
i64 compute_supernodes_ref(i64 n, const i32* parent, const i64* cp, i32* sn_id, i64* supernodes) {
    if (n == 0) {
        if (supernodes) supernodes[0] = 0;
        return 0;
    }
    i64 nsn = 0;
    if (supernodes) supernodes[0] = 0;
    i32 sid = 0;
    if (sn_id) sn_id[0] = 0;
    for (i64 j = 1; j < n; ++j) {
        bool same = false;
        if (parent[j - 1] == j) {
            i64 lenj = cp[j + 1] - cp[j], lenjm1 = cp[j] - cp[j - 1];
            if (lenj == lenjm1 - 1) same = true;
        }
        if (!same) {
            ++sid;
            if (supernodes) supernodes[sid] = j;
        }
        if (sn_id) sn_id[j] = sid;
    }
    nsn = (i64)sid + 1;
    if (supernodes) supernodes[nsn] = n;
    return nsn;
}

// atree (src/chol.cpp:102-136): parent supernode = min sn_id among rows >= end.
i64 atree_ref(i64 n, const i64* Lp, const i32* Li, const i32* sn_id, const i64* supernodes, i64 ns,
              i32* super_parent) {
    (void)n;
    for (i64 s = 0; s < ns; ++s) {
        super_parent[s] = -1;
        const i64 start = supernodes[s], end = supernodes[s + 1];
        for (i64 j = start; j < end; ++j)
            for (i64 p = Lp[j]; p < Lp[j + 1]; ++p) {
                i32 row = Li[p];
                if (row >= end) {
                    i32 t = sn_id[row];
                    if (t != s && (super_parent[s] == -1 || t < super_parent[s])) super_parent[s] = t;
                }
            }
    }
    return SC_OK;
}

// Deterministic geometric nested dissection of a k^3 grid:
// split the longest axis (ties x, then y, then z) at (lo+hi)/2; recurse on the
// low half, then the high half, then emit the separator slab; boxes with max
// extent <= 2 or volume <= 8 are emitted in z, y, x loop order.
static void nd_rec(i64 k, i64 x0, i64 x1, i64 y0, i64 y1, i64 z0, i64 z1, std::vector<i32>& out) {
    struct Box {
        i64 x0, x1, y0, y1, z0, z1;
        int stage;
    };
    std::vector<Box> st;
    st.push_back({x0, x1, y0, y1, z0, z1, 0});
    while (!st.empty()) {
        Box b = st.back();
        st.pop_back();
        const i64 ex = b.x1 - b.x0, ey = b.y1 - b.y0, ez = b.z1 - b.z0;
        if (ex <= 0 || ey <= 0 || ez <= 0) continue;
        const i64 mx = std::max(ex, std::max(ey, ez));
        if (mx <= 2 || ex * ey * ez <= 8) {
            for (i64 z = b.z0; z < b.z1; ++z)
                for (i64 y = b.y0; y < b.y1; ++y)
                    for (i64 x = b.x0; x < b.x1; ++x) out.push_back((i32)((z * k + y) * k + x));
            continue;
        }
        // children pushed in reverse: low, high, separator
        if (ex == mx) {
            i64 m = (b.x0 + b.x1) / 2;
            st.push_back({m, m + 1, b.y0, b.y1, b.z0, b.z1, 0});
            st.push_back({m + 1, b.x1, b.y0, b.y1, b.z0, b.z1, 0});
            st.push_back({b.x0, m, b.y0, b.y1, b.z0, b.z1, 0});
        } else if (ey == mx) {
            i64 m = (b.y0 + b.y1) / 2;
            st.push_back({b.x0, b.x1, m, m + 1, b.z0, b.z1, 0});
            st.push_back({b.x0, b.x1, m + 1, b.y1, b.z0, b.z1, 0});
            st.push_back({b.x0, b.x1, b.y0, m, b.z0, b.z1, 0});
        } else {
            i64 m = (b.z0 + b.z1) / 2;
            st.push_back({b.x0, b.x1, b.y0, b.y1, m, m + 1, 0});
            st.push_back({b.x0, b.x1, b.y0, b.y1, m + 1, b.z1, 0});
            st.push_back({b.x0, b.x1, b.y0, b.y1, b.z0, m, 0});
        }
    }
}

i64 laplacian3d(i64 k, int nd, i64* Ap, i32* Ai, double* Ax, i32* perm_out) {
    if (k <= 0) return SC_ERR_ARG;
    const i64 n = k * k * k;
    std::vector<i32> perm;
    perm.reserve((size_t)n);
    if (nd)
        nd_rec(k, 0, k, 0, k, 0, k, perm);
    else
        for (i64 i = 0; i < n; ++i) perm.push_back((i32)i);
    if ((i64)perm.size() != n) return SC_ERR_ARG;
    std::vector<i32> inew((size_t)n);
    for (i64 q = 0; q < n; ++q) inew[perm[q]] = (i32)q;
    if (perm_out) std::copy(perm.begin(), perm.end(), perm_out);
    const i64 nnz = n + 3 * k * k * (k - 1);
    if (!Ap) return nnz;
    // column j' (new) holds rows i' <= j' of the permuted stencil, ascending.
    i64 q = 0;
    Ap[0] = 0;
    i32 rowsbuf[7];
    for (i64 jn = 0; jn < n; ++jn) {
        const i64 old = perm[jn];
        const i64 x = old % k, y = (old / k) % k, z = old / (k * k);
        int cnt = 0;
        rowsbuf[cnt++] = (i32)jn;
        const i64 nb[6][3] = {{x - 1, y, z}, {x + 1, y, z}, {x, y - 1, z},
                              {x, y + 1, z}, {x, y, z - 1}, {x, y, z + 1}};
        for (auto& v : nb) {
            if (v[0] < 0 || v[0] >= k || v[1] < 0 || v[1] >= k || v[2] < 0 || v[2] >= k) continue;
            i32 in = inew[(v[2] * k + v[1]) * k + v[0]];
            if (in < jn) rowsbuf[cnt++] = in;
        }
        std::sort(rowsbuf, rowsbuf + cnt);
        for (int t = 0; t < cnt; ++t) {
            if (Ai) Ai[q] = rowsbuf[t];
            if (Ax) Ax[q] = (rowsbuf[t] == jn) ? 6.0 : -1.0;
            ++q;
        }
        Ap[jn + 1] = q;
    }
    return q;
}

}  // namespace sc
