// Host symbolic analysis -- see symbolic.hpp for the reference map.
#include "symbolic.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace sc {

// Liu's elimination tree with ancestor path compression (chol.hpp:377-410).
void etree(i64 n, const i64* Ap, const i32* Ai, i32* parent) {
    std::vector<i32> ancestor((size_t)n, -1);
    for (i64 k = 0; k < n; k++) {
        parent[k] = -1;
        for (i64 p = Ap[k]; p < Ap[k + 1]; p++) {
            i32 i = Ai[p];
            if (i > k) continue;  // upper triangle only
            while (i != -1 && i < k) {
                i32 inext = ancestor[i];
                ancestor[i] = (i32)k;
                if (inext == -1) {
                    parent[i] = (i32)k;
                    break;
                }
                i = inext;
            }
        }
    }
}

// Postorder with children visited in CSparse order (chol.hpp:445-499).
void post_order(i64 n, const i32* parent, i32* post) {
    std::vector<i32> head((size_t)n, -1), next((size_t)n, -1), stack((size_t)n + 1, -1);
    for (i64 j = n - 1; j >= 0; --j) {
        i32 p = parent[j];
        if (p == -1) continue;
        next[j] = head[p];
        head[p] = (i32)j;
    }
    i64 k = 0;
    for (i64 j = 0; j < n; ++j) {
        if (parent[j] != -1) continue;
        i64 top = 0;
        stack[0] = (i32)j;
        while (top >= 0) {
            i32 p = stack[top];
            i32 child = head[p];
            if (child == -1) {
                top--;
                post[k++] = p;
            } else {
                head[p] = next[child];
                stack[++top] = child;
            }
        }
    }
}

// Column counts, skeleton-matrix / least-common-ancestor method (chol.hpp:567-622).
void col_count(i64 n, const i64* Ap, const i32* Ai, const i32* parent, const i32* post,
               i64* colcount) {
    const i64 nnz = Ap[n];
    std::vector<i64> ATp((size_t)n + 1, 0);
    std::vector<i32> ATi((size_t)std::max<i64>(nnz, 1));
    for (i64 j = 0; j < n; ++j)
        for (i64 p = Ap[j]; p < Ap[j + 1]; ++p) ATp[Ai[p] + 1]++;
    for (i64 j = 0; j < n; ++j) ATp[j + 1] += ATp[j];
    {
        std::vector<i64> nxt(ATp);
        for (i64 j = 0; j < n; ++j)
            for (i64 p = Ap[j]; p < Ap[j + 1]; ++p) ATi[nxt[Ai[p]]++] = (i32)j;
    }
    std::vector<i32> first((size_t)n, -1), maxfirst((size_t)n, -1), prevleaf((size_t)n, -1),
        ancestor((size_t)n);
    std::vector<i64> delta((size_t)n, 0);
    for (i64 i = 0; i < n; ++i) ancestor[i] = (i32)i;
    for (i64 k = 0; k < n; ++k) {
        i32 j = post[k];
        delta[j] = (first[j] == -1) ? 1 : 0;
        for (; j != -1 && first[j] == -1; j = parent[j]) first[j] = (i32)k;
    }
    for (i64 k = 0; k < n; ++k) {
        i32 j = post[k];
        if (parent[j] != -1) delta[parent[j]]--;
        for (i64 p = ATp[j]; p < ATp[j + 1]; ++p) {
            i32 i = ATi[p];
            if (i <= j || first[j] <= maxfirst[i]) continue;
            maxfirst[i] = first[j];
            i32 jprev = prevleaf[i];
            delta[j]++;
            if (jprev != -1) {
                i32 q = jprev;
                while (q != ancestor[q]) q = ancestor[q];
                for (i32 s = jprev; s != q;) {
                    i32 sp = ancestor[s];
                    ancestor[s] = q;
                    s = sp;
                }
                delta[q]--;
            }
            prevleaf[i] = j;
        }
        if (parent[j] != -1) ancestor[j] = parent[j];
    }
    for (i64 j = 0; j < n; ++j) colcount[j] = delta[j];
    for (i64 j = 0; j < n; ++j) {
        i32 pj = parent[j];
        if (pj != -1) colcount[pj] += colcount[j];
    }
}

// Row reach (chol.hpp:686-739).  `path` is reusable scratch in place of the
// reference's per-nonzero std::vector (chol.hpp:701).
i64 ereach(i64 n, const i64* Ap, const i32* Ai, const double* Ax, i64 k, const i32* parent,
           i32* s, i32* w, double* x, std::vector<i32>& path) {
    i64 top = n;
    if ((i64)path.size() < n) path.resize((size_t)n);
    for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
        i32 i = Ai[p];
        if (i > k) continue;
        if (x && Ax) x[i] = Ax[p];
        i64 len = 0;
        while (i != -1 && w[i] != k) {
            path[len++] = i;
            w[i] = (i32)k;
            i = parent[i];
        }
        while (len > 0) s[--top] = path[--len];
    }
    return top;
}

// Depth-from-root levels, deepest first (src/chol.cpp:7-40).
i64 compute_levels(i64 n, const i32* parent, i32* level_of) {
    std::vector<i32> depth((size_t)n, -1);
    std::vector<i32> path;
    for (i64 j = 0; j < n; ++j) {
        if (depth[j] != -1) continue;
        path.clear();
        i32 v = (i32)j;
        while (v != -1 && depth[v] == -1) {
            path.push_back(v);
            v = parent[v];
        }
        i32 base = (v == -1) ? 0 : depth[v] + 1;
        for (i64 t = (i64)path.size() - 1; t >= 0; --t) depth[path[t]] = base++;
    }
    i32 maxd = 0;
    for (i64 j = 0; j < n; ++j) maxd = std::max(maxd, depth[j]);
    if (level_of)
        for (i64 j = 0; j < n; ++j) level_of[j] = maxd - depth[j];
    return n > 0 ? (i64)maxd + 1 : 0;
}

i64 etree_depth(i64 n, const i32* parent) { return compute_levels(n, parent, nullptr); }

static bool validate(i64 n, const i64* Ap, const i32* Ai, std::string& err) {
    if (n < 0 || n > (i64)INT32_MAX - 1) {
        err = "n out of range";
        return false;
    }
    if (!Ap || (n > 0 && !Ai && Ap[n] > 0)) {
        err = "null CSC arrays";
        return false;
    }
    if (Ap[0] != 0) {
        err = "Ap[0] != 0";
        return false;
    }
    for (i64 j = 0; j < n; ++j)
        if (Ap[j + 1] < Ap[j]) {
            err = "column pointers not monotone";
            return false;
        }
    for (i64 p = 0; p < Ap[n]; ++p)
        if (Ai[p] < 0 || Ai[p] >= n) {
            err = "row index out of range";
            return false;
        }
    return true;
}

i64 analyze(i64 n, const i64* Ap, const i32* Ai, const sc_options& opt, Symbolic& S,
            std::string& err) {
    if (!validate(n, Ap, Ai, err)) return SC_ERR_ARG;
    S.opt = opt;
    S.n = n;
    S.nnzA_in = Ap[n];
    S.Ap.assign(Ap, Ap + n + 1);
    S.Ai.assign(Ai, Ai + Ap[n]);
    const i64 nnz = Ap[n];

    // ---- natural-order symbolic (reference semantics) ----
    S.parent.resize((size_t)n);
    S.post.resize((size_t)n);
    S.ipost.resize((size_t)n);
    S.colcount.resize((size_t)n);
    etree(n, Ap, Ai, S.parent.data());
    post_order(n, S.parent.data(), S.post.data());
    col_count(n, Ap, Ai, S.parent.data(), S.post.data(), S.colcount.data());
    S.nnzL = 0;
    S.flops = 0.0;
    for (i64 j = 0; j < n; ++j) {
        S.nnzL += S.colcount[j];
        S.flops += (double)S.colcount[j] * (double)S.colcount[j];
    }
    S.depth = etree_depth(n, S.parent.data());
    for (i64 c = 0; c < n; ++c) S.ipost[S.post[c]] = (i32)c;

    // ---- internal (postorder) etree and counts ----
    std::vector<i32> iparent((size_t)n);
    std::vector<i64> icc((size_t)n);
    for (i64 c = 0; c < n; ++c) {
        i32 j = S.post[c];
        iparent[c] = S.parent[j] == -1 ? -1 : S.ipost[S.parent[j]];
        icc[c] = S.colcount[j];
    }

    // ---- fundamental supernodes: reference rule (src/chol.cpp:75-85) in postorder ----
    std::vector<i32> fstart;
    fstart.reserve((size_t)n + 1);
    for (i64 c = 0; c < n; ++c) {
        bool same = c > 0 && iparent[c - 1] == c && icc[c] == icc[c - 1] - 1;
        if (!same) fstart.push_back((i32)c);
    }
    const i32 nf = (i32)fstart.size();
    fstart.push_back((i32)n);
    S.n_fundamental = nf;
    std::vector<i32> fsn_of((size_t)n);
    for (i32 f = 0; f < nf; ++f)
        for (i32 c = fstart[f]; c < fstart[f + 1]; ++c) fsn_of[c] = f;
    std::vector<i32> fparent((size_t)nf, -1);
    for (i32 f = 0; f < nf; ++f) {
        i32 pc = iparent[fstart[f + 1] - 1];
        fparent[f] = pc == -1 ? -1 : fsn_of[pc];
    }

    // ---- relaxed amalgamation (CHOLMOD-style): merge f into f+1 when f+1 is its parent ----
    std::vector<i64> nscol((size_t)nf), snz((size_t)nf);
    std::vector<double> zeros((size_t)nf, 0.0);
    std::vector<char> absorbed((size_t)nf, 0);
    for (i32 f = 0; f < nf; ++f) {
        nscol[f] = fstart[f + 1] - fstart[f];
        snz[f] = icc[fstart[f]];
    }
    if (opt.relax) {
        std::vector<i32> gkids((size_t)nf, 0);  // children of each (merged) group
        for (i32 f = 0; f < nf; ++f)
            if (fparent[f] >= 0) gkids[fparent[f]]++;
        // heights in the fundamental tree (leaves 0) and, per node, how many children reach
        // its height minus one: a child is its parent's unique deepest child when it alone
        // sets the parent's height (children precede their parent in postorder)
        std::vector<i32> fh((size_t)nf, 0), nmax((size_t)nf, 0);
        for (i32 f = 0; f < nf; ++f) {
            const i32 p = fparent[f];
            if (p < 0) continue;
            if (fh[f] + 1 > fh[p]) {
                fh[p] = fh[f] + 1;
                nmax[p] = 1;
            } else if (fh[f] + 1 == fh[p]) {
                nmax[p]++;
            }
        }
        for (i32 j = nf - 2; j >= 0; --j) {
            if (fparent[j] != j + 1) continue;
            const i64 nscol0 = nscol[j], nscol1 = nscol[j + 1], ns = nscol0 + nscol1;
            const i64 lnz0 = snz[j], lnz1 = snz[j + 1];
            const double newzeros = (double)nscol0 * (double)(nscol0 + lnz1 - lnz0);
            const double totz = newzeros + zeros[j] + zeros[j + 1];
            bool merge = false;
            // a merged front that still runs in the one-workgroup register kernel (m <=
            // small_front_max) has no CB SYRK to keep the coupling in: such a merge is not
            // blocked by the wide-sibling rule, and when the child is its parent's unique
            // deepest child (the merge takes one dependent front off the tree's longest
            // path) it is held to the loosest zero threshold at any width.  1138_bus: 93 ->
            // 47 levels, 0.614 -> 0.436 ms with the pinned status word (numeric.cpp); 128^3:
            // 164,027 -> 163,933 supernodes, 19 levels, bench neutral; an unrestricted loose
            // threshold also merged 128^3's balanced small fronts (147,549 supernodes) and
            // grew the 8-rank work arena 7.73 -> 8.03 GB
            const bool small_merged = nscol0 + lnz1 <= opt.small_front_max;
            // ... and on the parent's one longest path (a merge there shortens the tree)
            const bool deepest = fh[j] + 1 == fh[j + 1] && nmax[j + 1] == 1;
            if (opt.relax_wmax > 0 && nscol0 > opt.relax_wmax && nscol1 > opt.relax_wmax && gkids[j + 1] > 1 &&
                !small_merged) {
                // a wide child of a wide parent with siblings stays apart: its coupling goes
                // through the CB SYRK and the siblings stay parallel.  Chains still merge.
                merge = false;
            } else if (ns <= opt.nrelax[0] || newzeros == 0.0) {
                merge = true;
            } else {
                const double denom =
                    (double)ns * (double)(ns + 1) / 2.0 + (double)ns * (double)(lnz1 - nscol1);
                const double z = totz / denom;
                merge = (ns <= opt.nrelax[1] && z < opt.zrelax[0]) ||
                        (ns <= opt.nrelax[2] && z < opt.zrelax[1]) || (z < opt.zrelax[2]) ||
                        (small_merged && deepest && z < opt.zrelax[0]);
            }
            if (merge) {
                zeros[j] = totz;
                nscol[j] = ns;
                snz[j] = nscol0 + lnz1;
                absorbed[j + 1] = 1;
                gkids[j] += gkids[j + 1] - 1;
            }
        }
    }
    S.sn_start.clear();
    for (i32 f = 0; f < nf; ++f)
        if (!absorbed[f]) S.sn_start.push_back(fstart[f]);
    const i32 ns = (i32)S.sn_start.size();
    S.ns = ns;
    S.sn_start.push_back((i32)n);
    S.sn_of.resize((size_t)n);
    for (i32 s = 0; s < ns; ++s)
        for (i32 c = S.sn_start[s]; c < S.sn_start[s + 1]; ++c) S.sn_of[c] = s;

    // ---- A in internal numbering, lower pattern by column (duplicates: last wins,
    //      as the reference's ereach scatter x[i] = Ax[p] does, chol.hpp:731) ----
    std::vector<i64> amap((size_t)nnz, -1);
    std::vector<i64>& acnt = S.a_ptr;
    acnt.assign((size_t)n + 1, 0);
    std::vector<i32> seen_col((size_t)n, -1);
    std::vector<i64> seen_p((size_t)n, -1);
    S.nnzA_used = 0;
    for (i64 k = 0; k < n; ++k) {
        for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
            i32 i = Ai[p];
            if (i > k) continue;
            if (seen_col[i] == k) {
                amap[seen_p[i]] = -2;  // superseded duplicate
                acnt[std::min(S.ipost[i], S.ipost[k]) + 1]--;
                S.nnzA_used--;
            }
            seen_col[i] = (i32)k;
            seen_p[i] = p;
            amap[p] = -3;  // live, placeholder
            acnt[std::min(S.ipost[i], S.ipost[k]) + 1]++;
            S.nnzA_used++;
        }
    }
    for (i64 c = 0; c < n; ++c) acnt[c + 1] += acnt[c];
    std::vector<i32> a_row((size_t)std::max<i64>(S.nnzA_used, 1));
    std::vector<i64>& a_src = S.a_src;
    a_src.assign((size_t)std::max<i64>(S.nnzA_used, 1), 0);
    S.a_pos.assign((size_t)std::max<i64>(S.nnzA_used, 1), 0);
    {
        std::vector<i64> nxt(acnt.begin(), acnt.end() - 1);
        for (i64 k = 0; k < n; ++k) {
            for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
                if (amap[p] != -3) continue;
                i32 i = Ai[p];
                i32 ri = S.ipost[i], rk = S.ipost[k];
                i32 c = std::min(ri, rk), r = std::max(ri, rk);
                i64 q = nxt[c]++;
                a_row[q] = r;
                a_src[q] = p;
            }
        }
    }

    // ---- row structures, assembly tree, relative indices, A map ----
    S.sn_m.assign((size_t)ns, 0);
    S.sn_parent.assign((size_t)ns, -1);
    S.rows_ptr.assign((size_t)ns + 1, 0);
    S.rel_ptr.assign((size_t)ns + 1, 0);
    S.panel_off.assign((size_t)ns + 1, 0);
    S.cb_off.assign((size_t)ns + 1, 0);
    S.level.assign((size_t)ns, 0);
    S.rows.clear();
    S.relind.clear();
    std::vector<std::vector<i32>> kids((size_t)ns);
    std::vector<i32> mark((size_t)n, -1);
    std::vector<i32> pos((size_t)n, -1);
    std::vector<i32> buf;
    for (i32 s = 0; s < ns; ++s) {
        const i32 c0 = S.sn_start[s], c1 = S.sn_start[s + 1], w = c1 - c0;
        buf.clear();
        for (i32 c = c0; c < c1; ++c) {
            buf.push_back(c);
            mark[c] = s;
        }
        for (i32 c = c0; c < c1; ++c)
            for (i64 q = acnt[c]; q < acnt[c + 1]; ++q) {
                i32 r = a_row[q];
                if (r >= c1 && mark[r] != s) {
                    mark[r] = s;
                    buf.push_back(r);
                }
            }
        i32 lev = 0;
        for (i32 ch : kids[s]) {
            lev = std::max(lev, S.level[ch] + 1);
            const i64 b0 = S.rows_ptr[ch] + S.w(ch), b1 = S.rows_ptr[ch + 1];
            for (i64 q = b0; q < b1; ++q) {
                i32 r = S.rows[q];
                if (r >= c1 && mark[r] != s) {
                    mark[r] = s;
                    buf.push_back(r);
                }
            }
        }
        S.level[s] = lev;
        std::sort(buf.begin() + w, buf.end());
        const i32 m = (i32)buf.size();
        S.sn_m[s] = m;
        S.rows_ptr[s + 1] = S.rows_ptr[s] + m;
        S.rows.insert(S.rows.end(), buf.begin(), buf.end());
        S.panel_off[s + 1] = S.panel_off[s] + (i64)m * w;
        S.cb_off[s + 1] = S.cb_off[s] + (i64)(m - w) * (m - w);
        S.rel_ptr[s + 1] = S.rel_ptr[s] + (m - w);
        if (m > w) {
            S.sn_parent[s] = S.sn_of[buf[w]];
            kids[S.sn_parent[s]].push_back(s);
        }
        // positions of this front's rows
        for (i32 t = 0; t < m; ++t) pos[buf[t]] = t;
        // children's relative indices into this front
        for (i32 ch : kids[s]) {
            const i64 b0 = S.rows_ptr[ch] + S.w(ch), b1 = S.rows_ptr[ch + 1];
            i64 dst = S.rel_ptr[ch];
            if ((i64)S.relind.size() < S.rel_ptr[ch + 1]) S.relind.resize(S.rel_ptr[ch + 1]);
            for (i64 q = b0; q < b1; ++q) S.relind[dst++] = pos[S.rows[q]];
        }
        // A entries of this supernode's columns
        for (i32 c = c0; c < c1; ++c)
            for (i64 q = acnt[c]; q < acnt[c + 1]; ++q)
                S.a_pos[q] = pos[a_row[q]];
    }
    S.relind.resize((size_t)S.rel_ptr[ns]);
    // per child, bounds of its CB rows by blocks of the parent front (the large-front
    // assembly and the CB SYRK's gather read them instead of binary-searching relind):
    // g(k) = first CB row whose parent position is >= base + k * blk, stored compactly
    // over the blocks the child touches: [k_lo, k_hi, g(k_lo), g(k_lo + 1) .. g(k_hi - 1)]
    // (g = g(k_lo) below k_lo, mbc from k_hi; kernels.hip bnd_at)
    auto bounds = [&](std::vector<i64>& ptr, std::vector<i32>& out, int blk, bool cb_only) {
        ptr.assign((size_t)ns + 1, 0);
        out.clear();
        for (i32 s = 0; s < ns; ++s) {
            const i32 p = S.sn_parent[s];
            if (p >= 0) {
                const i32 base = cb_only ? S.w(p) : 0;
                const i32* rel = S.relind.data() + S.rel_ptr[s];
                const i32 mbc = (i32)(S.rel_ptr[s + 1] - S.rel_ptr[s]);
                const i32 j0 = (i32)(std::lower_bound(rel, rel + mbc, base) - rel);
                const i32 klo = j0 < mbc ? (rel[j0] - base) / blk : 0;
                const i32 khi = j0 < mbc ? (rel[mbc - 1] - base) / blk + 1 : 0;
                out.push_back(klo);
                out.push_back(khi);
                out.push_back(j0);
                for (i32 k = klo + 1; k < khi; ++k)
                    out.push_back((i32)(std::lower_bound(rel, rel + mbc, base + blk * k) - rel));
            }
            ptr[s + 1] = (i64)out.size();
        }
    };
    bounds(S.rb_ptr, S.rel_bnd, kAsmRows, false);   // assembly row tiles
    bounds(S.cbk_ptr, S.col_bnd, kAsmCols, false);  // assembly column blocks
    bounds(S.tb_ptr, S.tile_bnd, 64, true);         // 64-row blocks of the parent's CB
    S.child_ptr.assign((size_t)ns + 1, 0);
    S.child_list.clear();
    for (i32 s = 0; s < ns; ++s) {
        S.child_ptr[s + 1] = S.child_ptr[s] + (i32)kids[s].size();
        S.child_list.insert(S.child_list.end(), kids[s].begin(), kids[s].end());
    }
    S.nlevels = 0;
    for (i32 s = 0; s < ns; ++s) S.nlevels = std::max(S.nlevels, S.level[s] + 1);

    // ---- front classes and statistics ----
    S.fclass.assign((size_t)ns, FRONT_SMALL);
    sc_symbolic_stats& st = S.stats;
    std::memset(&st, 0, sizeof(st));
    st.n = n;
    st.nnz_A = S.nnzA_used;
    st.nnz_L = S.nnzL;
    st.flops = S.flops;
    st.etree_depth = S.depth;
    st.n_fundamental = nf;
    st.n_supernodes = ns;
    st.n_levels = S.nlevels;
    st.panel_entries = S.panel_off[ns];
    st.cb_entries = S.cb_off[ns];
    for (i32 s = 0; s < ns; ++s) {
        const double m = S.sn_m[s], w = S.w(s), mb = m - w;
        st.max_front_m = std::max<i64>(st.max_front_m, S.sn_m[s]);
        st.max_front_w = std::max<i64>(st.max_front_w, S.w(s));
        S.fclass[s] = (S.sn_m[s] <= opt.small_front_max) ? FRONT_SMALL : FRONT_LARGE;
        if (S.fclass[s] == FRONT_SMALL)
            st.n_small_fronts++;
        else
            st.n_large_fronts++;
        // dense partial factorization of w pivots of an m-row front:
        // sum_{t<w} (m-t)^2 counted the same way as F (colcount^2 per column)
        double f = 0.0;
        for (double t = 0; t < w; t += 1.0) f += (m - t) * (m - t);
        st.flops_executed += f;
        if (w >= 256) st.flops_syrk_w256 += mb * (mb + 1.0) * w;
    }
    return SC_OK;
}

void pattern_L(const Symbolic& S, i64* Lp, i32* Li) {
    const i64 n = S.n;
    i64 nz = 0;
    for (i64 j = 0; j < n; ++j) {
        Lp[j] = nz;
        nz += S.colcount[j];
    }
    Lp[n] = nz;
    if (!Li) return;
    std::vector<i64> c(Lp, Lp + n);
    std::vector<i32> s((size_t)n), w((size_t)n, -1), path((size_t)n);
    // row-by-row ereach appends (chol.hpp:916-942); natural row order yields the
    // same ascending columns as the reference's level order.
    for (i64 j = 0; j < n; ++j) {
        w[j] = (i32)j;
        i64 top = ereach(n, S.Ap.data(), S.Ai.data(), nullptr, j, S.parent.data(), s.data(),
                         w.data(), nullptr, path);
        for (i64 t = top; t < n; ++t) Li[c[s[t]]++] = (i32)j;
        Li[c[j]++] = (i32)j;
    }
}

void export_L(const Symbolic& S, const double* panels, const i64* poff, i64* Lp, i32* Li, double* Lx) {
    const i64 n = S.n;
    std::vector<i64> Lp_loc;
    std::vector<i32> Li_loc;
    if (!Lp) {
        Lp_loc.resize((size_t)n + 1);
        Lp = Lp_loc.data();
    }
    if (!Li && Lx) {
        Li_loc.resize((size_t)std::max<i64>(S.nnzL, 1));
        Li = Li_loc.data();
    }
    pattern_L(S, Lp, Li);
    if (!Lx) return;
    std::vector<i32> pos((size_t)n, -1);
    for (i32 s = 0; s < S.ns; ++s) {
        const i32 c0 = S.sn_start[s], c1 = S.sn_start[s + 1];
        const i64 m = S.sn_m[s];
        const i32* rows = S.rows.data() + S.rows_ptr[s];
        for (i64 t = 0; t < m; ++t) pos[rows[t]] = (i32)t;
        const double* P = panels + poff[s];
        for (i32 c = c0; c < c1; ++c) {
            const i32 j = S.post[c];
            const double* col = P + (i64)(c - c0) * m;
            for (i64 p = Lp[j]; p < Lp[j + 1]; ++p) Lx[p] = col[pos[S.ipost[Li[p]]]];
        }
    }
}

}  // namespace sc
