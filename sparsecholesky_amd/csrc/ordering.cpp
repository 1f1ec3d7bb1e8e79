// Fill-reducing ordering.  The reference factors in the
// given order (no permutation anywhere in include/chol.hpp); this is an opt-in
// extension: sc_options.ordering = SC_ORDER_ND factors P A P^T instead.
//
// Nested dissection on the graph of A by level structures (George & Liu): in each
// connected part, a pseudo-peripheral vertex roots a BFS level structure; the
// middle level (by vertex count), trimmed to the vertices adjacent to the next
// level, separates the levels before it from the levels after it.  Parts are
// numbered first, separators last (so separators become the top supernodes and
// the two parts independent subtrees), recursively down to small leaves.
#include <algorithm>
#include <cmath>
#include <vector>

#include "symbolic.hpp"

namespace sc {

namespace {

struct Graph {
    std::vector<i64> xadj;
    std::vector<i32> adj;
};

// symmetric adjacency without the diagonal; entries below the diagonal of the
// upper-CSC input are ignored, as the reference does (chol.hpp:392,696)
Graph build_graph(i64 n, const i64* Ap, const i32* Ai) {
    Graph G;
    std::vector<i64> deg((size_t)n + 1, 0);
    for (i64 k = 0; k < n; ++k)
        for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
            const i32 i = Ai[p];
            if (i < k) {
                deg[i + 1]++;
                deg[k + 1]++;
            }
        }
    for (i64 v = 0; v < n; ++v) deg[v + 1] += deg[v];
    G.xadj = deg;
    G.adj.resize((size_t)deg[n]);
    std::vector<i64> nxt(deg.begin(), deg.end() - 1);
    for (i64 k = 0; k < n; ++k)
        for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
            const i32 i = Ai[p];
            if (i < k) {
                G.adj[nxt[i]++] = (i32)k;
                G.adj[nxt[k]++] = i;
            }
        }
    // drop duplicate edges (duplicate triplets)
    std::vector<i64> xnew((size_t)n + 1, 0);
    i64 w = 0;
    for (i64 v = 0; v < n; ++v) {
        const i64 b = G.xadj[v], e = G.xadj[v + 1];
        std::sort(G.adj.begin() + b, G.adj.begin() + e);
        i32 last = -1;
        for (i64 p = b; p < e; ++p)
            if (G.adj[p] != last) G.adj[w++] = last = G.adj[p];
        xnew[v + 1] = w;
    }
    G.adj.resize((size_t)w);
    G.xadj = xnew;
    return G;
}

constexpr i32 kLeaf = 64;  // parts at most this large are numbered as they are

}  // namespace

// perm[new] = old.  Returns SC_OK.
i64 nd_order(i64 n, const i64* Ap, const i32* Ai, i32* perm) {
    const Graph G = build_graph(n, Ap, Ai);
    std::vector<i32> tag((size_t)n, -1);    // id of the part a vertex currently belongs to
    std::vector<i32> mark((size_t)n, -1);   // BFS stamp
    std::vector<i32> level((size_t)n, 0);
    std::vector<i32> queue;
    queue.reserve((size_t)n);
    i32 stamp = 0, next_tag = 0;
    struct Item {
        std::vector<i32> verts;
        i64 hi;  // the part takes positions [hi - |verts|, hi)
    };
    std::vector<Item> stack;
    {
        Item all;
        all.verts.resize((size_t)n);
        for (i64 v = 0; v < n; ++v) all.verts[v] = (i32)v;
        all.hi = n;
        stack.push_back(std::move(all));
    }
    // BFS from r inside part t; returns the number of levels, fills queue in BFS order
    auto bfs = [&](i32 r, i32 t) {
        ++stamp;
        queue.clear();
        queue.push_back(r);
        mark[r] = stamp;
        level[r] = 0;
        i32 nlev = 1;
        for (size_t h = 0; h < queue.size(); ++h) {
            const i32 v = queue[h];
            for (i64 p = G.xadj[v]; p < G.xadj[v + 1]; ++p) {
                const i32 u = G.adj[p];
                if (tag[u] != t || mark[u] == stamp) continue;
                mark[u] = stamp;
                level[u] = level[v] + 1;
                nlev = std::max(nlev, level[u] + 1);
                queue.push_back(u);
            }
        }
        return nlev;
    };
    auto degree_in = [&](i32 v, i32 t) {
        i32 d = 0;
        for (i64 p = G.xadj[v]; p < G.xadj[v + 1]; ++p) d += tag[G.adj[p]] == t;
        return d;
    };
    while (!stack.empty()) {
        Item it = std::move(stack.back());
        stack.pop_back();
        const i64 cnt = (i64)it.verts.size();
        if (cnt == 0) continue;
        const i64 lo = it.hi - cnt;
        if (cnt <= kLeaf) {
            for (i64 q = 0; q < cnt; ++q) perm[lo + q] = it.verts[q];
            continue;
        }
        const i32 t = next_tag++;
        for (i32 v : it.verts) tag[v] = t;
        // connected components: number each separately
        i32 nlev = bfs(it.verts[0], t);
        if ((i64)queue.size() < cnt) {
            std::vector<i32> comp(queue.begin(), queue.end());
            std::vector<i32> rest;
            for (i32 v : it.verts)
                if (mark[v] != stamp) rest.push_back(v);
            stack.push_back({std::move(rest), it.hi - (i64)comp.size()});
            stack.push_back({std::move(comp), it.hi});
            continue;
        }
        // pseudo-peripheral root: restart from a minimum-degree vertex of the last
        // level while the eccentricity grows
        i32 root = it.verts[0];
        for (int iter = 0; iter < 4; ++iter) {
            i32 best = -1, bd = 0;
            for (size_t q = queue.size(); q-- > 0;) {
                const i32 v = queue[q];
                if (level[v] != nlev - 1) break;
                const i32 d = degree_in(v, t);
                if (best < 0 || d < bd) best = v, bd = d;
            }
            const i32 nl2 = bfs(best, t);
            if (nl2 <= nlev) {
                nlev = bfs(root, t);
                break;
            }
            root = best;
            nlev = nl2;
        }
        if (nlev < 3) {  // (nearly) a clique: no useful separator
            for (i64 q = 0; q < cnt; ++q) perm[lo + q] = queue[q];
            continue;
        }
        // middle level by count
        std::vector<i64> lcnt((size_t)nlev, 0);
        for (i32 v : queue) lcnt[level[v]]++;
        i32 k = 1;
        for (i64 acc = lcnt[0]; k < nlev - 2 && acc + lcnt[k] < (cnt + 1) / 2; ++k) acc += lcnt[k];
        std::vector<i32> A, B, Sep;
        for (i32 v : queue) {
            const i32 l = level[v];
            if (l < k) {
                A.push_back(v);
            } else if (l > k) {
                B.push_back(v);
            } else {
                bool touches_next = false;
                for (i64 p = G.xadj[v]; p < G.xadj[v + 1] && !touches_next; ++p) {
                    const i32 u = G.adj[p];
                    touches_next = tag[u] == t && mark[u] == stamp && level[u] == k + 1;
                }
                (touches_next ? Sep : A).push_back(v);
            }
        }
        for (size_t q = 0; q < Sep.size(); ++q) perm[it.hi - (i64)Sep.size() + (i64)q] = Sep[q];
        const i64 hb = it.hi - (i64)Sep.size();
        const i64 nbv = (i64)B.size();
        stack.push_back({std::move(A), hb - nbv});
        stack.push_back({std::move(B), hb});
    }
    return SC_OK;
}

// Approximate minimum degree (Amestoy, Davis & Duff, SIAM J. Matrix Anal. Appl. 17(4),
// 1996): greedy minimum-degree elimination on the quotient graph, where eliminated
// pivots become ELEMENTS (cliques stored by their variable lists) and a variable's
// exact external degree is replaced by the AMD bound
//   d_i <= min(n - k, d_i_old + |L_p \ i|, |A_i \ i| + |L_p \ i| + sum_{e in E_i, e != p} |L_e \ L_p|),
// with element absorption, indistinguishable-variable (supervariable) detection by
// hashing, mass elimination and the usual dense-row postponement.  The elimination
// order is then postordered over the element tree.  perm[new] = old.
//
// Storage: one integer array iw holds every list -- a variable's elements first
// (elen[i] of them) then its variables; an element's variables.  pe[i] is i's list
// start, len[i] its length.  An absorbed variable / element j gets pe[j] = flip(parent)
// (its representative supervariable or absorbing element), so the final tree is read
// back from pe.  nv[i]: supervariable size (0 = absorbed; negated while i is in the
// new element).  Degree lists: head[d] / next / prev.  w[]: marks for |L_e \ L_p|.
i64 amd_order(i64 n, const i64* Ap, const i32* Ai, i32* perm) {
    if (n <= 0) return SC_OK;
    const Graph G = build_graph(n, Ap, Ai);
    const i64 nnz = (i64)G.adj.size();
    auto flip = [](i64 x) { return -x - 2; };
    // dense rows: postponed to the end (absorbed into the dummy root n)
    i64 dense = std::max<i64>(16, (i64)(10.0 * std::sqrt((double)n)));
    dense = std::min<i64>(n - 2, dense);
    i64 cap = nnz + nnz / 5 + 2 * n + 1;  // elbow room for the new elements
    std::vector<i64> iw((size_t)cap);
    std::vector<i64> pe((size_t)n + 1), len((size_t)n + 1), nv((size_t)n + 1, 1), nxt((size_t)n + 1, -1),
        prv((size_t)n + 1, -1), head((size_t)n + 1, -1), elen((size_t)n + 1, 0), deg((size_t)n + 1),
        w((size_t)n + 1, 1), hhead((size_t)n + 1, -1);
    for (i64 i = 0; i < n; ++i) {
        pe[i] = G.xadj[i];
        len[i] = G.xadj[i + 1] - G.xadj[i];
    }
    std::copy(G.adj.begin(), G.adj.end(), iw.begin());
    i64 used = nnz;  // iw[0, used) in use
    len[n] = 0;
    nv[n] = 0;
    elen[n] = -2;
    pe[n] = -1;
    w[n] = 0;
    // w-marks: reset when the stamp would overflow
    i64 lemax = 0, mark = 2;
    auto wclear = [&](i64 m2) {
        if (m2 < 2 || m2 + lemax < 0) {
            for (i64 k = 0; k < n; ++k)
                if (w[k] != 0) w[k] = 1;
            m2 = 2;
        }
        return m2;
    };
    auto list_remove = [&](i64 i) {
        if (nxt[i] != -1) prv[nxt[i]] = prv[i];
        if (prv[i] != -1)
            nxt[prv[i]] = nxt[i];
        else
            head[deg[i]] = nxt[i];
    };
    auto list_insert = [&](i64 i, i64 d) {
        if (head[d] != -1) prv[head[d]] = i;
        nxt[i] = head[d];
        prv[i] = -1;
        head[d] = i;
    };
    i64 nel = 0, mindeg = 0;
    for (i64 i = 0; i < n; ++i) {
        deg[i] = len[i];
        if (deg[i] == 0) {  // isolated: an element at once
            elen[i] = -2;
            ++nel;
            pe[i] = -1;
            w[i] = 0;
        } else if (deg[i] > dense) {  // dense: absorbed into the root, ordered last
            nv[i] = 0;
            elen[i] = -1;
            ++nel;
            pe[i] = flip(n);
            nv[n]++;
        } else {
            list_insert(i, deg[i]);
        }
    }
    while (nel < n) {
        // pivot k of minimum approximate degree
        i64 k = -1;
        for (; mindeg < n && (k = head[mindeg]) == -1; ++mindeg) {
        }
        if (nxt[k] != -1) prv[nxt[k]] = -1;
        head[mindeg] = nxt[k];
        const i64 elenk = elen[k];
        i64 nvk = nv[k];
        nel += nvk;
        // compact iw when the new element might not fit after `used`
        if (elenk > 0 && used + mindeg >= cap) {
            for (i64 j = 0; j < n; ++j) {
                const i64 p = pe[j];
                if (p >= 0) {  // live list: mark its start with its owner
                    pe[j] = iw[p];
                    iw[p] = flip(j);
                }
            }
            i64 q = 0;
            for (i64 p = 0; p < used;) {
                const i64 j = flip(iw[p++]);
                if (j >= 0) {
                    iw[q] = pe[j];
                    pe[j] = q++;
                    for (i64 t = 0; t < len[j] - 1; ++t) iw[q++] = iw[p++];
                }
            }
            used = q;
        }
        // new element L_k: every variable reachable from k through its elements and
        // its own variable list, each once (nv negated to mark membership)
        i64 dk = 0;
        nv[k] = -nvk;
        i64 p = pe[k];
        const i64 pk1 = elenk == 0 ? p : used;  // no elements: build in place
        i64 pk2 = pk1;
        for (i64 k1 = 1; k1 <= elenk + 1; ++k1) {
            i64 e, pj, ln;
            if (k1 > elenk) {
                e = k;
                pj = p;
                ln = len[k] - elenk;
            } else {
                e = iw[p++];
                pj = pe[e];
                ln = len[e];
            }
            for (i64 k2 = 1; k2 <= ln; ++k2) {
                const i64 i = iw[pj++];
                const i64 nvi = nv[i];
                if (nvi <= 0) continue;  // absorbed, or already in L_k
                dk += nvi;
                nv[i] = -nvi;
                iw[pk2++] = i;
                list_remove(i);
            }
            if (e != k) {  // element e is absorbed into k
                pe[e] = flip(k);
                w[e] = 0;
            }
        }
        if (elenk != 0) used = pk2;
        deg[k] = dk;
        pe[k] = pk1;
        len[k] = pk2 - pk1;
        elen[k] = -2;  // k is an element now
        // |L_e \ L_k| for every element e adjacent to a variable of L_k: w[e] - mark
        mark = wclear(mark);
        for (i64 pk = pk1; pk < pk2; ++pk) {
            const i64 i = iw[pk];
            const i64 eln = elen[i];
            if (eln <= 0) continue;
            const i64 nvi = -nv[i];
            const i64 wnvi = mark - nvi;
            for (i64 q = pe[i]; q <= pe[i] + eln - 1; ++q) {
                const i64 e = iw[q];
                if (w[e] >= mark)
                    w[e] -= nvi;
                else if (w[e] != 0)
                    w[e] = deg[e] + wnvi;
            }
        }
        // approximate degrees of the variables of L_k; prune absorbed elements
        for (i64 pk = pk1; pk < pk2; ++pk) {
            const i64 i = iw[pk];
            const i64 p1 = pe[i], p2 = p1 + elen[i] - 1;
            i64 pn = p1, h = 0, d = 0;
            for (i64 q = p1; q <= p2; ++q) {
                const i64 e = iw[q];
                if (w[e] == 0) continue;
                const i64 dext = w[e] - mark;
                if (dext > 0) {
                    d += dext;
                    iw[pn++] = e;
                    h += e;
                } else {  // aggressive absorption: L_e is inside L_k
                    pe[e] = flip(k);
                    w[e] = 0;
                }
            }
            elen[i] = pn - p1 + 1;  // + the new element k
            const i64 p3 = pn, p4 = p1 + len[i];
            for (i64 q = p2 + 1; q < p4; ++q) {  // variables still in i's list
                const i64 j = iw[q];
                const i64 nvj = nv[j];
                if (nvj <= 0) continue;  // absorbed, or in L_k (covered by the element)
                d += nvj;
                iw[pn++] = j;
                h += j;
            }
            if (d == 0) {  // mass elimination: i is adjacent to L_k only
                pe[i] = flip(k);
                const i64 nvi = -nv[i];
                dk -= nvi;
                nvk += nvi;
                nel += nvi;
                nv[i] = 0;
                elen[i] = -1;
            } else {
                deg[i] = std::min(deg[i], d);
                iw[pn] = iw[p3];  // element k goes first in i's list
                iw[p3] = iw[p1];
                iw[p1] = k;
                len[i] = pn - p1 + 1;
                h %= n;
                nxt[i] = hhead[h];  // hash bucket (nxt / prv reused: i is off the degree lists)
                hhead[h] = i;
                prv[i] = h;
            }
        }
        deg[k] = dk;
        lemax = std::max(lemax, dk);
        mark = wclear(mark + lemax);
        // supervariables: variables of L_k with identical lists merge
        for (i64 pk = pk1; pk < pk2; ++pk) {
            i64 i = iw[pk];
            if (nv[i] >= 0) continue;
            const i64 h = prv[i];
            i = hhead[h];
            hhead[h] = -1;
            for (; i != -1 && nxt[i] != -1; i = nxt[i], ++mark) {
                const i64 ln = len[i], eln = elen[i];
                for (i64 q = pe[i] + 1; q <= pe[i] + ln - 1; ++q) w[iw[q]] = mark;
                i64 jlast = i;
                for (i64 j = nxt[i]; j != -1;) {
                    bool same = len[j] == ln && elen[j] == eln;
                    for (i64 q = pe[j] + 1; same && q <= pe[j] + ln - 1; ++q)
                        if (w[iw[q]] != mark) same = false;
                    if (same) {  // j joins supervariable i
                        pe[j] = flip(i);
                        nv[i] += nv[j];
                        nv[j] = 0;
                        elen[j] = -1;
                        j = nxt[j];
                        nxt[jlast] = j;
                    } else {
                        jlast = j;
                        j = nxt[j];
                    }
                }
            }
        }
        // finish L_k: its live variables back on the degree lists
        i64 pw = pk1;
        for (i64 pk = pk1; pk < pk2; ++pk) {
            const i64 i = iw[pk];
            const i64 nvi = -nv[i];
            if (nvi <= 0) continue;
            nv[i] = nvi;
            i64 d = deg[i] + dk - nvi;
            d = std::min(d, n - nel - nvi);
            list_insert(i, d);
            mindeg = std::min(mindeg, d);
            deg[i] = d;
            iw[pw++] = i;
        }
        nv[k] = nvk;
        if ((len[k] = pw - pk1) == 0) {  // an element with no variables: a tree root
            pe[k] = -1;
            w[k] = 0;
        }
        if (elenk != 0) used = pw;
    }
    // postorder the assembly tree read back from pe (parent = flip(pe)); absorbed
    // variables follow their representative
    for (i64 i = 0; i < n; ++i) pe[i] = flip(pe[i]);
    std::fill(head.begin(), head.end(), -1);
    for (i64 j = n - 1; j >= 0; --j) {  // absorbed variables: children of their representative (n: a root)
        if (nv[j] > 0) continue;
        nxt[j] = head[pe[j]];
        head[pe[j]] = j;
    }
    for (i64 e = n; e >= 0; --e) {  // elements: children of their absorbing element
        if (nv[e] <= 0) continue;
        if (pe[e] != -1) {
            nxt[e] = head[pe[e]];
            head[pe[e]] = e;
        }
    }
    std::vector<i64> stack;
    std::vector<i32> order;
    order.reserve((size_t)n + 1);
    for (i64 r = 0; r <= n; ++r) {
        if (pe[r] != -1) continue;  // not a root
        stack.push_back(r);
        while (!stack.empty()) {
            const i64 v = stack.back();
            const i64 c = head[v];
            if (c == -1) {
                stack.pop_back();
                if (v != n) order.push_back((i32)v);
            } else {
                head[v] = nxt[c];
                stack.push_back(c);
            }
        }
    }
    if ((i64)order.size() != n) return SC_ERR_ARG;  // cannot happen: every vertex is in the tree
    std::copy(order.begin(), order.end(), perm);
    return SC_OK;
}

// B = P A P^T as upper CSC (rows ascending; duplicates kept in input order so the
// reference's last-one-wins rule still applies), src[q] = index of B's entry q in
// A's arrays.  iperm[old] = new.
void permute_upper(i64 n, const i64* Ap, const i32* Ai, const i32* perm, std::vector<i64>& Bp,
                   std::vector<i32>& Bi, std::vector<i64>& src) {
    std::vector<i32> iperm((size_t)n);
    for (i64 q = 0; q < n; ++q) iperm[perm[q]] = (i32)q;
    Bp.assign((size_t)n + 1, 0);
    for (i64 k = 0; k < n; ++k)
        for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
            if (Ai[p] > k) continue;
            Bp[std::max(iperm[Ai[p]], iperm[k]) + 1]++;
        }
    for (i64 j = 0; j < n; ++j) Bp[j + 1] += Bp[j];
    Bi.resize((size_t)Bp[n]);
    src.resize((size_t)Bp[n]);
    std::vector<i64> nxt(Bp.begin(), Bp.end() - 1);
    for (i64 k = 0; k < n; ++k)
        for (i64 p = Ap[k]; p < Ap[k + 1]; ++p) {
            if (Ai[p] > k) continue;
            const i32 a = iperm[Ai[p]], b = iperm[k];
            const i64 q = nxt[std::max(a, b)]++;
            Bi[q] = std::min(a, b);
            src[q] = p;
        }
    // rows ascending per column, stable (duplicates keep their input order)
    std::vector<std::pair<i32, i64>> tmp;
    for (i64 j = 0; j < n; ++j) {
        const i64 b = Bp[j], e = Bp[j + 1];
        tmp.clear();
        for (i64 q = b; q < e; ++q) tmp.push_back({Bi[q], src[q]});
        std::stable_sort(tmp.begin(), tmp.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        for (i64 q = b; q < e; ++q) {
            Bi[q] = tmp[q - b].first;
            src[q] = tmp[q - b].second;
        }
    }
}

}  // namespace sc
