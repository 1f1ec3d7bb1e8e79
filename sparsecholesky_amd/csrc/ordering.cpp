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
