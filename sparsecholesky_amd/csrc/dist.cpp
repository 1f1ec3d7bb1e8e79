// Multi-GPU plan: proportional subtree-to-GPU mapping of the
// assembly tree, split top fronts, and the comm steps between ranks.
//
// Mapping.  The ranks form a continuous interval [0, P) of processor mass split
// among the children of every front in proportion to subtree work; rounded to
// whole ranks, a child whose interval holds at most one rank gets its whole
// subtree there (no communication inside).  Fronts whose interval holds more
// ranks are the subtree-merge ("shared") fronts; their rank groups nest and two
// fronts of the same level have disjoint groups.
//
// Split fronts.  A shared front with a contribution block is split over its
// group: its least-loaded rank (the owner) assembles it and factors its panel;
// the other ranks own column blocks of its contribution block.  The owner sends
// the assembled CB blocks once (STEP_INIT) and then rows [w, m) of every panel
// slab as soon as the slab is final (STEP_SLAB); each CB rank applies
// CB -= L21_k L21_k^T to its blocks per slab, so the CB update (the bulk of the
// front's flops) runs on the group in parallel and overlaps the owner's panel
// chain.  Shared fronts without a CB (the root) run on their owner.
//
// Distributed panels (dist_panel).  A shared front wider than one slab has its
// panel factored 1D slab-cyclic over its group (right-looking with lookahead, the
// reference's level loop include/chol.hpp:1423-1443 parallelised inside the front):
// the owner assembles the front and factors slab 0; slab k goes to group rank
// (owner + k) mod g, which receives its assembled columns once (STEP_INIT).  When
// slab k is final its owner sends its rows [need, m) (STEP_SLAB) to every rank that
// updates a later slab or a CB block with it; each rank applies the slab's update
// to the slabs and CB blocks it owns (the next slab first, on the critical path).
// This covers the root, whose panel is the whole front.
//
// Transfers.  After each level, every CB column block whose producer is not the
// executing rank of the parent goes there (STEP_DELIVER), packed (only rows
// >= the block's first column: the lower part), so several links feed one parent
// at once when its child was split.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "numeric.hpp"
#include "symbolic.hpp"

namespace sc {

// sum_{t<w} (m-t)^2, closed form: the front's dense partial-Cholesky work
static double front_work(const Symbolic& S, i32 s) {
    const double m = S.sn_m[s], w = S.w(s);
    return w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0;
}

// CB-update share of front_work: mb (mb + 1) w
static double cb_work(const Symbolic& S, i32 s) {
    const double mb = S.mb(s), w = S.w(s);
    return mb * (mb + 1.0) * w;
}

// Panel work of columns [c0, c1) in right-looking order: column c takes the
// updates of the c columns before it over rows [c, m)
static double slab_work(const Symbolic& S, i32 s, int c0, int c1) {
    const double m = S.sn_m[s];
    double v = 0.0;
    for (int c = c0; c < c1; ++c) v += 2.0 * (c + 1.0) * (m - c);
    return v;
}

bool DistPlan::holds(int32_t s, int r) const {
    if (owner[s] == r) return true;
    if (pd.empty() || pd[s] < 0) return false;
    const std::vector<int32_t>& h = holders[pd[s]];
    return std::binary_search(h.begin(), h.end(), r);
}

int DistPlan::col_owner(const Symbolic& S, int32_t p, int col) const {
    const int w = S.w(p);
    if (col < w) return pd[p] >= 0 ? slab_rank[pd[p]][col / nbo] : owner[p];
    return split[p] >= 0 ? cb_rank[split[p]][(col - w) / cbb] : owner[p];
}

bool DistPlan::receives(const Symbolic& S, int32_t c, int r) const {
    const int32_t p = S.sn_parent[c];
    if (p < 0) return false;
    if (!dasm[p]) return owner[p] == r;
    const int32_t* rel = S.relind.data() + S.rel_ptr[c];
    for (int j = 0; j < S.mb(c); ++j)
        if (col_owner(S, p, rel[j]) == r) return true;
    return false;
}

bool DistPlan::produces_cb(const Symbolic& S, int32_t s, int r) const {
    if (S.mb(s) <= 0) return false;
    if (split[s] < 0) return owner[s] == r;
    if (owner[s] == r && !dasm[s]) return true;  // assembles the whole CB, sends its blocks (STEP_INIT)
    for (int32_t q : cb_rank[split[s]])
        if (q == r) return true;
    return false;
}

int DistPlan::need_row(const Symbolic& S, int32_t s, int k, int r) const {
    const int m = S.sn_m[s];
    const std::vector<int32_t>& sr = slab_rank[pd[s]];
    for (int j = k + 1; j < (int)sr.size(); ++j)
        if (sr[j] == r) return j * nbo;
    if (split[s] >= 0) {
        for (i32 q : cb_rank[split[s]])
            if (q == r) return S.w(s);
    } else if (S.mb(s) > 0 && r == owner[s]) {  // unsplit: the owner updates the whole CB
        return S.w(s);
    }
    return m;
}

int64_t dist_plan(const Symbolic& S, int nranks, DistPlan& D) {
    if (nranks <= 0) return SC_ERR_ARG;
    D = DistPlan();
    D.nranks = nranks;
    D.cbb = std::max(64, S.opt.dist_cbb > 0 ? S.opt.dist_cbb : 1024);
    D.nbo = std::max(PNB, (S.opt.panel_nb_outer / PNB) * PNB);
    {
        const int np = std::max(1, S.opt.dist_pieces);
        D.pw = std::max(PNB, (D.nbo / np + PNB - 1) / PNB * PNB);
    }
    const i32 ns = S.ns;
    D.owner.assign((size_t)ns, 0);
    D.gsize.assign((size_t)ns, 1);
    D.split.assign((size_t)ns, -1);
    D.pd.assign((size_t)ns, -1);
    D.work.assign((size_t)nranks, 0.0);
    std::vector<double> sub((size_t)ns, 0.0);
    for (i32 s = 0; s < ns; ++s) {  // children precede parents (postorder)
        sub[s] += front_work(S, s);
        if (S.sn_parent[s] >= 0) sub[S.sn_parent[s]] += sub[s];
    }
    struct Item {
        i32 s;
        double a, b;   // processor interval
        i32 plo, phi;  // parent's rank group (single owners are clamped into it)
    };
    std::vector<Item> stack;
    {
        double W = 0.0, cum = 0.0;
        for (i32 s = 0; s < ns; ++s)
            if (S.sn_parent[s] < 0) W += sub[s];
        for (i32 s = 0; s < ns; ++s)
            if (S.sn_parent[s] < 0) {
                const double a = nranks * (W > 0 ? cum / W : 0.0);
                cum += sub[s];
                const double b = nranks * (W > 0 ? cum / W : 1.0);
                stack.push_back({s, a, b, 0, nranks});
            }
    }
    std::vector<i32> glo((size_t)ns, 0);
    std::vector<char> shared((size_t)ns, 0);
    auto rnd = [&](double x) { return std::min(nranks, std::max(0, (int)std::floor(x + 0.5))); };
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        const int lo = rnd(it.a), hi = rnd(it.b);
        if (hi - lo <= 1) {
            int r = std::min(lo, nranks - 1);
            r = std::max(it.plo, std::min(it.phi - 1, r));
            std::vector<i32> st {it.s};  // whole subtree on r
            while (!st.empty()) {
                const i32 v = st.back();
                st.pop_back();
                D.owner[v] = r;
                for (i32 q = S.child_ptr[v]; q < S.child_ptr[v + 1]; ++q) st.push_back(S.child_list[q]);
            }
            continue;
        }
        shared[it.s] = 1;
        glo[it.s] = lo;
        D.gsize[it.s] = hi - lo;
        double Wc = 0.0, cum = 0.0;
        for (i32 q = S.child_ptr[it.s]; q < S.child_ptr[it.s + 1]; ++q) Wc += sub[S.child_list[q]];
        for (i32 q = S.child_ptr[it.s]; q < S.child_ptr[it.s + 1]; ++q) {
            const i32 c = S.child_list[q];
            const double a = it.a + (it.b - it.a) * (Wc > 0 ? cum / Wc : 0.0);
            cum += sub[c];
            const double b = it.a + (it.b - it.a) * (Wc > 0 ? cum / Wc : 1.0);
            stack.push_back({c, a, b, lo, hi});
        }
    }
    for (i32 s = 0; s < ns; ++s)
        if (!shared[s]) D.work[D.owner[s]] += front_work(S, s);
    // shared fronts, children first: owner = least-loaded rank of the group; split
    // fronts deal their CB column blocks to the other ranks, largest block first
    for (i32 s = 0; s < ns; ++s) {
        if (!shared[s]) continue;
        const int lo = glo[s], hi = lo + D.gsize[s];
        int own = lo;
        for (int r = lo + 1; r < hi; ++r)
            if (D.work[r] < D.work[own]) own = r;
        D.owner[s] = own;
        const int mb = S.mb(s), w = S.w(s);
        const bool split = S.opt.dist_split != 0 && S.fclass[s] == FRONT_LARGE && mb > 0;
        const bool dpanel = S.opt.dist_panel != 0 && S.fclass[s] == FRONT_LARGE && w > D.nbo;
        if (dpanel) {
            // slab k on group rank (owner + k) mod g: the whole group is free at a
            // shared front (its subtrees are done), so the slabs go round the group
            // rather than to the ranks with the least total work
            // slab blocks of dist_slab_block consecutive slabs per rank: the hand-over from a
            // slab to the next (its owner's send, the next owner's update) leaves the critical
            // path inside a block; a front with fewer than two blocks per rank deals single
            // slabs (parallel trailing updates matter more there)
            const int g = hi - lo, nsl = (w + D.nbo - 1) / D.nbo;
            const int sb = std::max(1, std::min(S.opt.dist_slab_block, nsl / g));
            std::vector<i32> sr((size_t)nsl);
            for (int k = 0; k < nsl; ++k) {
                sr[k] = lo + (own - lo + k / sb) % g;
                D.work[sr[k]] += slab_work(S, s, k * D.nbo, std::min(w, (k + 1) * D.nbo));
            }
            D.pd[s] = (i32)D.pd_s.size();
            D.pd_s.push_back(s);
            D.slab_rank.push_back(std::move(sr));
            if (!split) D.work[own] += cb_work(S, s);
        }
        if (!split) {
            if (!dpanel) D.work[own] += front_work(S, s);
            continue;
        }
        if (!dpanel) D.work[own] += front_work(S, s) - cb_work(S, s);
        const int nblk = (mb + D.cbb - 1) / D.cbb;
        std::vector<int> ord((size_t)nblk);
        for (int b = 0; b < nblk; ++b) ord[b] = b;  // block b has mb - b*cbb rows: descending work
        std::vector<i32> cbr((size_t)nblk, -1);
        for (int b : ord) {
            const double rows = mb - (double)b * D.cbb, cols = std::min<double>(D.cbb, rows);
            int best = -1;  // a distributed panel's owner is free after slab 0: it may take blocks
            for (int r = lo; r < hi; ++r)
                if ((r != own || dpanel) && (best < 0 || D.work[r] < D.work[best])) best = r;
            cbr[b] = best;
            D.work[best] += w * (2.0 * rows * cols - cols * cols + cols);
        }
        D.split[s] = (i32)D.split_s.size();
        D.split_s.push_back(s);
        D.cb_rank.push_back(std::move(cbr));
    }
    D.holders.assign(D.pd_s.size(), std::vector<i32>());
    for (size_t q = 0; q < D.pd_s.size(); ++q) {
        const i32 s = D.pd_s[q];
        std::vector<i32> h(D.slab_rank[q]);
        if (D.split[s] >= 0) h.insert(h.end(), D.cb_rank[D.split[s]].begin(), D.cb_rank[D.split[s]].end());
        std::sort(h.begin(), h.end());
        h.erase(std::unique(h.begin(), h.end()), h.end());
        D.holders[q] = std::move(h);
    }

    D.dasm.assign((size_t)ns, 0);
    for (i32 s = 0; s < ns; ++s)
        D.dasm[s] = S.opt.dist_asm != 0 && shared[s] && (D.pd[s] >= 0 || D.split[s] >= 0);
    D.early_gw = 4 * D.cbb;
    D.early.assign((size_t)ns, 0);
    for (i32 c = 0; c < ns; ++c) {
        const i32 p = S.sn_parent[c];
        D.early[c] = S.opt.dist_early != 0 && p >= 0 && D.split[c] < 0 && D.pd[c] < 0 && D.owner[c] != D.owner[p] &&
                     S.fclass[c] == FRONT_LARGE && S.mb(c) >= 2 * D.cbb;
    }
    // comm steps in the global order: per level, the split fronts' INIT and SLAB
    // steps (ascending supernode), then the level's DELIVER sub-steps
    std::vector<std::vector<i32>> by_level((size_t)S.nlevels);
    for (i32 s = 0; s < ns; ++s) by_level[S.level[s]].push_back(s);
    // column block jb of c's contribution block: rows [jb cbb, mb), its cbb columns
    auto cb_block = [&](DistMsg& g, i32 c, int jb) {
        const int mbc = S.mb(c);
        g.skind = g.dkind = R_CB;
        g.srow = g.scol = g.drow = g.dcol = jb * D.cbb;
        g.rows = mbc - jb * D.cbb;
        g.cols = std::min(D.cbb, g.rows);
        g.s = c;
    };
    auto open_step = [&](int kind, int lev, int s, int k, int p = 0) {
        D.steps.push_back({kind, lev, s, k, p});
        return (int32_t)D.steps.size() - 1;
    };
    auto close_step = [&](int32_t id) {  // drop a step without messages
        if (D.msgs.empty() || D.msgs.back().step != id) D.steps.pop_back();
    };
    // a distributed panel's slab (panel columns [c0, c1), rows [r0, m)) from src to dst
    auto panel_msg = [&](int32_t id, i32 s, int src, int dst, int r0, int c0, int c1) {
        DistMsg g {};
        g.step = id;
        g.src = src;
        g.dst = dst;
        g.skind = g.dkind = R_PANEL;
        g.srow = g.drow = r0;
        g.scol = g.dcol = c0;
        g.rows = S.sn_m[s] - r0;
        g.cols = c1 - c0;
        g.s = s;
        D.msgs.push_back(g);
    };
    for (i32 lev = 0; lev < S.nlevels; ++lev) {
        for (i32 s : by_level[lev]) {
            if (D.pd[s] < 0) continue;
            const std::vector<i32>& sr = D.slab_rank[D.pd[s]];
            const int own = D.owner[s], w = S.w(s), nsl = (int)sr.size();
            // INIT (owner-assembled fronts only): assembled slab columns to their owners,
            // CB blocks to the CB ranks
            int32_t id = open_step(STEP_INIT, lev, s, 0);
            for (int k = 1; k < nsl && !D.dasm[s]; ++k)
                if (sr[k] != own) panel_msg(id, s, own, sr[k], k * D.nbo, k * D.nbo, std::min(w, (k + 1) * D.nbo));
            if (D.split[s] >= 0 && !D.dasm[s]) {
                const std::vector<i32>& cbr = D.cb_rank[D.split[s]];
                for (int jb = 0; jb < (int)cbr.size(); ++jb) {
                    if (cbr[jb] == own) continue;  // computed in place in the owner's CB
                    DistMsg g {};
                    g.step = id;
                    g.src = own;
                    g.dst = cbr[jb];
                    cb_block(g, s, jb);
                    D.msgs.push_back(g);
                }
            }
            close_step(id);
            // SLAB k: rows [need, m) of the final slab to every holder that uses them,
            // the next slab's owner first (its update is on the critical path), in column
            // pieces of pw (dist_pieces): a piece leaves as soon as the chain has finished
            // its columns, and the next owner applies it while the rest is computed
            for (int k = 0; k < nsl; ++k) {
                const int k0 = k * D.nbo, k1 = std::min(w, k0 + D.nbo);
                std::vector<i32> dsts;
                if (k + 1 < nsl && sr[k + 1] != sr[k]) dsts.push_back(sr[k + 1]);
                for (i32 r : D.holders[D.pd[s]])
                    if (r != sr[k] && (k + 1 >= nsl || r != sr[k + 1])) dsts.push_back(r);
                for (int p = 0, c0 = k0; c0 < k1; ++p, c0 += D.pw) {
                    id = open_step(STEP_SLAB, lev, s, k, p);
                    for (i32 r : dsts) {
                        const int need = D.need_row(S, s, k, r);
                        if (need < S.sn_m[s]) panel_msg(id, s, sr[k], r, std::max(need, k1), c0, std::min(k1, c0 + D.pw));
                    }
                    close_step(id);
                }
            }
        }
        for (i32 s : by_level[lev]) {
            if (D.split[s] < 0 || D.pd[s] >= 0) continue;
            const std::vector<i32>& cbr = D.cb_rank[D.split[s]];
            const int own = D.owner[s], m = S.sn_m[s], w = S.w(s), mb = m - w;
            int32_t id = open_step(STEP_INIT, lev, s, 0);
            for (int jb = 0; jb < (int)cbr.size() && !D.dasm[s]; ++jb) {
                DistMsg g {};
                g.step = id;
                g.src = own;
                g.dst = cbr[jb];
                cb_block(g, s, jb);
                D.msgs.push_back(g);
            }
            close_step(id);
            std::vector<i32> dsts(cbr);
            std::sort(dsts.begin(), dsts.end());
            dsts.erase(std::unique(dsts.begin(), dsts.end()), dsts.end());
            for (int k0 = 0, k = 0; k0 < w; k0 += D.nbo, ++k) {
                const int k1 = std::min(w, k0 + D.nbo);
                id = open_step(STEP_SLAB, lev, s, k);
                for (i32 r : dsts) {
                    DistMsg g {};
                    g.step = id;
                    g.src = own;
                    g.dst = r;
                    g.skind = R_PANEL;  // rows [w, m) of the owner's panel ...
                    g.srow = w;
                    g.scol = k0;
                    g.dkind = R_LAND;   // ... into the CB rank's copy of L21
                    g.drow = 0;
                    g.dcol = k0;
                    g.rows = mb;
                    g.cols = k1 - k0;
                    g.s = s;
                    D.msgs.push_back(g);
                }
                close_step(id);
            }
        }
        // child c's CB columns [j0, j1) (computed on src) to the ranks that assemble the
        // parent columns they map into: the parent's owner, or, distributed assembly,
        // each run of consecutive columns to the owner of its parent slab / CB block
        // (rows from the run's first column down; a run on src itself stays put)
        auto deliver_cols = [&](int32_t id, i32 c, int src, int j0, int j1) {
            const i32 p = S.sn_parent[c];
            const int mbc = S.mb(c);
            const int32_t* rel = S.relind.data() + S.rel_ptr[c];
            auto dst_of = [&](int j) { return D.dasm[p] ? D.col_owner(S, p, rel[j]) : D.owner[p]; };
            for (int a = j0; a < j1;) {
                const int r = dst_of(a);
                int b = a + 1;
                while (b < j1 && dst_of(b) == r) ++b;
                if (r != src) {
                    DistMsg g {};
                    g.step = id;
                    g.src = src;
                    g.dst = r;
                    g.skind = g.dkind = R_CB;
                    g.srow = g.scol = g.drow = g.dcol = a;
                    g.rows = mbc - a;
                    g.cols = b - a;
                    g.s = c;
                    D.msgs.push_back(g);
                }
                a = b;
            }
        };
        for (i32 c : by_level[lev]) {  // early children: one sub-step per column group
            if (!D.early[c]) continue;
            const int mbc = S.mb(c), per = D.early_gw / D.cbb;
            for (int g = 0; g * D.early_gw < mbc; ++g) {
                const int32_t id = open_step(STEP_DELIVER, lev, c, g);
                for (int jb = g * per; jb < (g + 1) * per && jb * D.cbb < mbc; ++jb)
                    deliver_cols(id, c, D.owner[c], jb * D.cbb, std::min(mbc, (jb + 1) * D.cbb));
                close_step(id);
            }
        }
        int32_t id = open_step(STEP_DELIVER, lev, -1, 0);
        for (i32 c : by_level[lev]) {
            const i32 p = S.sn_parent[c];
            const int mbc = S.mb(c);
            if (p < 0 || mbc <= 0 || D.early[c]) continue;
            for (int jb = 0; jb * D.cbb < mbc; ++jb) {
                const int src = D.split[c] >= 0 ? D.cb_rank[D.split[c]][jb] : D.owner[c];
                deliver_cols(id, c, src, jb * D.cbb, std::min(mbc, (jb + 1) * D.cbb));
            }
        }
        close_step(id);
    }
    return SC_OK;
}

i64 dist_owner_map(const Symbolic& S, int nranks, i32* owner, double* work_per_rank) {
    DistPlan D;
    i64 rc = dist_plan(S, nranks, D);
    if (rc != SC_OK) return rc;
    if (owner) std::memcpy(owner, D.owner.data(), sizeof(i32) * (size_t)S.ns);
    if (work_per_rank) std::memcpy(work_per_rank, D.work.data(), sizeof(double) * (size_t)nranks);
    return SC_OK;
}

// Messages of `rank` in posting order: (comm step, peer, bytes, is_send).
i64 dist_schedule(const Symbolic& S, int nranks, int rank, i32* step, i32* peer, i64* bytes, i32* is_send,
                  i64 cap) {
    DistPlan D;
    i64 rc = dist_plan(S, nranks, D);
    if (rc != SC_OK) return rc;
    i64 cnt = 0;
    for (const DistMsg& g : D.msgs) {
        if (g.src != rank && g.dst != rank) continue;
        if (step && cnt < cap) {
            step[cnt] = g.step;
            peer[cnt] = g.src == rank ? g.dst : g.src;
            bytes[cnt] = (i64)g.rows * g.cols * (i64)sizeof(double);
            is_send[cnt] = g.src == rank ? 1 : 0;
        }
        ++cnt;
    }
    return cnt;
}

// ---------------- transport ----------------
static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");

i64 dist_unique_id(void* id128) {
    if (!id128) return SC_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SC_ERR_COMM;
    std::memcpy(id128, &id, sizeof(id));
    return SC_OK;
}

// One transfer group: every message of msgs[off, off + count) (the packed slots are
// ready on stream st).  RCCL: one ncclGroupStart/End with each send / receive (both
// ends post a step's messages in the same plan order, so the per-peer matching is
// consistent; a 1-rank communicator sends to itself in the emulated mode).  Device
// copies: hosted-to-hosted messages of an emulated handle.  Host transport (tests):
// through host memory, synchronously.
static hipError_t transfer_group(Numeric& N, const Msg* msgs, int64_t count, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (N.dry_comm || count == 0) return hipSuccess;
    bool any_net = false;
    for (int64_t q = 0; q < count; ++q) {
        if (msgs[q].op != MSG_COPY) {
            any_net = true;
            continue;
        }
        e = hipMemcpyAsync(msgs[q].buf, msgs[q].src_buf, (size_t)msgs[q].count * sizeof(double),
                           hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    if (!any_net) return hipSuccess;
    if (N.xport) {
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        std::vector<std::vector<char>> host((size_t)count);
        for (int64_t q = 0; q < count; ++q) {
            const Msg& g = msgs[q];
            if (g.op == MSG_COPY) continue;
            const size_t nb = (size_t)g.count * sizeof(double);
            host[q].resize(std::max<size_t>(nb, 1));
            if (g.op == MSG_SEND && (e = hipMemcpy(host[q].data(), g.buf, nb, hipMemcpyDeviceToHost)) != hipSuccess)
                return e;
            if (N.xport(N.xport_ctx, g.op == MSG_SEND ? 0 : 1, g.peer, host[q].data(), (int64_t)nb) != 0) {
                N.err = "host transport: post failed";
                return hipErrorUnknown;
            }
        }
        if (N.xport(N.xport_ctx, 2, -1, nullptr, 0) != 0) {
            N.err = "host transport: completion failed";
            return hipErrorUnknown;
        }
        for (int64_t q = 0; q < count; ++q) {
            const Msg& g = msgs[q];
            if (g.op == MSG_RECV &&
                (e = hipMemcpy(g.buf, host[q].data(), (size_t)g.count * sizeof(double), hipMemcpyHostToDevice)) !=
                    hipSuccess)
                return e;
        }
        return hipSuccess;
    }
    if (!N.comm) {
        N.err = "no communicator";
        return hipErrorInvalidValue;
    }
    ncclComm_t comm = (ncclComm_t)N.comm;
    if (ncclGroupStart() != ncclSuccess) return hipErrorUnknown;
    for (int64_t q = 0; q < count; ++q) {
        const Msg& g = msgs[q];
        if (g.op == MSG_COPY) continue;
        ncclResult_t r = g.op == MSG_SEND ? ncclSend(g.buf, (size_t)g.count, ncclDouble, g.peer, comm, st)
                                          : ncclRecv(g.buf, (size_t)g.count, ncclDouble, g.peer, comm, st);
        if (r != ncclSuccess) {
            N.err = std::string("rccl p2p: ") + ncclGetErrorString(r);
            (void)ncclGroupEnd();
            return hipErrorUnknown;
        }
    }
    ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) {
        N.err = std::string("rccl group: ") + ncclGetErrorString(r);
        return hipErrorUnknown;
    }
    return hipSuccess;
}

// One comm step of the hosted ranks on the comm stream: pack the sends into their
// staging slots, the transfer group, unpack the receives.
hipError_t comm_launch(Numeric& N, const Launch& L) {
    hipStream_t st = N.stream3;
    hipError_t e = hipSuccess;
    if (L.pcount > 0 && (e = launch_copy2d(N.d_copy, N.d_ctiles + L.poff, L.pcount, false, st)) != hipSuccess)
        return e;
    if ((e = transfer_group(N, N.msgs.data() + L.off, L.count, st)) != hipSuccess) return e;
    if (L.ucount > 0) return launch_copy2d(N.d_copy, N.d_ctiles + L.uoff, L.ucount, true, st);
    return hipSuccess;
}

// Global status of a one-rank-per-process handle: the minimum failing column over
// the ranks (each rank's info word holds its own fronts' failures only).
int64_t dist_min_info(Numeric& N, int32_t& info) {
    if (N.xport) {
        std::vector<int32_t> got((size_t)N.nranks, info);
        for (int r = 0; r < N.nranks; ++r) {
            if (r == N.rank) continue;
            if (N.xport(N.xport_ctx, 0, r, &info, sizeof(int32_t)) != 0 ||
                N.xport(N.xport_ctx, 1, r, &got[r], sizeof(int32_t)) != 0) {
                N.err = "host transport: status exchange failed";
                return SC_ERR_COMM;
            }
        }
        if (N.xport(N.xport_ctx, 2, -1, nullptr, 0) != 0) {
            N.err = "host transport: status exchange failed";
            return SC_ERR_COMM;
        }
        for (int32_t v : got) info = std::min(info, v);
        return SC_OK;
    }
    if (!N.comm) return SC_OK;
    // info lives at d_info[0] (the value this rank saw); reduce into d_info[1]
    ncclResult_t r = ncclAllReduce(N.d_info, N.d_info + 1, 1, ncclInt32, ncclMin, (ncclComm_t)N.comm, N.stream);
    if (r != ncclSuccess) {
        N.err = std::string("rccl allreduce: ") + ncclGetErrorString(r);
        return SC_ERR_COMM;
    }
    if (hipMemcpyAsync(N.h_info + 1, N.d_info + 1, sizeof(int32_t), hipMemcpyDeviceToHost, N.stream) != hipSuccess ||
        hipStreamSynchronize(N.stream) != hipSuccess) {
        N.err = "status reduction: HIP error";
        return SC_ERR_HIP;
    }
    info = N.h_info[1];
    return SC_OK;
}

// Whole factor on every rank of a one-rank-per-process handle: each rank's panel
// arena is contiguous, so the exchange is one message per rank pair; every rank
// lands rank q's arena at gpanel + rank_base[q] (the gathered layout).
int64_t dist_gather_panels(Numeric& N) {
    const int64_t tot = N.rank_base.back();
    if (!N.gpanel) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, (size_t)std::max<int64_t>(tot, 1) * sizeof(double));
        if (e != hipSuccess) {
            N.err = std::string("hipMalloc(gathered factor): ") + hipGetErrorString(e);
            return SC_ERR_DEVMEM;
        }
        N.allocs.push_back(p);
        N.dev_bytes += tot * (int64_t)sizeof(double);
        N.gpanel = (double*)p;
        N.gpanel_owned = true;
    }
    const RankMem& R = N.R[0];
    hipStream_t st = N.stream3 ? N.stream3 : N.stream;
    if (hipMemcpyAsync(N.gpanel + N.rank_base[N.rank], R.P.panel_pool, (size_t)R.panel_total * sizeof(double),
                       hipMemcpyDeviceToDevice, st) != hipSuccess) {
        N.err = "gather: local copy failed";
        return SC_ERR_HIP;
    }
    std::vector<Msg> m;
    for (int q = 0; q < N.nranks; ++q) {
        if (q == N.rank) continue;
        // in rank order on both sides: pair (a, b) posts a's send and b's receive in the
        // same relative order
        Msg snd {};
        snd.buf = R.P.panel_pool;
        snd.count = R.panel_total;
        snd.peer = q;
        snd.op = MSG_SEND;
        Msg rcv {};
        rcv.buf = N.gpanel + N.rank_base[q];
        rcv.count = N.rank_base[q + 1] - N.rank_base[q];
        rcv.peer = q;
        rcv.op = MSG_RECV;
        m.push_back(snd);
        m.push_back(rcv);
    }
    if (transfer_group(N, m.data(), (int64_t)m.size(), st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        if (N.err.empty()) N.err = "gather: transfer failed";
        return SC_ERR_COMM;
    }
    return SC_OK;
}

void comm_destroy(Numeric& N) {
    if (N.comm) {
        (void)ncclCommDestroy((ncclComm_t)N.comm);
        N.comm = nullptr;
    }
}

// Multi-rank handle.  One process per GPU: this process is `rank` of `nranks`; id128
// != NULL: RCCL transport; xport != NULL: host-staged transport (tests); DIST_DRY:
// nothing moves (timing projection).  Emulated (emulate != 0): every rank in this
// process on one device, each with its own memory plan and arenas, transfers as
// device copies (emulate == 1) or as RCCL send / receive to self on a 1-rank
// communicator (emulate == 2), so the whole message plan is exercised.
i64 numeric_create_dist(const Symbolic& S, int device, int rank, int nranks, const void* id128,
                        int32_t (*xport)(void*, int32_t, int32_t, void*, int64_t), void* xport_ctx, int emulate,
                        Numeric*& out, std::string& err) {
    out = nullptr;
    Numeric* Np = new (std::nothrow) Numeric();
    if (!Np) return SC_ERR_NOMEM;
    Numeric& N = *Np;
    N.rank = rank;
    N.nranks = nranks;
    i64 rc = dist_plan(S, nranks, N.D);
    if (rc != SC_OK) {
        delete Np;
        return rc;
    }
    N.owner = N.D.owner;
    auto comm_init = [&](const ncclUniqueId& id, int n, int r) -> i64 {
        int dev = device;
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipSetDevice(dev) != hipSuccess) {
            err = "hipSetDevice failed";
            return SC_ERR_HIP;
        }
        ncclComm_t comm = nullptr;
        ncclResult_t r2 = ncclCommInitRank(&comm, n, id, r);
        if (r2 != ncclSuccess) {
            err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r2);
            return SC_ERR_COMM;
        }
        N.comm = comm;
        return SC_OK;
    };
    if (emulate) {
        N.emulated = true;
        N.rank = 0;
        N.emul_rccl = emulate == 2 ? 1 : 0;
        if (N.emul_rccl) {
            ncclUniqueId id;
            if (ncclGetUniqueId(&id) != ncclSuccess) {
                err = "ncclGetUniqueId failed";
                delete Np;
                return SC_ERR_COMM;
            }
            if ((rc = comm_init(id, 1, 0)) != SC_OK) {
                delete Np;
                return rc;
            }
        }
    } else if (xport == DIST_DRY) {
        N.dry_comm = true;
    } else if (xport) {
        N.xport = xport;
        N.xport_ctx = xport_ctx;
    } else if (id128) {
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof(id));
        if ((rc = comm_init(id, nranks, rank)) != SC_OK) {
            delete Np;
            return rc;
        }
    } else {
        err = "multi-rank handle without a transport";
        delete Np;
        return SC_ERR_ARG;
    }
    rc = numeric_init(N, S, device);
    if (rc != SC_OK) {
        err = N.err;
        numeric_free(Np);
        return rc;
    }
    out = Np;
    return SC_OK;
}

}  // namespace sc
