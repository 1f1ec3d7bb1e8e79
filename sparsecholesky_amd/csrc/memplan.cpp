// Device memory plan of one rank.
//
// The reference allocates each supernode's update block (UpdateBlock,
// include/chol.hpp:1161-1169) for the duration of one supernode and scatters it
// into the working matrix at once (apply_update, :1196-1216).  Here the
// contribution block (CB) of a front lives from its assembly (level L) until the last
// reader at its parent's level Lp -- the parent's assembly, or, when the parent's CB
// SYRK gathers its children's entries itself (cb_gather, schedule.cpp), that CB SYRK
// launch, the last launch of level Lp -- and every region's lifetime is a closed
// interval of assembly-tree levels, fixed by the static schedule.  A sweep over
// the levels places the regions in one work arena: regions dead before level t are
// freed before those born at t are placed (best fit, largest first), so offsets
// are static (hipGraph-capturable) and memory is reused across levels.
//
// Lifetimes (L = level of s, Lp = level of its parent):
//   single device           CB(s)                        [L, Lp]
//   multi-rank, comm steps  a region a comm step of level L' touches stays live
//                           through L' + 1: the comm stream runs ahead of or behind
//                           the main stream within that window, and the schedule
//                           makes the main stream wait for level L' 's steps before
//                           level L' + 2 starts (numeric.cpp)
//   owner of s, parent here CB(s)                        [L, Lp]
//   owner of s, parent away CB(s), sent after level L    [L, L+1]
//   parent's owner          CB(c) of a remote child c     [Lc, Lp] (received)
//   CB rank of split s      the column range of its blocks [L, L+1] (round 6: the range a
//                           rank touches, not the whole square; ld stays mb)
//                           R_LAND(s) (the L21 slabs)     [L, L+1]
//   holder of distributed s a full panel copy in the panel arena (permanent: its
//                           slabs are part of the factor; gathered for export)
#include <algorithm>
#include <map>
#include <queue>

#include "numeric.hpp"

namespace sc {

namespace {

constexpr int64_t kAlign = 64;  // doubles (512 B): region starts stay 512-B aligned

struct Req {
    int64_t size;   // doubles, aligned
    int32_t t0, t1; // closed lifetime
    int64_t* out;
};

int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Places the requests; returns the arena size; *live_max = the largest sum of
// sizes live at one level (no placement can use less).
int64_t place(std::vector<Req>& reqs, int64_t* live_max) {
    if (reqs.empty()) {
        if (live_max) *live_max = 0;
        return 0;
    }
    std::sort(reqs.begin(), reqs.end(), [](const Req& a, const Req& b) {
        return a.t0 != b.t0 ? a.t0 < b.t0 : a.size > b.size;
    });
    int32_t tmax = 0;
    for (const Req& r : reqs) tmax = std::max(tmax, r.t1);
    std::vector<int64_t> diff((size_t)tmax + 2, 0);
    for (const Req& r : reqs) {
        diff[r.t0] += r.size;
        diff[r.t1 + 1] -= r.size;
    }
    int64_t cur = 0, lm = 0;
    for (int32_t t = 0; t <= tmax; ++t) lm = std::max(lm, cur += diff[t]);
    if (live_max) *live_max = lm;

    // free list by offset (coalescing) and by size (best fit), kept in step
    std::map<int64_t, int64_t> by_off;
    std::multimap<int64_t, int64_t> by_size;
    auto drop = [&](std::map<int64_t, int64_t>::iterator it) {
        auto rg = by_size.equal_range(it->second);
        for (auto q = rg.first; q != rg.second; ++q)
            if (q->second == it->first) {
                by_size.erase(q);
                break;
            }
        by_off.erase(it);
    };
    auto add = [&](int64_t off, int64_t size) {
        by_off.emplace(off, size);
        by_size.emplace(size, off);
    };
    int64_t top = 0;
    using Live = std::pair<int32_t, std::pair<int64_t, int64_t>>;  // (t1, (off, size))
    std::priority_queue<Live, std::vector<Live>, std::greater<Live>> live;
    auto release = [&](int64_t off, int64_t size) {
        auto nx = by_off.lower_bound(off);
        if (nx != by_off.end() && off + size == nx->first) {
            size += nx->second;
            drop(nx);
        }
        auto pv = by_off.lower_bound(off);
        if (pv != by_off.begin()) {
            --pv;
            if (pv->first + pv->second == off) {
                off = pv->first;
                size += pv->second;
                drop(pv);
            }
        }
        if (off + size == top)  // free tail: lower the top
            top = off;
        else
            add(off, size);
    };
    int64_t peak = 0;
    for (size_t i = 0; i < reqs.size(); ++i) {
        Req& r = reqs[i];
        while (!live.empty() && live.top().first < r.t0) {
            release(live.top().second.first, live.top().second.second);
            live.pop();
        }
        auto bs = by_size.lower_bound(r.size);
        int64_t off;
        if (bs != by_size.end()) {
            off = bs->second;
            const int64_t rest = bs->first - r.size;
            drop(by_off.find(off));
            if (rest > 0) add(off + r.size, rest);
        } else {
            off = top;
            top += r.size;
            peak = std::max(peak, top);
        }
        *r.out = off;
        live.push({r.t1, {off, r.size}});
    }
    return peak;
}

// Greedy by size (largest region first, each at the lowest offset free over its whole
// lifetime) for the regions of at least `big` doubles, then the sweep above for the rest
// placed on top of them.  Returns the arena size.
int64_t place_by_size(std::vector<Req>& reqs, int64_t big) {
    std::vector<size_t> large, small;
    for (size_t i = 0; i < reqs.size(); ++i) (reqs[i].size >= big ? large : small).push_back(i);
    std::stable_sort(large.begin(), large.end(), [&](size_t a, size_t b) { return reqs[a].size > reqs[b].size; });
    int32_t tmax = 0;
    for (const Req& r : reqs) tmax = std::max(tmax, r.t1);
    // per level: placed (offset, end) intervals, sorted by offset
    std::vector<std::vector<std::pair<int64_t, int64_t>>> at((size_t)tmax + 1);
    int64_t top = 0;
    std::vector<std::pair<int64_t, int64_t>> busy;
    for (size_t i : large) {
        Req& r = reqs[i];
        busy.clear();
        for (int32_t t = r.t0; t <= r.t1; ++t) busy.insert(busy.end(), at[t].begin(), at[t].end());
        std::sort(busy.begin(), busy.end());
        int64_t off = 0;
        for (const auto& b : busy) {
            if (b.first >= off + r.size) break;  // the gap before b fits
            off = std::max(off, b.second);
        }
        *r.out = off;
        top = std::max(top, off + r.size);
        for (int32_t t = r.t0; t <= r.t1; ++t) {
            auto& v = at[t];
            v.insert(std::upper_bound(v.begin(), v.end(), std::make_pair(off, off + r.size)), {off, off + r.size});
        }
    }
    std::vector<Req> rest;
    for (size_t i : small) rest.push_back(reqs[i]);
    const int64_t base = align_up(top);
    const int64_t peak = place(rest, nullptr);
    for (size_t i : small) *reqs[i].out += base;
    return base + peak;
}

}  // namespace

int64_t plan_rank_panels(const Symbolic& S, const DistPlan* D, int rank, std::vector<int64_t>& panel_off) {
    panel_off.assign((size_t)S.ns, -1);
    int64_t off = 0;
    for (i32 s = 0; s < S.ns; ++s)
        if (D ? D->holds(s, rank) : rank == 0) {
            panel_off[s] = off;
            off += (int64_t)S.sn_m[s] * S.w(s);
        }
    return off + PNB;
}

int64_t plan_rank_memory(const Symbolic& S, const DistPlan* D, int rank, RankMem& R,
                         std::vector<PlacedRegion>* placed) {
    const i32 ns = S.ns;
    R.rank = rank;
    R.panel_off.assign((size_t)ns, -1);
    R.cb_off.assign((size_t)ns, -1);
    R.cb_col0.assign((size_t)ns, 0);
    R.land_off.assign((size_t)ns, -1);
    auto owner = [&](i32 s) { return D ? D->owner[s] : 0; };
    R.panel_total = plan_rank_panels(S, D, rank, R.panel_off);
    std::vector<Req> reqs;
    auto req = [&](int64_t size, i32 t0, i32 t1, int64_t* out) { reqs.push_back({align_up(size), t0, t1, out}); };
    for (i32 s = 0; s < ns; ++s) {
        const int64_t mb = S.mb(s);
        if (mb <= 0) continue;
        const i32 L = S.level[s], p = S.sn_parent[s], Lp = S.level[p];
        const int64_t sq = mb * mb;
        if (!D) {
            req(sq, L, Lp, &R.cb_off[s]);
            continue;
        }
        // CB(s) wherever part of it is computed (until it is sent after level L) or
        // received for the parent's assembly (until level Lp): only the column range the
        // rank touches -- a CB rank's column blocks, a receiver's columns that map into the
        // parent columns it assembles (ld stays mb, so every kernel addresses it as the square)
        const bool prod = D->produces_cb(S, s, rank), recv = D->receives(S, s, rank);
        if (!prod && !recv) continue;
        int64_t lo = mb, hi = 0;
        auto all = [&]() {
            lo = 0;
            hi = mb;
        };
        if (prod) {
            if (D->split[s] < 0 || (owner(s) == rank && !D->dasm[s])) {
                all();
            } else {
                const std::vector<i32>& cbr = D->cb_rank[D->split[s]];
                for (int jb = 0; jb < (int)cbr.size(); ++jb)
                    if (cbr[jb] == rank) {
                        lo = std::min<int64_t>(lo, (int64_t)jb * D->cbb);
                        hi = std::max<int64_t>(hi, std::min<int64_t>(mb, (int64_t)(jb + 1) * D->cbb));
                    }
            }
        }
        if (recv) {
            if (!D->dasm[p]) {
                all();
            } else {
                const i32* rel = S.relind.data() + S.rel_ptr[s];
                for (int64_t j = 0; j < mb; ++j)
                    if (D->col_owner(S, p, rel[j]) == rank) {
                        lo = std::min(lo, j);
                        hi = std::max(hi, j + 1);
                    }
            }
        }
        if (hi <= lo) all();  // cannot happen: a producer or receiver touches some column
        R.cb_col0[s] = (i32)lo;
        req((hi - lo) * mb, L, recv ? Lp : L + 1, &R.cb_off[s]);
        bool cbrank = false;
        if (D->split[s] >= 0)
            for (i32 r : D->cb_rank[D->split[s]]) cbrank |= r == rank;
        if (cbrank && D->pd[s] < 0 && owner(s) != rank)  // L21 slabs (a distributed panel: its copy)
            req(mb * S.w(s), L, L + 1, &R.land_off[s]);
    }
    // two placements, the smaller arena kept: the level sweep (best fit, regions born at a
    // level placed largest first), and greedy by size for the regions >= 1 MB (the sweep
    // for the small rest on top); offsets are static either way
    std::vector<int64_t> sweep_off(reqs.size());
    {
        std::vector<Req> r2 = reqs;
        for (size_t i = 0; i < r2.size(); ++i) r2[i].out = &sweep_off[i];
        R.work_total = place(r2, &R.work_live_max);
    }
    const int64_t gsz = place_by_size(reqs, 1 << 17);
    if (gsz < R.work_total)
        R.work_total = gsz;
    else
        for (size_t i = 0; i < reqs.size(); ++i) *reqs[i].out = sweep_off[i];
    if (placed)
        for (const Req& q : reqs) placed->push_back({*q.out, q.size, q.t0, q.t1});
    return SC_OK;
}

// Checks a plan: no two regions of one rank overlap in memory while both are live,
// every region lies inside the work arena, and every full-square CB held where its
// parent runs stays live through the parent's level (its last reader there is the
// parent's assembly or the parent's gathering CB SYRK, the level's last launch: a
// region placed at level Lp must never overlap it).  Returns the number of violations.
int64_t plan_check(const Symbolic& S, int nranks) {
    DistPlan D;
    if (nranks > 1 && dist_plan(S, nranks, D) != SC_OK) return -1;
    int64_t bad = 0;
    for (int r = 0; r < nranks; ++r) {
        RankMem R;
        std::vector<PlacedRegion> pl;
        plan_rank_memory(S, nranks > 1 ? &D : nullptr, r, R, &pl);
        // (offset, birth level) names a region: two regions born at one level at one
        // offset would overlap, which the sweep below counts anyway
        std::map<std::pair<int64_t, int32_t>, int32_t> t1_of;
        for (const PlacedRegion& q : pl) t1_of[{q.off, q.t0}] = q.t1;
        for (i32 s = 0; s < S.ns; ++s) {
            if (R.cb_off[s] < 0 || S.mb(s) <= 0) continue;
            const i32 p = S.sn_parent[s];
            if (nranks > 1 && !D.receives(S, s, r)) continue;
            auto it = t1_of.find({R.cb_off[s], S.level[s]});
            if (it == t1_of.end() || it->second < S.level[p]) ++bad;
        }
        int32_t tmax = 0;
        for (const PlacedRegion& q : pl) {
            tmax = std::max(tmax, q.t1);
            if (q.off < 0 || q.off + q.size > R.work_total) ++bad;
        }
        std::vector<std::vector<int32_t>> at((size_t)tmax + 1);
        for (size_t i = 0; i < pl.size(); ++i)
            for (int32_t t = pl[i].t0; t <= pl[i].t1; ++t) at[t].push_back((int32_t)i);
        for (auto& v : at) {
            std::sort(v.begin(), v.end(), [&](int32_t a, int32_t b) { return pl[a].off < pl[b].off; });
            for (size_t k = 1; k < v.size(); ++k)
                if (pl[v[k - 1]].off + pl[v[k - 1]].size > pl[v[k]].off) ++bad;
        }
    }
    return bad;
}

bool region_addr(const Symbolic& S, const DistPlan* D, const RankMem& R, int kind, int s, int row, int col,
                 int& arena, int64_t& off, int64_t& ld) {
    switch (kind) {
        case R_PANEL:
            if (R.panel_off[s] < 0) return false;
            arena = 0;
            ld = S.sn_m[s];
            off = R.panel_off[s] + (int64_t)col * ld + row;
            return true;
        case R_LAND:
            if (R.land_off[s] < 0) return false;
            arena = 1;
            ld = S.mb(s);
            off = R.land_off[s] + (int64_t)col * ld + row;
            return true;
        case R_CB:
            if (R.cb_off[s] < 0 || col < R.cb_col0[s]) return false;
            arena = 1;
            ld = S.mb(s);
            off = R.cb_base(S, s) + (int64_t)col * ld + row;
            return true;
    }
    (void)D;
    return false;
}

int64_t plan_memory_stats(const Symbolic& S, int nranks, int64_t* panel_doubles, int64_t* work_doubles,
                          int64_t* work_lower_bound) {
    if (nranks < 1) return SC_ERR_ARG;
    DistPlan D;
    if (nranks > 1) {
        const int64_t rc = dist_plan(S, nranks, D);
        if (rc != SC_OK) return rc;
    }
    for (int r = 0; r < nranks; ++r) {
        RankMem R;
        plan_rank_memory(S, nranks > 1 ? &D : nullptr, r, R, nullptr);
        if (panel_doubles) panel_doubles[r] = R.panel_total;
        if (work_doubles) work_doubles[r] = R.work_total;
        if (work_lower_bound) work_lower_bound[r] = R.work_live_max;
    }
    return SC_OK;
}

}  // namespace sc
