// Multi-GPU plan: proportional subtree-to-GPU mapping of the assembly tree
// (SURVEY.md 8e).  Every supernode gets one owner rank; a contribution block
// crosses GPUs only where a child and its parent have different owners (the
// subtree-merge fronts).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "numeric.hpp"
#include "symbolic.hpp"

namespace sc {

static void subtree_work(const Symbolic& S, std::vector<double>& work) {
    work.assign((size_t)S.ns, 0.0);
    for (i32 s = 0; s < S.ns; ++s) {  // children precede parents (postorder)
        const double m = S.sn_m[s], w = S.w(s);
        double f = 0.0;
        // sum_{t<w} (m-t)^2, closed form
        f = w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0;
        work[s] += f;
        if (S.sn_parent[s] >= 0) work[S.sn_parent[s]] += work[s];
    }
}

// Recursive proportional mapping: the ranks [r0, r1) are a continuous interval of
// processor mass split among the children in proportion to subtree work; a child
// whose share rounds to one rank owns its whole subtree there.
i64 dist_owner_map(const Symbolic& S, int nranks, i32* owner, double* work_per_rank) {
    std::vector<double> work;
    subtree_work(S, work);
    std::vector<i32> own((size_t)S.ns, 0);
    struct Item {
        i32 s;
        double a, b;  // processor interval
    };
    std::vector<Item> stack;
    // roots share the whole machine
    std::vector<i32> roots;
    double W = 0.0;
    for (i32 s = 0; s < S.ns; ++s)
        if (S.sn_parent[s] < 0) {
            roots.push_back(s);
            W += work[s];
        }
    {
        double cum = 0.0;
        for (i32 r : roots) {
            const double a = nranks * (W > 0 ? cum / W : 0.0);
            cum += work[r];
            const double b = nranks * (W > 0 ? cum / W : 1.0);
            stack.push_back({r, a, b});
        }
    }
    auto whole_subtree = [&](i32 s, i32 rank) {
        // subtree of s = contiguous supernode range ending at s (postorder)
        std::vector<i32> st {s};
        while (!st.empty()) {
            i32 v = st.back();
            st.pop_back();
            own[v] = rank;
            for (i32 q = S.child_ptr[v]; q < S.child_ptr[v + 1]; ++q) st.push_back(S.child_list[q]);
        }
    };
    const double eps = 1e-9;
    // multi-rank (merge) fronts, placed after the subtrees: least-loaded rank of
    // their interval, children before parents
    std::vector<std::pair<i32, std::pair<i32, i32>>> shared;
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        i32 lo = (i32)std::floor(it.a + eps);
        i32 hi = std::max(lo + 1, (i32)std::ceil(it.b - eps));
        lo = std::min(lo, nranks - 1);
        hi = std::min(hi, nranks);
        if (hi - lo <= 1) {
            whole_subtree(it.s, lo);
            continue;
        }
        own[it.s] = lo;
        shared.push_back({it.s, {lo, hi}});
        double Wc = 0.0;
        for (i32 q = S.child_ptr[it.s]; q < S.child_ptr[it.s + 1]; ++q) Wc += work[S.child_list[q]];
        double cum = 0.0;
        for (i32 q = S.child_ptr[it.s]; q < S.child_ptr[it.s + 1]; ++q) {
            i32 c = S.child_list[q];
            const double a = it.a + (it.b - it.a) * (Wc > 0 ? cum / Wc : 0.0);
            cum += work[c];
            const double b = it.a + (it.b - it.a) * (Wc > 0 ? cum / Wc : 1.0);
            stack.push_back({c, a, b});
        }
    }
    {
        std::vector<double> load((size_t)nranks, 0.0);
        std::vector<char> is_shared((size_t)S.ns, 0);
        for (auto& sh : shared) is_shared[sh.first] = 1;
        for (i32 s = 0; s < S.ns; ++s) {
            if (is_shared[s]) continue;
            const double m = S.sn_m[s], w = S.w(s);
            load[own[s]] += w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0;
        }
        std::sort(shared.begin(), shared.end());  // postorder: children first
        for (auto& sh : shared) {
            const i32 s = sh.first, lo = sh.second.first, hi = sh.second.second;
            i32 best = lo;
            for (i32 r = lo + 1; r < hi; ++r)
                if (load[r] < load[best]) best = r;
            own[s] = best;
            const double m = S.sn_m[s], w = S.w(s);
            load[best] += w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0;
        }
    }
    if (owner) std::memcpy(owner, own.data(), sizeof(i32) * (size_t)S.ns);
    if (work_per_rank) {
        std::fill(work_per_rank, work_per_rank + nranks, 0.0);
        for (i32 s = 0; s < S.ns; ++s) {
            const double m = S.sn_m[s], w = S.w(s);
            work_per_rank[own[s]] += w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0;
        }
    }
    return SC_OK;
}

// Messages of `rank` in global order (level of the sending child, then child id):
// a child's CB goes from owner(child) to owner(parent) after the child's level.
i64 dist_schedule(const Symbolic& S, int nranks, int rank, i32* level, i32* peer, i64* bytes, i32* is_send,
                  i64 cap) {
    std::vector<i32> own((size_t)S.ns);
    dist_owner_map(S, nranks, own.data(), nullptr);
    std::vector<i32> order((size_t)S.ns);
    for (i32 s = 0; s < S.ns; ++s) order[s] = s;
    std::stable_sort(order.begin(), order.end(), [&](i32 a, i32 b) { return S.level[a] < S.level[b]; });
    i64 cnt = 0;
    for (i32 c : order) {
        const i32 p = S.sn_parent[c];
        if (p < 0 || own[c] == own[p]) continue;
        const bool snd = own[c] == rank, rcv = own[p] == rank;
        if (!snd && !rcv) continue;
        if (level && cnt < cap) {
            level[cnt] = S.level[c];
            peer[cnt] = snd ? own[p] : own[c];
            const i64 mb = S.mb(c);
            bytes[cnt] = mb * mb * (i64)sizeof(double);
            is_send[cnt] = snd ? 1 : 0;
        }
        ++cnt;
    }
    return cnt;
}

// ---------------- RCCL transport ----------------
static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");

i64 dist_unique_id(void* id128) {
    if (!id128) return SC_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SC_ERR_COMM;
    std::memcpy(id128, &id, sizeof(id));
    return SC_OK;
}

// All CB transfers of one level as one RCCL group on the library stream: both
// sides post them in the same global order (level, then child id), so the
// point-to-point matching per peer pair is consistent.
hipError_t comm_launch(Numeric& N, const Launch& L) {
    if (!N.comm) return hipErrorInvalidValue;
    ncclComm_t comm = (ncclComm_t)N.comm;
    if (ncclGroupStart() != ncclSuccess) return hipErrorUnknown;
    for (int64_t q = L.off; q < L.off + L.count; ++q) {
        const Msg& g = N.msgs[q];
        ncclResult_t r = g.is_send ? ncclSend(g.buf, (size_t)g.count, ncclDouble, g.peer, comm, N.stream)
                                   : ncclRecv(g.buf, (size_t)g.count, ncclDouble, g.peer, comm, N.stream);
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

void comm_destroy(Numeric& N) {
    if (N.comm) {
        (void)ncclCommDestroy((ncclComm_t)N.comm);
        N.comm = nullptr;
    }
}

// Real multi-GPU handle: this process is `rank` of `nranks` (one GPU each).
// Every rank allocates the full pools (288 GB HBM per GPU holds them) but only
// computes the supernodes the proportional mapping gives it.
i64 numeric_create_dist(const Symbolic& S, int device, int rank, int nranks, const void* id128, Numeric*& out,
                        std::string& err) {
    out = nullptr;
    Numeric* Np = new (std::nothrow) Numeric();
    if (!Np) return SC_ERR_NOMEM;
    Numeric& N = *Np;
    N.rank = rank;
    N.nranks = nranks;
    N.owner.resize((size_t)S.ns);
    dist_owner_map(S, nranks, N.owner.data(), nullptr);
    if (!id128) {
        // in-process emulation of all ranks (shared pools, no transfers)
        N.virt_ranks = nranks;
    } else if (nranks > 1) {
        int dev = device;
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipSetDevice(dev) != hipSuccess) {
            err = "hipSetDevice failed";
            delete Np;
            return SC_ERR_HIP;
        }
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof(id));
        ncclComm_t comm = nullptr;
        ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
        if (r != ncclSuccess) {
            err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            delete Np;
            return SC_ERR_COMM;
        }
        N.comm = comm;
    }
    i64 rc = numeric_init(N, S, device);
    if (rc != SC_OK) {
        err = N.err;
        numeric_free(Np);
        return rc;
    }
    out = Np;
    return SC_OK;
}

}  // namespace sc
