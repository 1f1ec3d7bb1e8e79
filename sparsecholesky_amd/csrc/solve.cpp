// Export of the supernodal factor in the reference CSC layout and the triangular
// solves on the GPU; multi-rank handles gather the panels first.
#include "numeric_impl.hpp"

namespace sc {

int64_t numeric_gather(Numeric& N) {
    if (!N.factored) return SC_ERR_STATE;
    const int64_t st = numeric_status(N);
    if (st < 0) return st;
    if (N.owner.empty()) return SC_OK;  // single device: the arena is the factor
    if (N.gather_gen == N.factor_gen) return SC_OK;
    // emulated handles: the hosted arenas, back to back, are the gathered layout
    if (!N.emulated) TRY(dist_gather_panels(N));
    // slabs of distributed panels into their owners' copies
    for (const Numeric::SlabFix& f : N.fix)
        HIP_TRY(hipMemcpy2DAsync(N.gpanel + f.dst, (size_t)f.ld * sizeof(double), N.gpanel + f.src,
                                 (size_t)f.ld * sizeof(double), (size_t)f.rows * sizeof(double), (size_t)f.cols,
                                 hipMemcpyDeviceToDevice, N.stream));
    HIP_TRY(hipStreamSynchronize(N.stream));
    N.gather_gen = N.factor_gen;
    return SC_OK;
}

int64_t numeric_export(Numeric& N, int64_t* Lp, int32_t* Li, double* Lx) {
    if (!N.factored) return SC_ERR_STATE;
    const int64_t st = numeric_status(N);
    if (st < 0) return st;
    const Symbolic& S = *N.S;
    std::vector<double> host;
    if (Lx) {
        TRY(numeric_gather(N));
        const int64_t tot = N.rank_base.back();
        host.resize((size_t)std::max<int64_t>(tot, 1));
        HIP_TRY(hipMemcpy(host.data(), N.gpanel, (size_t)tot * sizeof(double), hipMemcpyDeviceToHost));
    }
    export_L(S, Lx ? host.data() : nullptr, N.gpo.data(), Lp, Li, Lx);
    return st;
}

int64_t numeric_export_cols(Numeric& N, int64_t j0, int64_t j1, int64_t* cp, int32_t* ri, double* rx) {
    if (!N.factored) return SC_ERR_STATE;
    const int64_t st = numeric_status(N);
    if (st < 0) return st;
    const Symbolic& S = *N.S;
    if (j0 < 0 || j1 < j0 || j1 > S.n || !cp) return SC_ERR_ARG;
    HIP_TRY(hipSetDevice(N.device));
    if (rx) TRY(numeric_gather(N));
    // per supernode touched, only the columns [lo, hi] the request needs, each copied
    // once (a column of supernode s holds rows [off, m) of its front: the copy starts
    // at the diagonal of column lo)
    std::vector<int64_t> lo, hi;
    std::vector<int32_t> touched;
    if (rx) {
        lo.assign((size_t)S.ns, INT64_MAX);
        hi.assign((size_t)S.ns, -1);
        for (int64_t j = j0; j < j1; ++j) {
            const int32_t c = S.ipost[j], s = S.sn_of[c];
            const int64_t off = c - S.sn_start[s];
            if (hi[s] < 0) touched.push_back(s);
            lo[s] = std::min(lo[s], off);
            hi[s] = std::max(hi[s], off);
        }
    }
    std::vector<int64_t> base((size_t)(rx ? S.ns : 0), -1);
    std::vector<double> buf;
    for (int32_t s : touched) {
        const int64_t m = S.sn_m[s];
        const int64_t first = lo[s] * m + lo[s], last = hi[s] * m + m;  // [first, last) in the panel
        base[s] = (int64_t)buf.size() - first;
        const size_t at = buf.size();
        buf.resize(at + (size_t)(last - first));
        HIP_TRY(hipMemcpy(buf.data() + at, N.gpanel + N.gpo[s] + first, (size_t)(last - first) * sizeof(double),
                          hipMemcpyDeviceToHost));
    }
    int64_t tot = 0;
    cp[0] = 0;
    for (int64_t j = j0; j < j1; ++j) {
        const int32_t c = S.ipost[j], s = S.sn_of[c];
        const int64_t m = S.sn_m[s], off = c - S.sn_start[s];
        if (ri) {
            const int32_t* rows = S.rows.data() + S.rows_ptr[s];
            for (int64_t t = off; t < m; ++t) {
                ri[tot + t - off] = S.post[rows[t]];
                if (rx) rx[tot + t - off] = buf[(size_t)(base[s] + off * m + t)];
            }
        }
        tot += m - off;
        cp[j - j0 + 1] = tot;
    }
    return tot;
}

// ---------------- triangular solves ----------------
// A = P^T L L^T P (P = etree postorder): c = P b; L y = c (levels up); L^T x = y
// (levels down); x = P^T c.  Per level and 64-column step, over every supernode with
// w > k0: forward, one fused launch (each workgroup solves the diagonal block and
// applies its SOLVE_ROWS rows below); backward, in reverse order, the transposed
// GEMV over the rows below, then the one-wave diagonal solve.
static int64_t solve_build(Numeric& N) {
    const Symbolic& S = *N.S;
    std::vector<std::vector<int32_t>> by_level((size_t)S.nlevels);
    for (int32_t s = 0; s < S.ns; ++s) by_level[S.level[s]].push_back(s);
    std::vector<int2> inv64, inv128;
    std::vector<int4> diag, bwd, fwd;
    std::vector<int32_t> gather;  // per level: the fronts with children (forward gather)
    int64_t max_g = 1;            // most GEMV workgroups in one backward step
    // internal index -> index in the caller's order (postorder, then the fill-reducing
    // permutation when one is in effect)
    std::vector<int32_t> solve_perm(S.post);
    if (!S.perm.empty())
        for (auto& v : solve_perm) v = S.perm[v];
    for (int32_t lev = 0; lev < S.nlevels; ++lev) {
        int maxw = 0;
        for (int32_t s : by_level[lev]) maxw = std::max(maxw, S.w(s));
        const int64_t g_off = (int64_t)gather.size();
        for (int32_t s : by_level[lev])
            if (S.child_ptr[s + 1] > S.child_ptr[s]) gather.push_back(s);
        for (int k0 = 0; k0 < maxw; k0 += SOLVE_NB) {
            Numeric::SolveStep st {};
            st.doff = (int64_t)diag.size();
            st.goff = (int64_t)bwd.size();
            st.foff = (int64_t)fwd.size();
            st.gaoff = g_off;
            st.gacount = k0 == 0 ? (int32_t)((int64_t)gather.size() - g_off) : 0;  // before the level's first step
            for (int32_t s : by_level[lev]) {
                const int w = S.w(s), m = S.sn_m[s];
                if (w <= k0) continue;
                const int rb0 = std::min(w, k0 + SOLVE_NB);
                const int ng = rb0 < m ? (m - rb0 + SOLVE_ROWS - 1) / SOLVE_ROWS : 0;
                diag.push_back(make_int4(s, k0, (int)((int64_t)bwd.size() - st.goff), ng));
                inv64.push_back(make_int2(s, k0));
                if (w > k0 + PNB) {
                    inv64.push_back(make_int2(s, k0 + PNB));
                    inv128.push_back(make_int2(s, k0));
                }
                const int rb = std::min(w, k0 + SOLVE_NB);
                if (rb >= m) fwd.push_back(make_int4(s, k0, -1, 1));
                for (int r0 = rb; r0 < m; r0 += SOLVE_ROWS) {
                    bwd.push_back(make_int4(s, k0, r0, 0));
                    fwd.push_back(make_int4(s, k0, r0, r0 == rb ? 1 : 0));
                }
            }
            st.dcount = (int32_t)((int64_t)diag.size() - st.doff);
            st.gcount = (int32_t)((int64_t)bwd.size() - st.goff);
            st.fcount = (int32_t)((int64_t)fwd.size() - st.foff);
            max_g = std::max<int64_t>(max_g, st.gcount);
            N.solve_steps.push_back(st);
        }
    }
    int64_t rc;
    int32_t* d_rows = nullptr;
    int64_t* d_rows_ptr = nullptr;
    N.n_sinv = (int32_t)inv64.size();
    N.n_sinv2 = (int32_t)inv128.size();
    if ((rc = upload(N, diag, N.d_sdiag)) || (rc = upload(N, inv64, N.d_sinv)) || (rc = upload(N, inv128, N.d_sinv2)) ||
        (rc = upload(N, bwd, N.d_sgemv)) || (rc = upload(N, fwd, N.d_sfwd)) || (rc = upload(N, gather, N.d_sgather)) ||
        (rc = upload(N, S.rows, d_rows)) ||
        (rc = upload(N, S.rows_ptr, d_rows_ptr)) || (rc = upload(N, solve_perm, N.d_post)))
        return rc;
    void* p = nullptr;
    if ((rc = dalloc(N, (size_t)std::max<int64_t>(S.n, 1) * 3 * sizeof(double), p))) return rc;
    N.d_sbuf = (double*)p;
    N.SP.y = N.d_sbuf + 2 * S.n;  // forward result of the fused steps
    N.SP.sn_start = N.R[0].P.sn_start;
    N.SP.sn_m = N.R[0].P.sn_m;
    N.SP.panel_off = N.d_gpo;
    N.SP.rows_ptr = d_rows_ptr;
    N.SP.rows = d_rows;
    N.SP.panel_pool = N.gpanel;
    N.SP.c = N.d_sbuf + S.n;  // internal-order work vector
    // u: each front's contribution-block rows (sum mb); part: the backward GEMV partials
    std::vector<int64_t> u_off((size_t)S.ns);
    int64_t u_tot = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        u_off[s] = u_tot;
        u_tot += S.mb(s);
    }
    int64_t* d_u_off = nullptr;
    if ((rc = upload(N, u_off, d_u_off))) return rc;
    if ((rc = dalloc(N, (size_t)std::max<int64_t>(u_tot, 1) * sizeof(double), p))) return rc;
    N.SP.u = (double*)p;
    N.u_total = u_tot;
    if ((rc = dalloc(N, (size_t)max_g * SOLVE_NB * sizeof(double), p))) return rc;
    N.SP.part = (double*)p;
    N.SP.u_off = d_u_off;
    N.SP.child_ptr = N.R[0].P.child_ptr;
    N.SP.child_list = N.R[0].P.child_list;
    N.SP.rel_ptr = N.R[0].P.rel_ptr;
    N.SP.relind = N.R[0].P.relind;
    N.solve_ready = true;
    return SC_OK;
}

int64_t numeric_solve_device(Numeric& N, const double* d_b, double* d_x) {
    if (!N.factored) return SC_ERR_STATE;
    const int64_t st = numeric_status(N);
    if (st != SC_OK) return st;
    HIP_TRY(hipSetDevice(N.device));
    TRY(numeric_gather(N));  // multi-rank: every rank solves with the whole factor
    if (N.solve_ready && N.SP.panel_pool != N.gpanel) {
        N.SP.panel_pool = N.gpanel;  // gathered buffer allocated after the plan was built
        if (N.solve_gexec) (void)hipGraphExecDestroy(N.solve_gexec);
        if (N.solve_graph) (void)hipGraphDestroy(N.solve_graph);
        N.solve_gexec = nullptr;
        N.solve_graph = nullptr;
    }
    if (!N.solve_ready) TRY(solve_build(N));
    const int64_t n = N.S->n;
    if (n == 0) return SC_OK;
    hipStream_t s0 = N.stream;
    // the graph reads b from and writes x to the handle's own vector io = d_sbuf[0, n),
    // so it is captured once, whatever buffers the caller passes
    double* io = N.d_sbuf;
    auto sweeps = [&]() -> hipError_t {
        hipError_t e = launch_permute(N.SP.c, io, N.d_post, n, false, s0);
        if (e == hipSuccess) e = hipMemsetAsync(N.SP.u, 0, (size_t)std::max<int64_t>(N.u_total, 1) * sizeof(double), s0);
        // forward: per level the children's u gathered, then one fused launch per step
        // (y to SP.y), then y -> c
        for (size_t i = 0; e == hipSuccess && i < N.solve_steps.size(); ++i) {
            const Numeric::SolveStep& t = N.solve_steps[i];
            e = launch_solve_fwd_gather(N.SP, N.d_sgather + t.gaoff, t.gacount, s0);
            if (e == hipSuccess) e = launch_solve_fwd(N.SP, N.d_sfwd + t.foff, t.fcount, s0);
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(N.SP.c, N.SP.y, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s0);
        for (size_t i = N.solve_steps.size(); e == hipSuccess && i-- > 0;) {
            const Numeric::SolveStep& t = N.solve_steps[i];
            e = launch_solve_gemv(N.SP, N.d_sgemv + t.goff, t.gcount, s0);
            if (e == hipSuccess) e = launch_solve_diag(N.SP, N.d_sdiag + t.doff, t.dcount, s0);
        }
        if (e == hipSuccess) e = launch_permute(io, N.SP.c, N.d_post, n, true, s0);
        return e;
    };
    if (!N.solve_gexec && !N.solve_eager) {
        // ~700 dependent steps per sweep at 128^3: replayed as one hipGraph
        HIP_TRY(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
        hipError_t e = sweeps();
        hipGraph_t g = nullptr;
        hipError_t e2 = hipStreamEndCapture(s0, &g);
        HIP_TRY(e);
        HIP_TRY(e2);
        N.solve_graph = g;
        HIP_TRY(hipGraphInstantiate(&N.solve_gexec, g, nullptr, nullptr, 0));
    }
    if (N.inv_gen != N.factor_gen) {  // inverses of the diagonal blocks, once per factorization
        HIP_TRY(launch_solve_inv(N.SP, N.d_sinv, N.n_sinv, N.d_sinv2, N.n_sinv2, s0));
        N.inv_gen = N.factor_gen;
    }
    const size_t nb = (size_t)n * sizeof(double);
    if (d_b != io) HIP_TRY(hipMemcpyAsync(io, d_b, nb, hipMemcpyDeviceToDevice, s0));
    if (N.solve_eager)
        HIP_TRY(sweeps());
    else
        HIP_TRY(hipGraphLaunch(N.solve_gexec, s0));
    if (d_x != io) HIP_TRY(hipMemcpyAsync(d_x, io, nb, hipMemcpyDeviceToDevice, s0));
    HIP_TRY(hipStreamSynchronize(s0));
    return SC_OK;
}

int64_t numeric_solve_host(Numeric& N, const double* b, double* x) {
    if (!N.factored) return SC_ERR_STATE;
    const int64_t st = numeric_status(N);
    if (st != SC_OK) return st;
    HIP_TRY(hipSetDevice(N.device));
    if (!N.solve_ready) TRY(solve_build(N));
    const size_t nb = (size_t)N.S->n * sizeof(double);
    if (nb == 0) return SC_OK;
    HIP_TRY(hipMemcpy(N.d_sbuf, b, nb, hipMemcpyHostToDevice));
    TRY(numeric_solve_device(N, N.d_sbuf, N.d_sbuf));
    HIP_TRY(hipMemcpy(x, N.d_sbuf, nb, hipMemcpyDeviceToHost));
    return SC_OK;
}

}  // namespace sc
