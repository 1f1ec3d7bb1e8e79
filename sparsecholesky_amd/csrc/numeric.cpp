// Device numeric factorization handle: plan upload, memory pools, launch of the
// static schedule (schedule.cpp) eagerly or as one captured hipGraph, status and
// per-launch timing.
//
// Layout in HBM (one allocation each, doubles):
//   panel pool  sum_s m_s*w_s      L panels, column-major, ld = m_s (the output)
//   work arena  liveness-planned contribution blocks (memplan.cpp), ld = mb_s
#include "numeric_impl.hpp"

#include <chrono>

namespace sc {

int64_t dalloc(Numeric& N, size_t bytes, void*& p) {
    p = nullptr;
    hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 8));
    if (e != hipSuccess) {
        N.err = std::string("hipMalloc(pool ") + std::to_string(bytes) + " B): " + hipGetErrorString(e);
        return SC_ERR_DEVMEM;
    }
    N.allocs.push_back(p);
    N.dev_bytes += (int64_t)std::max<size_t>(bytes, 8);
    return SC_OK;
}

int64_t numeric_create(const Symbolic& S, int device, Numeric*& out, std::string& err) {
    out = nullptr;
    Numeric* Np = new (std::nothrow) Numeric();
    if (!Np) return SC_ERR_NOMEM;
    int64_t rc = numeric_init(*Np, S, device);
    if (rc != SC_OK) {
        err = Np->err;
        numeric_free(Np);
        return rc;
    }
    out = Np;
    return SC_OK;
}

// Gathered panel layout: every rank's panel arena back to back (rank_base), each as
// plan_rank_panels lays it out; a supernode's factor is its owner's copy (gpo).  The
// slabs of a distributed panel that other ranks factored are copied into the owner's
// copy after the exchange (fix).
static void panel_layout(Numeric& N, const Symbolic& S, int nranks) {
    const DistPlan* D = N.owner.empty() ? nullptr : &N.D;
    std::vector<std::vector<int64_t>> po((size_t)nranks);
    N.rank_base.assign((size_t)nranks + 1, 0);
    for (int r = 0; r < nranks; ++r) N.rank_base[r + 1] = N.rank_base[r] + plan_rank_panels(S, D, r, po[r]);
    N.gpo.assign((size_t)S.ns, 0);
    for (int32_t s = 0; s < S.ns; ++s) {
        const int r = D ? D->owner[s] : 0;
        N.gpo[s] = N.rank_base[r] + po[r][s];
    }
    N.fix.clear();
    if (!D) return;
    for (size_t q = 0; q < D->pd_s.size(); ++q) {
        const int32_t s = D->pd_s[q];
        const int m = S.sn_m[s], w = S.w(s);
        for (int k = 0; k < (int)D->slab_rank[q].size(); ++k) {
            const int r = D->slab_rank[q][k];
            if (r == D->owner[s]) continue;
            const int k0 = k * D->nbo, k1 = std::min(w, k0 + D->nbo);
            Numeric::SlabFix f {};
            f.src = N.rank_base[r] + po[r][s] + (int64_t)k0 * m + k0;
            f.dst = N.gpo[s] + (int64_t)k0 * m + k0;
            f.ld = m;
            f.rows = m - k0;
            f.cols = k1 - k0;
            N.fix.push_back(f);
        }
    }
}

int64_t numeric_init(Numeric& N, const Symbolic& S, int device) {
    N.S = &S;
    auto fail = [&](int64_t rc) { return rc; };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        N.err = "no HIP device available";
        return fail(SC_ERR_HIP);
    }
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) device = 0;
    }
    if (device >= ndev) {
        N.err = "device index out of range";
        return fail(SC_ERR_ARG);
    }
    N.device = device;
    if (hipSetDevice(device) != hipSuccess) {
        N.err = "hipSetDevice failed";
        return fail(SC_ERR_HIP);
    }
    const bool multi = !N.owner.empty();
    // critical path (assembly, POTRF/TRSM chain, next-slab updates) on the high
    // priority stream; the overlapped trailing updates on the low priority one
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    bool ok = hipStreamCreateWithPriority(&N.stream, hipStreamNonBlocking, prio_hi) == hipSuccess;
    if (ok) ok = hipStreamCreateWithPriority(&N.stream2, hipStreamNonBlocking, prio_lo) == hipSuccess;
    // comm stream only on multi-rank handles: one more stream on the device costs 13.5%
    // under hipGraph replay (569 -> 649 ms at 128^3, any priority, any
    // GPU_MAX_HW_QUEUES) though nothing runs on it; eager runs (multi-rank) see 0.5%.
    if (ok && multi) ok = hipStreamCreateWithPriority(&N.stream3, hipStreamNonBlocking, prio_hi) == hipSuccess;
    if (!ok) {
        N.err = "hipStreamCreate failed";
        return fail(SC_ERR_HIP);
    }
    N.use_graph = S.opt.use_graph != 0;
    const int32_t ns = S.ns;
    int64_t rc;
    static_assert(ASM_ROWS == kAsmRows, "assembly row tile");
    static_assert(ASM_COLS == kAsmCols, "assembly column block");
    for (int32_t s = 0; s < S.ns; ++s)
        if (S.sn_m[s] >= (1 << 20)) {  // assembly task encoding: 16-bit column block index
            N.err = "front with >= 2^20 rows is not supported";
            return fail(SC_ERR_NOTIMPL);
        }
    // ---- memory plan of the hosted ranks ----
    N.R.clear();
    if (!multi) {
        N.R.resize(1);
    } else if (N.emulated) {
        N.R.resize((size_t)N.nranks);
    } else {
        N.R.resize(1);
    }
    for (size_t v = 0; v < N.R.size(); ++v) {
        const int r = (multi && N.emulated) ? (int)v : (multi ? N.rank : 0);
        plan_rank_memory(S, multi ? &N.D : nullptr, r, N.R[v]);
    }
    panel_layout(N, S, multi ? N.nranks : 1);
    // ---- shared plan arrays ----
    DevPlan P0 {};
    int32_t *d_sn_start, *d_sn_m, *d_child_ptr, *d_child_list, *d_relind, *d_apos, *d_relbnd, *d_colbnd, *d_tilebnd;
    int64_t *d_rel_ptr, *d_aptr, *d_asrc, *d_rbptr, *d_cbkptr, *d_tbptr;
    if ((rc = upload(N, S.sn_start, d_sn_start)) || (rc = upload(N, S.sn_m, d_sn_m)) ||
        (rc = upload(N, S.child_ptr, d_child_ptr)) || (rc = upload(N, S.child_list, d_child_list)) ||
        (rc = upload(N, S.rel_ptr, d_rel_ptr)) || (rc = upload(N, S.relind, d_relind)) ||
        (rc = upload(N, S.rb_ptr, d_rbptr)) || (rc = upload(N, S.rel_bnd, d_relbnd)) ||
        (rc = upload(N, S.cbk_ptr, d_cbkptr)) || (rc = upload(N, S.col_bnd, d_colbnd)) ||
        (rc = upload(N, S.tb_ptr, d_tbptr)) || (rc = upload(N, S.tile_bnd, d_tilebnd)) ||
        (rc = upload(N, S.a_ptr, d_aptr)) || (rc = upload(N, S.a_pos, d_apos)) ||
        (rc = upload(N, S.a_src, d_asrc)) || (rc = upload(N, N.gpo, N.d_gpo)))
        return fail(rc);
    P0.sn_start = d_sn_start;
    P0.sn_m = d_sn_m;
    P0.child_ptr = d_child_ptr;
    P0.child_list = d_child_list;
    P0.rel_ptr = d_rel_ptr;
    P0.relind = d_relind;
    P0.rb_ptr = d_rbptr;
    P0.rel_bnd = d_relbnd;
    P0.cbk_ptr = d_cbkptr;
    P0.col_bnd = d_colbnd;
    P0.tb_ptr = d_tbptr;
    P0.tile_bnd = d_tilebnd;
    P0.a_ptr = d_aptr;
    P0.a_pos = d_apos;
    P0.a_src = d_asrc;
    void* p = nullptr;
    if ((rc = dalloc(N, 64, p))) return fail(rc);
    N.d_info = (int32_t*)p;
    P0.info = N.d_info;
    if (hipHostMalloc((void**)&N.h_info, sizeof(int32_t) * 16, hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess) {
        N.err = "hipHostMalloc failed";
        return fail(SC_ERR_NOMEM);
    }
    // ---- pools: the hosted ranks' panel arenas back to back in one allocation (so an
    // emulated handle's allocation IS the gathered factor), work arenas likewise ----
    int64_t ptot = 0, wtot = 0;
    for (const RankMem& R : N.R) {
        ptot += R.panel_total;
        wtot += R.work_total;
    }
    if ((rc = dalloc(N, (size_t)ptot * sizeof(double), p))) return fail(rc);
    double* pbase = (double*)p;
    if ((rc = dalloc(N, (size_t)std::max<int64_t>(wtot, 1) * sizeof(double), p))) return fail(rc);
    double* wbase = (double*)p;
    int64_t po = 0, wo = 0;
    for (RankMem& R : N.R) {
        R.P = P0;
        R.P.panel_pool = pbase + po;
        R.P.cb_pool = wbase + wo;
        po += R.panel_total;
        wo += R.work_total;
        int64_t* dp = nullptr;
        if ((rc = upload(N, R.panel_off, dp))) return fail(rc);
        R.P.panel_off = dp;
        // the kernels address a CB as the full square from its (virtual) origin
        std::vector<int64_t> base((size_t)S.ns, 0);
        for (int32_t s = 0; s < S.ns; ++s)
            if (R.cb_off[s] >= 0) base[s] = R.cb_base(S, s);
        if ((rc = upload(N, base, dp))) return fail(rc);
        R.P.cb_off = dp;
    }
    if (!multi || N.emulated) N.gpanel = pbase;  // gathered layout == the arenas

    SchedBuild B;
    if ((rc = build_schedule(N, B))) return fail(rc);
    CommBuild& cbld = B.cb;
    if (cbld.stage_total > 0) {  // multi-rank: packed staging slots of the hosted ranks' messages
        if ((rc = dalloc(N, (size_t)cbld.stage_total * sizeof(double), p))) return fail(rc);
        N.staging = (double*)p;
        for (size_t q = 0; q < N.msgs.size(); ++q) {
            if (cbld.msg_slot[q] >= 0) N.msgs[q].buf = N.staging + cbld.msg_slot[q];
            if (cbld.msg_src_slot[q] >= 0) N.msgs[q].src_buf = N.staging + cbld.msg_src_slot[q];
        }
        for (size_t q = 0; q < cbld.copies.size(); ++q) cbld.copies[q].b = N.staging + cbld.copy_slot[q];
    }
    if ((rc = upload(N, cbld.copies, N.d_copy)) || (rc = upload(N, cbld.ctiles, N.d_ctiles))) return fail(rc);
    N.stamp_of.assign(N.sched.size(), -1);
    int nstamp = 0;
    for (size_t i = 0; i < N.sched.size(); ++i)
        if (N.sched[i].kind == L_CB) N.stamp_of[i] = nstamp++;
    if ((rc = dalloc(N, (size_t)std::max(1, 2 * nstamp) * sizeof(uint64_t), p))) return fail(rc);
    N.d_stamps = (uint64_t*)p;
    N.sync_ev.assign((size_t)N.n_sync_events, nullptr);
    for (auto& e : N.sync_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            N.err = "hipEventCreate failed";
            return fail(SC_ERR_HIP);
        }
    {
        ChainDesc* dd = nullptr;
        uint32_t* dr = nullptr;
        if ((rc = upload(N, B.cdesc, dd)) || (rc = upload(N, B.crelp, dr))) return fail(rc);
        N.CP.desc = dd;
        N.CP.relp = dr;
        N.n_chain = (int64_t)B.cdesc.size();
        if ((rc = dalloc(N, (size_t)std::max<int64_t>(B.chain_init, 1) * sizeof(double), p))) return fail(rc);
        N.CP.init = (double*)p;
        TinyFront* tf = nullptr;
        int2 *t1 = nullptr, *t2 = nullptr, *t3 = nullptr;
        if ((rc = upload(N, B.tfr, tf)) || (rc = upload(N, B.ta, t1)) || (rc = upload(N, B.tph, t2)) ||
            (rc = upload(N, B.tpr, t3)))
            return fail(rc);
        N.TP.fr = tf;
        N.TP.a = t1;
        N.TP.ph = t2;
        N.TP.pr = t3;
        N.TP.nf = (int32_t)B.tfr.size();
        N.TP.na = (int32_t)B.ta.size();
        N.TP.nph = (int32_t)B.tph.size();
        N.TP.npr = (int32_t)B.tpr.size();
        N.TP.lds = B.tiny_lds;
        N.TP.nax = (int32_t)std::min<int64_t>(S.nnzA_in, INT32_MAX);
        N.TP.npan = (int32_t)std::min<int64_t>(N.R[0].panel_total, INT32_MAX);
        // a tiny-tree handle is one launch: the kernel owns the status word (initial
        // value, failures, the copy to pinned host memory), so a factorization is one
        // dispatch with no reset / copy around it
        if (N.sched.size() == 1 && N.sched[0].kind == L_SMALL && N.sched[0].big >= 2) {
            void* dp = nullptr;
            if (hipHostGetDevicePointer(&dp, N.h_info, 0) != hipSuccess) {
                N.err = "hipHostGetDevicePointer failed";
                return fail(SC_ERR_HIP);
            }
            N.TP.host_info = (int32_t*)dp;
        }
    }
    // single-rank handles other than the tiny path: the status word published by a
    // one-thread kernel at the end of the schedule, d_info armed once here and re-armed by
    // that kernel (multi-rank handles keep the copy: the status is reduced over ranks)
    if (!N.TP.host_info && N.owner.empty()) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, N.h_info, 0) != hipSuccess || hipMemset(N.d_info, 0x7f, sizeof(int32_t)) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) {
            N.err = "status word setup failed";
            return fail(SC_ERR_HIP);
        }
        N.status_dp = (int32_t*)dp;
    }
    B.asml.resize(B.asmv.size(), make_int2(0, INT32_MAX));
    {  // the CB gather's segment tables
        int64_t* dgb = nullptr;
        GSeg* dgs = nullptr;
        if ((rc = upload(N, B.gblk, dgb)) || (rc = upload(N, B.gseg, dgs))) return fail(rc);
        N.gtab.blk = dgb;
        N.gtab.seg = dgs;
    }
    if ((rc = upload(N, B.small, N.d_small)) || (rc = upload(N, B.asmv, N.d_asm)) || (rc = upload(N, B.asml, N.d_asml)) ||
        (rc = upload(N, B.potrf, N.d_potrf)) || (rc = upload(N, B.trsm, N.d_trsm)) ||
        (rc = upload(N, std::vector<int32_t>(B.trsm.size() + 1, 0), N.d_arrive)) ||
        (rc = upload(N, B.gemm, N.d_gemm)) || (rc = upload(N, B.tiles, N.d_tiles)))
        return fail(rc);
    (void)ns;
    return SC_OK;
}


static hipStream_t stream_of(const Numeric& N, int strm) {
    return strm == 2 ? N.stream3 : strm == 1 ? N.stream2 : N.stream;
}

static hipError_t launch_one(Numeric& N, const Launch& L, const double* d_Ax) {
    hipStream_t st = stream_of(N, L.strm);  // every kind on the stream its schedule entry names
    switch (L.kind) {
        case L_RECORD:
            return hipEventRecord(N.sync_ev[L.count], st);
        case L_WAIT:
            return hipStreamWaitEvent(st, N.sync_ev[L.count], 0);
        case L_SMALL:
            if (L.big == 1) return launch_front_chain(N.R[L.vr].P, N.CP, (int)L.off, L.count, L.maxm, d_Ax, st);
            if (L.big == 2) return launch_tiny_tree(N.R[L.vr].P, N.TP, L.maxm, d_Ax, st);
            if (L.big == 3) return launch_tiny_dense(N.R[L.vr].P, N.TP, L.maxm, d_Ax, st);
            return launch_front_small(N.R[L.vr].P, N.d_small + L.off, L.count, L.maxm, false, d_Ax, st);
        case L_ASM:
            // epi = 1: distributed-assembly launch, column limits parallel to the tasks
            return launch_assemble_large(N.R[L.vr].P, N.d_asm + L.off, L.count, d_Ax, st, L.big != 0,
                                         L.epi ? N.d_asml + L.off : nullptr);
        case L_POTRF:
            return launch_potrf_diag(N.R[L.vr].P, N.d_potrf + L.off, L.count, st);
        case L_TRSM:
            return launch_trsm_panel(N.R[L.vr].P, N.d_trsm + L.off, L.count, st, L.big != 0, N.d_arrive,
                                     L.epi);
        case L_PANEL:
        case L_CB:
        {
            GatherTab gt = N.gtab;
            gt.info = N.d_info;
            return launch_syrk(N.d_gemm + L.off, N.d_tiles + L.toff, L.count, L.bt, L.kind == L_CB ? 1 : 0, st, L.epi,
                               gt, L.lean != 0, L.pf != 0);
        }
        case L_COMM:
            return comm_launch(N, L);
    }
    return hipErrorInvalidValue;
}

static int64_t enqueue_all(Numeric& N, const double* d_Ax, int prof) {
    // tiny path: the kernel writes the status; single-rank: the publish kernel at the end
    const bool own_status = N.TP.host_info != nullptr || N.status_dp != nullptr;
    if (!own_status) HIP_TRY(hipMemsetAsync(N.d_info, 0x7f, sizeof(int32_t), N.stream));
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& L = N.sched[i];
        const bool timed = prof == 1 && L.kind < L_RECORD;
        const bool stamped = prof == 2 && N.stamp_of[i] >= 0;
        hipStream_t st = stream_of(N, L.strm);
        if (timed) HIP_TRY(hipEventRecord(N.ev[2 * i], st));
        if (stamped) HIP_TRY(launch_stamp(N.d_stamps + 2 * N.stamp_of[i], st));
        HIP_TRY(launch_one(N, L, d_Ax));
        if (stamped) HIP_TRY(launch_stamp(N.d_stamps + 2 * N.stamp_of[i] + 1, st));
        if (timed) HIP_TRY(hipEventRecord(N.ev[2 * i + 1], st));
    }
    // the status word to pinned host memory on the main stream, which every other
    // stream has joined by now: the status read needs one stream sync, no extra copy
    if (!own_status) HIP_TRY(hipMemcpyAsync(N.h_info, N.d_info, sizeof(int32_t), hipMemcpyDeviceToHost, N.stream));
    if (N.status_dp) HIP_TRY(launch_status_publish(N.d_info, N.status_dp, N.stream));
    return SC_OK;
}

// Duration (ms) of launch i in the last profiled factorization, or -1.
static double launch_ms(Numeric& N, size_t i, const std::vector<uint64_t>& stamps) {
    if (N.profile == 1) {
        if (N.ev.size() != 2 * N.sched.size() || N.sched[i].kind >= L_RECORD) return -1.0;
        float t = 0.f;
        if (hipEventElapsedTime(&t, N.ev[2 * i], N.ev[2 * i + 1]) != hipSuccess) return -1.0;
        return t;
    }
    if (N.profile == 2 && N.stamp_of[i] >= 0 && !stamps.empty()) {
        const int q = N.stamp_of[i];
        return (double)(stamps[2 * q + 1] - stamps[2 * q]) * 1e-5;  // 100 MHz ticks -> ms
    }
    return -1.0;
}

static std::vector<uint64_t> read_stamps(Numeric& N) {
    std::vector<uint64_t> h;
    if (N.profile != 2 || !N.d_stamps) return h;
    int n = 0;
    for (int32_t v : N.stamp_of) n = std::max(n, v + 1);
    h.resize((size_t)2 * n);
    if (n && hipMemcpy(h.data(), N.d_stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        h.clear();
    return h;
}

int64_t numeric_factor(Numeric& N, const double* d_Ax, bool sync) {
    HIP_TRY(hipSetDevice(N.device));
    // tiny path: an earlier factorization still in flight (async, status never read) may
    // store its status word after the host re-arms it below, and that word would then be
    // read as this factorization's status -- drain it first
    const bool pinned = N.TP.host_info || N.status_dp;
    if (pinned && N.factored && !N.status_valid) HIP_TRY(hipStreamSynchronize(N.stream));
    N.status_valid = false;
    N.last_Ax = d_Ax;
    if (N.profile == 1 && N.ev.size() != 2 * N.sched.size()) {
        for (auto e : N.ev) (void)hipEventDestroy(e);
        N.ev.assign(2 * N.sched.size(), nullptr);
        for (auto& e : N.ev) HIP_TRY(hipEventCreate(&e));
    }
    // tiny path (the kernel stores the status word to pinned host memory itself): mark
    // it pending, so that numeric_status can wait on the word instead of the stream
    if (pinned) *(volatile int32_t*)N.h_info = Numeric::STATUS_PENDING;
    if (N.use_graph && N.profile != 1) {
        // the whole level schedule (both streams, and the timing events when
        // profiling) as one hipGraph, re-captured only when its inputs change
        if (!N.gexec || N.graph_Ax != d_Ax || N.graph_profiled != N.profile) {
            if (N.gexec) {
                (void)hipGraphExecDestroy(N.gexec);
                N.gexec = nullptr;
            }
            if (N.graph) {
                (void)hipGraphDestroy(N.graph);
                N.graph = nullptr;
            }
            HIP_TRY(hipStreamBeginCapture(N.stream, hipStreamCaptureModeThreadLocal));
            int64_t rc = enqueue_all(N, d_Ax, N.profile);
            hipGraph_t g = nullptr;
            hipError_t e2 = hipStreamEndCapture(N.stream, &g);
            if (rc != SC_OK) return rc;
            HIP_TRY(e2);
            N.graph = g;
            HIP_TRY(hipGraphInstantiate(&N.gexec, N.graph, nullptr, nullptr, 0));
            N.graph_Ax = d_Ax;
            N.graph_profiled = N.profile;
        }
        HIP_TRY(hipGraphLaunch(N.gexec, N.stream));
    } else {
        TRY(enqueue_all(N, d_Ax, N.profile));
    }
    N.factored = true;
    N.factor_gen++;
    if (sync) return numeric_status(N);
    return SC_OK;
}

int64_t numeric_status(Numeric& N) {
    if (!N.factored) return SC_ERR_STATE;
    if (N.status_valid) return N.status;
    HIP_TRY(hipSetDevice(N.device));
    // tiny path, unprofiled: the kernel's last act is the system-scope release store of
    // the status word (every panel store of its one wave is visible before it), so the
    // host polls the pinned word -- a few microseconds sooner than the stream's
    // completion signal; after ~2 ms of polling it falls back to the stream sync
    bool seen = false;
    if ((N.TP.host_info || N.status_dp) && N.profile == 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t it = 1;; ++it) {
            if (*(volatile int32_t*)N.h_info != Numeric::STATUS_PENDING) {
                seen = true;
                break;
            }
            if ((it & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        }
    }
    // every stream's work is joined into the main stream before the status copy
    if (!seen) HIP_TRY(hipStreamSynchronize(N.stream));
    int32_t info = *(volatile int32_t*)N.h_info;
    if (!N.owner.empty() && !N.emulated && !N.dry_comm) {  // one rank per process: the global minimum
        const int64_t rc = dist_min_info(N, info);
        if (rc != SC_OK) return rc;
    }
    if (info == 0x7f7f7f7f || info <= 0)
        N.status = 0;
    else
        N.status = (int64_t)N.S->post[info - 1] + 1;
    N.status_valid = true;
    if (N.profile == 1) {
        std::memset(N.phase_ms, 0, sizeof(N.phase_ms));
        hipEvent_t first = nullptr, last = nullptr;
        for (size_t i = 0; i < N.sched.size(); ++i) {
            if (N.sched[i].kind >= L_RECORD) continue;
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, N.ev[2 * i], N.ev[2 * i + 1]));
            int slot = 0;
            switch (N.sched[i].kind) {
                case L_SMALL: slot = 2; break;
                case L_ASM: slot = 3; break;
                case L_POTRF: slot = 4; break;
                case L_TRSM: slot = 5; break;
                case L_PANEL: slot = 6; break;
                case L_CB: slot = 7; break;
                case L_COMM: slot = 1; break;
            }
            N.phase_ms[slot] += ms;
            if (N.sched[i].strm == 0) {
                if (!first) first = N.ev[2 * i];
                last = N.ev[2 * i + 1];
            }
        }
        if (first) {
            float tot = 0.f;
            HIP_TRY(hipEventElapsedTime(&tot, first, last));
            N.phase_ms[0] = tot;
        }
    }
    return N.status;
}

// Wall time per assembly-tree level (first main-stream launch start to last end).
int64_t numeric_level_times(Numeric& N, double* ms, int nl) {
    if (N.profile != 1 || !N.status_valid) return SC_ERR_STATE;
    const int L = N.S->nlevels;
    std::vector<int> first(L, -1), last(L, -1);
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& l = N.sched[i];
        if (l.kind >= L_RECORD || l.strm != 0) continue;
        if (first[l.level] < 0) first[l.level] = (int)i;
        last[l.level] = (int)i;
    }
    for (int v = 0; v < L && v < nl; ++v) {
        float t = 0.f;
        if (first[v] >= 0) HIP_TRY(hipEventElapsedTime(&t, N.ev[2 * first[v]], N.ev[2 * last[v] + 1]));
        ms[v] = t;
    }
    return L;
}

// Per-launch trace of the last profiled factorization: kind, level, stream, ms, flops.
int64_t numeric_launch_trace(Numeric& N, int32_t* kind, int32_t* level, int32_t* strm, double* ms, double* flops,
                             int64_t cap) {
    if (N.profile != 1 || !N.status_valid) return SC_ERR_STATE;
    int64_t n = 0;
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& l = N.sched[i];
        if (l.kind >= L_RECORD) continue;
        if (n < cap && kind) {
            float t = 0.f;
            HIP_TRY(hipEventElapsedTime(&t, N.ev[2 * i], N.ev[2 * i + 1]));
            kind[n] = l.kind;
            level[n] = l.level;
            strm[n] = l.strm;
            ms[n] = t;
            flops[n] = l.flops;
        }
        ++n;
    }
    return n;
}

// Start / end (ms from the first main-stream launch) of every launch of the last
// profiled factorization, the launch kind and, for comm launches, the comm step.
int64_t numeric_launch_times(Numeric& N, double* t0, double* t1, int32_t* kind, int32_t* step, int32_t* strm,
                             int64_t cap) {
    if (N.profile != 1 || !N.status_valid) return SC_ERR_STATE;
    hipEvent_t origin = nullptr;
    for (size_t i = 0; i < N.sched.size() && !origin; ++i)
        if (N.sched[i].kind < L_RECORD && N.sched[i].strm == 0) origin = N.ev[2 * i];
    int64_t n = 0;
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& l = N.sched[i];
        if (l.kind >= L_RECORD) continue;
        if (n < cap && t0) {
            float a = 0.f, b = 0.f;
            HIP_TRY(hipEventElapsedTime(&a, origin, N.ev[2 * i]));
            HIP_TRY(hipEventElapsedTime(&b, origin, N.ev[2 * i + 1]));
            t0[n] = a;
            t1[n] = b;
            kind[n] = l.kind;
            step[n] = l.kind == L_COMM ? l.step : -1;
            strm[n] = l.strm;
        }
        ++n;
    }
    return n;
}

int64_t numeric_timing(Numeric& N, double* t, int nt) {
    if (N.profile != 1 || !N.status_valid) return SC_ERR_STATE;
    for (int i = 0; i < nt && i < 8; ++i) t[i] = N.phase_ms[i];
    return SC_OK;
}

// CB SYRK launches are split by w >= 256; wmin selects them (0: all CB launches, -1:
// the panel-update launches instead, -2: the CB launches on 128 x 128 tiles with the
// trickle epilogue, i.e. exactly the syrk_mfma_kernel<128,2,4,1,0,0> dispatches a kernel
// trace lists)
static bool syrk_selected(const Launch& L, int wmin) {
    if (L.kind != (wmin == -1 ? L_PANEL : L_CB)) return false;
    if (wmin >= 256 && !L.big) return false;
    if (wmin == -2 && (L.bt != SYRK_BT_LARGE || L.epi)) return false;
    return true;
}

int64_t numeric_syrk_bytes(Numeric& N, int wmin, double* bytes) {
    double b = 0.0;
    for (const Launch& L : N.sched)
        if (syrk_selected(L, wmin)) b += L.bytes;
    *bytes = b;
    return SC_OK;
}

int64_t numeric_syrk_stats(Numeric& N, int wmin, double* flops, double* ms, int64_t* launches) {
    double fl = 0.0, t = 0.0;
    int64_t cnt = 0;
    bool have_t = N.status_valid && N.profile != 0;
    const std::vector<uint64_t> stamps = read_stamps(N);
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& L = N.sched[i];
        if (!syrk_selected(L, wmin)) continue;
        fl += L.flops;
        ++cnt;
        if (have_t) {
            const double e = launch_ms(N, i, stamps);
            if (e < 0)
                have_t = false;
            else
                t += e;
        }
    }
    if (flops) *flops = fl;
    if (ms) *ms = have_t ? t : -1.0;
    if (launches) *launches = cnt;
    return SC_OK;
}


void numeric_free(Numeric* Np) {
    if (!Np) return;
    Numeric& N = *Np;
    (void)hipSetDevice(N.device);
    if (N.stream) (void)hipStreamSynchronize(N.stream);
    comm_destroy(N);
    if (N.solve_gexec) (void)hipGraphExecDestroy(N.solve_gexec);
    if (N.solve_graph) (void)hipGraphDestroy(N.solve_graph);
    if (N.gexec) (void)hipGraphExecDestroy(N.gexec);
    if (N.graph) (void)hipGraphDestroy(N.graph);
    for (auto e : N.ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : N.sync_ev)
        if (e) (void)hipEventDestroy(e);
    for (void* p : N.allocs) (void)hipFree(p);
    if (N.h_info) (void)hipHostFree(N.h_info);
    if (N.d_Ax_owned) (void)hipFree(N.d_Ax_owned);
    if (N.stream) (void)hipStreamDestroy(N.stream);
    if (N.stream2) (void)hipStreamDestroy(N.stream2);
    if (N.stream3) (void)hipStreamDestroy(N.stream3);
    delete Np;
}

int64_t numeric_chain_stamps(Numeric& N, int enable, uint64_t* out, int64_t cap) {
    const int64_t cnt = 8 * N.n_chain;
    if (enable) {
        if (!N.CP.stamps && cnt > 0) {
            void* p = nullptr;
            TRY(dalloc(N, (size_t)cnt * sizeof(uint64_t), p));
            N.CP.stamps = (uint64_t*)p;
        }
        return cnt;
    }
    if (!N.CP.stamps) return 0;
    HIP_TRY(hipStreamSynchronize(N.stream));
    if (out && cap > 0)
        HIP_TRY(hipMemcpy(out, N.CP.stamps, (size_t)std::min(cap, cnt) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return cnt;
}

}  // namespace sc
