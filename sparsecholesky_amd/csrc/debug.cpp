// Debug and microbenchmark hooks (sc_debug_syrk, sc_debug_bench): the SYRK kernel on
// caller data, kernel ceilings on synthetic operands.
#include "numeric_impl.hpp"

namespace sc {

int64_t debug_syrk(double* dC, int ldc, const double* dA, int lda, int M, int Nn, int K) {
    GemmTask t {};
    t.C = dC;
    t.A = dA;
    t.ldc = ldc;
    t.lda = lda;
    t.M = M;
    t.N = Nn;
    t.K = K;
    const int bt = SYRK_BT_SMALL;
    std::vector<int2> tiles;
    append_tiles(tiles, 0, M, Nn, bt);
    xcd_order(tiles.data(), (int64_t)tiles.size());
    GemmTask* d = nullptr;
    int2* dt = nullptr;
    if (hipMalloc(&d, sizeof(GemmTask)) != hipSuccess) return SC_ERR_DEVMEM;
    if (hipMalloc(&dt, std::max<size_t>(tiles.size(), 1) * sizeof(int2)) != hipSuccess) {
        (void)hipFree(d);
        return SC_ERR_DEVMEM;
    }
    hipError_t e = hipMemcpy(d, &t, sizeof(t), hipMemcpyHostToDevice);
    if (e == hipSuccess && !tiles.empty())
        e = hipMemcpy(dt, tiles.data(), tiles.size() * sizeof(int2), hipMemcpyHostToDevice);
    // K <= 128: the lean instance (as the schedule's default syrk_lean_kmax picks it)
    if (e == hipSuccess) e = launch_syrk(d, dt, (int)tiles.size(), bt, 0, nullptr, 0, GatherTab {}, K <= 128);
    hipError_t e2 = hipDeviceSynchronize();
    (void)hipFree(d);
    (void)hipFree(dt);
    return (e == hipSuccess && e2 == hipSuccess) ? SC_OK : SC_ERR_HIP;
}

// Panel-kernel microbenchmarks on one synthetic front (m = M rows, w = 64):
// which 2 = POTRF (us per launch), 3 = TRSM with the fused POTRF (us per launch).
static int64_t bench_panel(int which, int M, int reps, double* out) {
    const int w = PNB;
    if (M < w || reps < 1) return SC_ERR_ARG;
    const size_t nel = (size_t)M * w;
    std::vector<double> h(nel + PNB, 0.0);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return (double)(x >> 11) / 9007199254740992.0 - 0.5;
    };
    for (int j = 0; j < w; ++j)
        for (int i = 0; i < M; ++i) h[(size_t)j * M + i] = (i == j) ? 64.0 : rnd();
    int32_t hs[2] = {0, w}, hm[1] = {M};
    int64_t ho[2] = {0, (int64_t)nel};
    std::vector<TrsmTask> tr;
    for (int r0 = w; r0 < M; r0 += TRSM_ROWS) tr.push_back(TrsmTask {0, 0, r0, M, 1});
    int2 pt = make_int2(0, 0);
    void *d_pan = nullptr, *d_ref = nullptr, *d_s = nullptr, *d_m = nullptr, *d_o = nullptr, *d_info = nullptr,
         *d_pt = nullptr, *d_tr = nullptr, *d_arr = nullptr;
    const size_t bytes = (nel + PNB) * sizeof(double);
    int64_t rc = SC_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&d_pan, bytes) || hipMalloc(&d_ref, bytes) || hipMalloc(&d_s, 8) || hipMalloc(&d_m, 4) ||
        hipMalloc(&d_o, 16) || hipMalloc(&d_info, 4) || hipMalloc(&d_pt, 8) ||
        hipMalloc(&d_tr, std::max<size_t>(1, tr.size()) * sizeof(TrsmTask)) || hipMalloc(&d_arr, 4) ||
        hipMemset(d_arr, 0, 4) || hipEventCreate(&e0) ||
        hipEventCreate(&e1)) {
        rc = SC_ERR_DEVMEM;
    } else {
        (void)hipMemcpy(d_ref, h.data(), bytes, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_s, hs, 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_m, hm, 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_o, ho, 16, hipMemcpyHostToDevice);
        (void)hipMemset(d_info, 0, 4);
        (void)hipMemcpy(d_pt, &pt, 8, hipMemcpyHostToDevice);
        if (!tr.empty()) (void)hipMemcpy(d_tr, tr.data(), tr.size() * sizeof(TrsmTask), hipMemcpyHostToDevice);
        DevPlan P {};
        P.sn_start = (const int32_t*)d_s;
        P.sn_m = (const int32_t*)d_m;
        P.panel_off = (const int64_t*)d_o;
        P.info = (int32_t*)d_info;
        P.panel_pool = (double*)d_pan;
        const int nt = (int)tr.size();
        (void)hipMemcpy(d_pan, d_ref, bytes, hipMemcpyDeviceToDevice);
        (void)launch_potrf_diag(P, (const int2*)d_pt, 1, nullptr);
        double tot = 0.0;
        for (int r = 0; r < reps + 1; ++r) {
            if (which == 2) (void)hipMemcpy(d_pan, d_ref, bytes, hipMemcpyDeviceToDevice);
            (void)hipEventRecord(e0, nullptr);
            if (which == 2)
                (void)launch_potrf_diag(P, (const int2*)d_pt, 1, nullptr);
            else
                (void)launch_trsm_panel(P, (const TrsmTask*)d_tr, nt, nullptr, false, (int32_t*)d_arr);
            (void)hipEventRecord(e1, nullptr);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r > 0) tot += ms;
        }
        *out = 1e3 * tot / reps;
        if (hipGetLastError() != hipSuccess) rc = SC_ERR_HIP;
    }
    for (void* p : {d_pan, d_ref, d_s, d_m, d_o, d_info, d_pt, d_tr, d_arr})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

// Dispatch-contention probe (the chain-vs-lookahead question of DESIGN.md 5): a "hog" --
// the 128-tile panel-update SYRK (TAG 0, trickle epilogue) on an M x M triangle, K deep,
// on a low-priority stream -- and a "chain" of nchain dependent fused POTRF + TRSM
// launches on a chain_rows x 64 front, on the high-priority stream.  mode bit 0: the hog
// stream is CU-masked (every mask_stride-th CU off); bit 1: the hog is replayed from a
// captured hipGraph; bit 2: the chain too (its own graph).  out[0] chain alone, out[1] hog
// alone, out[2] chain under the hog (first chain start -> last chain end), out[3] hog
// under the chain, out[4] both (wall), all ms; out[5] CUs the hog may use.
int64_t debug_contention(int M, int K, int chain_rows, int nchain, int mode, int mask_stride, double* out) {
    for (int i = 0; i < 8; ++i) out[i] = 0.0;
    if (M < 128 || K < 16 || chain_rows < 128 || nchain < 1 || nchain > 4096) return SC_ERR_ARG;
    int64_t rc = SC_OK;
    hipStream_t s_chain = nullptr, s_hog = nullptr;
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    hipDeviceProp_t prop {};
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    int used = ncu;
    if (hipStreamCreateWithPriority(&s_chain, hipStreamNonBlocking, prio_hi) != hipSuccess) return SC_ERR_HIP;
    if (mode & 1) {
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        used = 0;
        for (int c = 0; c < ncu; ++c)
            if (mask_stride <= 0 || c % mask_stride != 0) {
                mask[c / 32] |= 1u << (c % 32);
                ++used;
            }
        if (hipExtStreamCreateWithCUMask(&s_hog, (uint32_t)mask.size(), mask.data()) != hipSuccess) rc = SC_ERR_HIP;
    } else if (hipStreamCreateWithPriority(&s_hog, hipStreamNonBlocking, prio_lo) != hipSuccess) {
        rc = SC_ERR_HIP;
    }
    out[5] = used;
    // hog operands
    const size_t na = (size_t)M * K, nc = (size_t)M * M;
    void *bufA = nullptr, *bufC = nullptr, *bt = nullptr, *bl = nullptr;
    int ntiles = 0;
    // chain front (as bench_panel)
    const int w = PNB, Mc = chain_rows;
    const size_t nel = (size_t)Mc * w;
    void *d_pan = nullptr, *d_s = nullptr, *d_m = nullptr, *d_o = nullptr, *d_info = nullptr, *d_tr = nullptr,
         *d_arr = nullptr;
    std::vector<TrsmTask> tr;
    for (int r0 = w; r0 < Mc; r0 += TRSM_ROWS) tr.push_back(TrsmTask {0, 0, r0, Mc, 1});
    hipEvent_t ev[8] = {};
    hipGraph_t g_hog = nullptr, g_chain = nullptr;
    hipGraphExec_t x_hog = nullptr, x_chain = nullptr;
    DevPlan P {};
    auto hog_direct = [&]() { return launch_syrk((GemmTask*)bt, (int2*)bl, ntiles, SYRK_BT_LARGE, 0, s_hog); };
    auto hog = [&]() {
        if (x_hog) return hipGraphLaunch(x_hog, s_hog);
        return hog_direct();
    };
    auto chain_direct = [&]() {
        hipError_t e = hipSuccess;
        for (int i = 0; i < nchain && e == hipSuccess; ++i)
            e = launch_trsm_panel(P, (const TrsmTask*)d_tr, (int)tr.size(), s_chain, false, (int32_t*)d_arr);
        return e;
    };
    auto chain = [&]() { return x_chain ? hipGraphLaunch(x_chain, s_chain) : chain_direct(); };
    auto elapsed = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ev[a], ev[b]);
        return (double)ms;
    };
    if (rc == SC_OK) {
        if (hipMalloc(&bufA, na * 8) || hipMalloc(&bufC, nc * 8) || hipMalloc(&d_pan, (nel + PNB) * 8) ||
            hipMalloc(&d_s, 8) || hipMalloc(&d_m, 4) || hipMalloc(&d_o, 16) || hipMalloc(&d_info, 4) ||
            hipMalloc(&d_tr, tr.size() * sizeof(TrsmTask)) || hipMalloc(&d_arr, 4))
            rc = SC_ERR_DEVMEM;
    }
    if (rc == SC_OK) {
        (void)launch_fill_random((double*)bufA, (int64_t)na, nullptr);
        (void)launch_fill_random((double*)bufC, (int64_t)nc, nullptr);
        GemmTask t {};
        t.C = (double*)bufC;
        t.A = (const double*)bufA;
        t.ldc = M;
        t.lda = M;
        t.M = M;
        t.N = M;
        t.K = K;
        std::vector<int2> tiles;
        append_tiles(tiles, 0, M, M, SYRK_BT_LARGE);
        xcd_order(tiles.data(), (int64_t)tiles.size());
        ntiles = (int)tiles.size();
        (void)hipMalloc(&bt, sizeof(GemmTask));
        (void)hipMalloc(&bl, tiles.size() * sizeof(int2));
        (void)hipMemcpy(bt, &t, sizeof(t), hipMemcpyHostToDevice);
        (void)hipMemcpy(bl, tiles.data(), tiles.size() * sizeof(int2), hipMemcpyHostToDevice);
        // chain front: a diagonally dominant 64-column panel
        std::vector<double> h(nel + PNB, 0.0);
        for (int j = 0; j < w; ++j)
            for (int i = 0; i < Mc; ++i) h[(size_t)j * Mc + i] = (i == j) ? 64.0 : 1e-3 * ((i * 7 + j * 3) % 11);
        int32_t hs[2] = {0, w}, hm[1] = {Mc};
        int64_t ho[2] = {0, (int64_t)nel};
        (void)hipMemcpy(d_pan, h.data(), h.size() * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_s, hs, 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_m, hm, 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_o, ho, 16, hipMemcpyHostToDevice);
        (void)hipMemset(d_info, 0, 4);
        (void)hipMemset(d_arr, 0, 4);
        (void)hipMemcpy(d_tr, tr.data(), tr.size() * sizeof(TrsmTask), hipMemcpyHostToDevice);
        P.sn_start = (const int32_t*)d_s;
        P.sn_m = (const int32_t*)d_m;
        P.panel_off = (const int64_t*)d_o;
        P.info = (int32_t*)d_info;
        P.panel_pool = (double*)d_pan;
        for (auto& e : ev) (void)hipEventCreate(&e);
        (void)hipDeviceSynchronize();
        if (mode & 2) {  // the hog as a captured graph
            (void)hipStreamBeginCapture(s_hog, hipStreamCaptureModeThreadLocal);
            (void)hog_direct();
            (void)hipStreamEndCapture(s_hog, &g_hog);
            if (!g_hog || hipGraphInstantiate(&x_hog, g_hog, nullptr, nullptr, 0) != hipSuccess) rc = SC_ERR_HIP;
        }
        if (rc == SC_OK && (mode & 4)) {
            (void)hipStreamBeginCapture(s_chain, hipStreamCaptureModeThreadLocal);
            (void)chain_direct();
            (void)hipStreamEndCapture(s_chain, &g_chain);
            if (!g_chain || hipGraphInstantiate(&x_chain, g_chain, nullptr, nullptr, 0) != hipSuccess) rc = SC_ERR_HIP;
        }
    }
    if (rc == SC_OK) {
        // warm up both, then alone, alone, together (best of 3 for each)
        (void)hog();
        (void)chain();
        (void)hipDeviceSynchronize();
        double best[5] = {1e30, 1e30, 1e30, 1e30, 1e30};
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(ev[0], s_chain);
            (void)chain();
            (void)hipEventRecord(ev[1], s_chain);
            (void)hipDeviceSynchronize();
            best[0] = std::min(best[0], elapsed(0, 1));
            (void)hipEventRecord(ev[2], s_hog);
            (void)hog();
            (void)hipEventRecord(ev[3], s_hog);
            (void)hipDeviceSynchronize();
            best[1] = std::min(best[1], elapsed(2, 3));
            // together: the hog first (its workgroups fill the GPU), the chain right after
            (void)hipEventRecord(ev[2], s_hog);
            (void)hog();
            (void)hipEventRecord(ev[3], s_hog);
            (void)hipStreamWaitEvent(s_chain, ev[2], 0);
            (void)hipEventRecord(ev[0], s_chain);
            (void)chain();
            (void)hipEventRecord(ev[1], s_chain);
            (void)hipDeviceSynchronize();
            best[2] = std::min(best[2], elapsed(0, 1));
            best[3] = std::min(best[3], elapsed(2, 3));
            best[4] = std::min(best[4], std::max(elapsed(2, 1), elapsed(2, 3)));
        }
        for (int i = 0; i < 5; ++i) out[i] = best[i];
        if (hipGetLastError() != hipSuccess) rc = SC_ERR_HIP;
    }
    (void)hipDeviceSynchronize();
    if (x_hog) (void)hipGraphExecDestroy(x_hog);
    if (g_hog) (void)hipGraphDestroy(g_hog);
    if (x_chain) (void)hipGraphExecDestroy(x_chain);
    if (g_chain) (void)hipGraphDestroy(g_chain);
    for (void* p : {bufA, bufC, bt, bl, d_pan, d_s, d_m, d_o, d_info, d_tr, d_arr})
        if (p) (void)hipFree(p);
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    if (s_chain) (void)hipStreamDestroy(s_chain);
    if (s_hog) (void)hipStreamDestroy(s_hog);
    return rc;
}

// which 0: register-only fp64 MFMA peak probe (M blocks of 4 waves, K iterations,
// arg accumulators); 1 / 5: the SYRK kernel on an M x M triangle, K deep, tile arg
// (64 / 128), with / without the XCD tile order; 2 / 3: bench_panel.  TFLOP/s or us.
int64_t debug_bench(int which, int M, int K, int reps, int arg, double* tflops) {
    *tflops = 0.0;
    if (which == 2 || which == 3) return bench_panel(which, M, reps, tflops);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return SC_ERR_HIP;
    double flops = 0.0;
    void *bufA = nullptr, *bufC = nullptr, *bt = nullptr, *bl = nullptr;
    int64_t rc = SC_OK;
    if (which == 0) {
        if (hipMalloc(&bufC, 8 * (size_t)std::max(M, 1)) != hipSuccess) return SC_ERR_DEVMEM;
        (void)launch_mfma_peak((double*)bufC, M, K, arg, nullptr);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, nullptr);
        for (int r = 0; r < reps; ++r) (void)launch_mfma_peak((double*)bufC, M, K, arg, nullptr);
        (void)hipEventRecord(e1, nullptr);
        flops = 2.0 * 16 * 16 * 4 * (double)arg * K * M * 4.0 * reps;  // 4 waves per block
    } else {
        const size_t na = (size_t)M * K, nc = (size_t)M * M;
        if (hipMalloc(&bufA, na * 8) != hipSuccess || hipMalloc(&bufC, nc * 8) != hipSuccess) {
            rc = SC_ERR_DEVMEM;
            goto done;
        }
        (void)launch_fill_random((double*)bufA, (int64_t)na, nullptr);
        (void)launch_fill_random((double*)bufC, (int64_t)nc, nullptr);
        {
            GemmTask t {};
            t.C = (double*)bufC;
            t.A = (const double*)bufA;
            t.ldc = M;
            t.lda = M;
            t.M = M;
            t.N = M;
            t.K = K;
            const int tb = arg == 128 ? 128 : 64;
            std::vector<int2> tiles;
            append_tiles(tiles, 0, M, M, tb);
            if (which != 5) xcd_order(tiles.data(), (int64_t)tiles.size());
            (void)hipMalloc(&bt, sizeof(GemmTask));
            (void)hipMalloc(&bl, tiles.size() * sizeof(int2));
            (void)hipMemcpy(bt, &t, sizeof(t), hipMemcpyHostToDevice);
            (void)hipMemcpy(bl, tiles.data(), tiles.size() * sizeof(int2), hipMemcpyHostToDevice);
            (void)launch_syrk((GemmTask*)bt, (int2*)bl, (int)tiles.size(), tb, 1, nullptr);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0, nullptr);
            for (int r = 0; r < reps; ++r) (void)launch_syrk((GemmTask*)bt, (int2*)bl, (int)tiles.size(), tb, 1, nullptr);
            (void)hipEventRecord(e1, nullptr);
            flops = (double)M * (M + 1.0) * K * reps;
        }
    }
    {
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        *tflops = flops / (ms * 1e-3) / 1e12;
        if (hipGetLastError() != hipSuccess) rc = SC_ERR_HIP;
    }
done:
    if (bufA) (void)hipFree(bufA);
    if (bufC) (void)hipFree(bufC);
    if (bt) (void)hipFree(bt);
    if (bl) (void)hipFree(bl);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

}  // namespace sc
