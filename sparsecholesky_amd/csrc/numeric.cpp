// Device numeric factorization driver.
//
// Layout in HBM (one allocation each, doubles):
//   panel pool  sum_s m_s*w_s      L panels, column-major, ld = m_s (the output)
//   CB pool     sum_s (m_s-w_s)^2  contribution blocks, column-major, ld = mb_s
// Schedule: assembly-tree levels, leaves first.  Per level:
//   small fronts (m <= small_front_max): one fused kernel per LDS size bucket;
//   large fronts: assemble, then per 64-column step potrf -> trsm -> panel
//   SYRK update (inner 64-wide within a 256-wide slab, outer at slab ends),
//   then one CB SYRK with K = w (the north-star MFMA kernel).
#include "numeric.hpp"

#include <algorithm>
#include <climits>
#include <cstring>

namespace sc {

// CB launches with every K below this use the batched SYRK epilogue (measured per
// level at 128^3: K <= 121 gains, K = 226 loses)
#ifndef SC_EPI_KMAX
#define SC_EPI_KMAX 192
#endif

#define HIP_TRY(x)                                                                \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            N.err = std::string(#x) + ": " + hipGetErrorString(e_);               \
            return SC_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

template <class T>
static int64_t upload(Numeric& N, const std::vector<T>& v, T*& dptr) {
    dptr = nullptr;
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(T);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        N.err = std::string("hipMalloc(plan): ") + hipGetErrorString(e);
        return SC_ERR_DEVMEM;
    }
    N.allocs.push_back(p);
    N.dev_bytes += (int64_t)bytes;
    if (!v.empty()) {
        e = hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            N.err = std::string("hipMemcpy(plan): ") + hipGetErrorString(e);
            return SC_ERR_HIP;
        }
    }
    dptr = (T*)p;
    return SC_OK;
}

static int64_t dalloc(Numeric& N, size_t bytes, void*& p) {
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

#define TRY(x)                        \
    do {                              \
        int64_t r_ = (x);             \
        if (r_ != SC_OK) return r_;   \
    } while (0)

static int bucket_of(int m) {
    if (m <= 32) return 32;
    if (m <= 64) return 64;
    if (m <= 96) return 96;
    return 128;
}

// register width of the small-front POTRF / TRSM (w > 64: right-looking path)
static int wbucket_of(int w) {
    if (w <= 16) return 16;
    if (w <= 32) return 32;
    if (w <= 64) return 64;
    return 128;
}

// Build the static launch schedule (host).  Task pointers into the pools are
// final device addresses, so the schedule can be replayed or graph-captured.
void append_tiles(std::vector<int2>& out, int task, int M, int N, int bt, int G) {
    const int TM = (M + bt - 1) / bt, TN = (N + bt - 1) / bt;
    for (int sj = 0; sj < TN; sj += G)
        for (int si = sj; si < TM; si += G)
            for (int tj = sj; tj < std::min(TN, sj + G); ++tj)
                for (int ti = std::max(si, tj); ti < std::min(TM, si + G); ++ti)
                    out.push_back(make_int2(task, (ti << 16) | tj));
}

void xcd_order(int2* tiles, int64_t n) {
    if (n <= 8) return;
    std::vector<int2> src(tiles, tiles + n);
    const int64_t q = n / 8, r = n % 8;
    for (int64_t b = 0; b < n; ++b) {
        const int64_t x = b % 8, j = b / 8;
        tiles[b] = src[x * q + std::min(x, r) + j];
    }
}

// Work-balanced XCD order of a multi-task launch (workgroup b runs on XCD b % 8,
// each XCD has its own L2).  The tiles arrive task-contiguous, each task in
// supertile order.  Every task is cut into 8 contiguous chunks, one per XCD, with
// the remainders dealt round robin across tasks so that each XCD receives exactly
// its ceil((n - x) / 8) tiles; an XCD walks its chunks in decreasing K (longest
// tiles first).  With one task this is xcd_order.
void xcd_order_tasks(int2* tiles, int64_t n, const GemmTask* tasks, int ntasks) {
    if (n <= 8) return;
    std::vector<int64_t> beg((size_t)ntasks + 1, 0);
    for (int64_t i = 0; i < n; ++i) beg[(size_t)tiles[i].x + 1]++;
    for (int t = 0; t < ntasks; ++t) beg[t + 1] += beg[t];
    std::vector<int> ord((size_t)ntasks);
    for (int t = 0; t < ntasks; ++t) ord[t] = t;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return tasks[a].K > tasks[b].K; });
    std::vector<std::vector<int2>> per(8);
    int p = 0;
    for (int t : ord) {
        const int64_t nt = beg[t + 1] - beg[t], base = nt / 8, rem = nt % 8;
        int64_t off = beg[t];
        for (int x = 0; x < 8; ++x) {
            const int64_t cnt = base + (((x - p + 8) % 8) < rem ? 1 : 0);
            per[x].insert(per[x].end(), tiles + off, tiles + off + cnt);
            off += cnt;
        }
        p = (int)((p + rem) % 8);
    }
    for (int x = 0; x < 8; ++x)
        if ((int64_t)per[x].size() != (n - x + 7) / 8) return xcd_order(tiles, n);  // cannot happen
    for (int64_t b = 0; b < n; ++b) tiles[b] = per[b % 8][b / 8];
}

// Staging slots of the hosted ranks' messages (patched to device addresses once
// the staging pool is allocated): slot < 0 = the buffer is the region itself.
struct CommBuild {
    std::vector<Copy2D> copies;
    std::vector<int64_t> copy_slot;
    std::vector<int2> ctiles;
    std::vector<int64_t> msg_slot, msg_src_slot;
    int64_t stage_total = 0;
};

struct SchedBuild {
    std::vector<ChainDesc> cdesc;
    std::vector<uint32_t> crelp;
    int64_t chain_init = 0;  // doubles of the chained fronts' packed images
    std::vector<TinyFront> tfr;  // tiny-tree plan
    std::vector<int2> ta, tph, tpr;
    int32_t tiny_lds = 0;
    std::vector<int32_t> small;
    std::vector<int2> asmv, potrf, inv;
    std::vector<TrsmTask> trsm;
    std::vector<int4> tall;
    std::vector<GemmTask> gemm;
    std::vector<int2> tiles;
    CommBuild cb;
};

static int64_t build_schedule(Numeric& N, SchedBuild& B) {
    const Symbolic& S = *N.S;
    std::vector<int32_t>& small = B.small;
    std::vector<int2>& asmv = B.asmv;
    std::vector<int2>& potrf = B.potrf;
    std::vector<TrsmTask>& trsm = B.trsm;
    std::vector<GemmTask>& gemm = B.gemm;
    std::vector<int2>& tiles = B.tiles;
    CommBuild& cbld = B.cb;
    const int NBO = std::max(PNB, (S.opt.panel_nb_outer / PNB) * PNB);
    std::vector<std::vector<int32_t>> by_level((size_t)S.nlevels);
    for (int32_t s = 0; s < S.ns; ++s) by_level[S.level[s]].push_back(s);
    // multi-rank plan lookups
    const DistPlan& D = N.D;
    const bool multi = !N.owner.empty();
    const DistPlan* Dp = multi ? &D : nullptr;
    auto is_split = [&](int32_t s) { return multi && D.split[s] >= 0; };
    auto is_dpanel = [&](int32_t s) { return multi && D.pd[s] >= 0; };
    std::vector<int32_t> hosted_of((size_t)std::max(N.nranks, 1), -1);  // rank -> index into N.R
    for (size_t v = 0; v < N.R.size(); ++v) hosted_of[N.R[v].rank] = (int32_t)v;
    std::vector<int32_t> init_step, slab_step0, early_step0, deliver_step((size_t)S.nlevels, -1);
    std::vector<std::vector<int32_t>> slab_step;  // distributed panels: step of slab k, -1 = none
    std::vector<std::vector<int>> early_ev((size_t)S.ns);  // sender: event after each CB column group
    std::vector<int64_t> step_beg;
    std::vector<char> emitted;
    if (multi) {
        init_step.assign((size_t)S.ns, -1);
        slab_step0.assign((size_t)S.ns, -1);
        slab_step.assign((size_t)S.ns, std::vector<int32_t>());
        for (size_t q = 0; q < D.pd_s.size(); ++q) slab_step[D.pd_s[q]].assign(D.slab_rank[q].size(), -1);
        early_step0.assign((size_t)S.ns, -1);
        for (int32_t id = 0; id < (int32_t)D.steps.size(); ++id) {
            const DistStep& t = D.steps[id];
            if (t.kind == STEP_INIT) init_step[t.s] = id;
            if (t.kind == STEP_SLAB && t.k == 0) slab_step0[t.s] = id;
            if (t.kind == STEP_SLAB && D.pd[t.s] >= 0) slab_step[t.s][t.k] = id;
            if (t.kind == STEP_DELIVER && t.s < 0) deliver_step[t.level] = id;
            if (t.kind == STEP_DELIVER && t.s >= 0 && t.k == 0) early_step0[t.s] = id;
        }
        step_beg.assign(D.steps.size() + 1, 0);
        for (const DistMsg& g : D.msgs) step_beg[g.step + 1]++;
        for (size_t i = 0; i < D.steps.size(); ++i) step_beg[i + 1] += step_beg[i];
        emitted.assign(D.steps.size(), 0);
    }
    // device address of logical element (row, col) of a region on hosted rank v
    auto addr = [&](int v, int kind, int s, int row, int col, int64_t& ld) -> double* {
        int arena = 0;
        int64_t off = 0;
        if (!region_addr(S, Dp, N.R[v], kind, s, row, col, arena, off, ld)) return nullptr;
        return (arena == 0 ? N.R[v].P.panel_pool : N.R[v].P.cb_pool) + off;
    };
    auto push_gemm_launch = [&](int kind, int level, const std::vector<GemmTask>& tasks, int big,
                                double flops, int strm = 0) {
        if (tasks.empty()) return;
        Launch L {};
        L.kind = kind;
        L.level = level;
        L.strm = strm;
        L.off = (int64_t)gemm.size();
        // 128x128 tiles on 8 waves when every task is at least 256 wide (random data,
        // 16384 x 4096: 61 vs 52 TF/s for 64x64); 64x64 on 4 waves for narrow updates
        int minN = INT32_MAX, maxK = 0;
        for (auto& t : tasks) {
            minN = std::min(minN, (int)t.N);
            maxK = std::max(maxK, (int)t.K);
        }
        const bool wide = minN >= 256;
        L.bt = (S.opt.syrk_tile == 128 || (S.opt.syrk_tile == 0 && wide)) ? SYRK_BT_LARGE : SYRK_BT_SMALL;
        // batched C epilogue on the critical path (main-stream panel updates) and where
        // K is short enough that the epilogue dominates a tile (CB of levels 4-7 at
        // 128^3); deep-K CB updates and the lookahead stream keep the trickle epilogue
        L.epi = (kind == L_PANEL && strm == 0) || (kind == L_CB && maxK < SC_EPI_KMAX);
        L.toff = (int64_t)tiles.size();
        for (size_t q = 0; q < tasks.size(); ++q) {
            append_tiles(tiles, (int)q, tasks[q].M, tasks[q].N, L.bt);
            gemm.push_back(tasks[q]);
        }
        L.count = (int32_t)((int64_t)tiles.size() - L.toff);
        xcd_order_tasks(tiles.data() + L.toff, L.count, tasks.data(), (int)tasks.size());
        L.ntasks = (int32_t)tasks.size();
        L.big = big;
        L.flops = flops;
        N.sched.push_back(L);
    };
    // cross-stream dependencies: record an event on a stream / make a stream wait on it
    auto push_record = [&](int strm) -> int {
        Launch L {};
        L.kind = L_RECORD;
        L.strm = strm;
        L.count = N.n_sync_events++;
        N.sched.push_back(L);
        return L.count;
    };
    auto push_wait = [&](int strm, int ev) {
        Launch L {};
        L.kind = L_WAIT;
        L.strm = strm;
        L.count = ev;
        N.sched.push_back(L);
    };
    // The hosted ranks' part of comm step `id` on the comm stream (strm 2), emitted
    // once, at the first call (the sender's point in an emulated schedule).  Sends
    // wait for the main stream's work so far (their data); the main stream waits
    // for the step when it receives.  Messages keep the plan order, so every peer
    // pair posts its matching sends and receives in the same order.
    auto emit_step = [&](int32_t id, int send_ev = -1) {
        if (!multi || id < 0 || emitted[id]) return;
        emitted[id] = 1;
        Launch L {};
        L.kind = L_COMM;
        L.level = D.steps[id].level;
        L.strm = 2;
        L.step = id;
        L.off = (int64_t)N.msgs.size();
        bool any_send = false, any_recv = false;
        std::vector<int32_t> pack_d, unpack_d;  // copy descriptors of the sends / receives
        // (buffer, staging slot) of one end: the region itself when contiguous
        auto end_of = [&](int v, int kind, int s, int row, int col, int rows, int cols, bool pack, double*& buf,
                          int64_t& slot) {
            int64_t ld = 0;
            double* a = addr(v, kind, s, row, col, ld);
            if (!a) return false;
            if (ld == rows || cols == 1) {
                buf = a;
                slot = -1;
                return true;
            }
            buf = nullptr;
            slot = cbld.stage_total;
            Copy2D c {};
            c.a = a;
            c.lda = ld;
            c.rows = rows;
            c.cols = cols;
            (pack ? pack_d : unpack_d).push_back((int32_t)cbld.copies.size());
            cbld.copies.push_back(c);
            cbld.copy_slot.push_back(slot);
            cbld.stage_total += (int64_t)rows * cols;
            return true;
        };
        for (int64_t q = step_beg[id]; q < step_beg[id + 1]; ++q) {
            const DistMsg& g = D.msgs[q];
            const int vs = hosted_of[g.src], vd = hosted_of[g.dst];
            if (vs < 0 && vd < 0) continue;
            const int64_t cnt = (int64_t)g.rows * g.cols;
            double *sb = nullptr, *db = nullptr;
            int64_t ss = -1, ds = -1;
            if (vs >= 0 && !end_of(vs, g.skind, g.s, g.srow, g.scol, g.rows, g.cols, true, sb, ss)) {
                N.err = "comm plan: send region missing";
                return;
            }
            if (vd >= 0 && !end_of(vd, g.dkind, g.s, g.drow, g.dcol, g.rows, g.cols, false, db, ds)) {
                N.err = "comm plan: receive region missing";
                return;
            }
            any_send |= vs >= 0;
            any_recv |= vd >= 0;
            auto push = [&](double* b, int64_t slot, double* src, int64_t src_slot, int peer, int op) {
                Msg m {};
                m.buf = b;
                m.src_buf = src;
                m.count = cnt;
                m.peer = peer;
                m.op = op;
                N.msgs.push_back(m);
                cbld.msg_slot.push_back(slot);
                cbld.msg_src_slot.push_back(src_slot);
            };
            if (vs >= 0 && vd >= 0) {  // both ends in this process (emulated ranks)
                if (N.emul_rccl) {
                    push(sb, ss, nullptr, -1, 0, MSG_SEND);
                    push(db, ds, nullptr, -1, 0, MSG_RECV);
                } else {
                    push(db, ds, sb, ss, 0, MSG_COPY);
                }
            } else if (vs >= 0) {
                push(sb, ss, nullptr, -1, g.dst, MSG_SEND);
            } else {
                push(db, ds, nullptr, -1, g.src, MSG_RECV);
            }
        }
        L.count = (int32_t)((int64_t)N.msgs.size() - L.off);
        if (L.count == 0) return;
        auto add_tiles = [&](const std::vector<int32_t>& ds) {
            for (int32_t d : ds)
                for (int j = 0; j < cbld.copies[d].cols; j += COPY_COLS) cbld.ctiles.push_back(make_int2(d, j));
        };
        L.poff = (int64_t)cbld.ctiles.size();
        add_tiles(pack_d);
        L.pcount = (int32_t)((int64_t)cbld.ctiles.size() - L.poff);
        L.uoff = (int64_t)cbld.ctiles.size();
        add_tiles(unpack_d);
        L.ucount = (int32_t)((int64_t)cbld.ctiles.size() - L.uoff);
        // sends wait for the data (default: everything the main stream has so far);
        // receive-only steps post as soon as the main stream has finished the previous
        // level (the per-level guard below)
        if (any_send) push_wait(2, send_ev >= 0 ? send_ev : push_record(0));
        N.sched.push_back(L);
        if (any_recv) push_wait(0, push_record(2));
    };
    auto is_early_sender = [&](int32_t s, int v) {
        return multi && D.early[s] && D.owner[s] == N.R[v].rank;
    };
    // CB rank (hosted index v) of split front s: per final panel slab, CB -= L21_k
    // L21_k^T on the column blocks it owns (K = slab width), from its R_LAND copy
    auto emit_cb_rank = [&](int32_t lev, int32_t s, int v) {
        const int who = N.R[v].rank;
        const std::vector<int32_t>& cbr = D.cb_rank[D.split[s]];
        const int w = S.w(s), m = S.sn_m[s], mb = m - w;
        emit_step(init_step[s]);
        for (int k0 = 0, k = 0; k0 < w; k0 += D.nbo, ++k) {
            const int k1 = std::min(w, k0 + D.nbo);
            emit_step(slab_step0[s] < 0 ? -1 : slab_step0[s] + k);
            std::vector<GemmTask> cbt;
            double fl = 0.0;
            for (int jb = 0; jb < (int)cbr.size(); ++jb) {
                if (cbr[jb] != who) continue;
                const int r0 = jb * D.cbb;
                GemmTask t {};
                int64_t ldc = 0, lda = 0;
                t.C = addr(v, R_CB, s, r0, r0, ldc);
                t.A = addr(v, R_LAND, s, r0, k0, lda);
                t.ldc = ldc;
                t.lda = lda;
                t.M = mb - r0;
                t.N = std::min(D.cbb, mb - r0);
                t.K = k1 - k0;
                cbt.push_back(t);
                fl += 2.0 * t.K * ((double)t.N * t.M - (double)t.N * (t.N - 1) / 2.0);
            }
            push_gemm_launch(L_CB, lev, cbt, w >= 256 ? 1 : 0, fl);
        }
    };
    // one level's fronts of hosted rank v
    auto emit_level = [&](int32_t lev, const std::vector<int32_t>& nodes, int v) {
        double* panel_pool = N.R[v].P.panel_pool;
        double* cb_pool = N.R[v].P.cb_pool;
        const std::vector<int64_t>& poff = N.R[v].panel_off;
        const std::vector<int64_t>& coff = N.R[v].cb_off;
        // small fronts: one launch sized for the level's largest front when the level
        // fits one workgroup per CU (fewer dependent launches on thin levels), else one
        // launch per LDS bucket (small fronts keep their occupancy on wide levels)
        int nsmall = 0, bmax = 0;
        for (int32_t s : nodes)
            if (S.fclass[s] == FRONT_SMALL) {
                ++nsmall;
                bmax = std::max(bmax, bucket_of(S.sn_m[s]));
            }
        for (int b : {32, 64, 96, 128}) {
            if (nsmall <= 256 && b != bmax) continue;
            Launch L {};
            L.kind = L_SMALL;
            L.level = lev;
            L.vr = v;
            L.off = (int64_t)small.size();
            L.maxm = b;
            L.bt = 16;
            for (int32_t s : nodes)
                if (S.fclass[s] == FRONT_SMALL && (nsmall <= 256 || bucket_of(S.sn_m[s]) == b)) {
                    small.push_back(s);
                    L.bt = std::max(L.bt, wbucket_of(S.w(s)));
                }
            L.count = (int32_t)((int64_t)small.size() - L.off);
            if (L.count > 0) N.sched.push_back(L);
        }
        std::vector<int32_t> large;
        for (int32_t s : nodes)
            if (S.fclass[s] == FRONT_LARGE) large.push_back(s);
        if (large.empty()) return;
        // fronts whose CB SYRK gathers the children's CB entries itself (one CB launch
        // task covering the whole CB): their assembly stops at the panel columns
        auto gather = [&](int32_t s) { return S.opt.cb_gather && S.mb(s) > 0 && !is_split(s) && !is_early_sender(s, v); };
        // assembly: fronts with m >= ASM_TILE_MIN_M one workgroup per (front, 16
        // columns, 256-row tile), write-once (big = 1); smaller fronts one workgroup per
        // (front, 16 columns) streaming child columns (measured faster below ~8k rows)
        const int tile_min_m = S.opt.asm_tile_min_m > 0 ? S.opt.asm_tile_min_m : ASM_TILE_MIN_M;
        for (int tiled = 1; tiled >= 0; --tiled) {
            Launch L {};
            L.kind = L_ASM;
            L.level = lev;
            L.vr = v;
            L.big = tiled;
            L.off = (int64_t)asmv.size();
            for (int32_t s : large) {
                const int m = S.sn_m[s];
                if ((m >= tile_min_m) != (tiled == 1)) continue;
                const int ncol = gather(s) ? S.w(s) : m;  // assembled columns
                for (int cb = 0; cb * ASM_COLS < ncol; ++cb) {
                    if (!tiled) {
                        asmv.push_back(make_int2(s, cb));
                        continue;
                    }
                    for (int k = cb * ASM_COLS / ASM_ROWS; k * ASM_ROWS < m; ++k)
                        asmv.push_back(make_int2(s, (k << 16) | cb));
                }
            }
            L.count = (int32_t)((int64_t)asmv.size() - L.off);
            if (L.count > 0) N.sched.push_back(L);
        }
        for (int32_t s : large)
            if (is_split(s)) emit_step(init_step[s]);
        int maxw = 0;
        for (int32_t s : large) maxw = std::max(maxw, S.w(s));
        // Lookahead: at a slab end the outer rank-NBO update is split into the next
        // slab's columns (stream 0, needed by the next POTRF/TRSM) and the rest
        // (stream 1), which overlaps the next slab's factorization.  A later outer
        // update of overlapping columns waits for the stream-1 work first.
        int b_pending = -1;
        // rows [c_lo, r_hi) of columns [c_lo, c_hi) -= their product over columns [ka, kb)
        auto add_update = [&](std::vector<GemmTask>& vec, double& fl, double* pan, int m, int r_hi, int c_lo, int c_hi,
                              int ka, int kb) {
            if (c_hi <= c_lo || kb <= ka || r_hi <= c_lo) return;
            GemmTask t {};
            t.C = pan + (int64_t)c_lo * m + c_lo;
            t.A = pan + (int64_t)ka * m + c_lo;
            t.ldc = m;
            t.lda = m;
            t.M = r_hi - c_lo;
            t.N = c_hi - c_lo;
            t.K = kb - ka;
            vec.push_back(t);
            fl += 2.0 * t.K * ((double)t.N * t.M - (double)t.N * (t.N - 1) / 2.0);
        };
        // tall mode (a front of more than one 64-column block): the 64-column chain
        // (POTRF / TRSM / inner updates) runs on the slab's diagonal-block rows only; at
        // the slab end the block inverses and one tall-TRSM launch solve every row below
        // the slab (panel_tall_kernel), then the outer updates as before
        auto tall = [&](int32_t s) { return S.opt.panel_tall && S.w(s) > PNB; };
        for (int k0 = 0; k0 < maxw; k0 += PNB) {
            Launch Lp {};
            Lp.kind = L_POTRF;
            Lp.level = lev;
            Lp.vr = v;
            Lp.off = (int64_t)potrf.size();
            Launch Lt {};
            Lt.kind = L_TRSM;
            Lt.level = lev;
            Lt.vr = v;
            Lt.off = (int64_t)trsm.size();
            std::vector<GemmTask> upd, outer_a, outer_b;
            std::vector<TrsmTask> trsm_part;  // partial last blocks: own launch (big = 1)
            std::vector<int2> inv_t;           // tall mode, slab end: diagonal-block inverses
            std::vector<int4> tall_t;          // ... and the tall TRSM of the rows below
            double uflops = 0.0, afl = 0.0, bfl = 0.0;
            for (int32_t s : large) {
                const int w = S.w(s), m = S.sn_m[s];
                if (w <= k0) continue;
                const int nb = std::min(PNB, w - k0);
                const int k1 = k0 + nb;
                const int slab0 = (k0 / NBO) * NBO;
                const int slab1 = std::min(w, slab0 + NBO);
                const int rend = tall(s) ? slab1 : m;  // rows of this step's TRSM and inner update
                if (nb < PNB) {
                    potrf.push_back(make_int2(s, k0));
                    for (int r0 = k1; r0 < rend; r0 += TRSM_ROWS) trsm_part.push_back(TrsmTask {s, k0, r0, rend, 0});
                } else {  // fused POTRF (one task if no rows below); ctr - 1: arrival counter
                    const int ctr = (int)trsm.size() + 1;
                    for (int r0 = k1; r0 < std::max(rend, k1 + 1); r0 += TRSM_ROWS)
                        trsm.push_back(TrsmTask {s, k0, r0, rend, ctr});
                }
                double* pan = panel_pool + poff[s];
                if (k1 < slab1 && S.opt.inner_order == 1) {
                    // recursive order: block b of the slab closes a run of 2^t blocks
                    // (t = trailing zeros of b + 1); that run updates the next 2^t
                    // blocks (K = 64 * 2^t).  Same flops and dependencies as
                    // right-looking, 768 instead of 1792 C columns rewritten per slab.
                    const int b = (k0 - slab0) / PNB;
                    const int span = PNB << __builtin_ctz((unsigned)(b + 1));
                    add_update(upd, uflops, pan, m, rend, k1, std::min(slab1, k1 + span), k1 - span, k1);
                } else if (k1 < slab1) {
                    add_update(upd, uflops, pan, m, rend, k1, slab1, k0, k1);
                }
                if (k1 == slab1 && tall(s)) {
                    for (int kb = slab0; kb < slab1; kb += PNB) inv_t.push_back(make_int2(s, kb));
                    for (int r0 = slab1; r0 < m; r0 += TALL_ROWS) tall_t.push_back(make_int4(s, slab0, r0, slab1));
                }
                if (k1 == slab1 && slab1 < w) {
                    // outer_a is the last update of block slab1: a pending stream-1 outer
                    // update of those columns is waited for before outer_a runs
                    const int nxt = S.opt.lookahead ? std::min(w, slab1 + NBO) : w;
                    add_update(outer_a, afl, pan, m, m, slab1, nxt, slab0, slab1);
                    add_update(outer_b, bfl, pan, m, m, nxt, w, slab0, slab1);
                }
            }
            Lp.count = (int32_t)((int64_t)potrf.size() - Lp.off);
            Lt.count = (int32_t)((int64_t)trsm.size() - Lt.off);
            if (Lp.count > 0) N.sched.push_back(Lp);
            if (Lt.count > 0) N.sched.push_back(Lt);
            if (!trsm_part.empty()) {
                Launch Lq = Lt;
                Lq.off = (int64_t)trsm.size();
                Lq.count = (int32_t)trsm_part.size();
                Lq.big = 1;
                trsm.insert(trsm.end(), trsm_part.begin(), trsm_part.end());
                N.sched.push_back(Lq);
            }
            push_gemm_launch(L_PANEL, lev, upd, 0, uflops);
            if (!tall_t.empty() || !inv_t.empty()) {
                Launch Li {};
                Li.kind = L_INV;
                Li.level = lev;
                Li.vr = v;
                Li.off = (int64_t)B.inv.size();
                Li.count = (int32_t)inv_t.size();
                B.inv.insert(B.inv.end(), inv_t.begin(), inv_t.end());
                if (Li.count > 0) N.sched.push_back(Li);
                Launch Lt2 {};
                Lt2.kind = L_TALL;
                Lt2.level = lev;
                Lt2.vr = v;
                Lt2.off = (int64_t)B.tall.size();
                Lt2.count = (int32_t)tall_t.size();
                B.tall.insert(B.tall.end(), tall_t.begin(), tall_t.end());
                if (Lt2.count > 0) N.sched.push_back(Lt2);
            }
            // split fronts: a slab is final after the TRSM of its last block (tall mode:
            // after the slab's tall TRSM); at a slab end no inner update is pending
            for (int32_t s : large) {
                const int w = S.w(s);
                if (!is_split(s) || w <= k0 || slab_step0[s] < 0) continue;
                const int k1 = std::min(w, k0 + PNB);
                if (k1 == w || k1 % D.nbo == 0) emit_step(slab_step0[s] + k0 / D.nbo);
            }
            int e_trsm = -1;
            if (!outer_b.empty()) e_trsm = push_record(0);
            if (!outer_a.empty()) {
                if (b_pending >= 0) {
                    push_wait(0, b_pending);
                    b_pending = -1;
                }
                push_gemm_launch(L_PANEL, lev, outer_a, 0, afl);
            }
            if (!outer_b.empty()) {
                push_wait(1, e_trsm);
                push_gemm_launch(L_PANEL, lev, outer_b, 0, bfl, 1);
                b_pending = push_record(1);
            }
        }
        if (b_pending >= 0) push_wait(0, b_pending);
        // early-delivery children: the CB SYRK in column groups, an event after each
        // (the group's comm sub-step waits for exactly that event)
        for (int32_t s : large) {
            if (!is_early_sender(s, v)) continue;
            const int w = S.w(s), m = S.sn_m[s], mb = m - w;
            for (int j0 = 0; j0 < mb; j0 += D.early_gw) {
                GemmTask t {};
                t.C = cb_pool + coff[s] + (int64_t)j0 * mb + j0;
                t.A = panel_pool + poff[s] + w + j0;
                t.ldc = mb;
                t.lda = m;
                t.M = mb - j0;
                t.N = std::min(D.early_gw, mb - j0);
                t.K = w;
                const double fl = 2.0 * t.K * ((double)t.N * t.M - (double)t.N * (t.N - 1) / 2.0);
                push_gemm_launch(L_CB, lev, std::vector<GemmTask> {t}, w >= 256 ? 1 : 0, fl);
                early_ev[s].push_back(push_record(0));
            }
        }
        // contribution-block SYRK, K = w; fronts with w >= 256 in their own launch
        for (int big = 1; big >= 0; --big) {
            std::vector<GemmTask> cbt;
            double fl = 0.0;
            for (int32_t s : large) {
                const int w = S.w(s), m = S.sn_m[s], mb = m - w;
                if (mb <= 0 || (w >= 256) != (big == 1) || is_split(s) || is_early_sender(s, v)) continue;
                GemmTask t {};
                t.C = cb_pool + coff[s];
                t.A = panel_pool + poff[s] + w;
                t.ldc = mb;
                t.lda = m;
                t.M = mb;
                t.N = mb;
                t.K = w;
                if (gather(s)) {
                    t.gs = s;
                    t.gv = v;
                }
                cbt.push_back(t);
                fl += (double)mb * (mb + 1.0) * t.K;
            }
            push_gemm_launch(L_CB, lev, cbt, big, fl);
        }
    };
    // Distributed panel of front s (dist.cpp): every hosted rank of its holders.  Per
    // slab k: its owner factors it (the 64-column POTRF / TRSM / inner-update chain
    // on the main stream), the SLAB step moves it, then every rank that needs it
    // updates its own next slab on the main stream (critical path) and its other
    // later slabs and CB blocks on the lookahead stream.  A lookahead-stream update
    // of slab j (from slab k <= j - 2) is waited for before the main stream touches
    // slab j (event after the lookahead launch of step j - 2, covering all earlier
    // ones: the stream is in order).
    auto emit_dist_front = [&](int32_t lev, int32_t s) {
        const int q = D.pd[s];
        const std::vector<int32_t>& sr = D.slab_rank[q];
        const int w = S.w(s), m = S.sn_m[s], mb = m - w, nsl = (int)sr.size();
        const int own = D.owner[s];
        std::vector<int> vs;  // hosted holders
        for (int32_t r : D.holders[q])
            if (hosted_of[r] >= 0) vs.push_back(hosted_of[r]);
        if (hosted_of[own] >= 0 && std::find(vs.begin(), vs.end(), hosted_of[own]) == vs.end())
            vs.push_back(hosted_of[own]);
        if (vs.empty()) return;
        auto pan_of = [&](int v) { return N.R[v].P.panel_pool + N.R[v].panel_off[s]; };
        auto slab_c0 = [&](int k) { return k * D.nbo; };
        auto slab_c1 = [&](int k) { return std::min(w, (k + 1) * D.nbo); };
        const int vo = hosted_of[own];
        if (vo >= 0) {  // the owner assembles the whole front (tiled or column-streaming)
            const int tile_min_m = S.opt.asm_tile_min_m > 0 ? S.opt.asm_tile_min_m : ASM_TILE_MIN_M;
            Launch L {};
            L.kind = L_ASM;
            L.level = lev;
            L.vr = vo;
            L.big = m >= tile_min_m ? 1 : 0;
            L.off = (int64_t)asmv.size();
            for (int cb = 0; cb * ASM_COLS < m; ++cb) {
                if (!L.big) {
                    asmv.push_back(make_int2(s, cb));
                    continue;
                }
                for (int kk = cb * ASM_COLS / ASM_ROWS; kk * ASM_ROWS < m; ++kk)
                    asmv.push_back(make_int2(s, (kk << 16) | cb));
            }
            L.count = (int32_t)((int64_t)asmv.size() - L.off);
            N.sched.push_back(L);
        }
        emit_step(init_step[s]);
        std::vector<std::vector<int>> ev1((size_t)N.R.size(), std::vector<int>((size_t)nsl, -1));
        auto last_ev1 = [&](int v, int kmax) {  // latest lookahead event of steps <= kmax
            for (int k = std::min(kmax, nsl - 1); k >= 0; --k)
                if (ev1[v][k] >= 0) return ev1[v][k];
            return -1;
        };
        auto upd_task = [&](std::vector<GemmTask>& vec, double& fl, double* C, int64_t ldc, const double* A,
                            int64_t lda, int M, int Nn, int K) {
            if (M <= 0 || Nn <= 0 || K <= 0) return;
            GemmTask t {};
            t.C = C;
            t.A = A;
            t.ldc = ldc;
            t.lda = lda;
            t.M = M;
            t.N = Nn;
            t.K = K;
            vec.push_back(t);
            fl += 2.0 * t.K * ((double)t.N * t.M - (double)t.N * (t.N - 1) / 2.0);
        };
        for (int k = 0; k < nsl; ++k) {
            const int k0s = slab_c0(k), k1s = slab_c1(k);
            const int vk = hosted_of[sr[k]];
            if (vk >= 0) {
                // factor slab k: per 64 columns POTRF, TRSM of the rows below, and the
                // update of the slab's next columns (recursive order, as emit_level)
                const int e = last_ev1(vk, k - 2);
                if (e >= 0) push_wait(0, e);
                double* pan = pan_of(vk);
                for (int k0 = k0s; k0 < k1s; k0 += PNB) {
                    const int nb = std::min(PNB, k1s - k0), k1 = k0 + nb;
                    Launch Lp {};
                    Lp.kind = L_POTRF;
                    Lp.level = lev;
                    Lp.vr = vk;
                    Lp.off = (int64_t)potrf.size();
                    Lp.count = 1;
                    if (nb < PNB) {  // full blocks: POTRF fused into the TRSM
                        potrf.push_back(make_int2(s, k0));
                        N.sched.push_back(Lp);
                    }
                    Launch Lt {};
                    Lt.kind = L_TRSM;
                    Lt.level = lev;
                    Lt.vr = vk;
                    Lt.off = (int64_t)trsm.size();
                    Lt.big = nb < PNB ? 1 : 0;
                    const int ctr = nb < PNB ? 0 : (int)trsm.size() + 1;  // fused POTRF: arrival counter
                    for (int r0 = k1; r0 < (nb < PNB ? m : std::max(m, k1 + 1)); r0 += TRSM_ROWS)
                        trsm.push_back(TrsmTask {s, k0, r0, m, ctr});
                    Lt.count = (int32_t)((int64_t)trsm.size() - Lt.off);
                    if (Lt.count > 0) N.sched.push_back(Lt);
                    if (k1 < k1s) {
                        std::vector<GemmTask> upd;
                        double fl = 0.0;
                        if (S.opt.inner_order == 1) {
                            const int b = (k0 - k0s) / PNB;
                            const int span = PNB << __builtin_ctz((unsigned)(b + 1));
                            const int c1 = std::min(k1s, k1 + span);
                            upd_task(upd, fl, pan + (int64_t)k1 * m + k1, m, pan + (int64_t)(k1 - span) * m + k1, m,
                                     m - k1, c1 - k1, span);
                        } else {
                            upd_task(upd, fl, pan + (int64_t)k1 * m + k1, m, pan + (int64_t)k0 * m + k1, m, m - k1,
                                     k1s - k1, nb);
                        }
                        push_gemm_launch(L_PANEL, lev, upd, 0, fl);
                    }
                }
            }
            if (slab_step[s].size() > (size_t)k) emit_step(slab_step[s][k]);
            // slab k's update on every hosted rank that needs it
            for (int v : vs) {
                const int r = N.R[v].rank;
                if (D.need_row(S, s, k, r) >= m) continue;
                double* pan = pan_of(v);
                const double* Lk = pan + (int64_t)k0s * m;  // column k0s of the slab, row 0
                const int K = k1s - k0s;
                if (k + 1 < nsl && sr[k + 1] == r) {  // the next slab: critical path
                    const int e = last_ev1(v, k - 1);
                    if (e >= 0) push_wait(0, e);
                    const int j0 = slab_c0(k + 1), j1 = slab_c1(k + 1);
                    std::vector<GemmTask> t0;
                    double fl = 0.0;
                    upd_task(t0, fl, pan + (int64_t)j0 * m + j0, m, Lk + j0, m, m - j0, j1 - j0, K);
                    push_gemm_launch(L_PANEL, lev, t0, 0, fl);
                }
                std::vector<GemmTask> t1;
                double fl = 0.0;
                for (int j = k + 2; j < nsl; ++j) {
                    if (sr[j] != r) continue;
                    const int j0 = slab_c0(j), j1 = slab_c1(j);
                    upd_task(t1, fl, pan + (int64_t)j0 * m + j0, m, Lk + j0, m, m - j0, j1 - j0, K);
                }
                if (is_split(s)) {  // CB blocks: CB -= L21_k L21_k^T
                    const std::vector<int32_t>& cbr = D.cb_rank[D.split[s]];
                    for (int jb = 0; jb < (int)cbr.size(); ++jb) {
                        if (cbr[jb] != r) continue;
                        const int r0 = jb * D.cbb;
                        int64_t ldc = 0;
                        double* C = addr(v, R_CB, s, r0, r0, ldc);
                        upd_task(t1, fl, C, ldc, Lk + w + r0, m, mb - r0, std::min(D.cbb, mb - r0), K);
                    }
                } else if (!is_split(s) && mb > 0 && r == own) {  // unsplit: the owner's whole CB
                    int64_t ldc = 0;
                    double* C = addr(v, R_CB, s, 0, 0, ldc);
                    upd_task(t1, fl, C, ldc, Lk + w, m, mb, mb, K);
                }
                if (t1.empty()) continue;
                push_wait(1, push_record(0));
                push_gemm_launch(L_PANEL, lev, t1, 0, fl, 1);
                ev1[v][k] = push_record(1);
            }
        }
        for (int v : vs) {  // join the lookahead stream before the level's deliveries
            const int e = last_ev1(v, nsl - 1);
            if (e >= 0) push_wait(0, e);
        }
    };
    if (multi) push_wait(2, push_record(0));  // previous factorization's reads are done
    // multi-rank work-arena reuse guard (memplan.cpp): the comm steps of level L run
    // after the main stream has finished level L - 1, and the main stream starts level
    // L + 2 only after the comm steps of level L, so a region a step of level L touches
    // is never reused before level L + 2
    std::vector<int> comm_done((size_t)S.nlevels, -1);
    // single device: a run of >= 2 levels holding one small front each (a chain: each
    // front the parent of the one before) runs as one single-workgroup launch
    auto chain_front = [&](int32_t lev) {
        return !multi && by_level[lev].size() == 1 && S.fclass[by_level[lev][0]] == FRONT_SMALL;
    };
    // single device, a tiny tree (at most TINY_MAX_FRONTS fronts, all small with m <= 64,
    // every image and CB fitting LDS): the whole factorization as one single-workgroup
    // launch, postorder (the internal numbering), everything in LDS
    bool tiny = !multi && S.ns > 1 && S.ns <= TINY_MAX_FRONTS;
    {
        int64_t lds = 0;
        for (int32_t s = 0; tiny && s < S.ns; ++s) {
            const int64_t m = S.sn_m[s], mb = S.mb(s);
            tiny = S.fclass[s] == FRONT_SMALL && m <= 64;
            lds += m * (m + 1) / 2 + mb * (mb + 1) / 2;
        }
        tiny = tiny && lds <= TINY_MAX_LDS;
    }
    if (tiny) {
        auto pk = [](int64_t m, int64_t j) { return j * m - j * (j - 1) / 2; };
        std::vector<int32_t> img((size_t)S.ns), cbo((size_t)S.ns);
        int32_t off = 0;
        for (int32_t s = 0; s < S.ns; ++s) {
            img[s] = off;
            off += S.sn_m[s] * (S.sn_m[s] + 1) / 2;
            cbo[s] = off;
            off += S.mb(s) * (S.mb(s) + 1) / 2;
        }
        B.tiny_lds = off;
        for (int32_t s = 0; s < S.ns; ++s) {
            const int m = S.sn_m[s], w = S.w(s), c0 = S.sn_start[s];
            TinyFront f {};
            f.s = s;
            f.c0 = c0;
            f.w = w;
            f.m = m;
            f.img = img[s];
            f.cb = cbo[s];
            f.e0 = (int32_t)B.tph.size();
            f.panel_off = N.R[0].panel_off[s];
            for (int lc = 0; lc < w; ++lc)
                for (int64_t q = S.a_ptr[c0 + lc]; q < S.a_ptr[c0 + lc + 1]; ++q)
                    B.ta.push_back(make_int2((int32_t)S.a_src[q], img[s] + (int32_t)(pk(m, lc) + S.a_pos[q] - lc)));
            for (int32_t ci = S.child_ptr[s]; ci < S.child_ptr[s + 1]; ++ci) {
                const int32_t c = S.child_list[ci];
                const int mbc = S.mb(c);
                const int32_t* rel = S.relind.data() + S.rel_ptr[c];
                const int32_t beg = (int32_t)B.tpr.size();
                for (int jc = 0; jc < mbc; ++jc)
                    for (int ic = jc; ic < mbc; ++ic)
                        B.tpr.push_back(make_int2(cbo[c] + (int32_t)(pk(mbc, jc) + ic - jc),
                                                  img[s] + (int32_t)(pk(m, rel[jc]) + rel[ic] - rel[jc])));
                B.tph.push_back(make_int2(beg, (int32_t)B.tpr.size()));
            }
            f.np = (int32_t)B.tph.size() - f.e0;
            B.tfr.push_back(f);
        }
        Launch L {};
        L.kind = L_SMALL;
        L.level = 0;
        L.maxm = 64;
        L.big = 2;  // tiny tree
        L.count = 1;
        N.sched.push_back(L);
    }
    for (int32_t lev = tiny ? S.nlevels : 0; lev < S.nlevels; ++lev) {
        if (chain_front(lev) && lev + 1 < S.nlevels && chain_front(lev + 1)) {
            Launch L {};
            L.kind = L_SMALL;
            L.level = lev;
            L.off = (int64_t)B.cdesc.size();
            L.maxm = 32;
            L.big = 1;  // chain
            int32_t sp = -1;
            for (; lev < S.nlevels && chain_front(lev) && (int64_t)B.cdesc.size() - L.off < CHAIN_MAXF; ++lev) {
                const int32_t s = by_level[lev][0];
                const int w = S.w(s), m = S.sn_m[s];
                L.maxm = std::max(L.maxm, bucket_of(m));
                ChainDesc d {};
                d.s = s;
                d.c0 = S.sn_start[s];
                d.w = w;
                d.m = m;
                d.sp = sp;
                d.panel_off = N.R[0].panel_off[s];
                d.cb_off = N.R[0].cb_off[s] < 0 ? 0 : N.R[0].cb_off[s];
                d.init_off = B.chain_init;
                d.relp_off = (int64_t)B.crelp.size();
                for (int t0 = 0; t0 < m; t0 += 4) {  // parent rows of CB rows, packed per tile row
                    uint32_t wd = 0;
                    for (int t = 0; t < 4; ++t) {
                        const int i = t0 + t;
                        const int32_t pr = (i >= w && i < m) ? S.relind[(size_t)S.rel_ptr[s] + (i - w)] : 0;
                        wd |= (uint32_t)(pr & 255) << (8 * t);
                    }
                    B.crelp.push_back(wd);
                }
                B.chain_init += ((int64_t)m * (m + 1) / 2 + 63) / 64 * 64;
                B.cdesc.push_back(d);
                sp = s;
            }
            L.count = (int32_t)((int64_t)B.cdesc.size() - L.off);
            N.sched.push_back(L);
            --lev;
            continue;
        }
        if (multi) {
            if (lev >= 2 && comm_done[lev - 2] >= 0) push_wait(0, comm_done[lev - 2]);
            push_wait(2, push_record(0));
        }
        for (size_t v = 0; v < N.R.size(); ++v) {
            if (!multi) {
                emit_level(lev, by_level[lev], (int)v);
                continue;
            }
            std::vector<int32_t> mine;
            for (int32_t s : by_level[lev])
                if (D.owner[s] == N.R[v].rank && !is_dpanel(s)) mine.push_back(s);
            if (!mine.empty()) emit_level(lev, mine, (int)v);
        }
        if (!multi) continue;
        for (int32_t s : by_level[lev])
            if (is_dpanel(s)) emit_dist_front(lev, s);
        // contribution-block ranks of this level's split fronts (emulated: after the
        // owners' panels, whose steps already moved the data)
        for (int32_t s : by_level[lev]) {
            if (!is_split(s) || is_dpanel(s)) continue;
            const std::vector<int32_t>& cbr = D.cb_rank[D.split[s]];
            for (size_t v = 0; v < N.R.size(); ++v) {
                const int who = N.R[v].rank;
                if (who != D.owner[s] && std::find(cbr.begin(), cbr.end(), who) != cbr.end())
                    emit_cb_rank(lev, s, (int)v);
            }
        }
        // contribution blocks that leave / enter the hosted ranks after this level:
        // early children's column groups first, then the rest
        for (int32_t c : by_level[lev]) {
            if (!D.early[c] || early_step0[c] < 0) continue;
            const int ng = (S.mb(c) + D.early_gw - 1) / D.early_gw;
            const int vs = hosted_of[D.owner[c]];
            for (int g = 0; g < ng; ++g)
                emit_step(early_step0[c] + g, vs >= 0 && !early_ev[c].empty() ? early_ev[c][g] : -1);
        }
        emit_step(deliver_step[lev]);
        comm_done[lev] = push_record(2);
    }
    if (multi) push_wait(0, push_record(2));  // join the comm stream (its last sends)
    if (!N.err.empty()) return SC_ERR_ARG;
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
    if (hipHostMalloc((void**)&N.h_info, sizeof(int32_t) * 16, hipHostMallocDefault) != hipSuccess) {
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
        if ((rc = upload(N, R.cb_off, dp))) return fail(rc);
        R.P.cb_off = dp;
    }
    if (!multi || N.emulated) N.gpanel = pbase;  // gathered layout == the arenas
    {
        std::vector<DevPlan> plans;
        for (const RankMem& R : N.R) plans.push_back(R.P);
        if ((rc = upload(N, plans, N.d_plans))) return fail(rc);
    }

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
    }
    if ((rc = upload(N, B.small, N.d_small)) || (rc = upload(N, B.asmv, N.d_asm)) ||
        (rc = upload(N, B.potrf, N.d_potrf)) || (rc = upload(N, B.trsm, N.d_trsm)) ||
        (rc = upload(N, B.inv, N.d_inv)) || (rc = upload(N, B.tall, N.d_tall)) ||
        (rc = upload(N, std::vector<int32_t>(B.trsm.size() + 1, 0), N.d_arrive)) ||
        (rc = upload(N, B.gemm, N.d_gemm)) || (rc = upload(N, B.tiles, N.d_tiles)))
        return fail(rc);
    (void)ns;
    return SC_OK;
}

hipError_t comm_launch(Numeric& N, const Launch& L);  // dist.cpp
int64_t dist_min_info(Numeric& N, int32_t& info);      // dist.cpp
int64_t dist_gather_panels(Numeric& N);                // dist.cpp

static hipStream_t stream_of(const Numeric& N, int strm) {
    return strm == 2 ? N.stream3 : strm == 1 ? N.stream2 : N.stream;
}

static hipError_t launch_one(Numeric& N, const Launch& L, const double* d_Ax) {
    hipStream_t st = stream_of(N, L.strm);
    switch (L.kind) {
        case L_RECORD:
            return hipEventRecord(N.sync_ev[L.count], st);
        case L_WAIT:
            return hipStreamWaitEvent(st, N.sync_ev[L.count], 0);
        case L_SMALL:
            if (L.big == 1) return launch_front_chain(N.R[L.vr].P, N.CP, (int)L.off, L.count, L.maxm, d_Ax, N.stream);
            if (L.big == 2) return launch_tiny_tree(N.R[L.vr].P, N.TP, L.maxm, d_Ax, N.stream);
            return launch_front_small(N.R[L.vr].P, N.d_small + L.off, L.count, L.maxm, false, d_Ax, N.stream);
        case L_ASM:
            return launch_assemble_large(N.R[L.vr].P, N.d_asm + L.off, L.count, d_Ax, N.stream, L.big != 0);
        case L_POTRF:
            return launch_potrf_diag(N.R[L.vr].P, N.d_potrf + L.off, L.count, N.stream);
        case L_TRSM:
            return launch_trsm_panel(N.R[L.vr].P, N.d_trsm + L.off, L.count, N.stream, L.big != 0, N.d_arrive);
        case L_PANEL:
        case L_CB:
            return launch_syrk(N.d_gemm + L.off, N.d_tiles + L.toff, L.count, L.bt, L.kind == L_CB ? 1 : 0, st, L.epi,
                               N.d_plans);
        case L_COMM:
            return comm_launch(N, L);
        case L_INV:
            return launch_panel_inv(N.R[L.vr].P, N.d_inv + L.off, L.count, N.stream);
        case L_TALL:
            return launch_panel_tall(N.R[L.vr].P, N.d_tall + L.off, L.count, N.stream);
    }
    return hipErrorInvalidValue;
}

static int64_t enqueue_all(Numeric& N, const double* d_Ax, int prof) {
    HIP_TRY(hipMemsetAsync(N.d_info, 0x7f, sizeof(int32_t), N.stream));
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
    HIP_TRY(hipMemcpyAsync(N.h_info, N.d_info, sizeof(int32_t), hipMemcpyDeviceToHost, N.stream));
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
    N.status_valid = false;
    N.last_Ax = d_Ax;
    if (N.profile == 1 && N.ev.size() != 2 * N.sched.size()) {
        for (auto e : N.ev) (void)hipEventDestroy(e);
        N.ev.assign(2 * N.sched.size(), nullptr);
        for (auto& e : N.ev) HIP_TRY(hipEventCreate(&e));
    }
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
    // every stream's work is joined into the main stream before the status copy
    HIP_TRY(hipStreamSynchronize(N.stream));
    int32_t info = *N.h_info;
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
                case L_TRSM:
                case L_INV:
                case L_TALL: slot = 5; break;
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

int64_t numeric_timing(Numeric& N, double* t, int nt) {
    if (N.profile != 1 || !N.status_valid) return SC_ERR_STATE;
    for (int i = 0; i < nt && i < 8; ++i) t[i] = N.phase_ms[i];
    return SC_OK;
}

int64_t numeric_syrk_stats(Numeric& N, int wmin, double* flops, double* ms, int64_t* launches) {
    // CB SYRK launches are split by w >= 256; wmin selects them (0: all CB launches,
    // -1: the panel-update launches instead, -2: the CB launches on 128 x 128 tiles with
    // the trickle epilogue, i.e. exactly the syrk_mfma_kernel<128,2,4,1,0> dispatches a
    // kernel trace lists)
    double fl = 0.0, t = 0.0;
    int64_t cnt = 0;
    bool have_t = N.status_valid && N.profile != 0;
    const std::vector<uint64_t> stamps = read_stamps(N);
    for (size_t i = 0; i < N.sched.size(); ++i) {
        const Launch& L = N.sched[i];
        if (L.kind != (wmin == -1 ? L_PANEL : L_CB)) continue;
        if (wmin >= 256 && !L.big) continue;
        if (wmin == -2 && (L.bt != SYRK_BT_LARGE || L.epi)) continue;
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
    std::vector<int2> diag, inv64, inv128;
    std::vector<int4> bwd, fwd;
    // internal index -> index in the caller's order (postorder, then the fill-reducing
    // permutation when one is in effect)
    std::vector<int32_t> solve_perm(S.post);
    if (!S.perm.empty())
        for (auto& v : solve_perm) v = S.perm[v];
    for (int32_t lev = 0; lev < S.nlevels; ++lev) {
        int maxw = 0;
        for (int32_t s : by_level[lev]) maxw = std::max(maxw, S.w(s));
        for (int k0 = 0; k0 < maxw; k0 += SOLVE_NB) {
            Numeric::SolveStep st {};
            st.doff = (int64_t)diag.size();
            st.goff = (int64_t)bwd.size();
            st.foff = (int64_t)fwd.size();
            for (int32_t s : by_level[lev]) {
                const int w = S.w(s), m = S.sn_m[s];
                if (w <= k0) continue;
                diag.push_back(make_int2(s, k0));
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
            N.solve_steps.push_back(st);
        }
    }
    int64_t rc;
    int32_t* d_rows = nullptr;
    int64_t* d_rows_ptr = nullptr;
    N.n_sinv = (int32_t)inv64.size();
    N.n_sinv2 = (int32_t)inv128.size();
    if ((rc = upload(N, diag, N.d_sdiag)) || (rc = upload(N, inv64, N.d_sinv)) || (rc = upload(N, inv128, N.d_sinv2)) ||
        (rc = upload(N, bwd, N.d_sgemv)) || (rc = upload(N, fwd, N.d_sfwd)) ||
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
        // forward: one fused launch per step (y to SP.y), then y -> c
        for (size_t i = 0; e == hipSuccess && i < N.solve_steps.size(); ++i) {
            const Numeric::SolveStep& t = N.solve_steps[i];
            e = launch_solve_fwd(N.SP, N.d_sfwd + t.foff, t.fcount, s0);
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

void comm_destroy(Numeric& N);  // dist.cpp

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
    if (e == hipSuccess) e = launch_syrk(d, dt, (int)tiles.size(), bt, 0, nullptr);
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
