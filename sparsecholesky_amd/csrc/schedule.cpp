// Static launch schedule of the numeric factorization (host).  Per assembly-tree
// level: small fronts (register kernels, chains, tiny trees), then the large fronts'
// assembly, the 64-column POTRF / TRSM chain with recursive inner updates and
// lookahead outer updates, and the CB SYRK (K = w, the children's CB entries
// gathered per tile).  Multi-rank handles add the comm steps of the plan (dist.cpp)
// and the distributed panels' slab schedule.  Task pointers are final device
// addresses, so the whole schedule can be captured once into a hipGraph.
#include "numeric_impl.hpp"

namespace sc {

// LDS edge of a small front's launch.  88: the widest front whose 4 x 4 tiles fit one
// per thread (KT = 1, 124 VGPRs, 4 workgroups per CU; 96 needs KT = 2 at 2 per CU)
static int bucket_of(int m) {
    if (m <= 32) return 32;
    if (m <= 64) return 64;
    if (m <= 88) return 88;
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

int64_t build_schedule(Numeric& N, SchedBuild& B) {
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
    std::vector<int32_t> init_step, deliver_step((size_t)S.nlevels, -1);
    // early children: early_step[c][g] = the DELIVER step of column group g (-1: none; a
    // group whose columns all stay on the producer has no messages and no step)
    std::vector<std::vector<int32_t>> early_step;
    // split fronts / distributed panels: slab_step[s][k] = the steps of slab k's pieces (dist_pieces)
    std::vector<std::vector<std::vector<int32_t>>> slab_step;
    std::vector<std::vector<int>> early_ev((size_t)S.ns);  // sender: event after each CB column group
    std::vector<int64_t> step_beg;
    std::vector<char> emitted;
    if (multi) {
        init_step.assign((size_t)S.ns, -1);
        slab_step.assign((size_t)S.ns, {});
        early_step.assign((size_t)S.ns, {});
        for (int32_t id = 0; id < (int32_t)D.steps.size(); ++id) {
            const DistStep& t = D.steps[id];
            if (t.kind == STEP_INIT) init_step[t.s] = id;
            if (t.kind == STEP_SLAB) {
                auto& ks = slab_step[t.s];
                if ((int)ks.size() <= t.k) ks.resize((size_t)t.k + 1);
                if ((int)ks[t.k].size() <= t.p) ks[t.k].resize((size_t)t.p + 1, -1);
                ks[t.k][t.p] = id;
            }
            if (t.kind == STEP_DELIVER && t.s < 0) deliver_step[t.level] = id;
            if (t.kind == STEP_DELIVER && t.s >= 0) {
                auto& es = early_step[t.s];
                if ((int)es.size() <= t.k) es.resize((size_t)t.k + 1, -1);
                es[t.k] = id;
            }
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
    // algorithmic HBM bytes of one SYRK task: its operand rows once, C written once when
    // the children are gathered (plus every child's CB entries read once), else C read
    // and written
    auto task_bytes = [&](const GemmTask& t) {
        const double pairs = (double)t.N * t.M - (double)t.N * (t.N - 1) / 2.0;
        double b = 8.0 * t.M * (double)t.K;
        if (t.gs < 0) return b + 16.0 * pairs;
        b += 8.0 * pairs;
        for (int32_t ci = S.child_ptr[t.gs]; ci < S.child_ptr[t.gs + 1]; ++ci) {
            const double mbc = S.mb(S.child_list[ci]);
            b += 8.0 * mbc * (mbc + 1.0) / 2.0;
        }
        return b;
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
        // CB launches of 64 < K <= syrk_lean_kmax (level 7 at 128^3) on the lean 64-tile
        // instance even when wide: 2.44 -> 2.24 ms (64-tiles up to K = 256 / 512 made levels
        // 8-10 slower, profiles/r06/ab_cb64.txt)
        if (kind == L_CB && S.opt.syrk_tile == 0 && maxK > 64 && maxK <= S.opt.syrk_lean_kmax) L.bt = SYRK_BT_SMALL;
        // instance tag (profiles): the critical path (main-stream panel updates) and the
        // short-K CB launches (levels 4-7 at 128^3) apart from the deep-K CB and the
        // lookahead stream -- the epilogue choice it used to make went with round 6's
        // staged epilogues (kernels.hip)
        L.epi = (kind == L_PANEL && strm == 0) || (kind == L_CB && maxK < SC_EPI_KMAX);
        // (CB launches with K <= 64 -- levels 4-6 at 128^3 -- are gather-bound and lose
        // more to the lean instance's smaller gather batches than they gain in occupancy)
        L.lean = L.bt == SYRK_BT_SMALL && S.opt.syrk_lean_kmax > 0 && maxK <= S.opt.syrk_lean_kmax &&
                 (kind == L_PANEL || maxK > 64);
        // panel-chain lookahead: a task whose pre-factor workgroup forms and factors the next
        // step's diagonal block (tile (0, 0), marker y = -1) -- 64 x 64 tiles, batched epilogue
        for (auto& t : tasks) L.pf |= t.pf >= 0 ? 1 : 0;
        if (L.pf) {
            L.bt = SYRK_BT_SMALL;
            L.lean = 0;
            L.epi = 1;
        }
        L.toff = (int64_t)tiles.size();
        L.bytes = 0.0;
        for (size_t q = 0; q < tasks.size(); ++q) {
            const size_t first = tiles.size();
            append_tiles(tiles, (int)q, tasks[q].M, tasks[q].N, L.bt);
            if (tasks[q].pf >= 0) tiles[first].y = -1;  // append_tiles emits tile (0, 0) first
            gemm.push_back(tasks[q]);
            L.bytes += task_bytes(tasks[q]);
        }
        L.count = (int32_t)((int64_t)tiles.size() - L.toff);
        xcd_order_tasks(tiles.data() + L.toff, L.count, tasks.data(), (int)tasks.size());
        if (L.pf)  // the pre-factor workgroups (the longest, on the chain) are dispatched first
            std::stable_partition(tiles.begin() + L.toff, tiles.end(), [](const int2& t) { return t.y < 0; });
        L.ntasks = (int32_t)tasks.size();
        L.big = big;
        L.flops = flops;
        // Deep-K CB launch on 128-tiles: every tile takes about the same time and 512 run
        // at once (two per CU), so a last partial round leaves most CUs idle for one whole
        // tile time (~2 ms at K = 8192).  Its tiles -- the last ones dispatched -- are re-cut
        // into 64 x 64 tiles in a launch of their own (up to 1024 at once, each ~1/4 of
        // the work): the tail shrinks to about a third (cb_tail_split).
        constexpr int64_t SLOTS = 512;
        const int64_t rem = L.count % SLOTS;
        if (kind == L_CB && L.bt == SYRK_BT_LARGE && S.opt.cb_tail_split && !L.epi && L.count > SLOTS && rem > 0 &&
            rem * 4 <= SLOTS * 3) {
            std::vector<int2> tail(tiles.end() - rem, tiles.end());
            tiles.resize(tiles.size() - (size_t)rem);
            L.count -= (int32_t)rem;
            std::stable_sort(tail.begin(), tail.end(), [](const int2& a, const int2& b) { return a.x < b.x; });
            Launch T = L;
            T.bt = SYRK_BT_SMALL;
            T.off = (int64_t)gemm.size();
            T.toff = (int64_t)tiles.size();
            gemm.insert(gemm.end(), tasks.begin(), tasks.end());
            double tfl = 0.0;
            for (const int2& t : tail) {
                const GemmTask& g = tasks[t.x];
                const int ti = t.y >> 16, tj = t.y & 0xffff;
                for (int a = 0; a < 2; ++a)
                    for (int b = 0; b < 2; ++b) {
                        const int si = 2 * ti + a, sj = 2 * tj + b;
                        if (si < sj || si * SYRK_BT_SMALL >= g.M || sj * SYRK_BT_SMALL >= g.N) continue;
                        tiles.push_back(make_int2(t.x, (si << 16) | sj));
                        // lower-triangle pairs of the sub-tile, 2 K flops each
                        const int64_t i0 = (int64_t)si * SYRK_BT_SMALL, i1 = std::min<int64_t>(i0 + SYRK_BT_SMALL, g.M);
                        const int64_t j0 = (int64_t)sj * SYRK_BT_SMALL, j1 = std::min<int64_t>(j0 + SYRK_BT_SMALL, g.N);
                        int64_t pairs = 0;
                        for (int64_t j = j0; j < j1; ++j) pairs += std::max<int64_t>(0, i1 - std::max(i0, j));
                        tfl += 2.0 * g.K * (double)pairs;
                    }
            }
            T.count = (int32_t)((int64_t)tiles.size() - T.toff);
            xcd_order_tasks(tiles.data() + T.toff, T.count, tasks.data(), (int)tasks.size());
            T.bytes = L.flops > 0.0 ? L.bytes * tfl / L.flops : 0.0;
            L.bytes -= T.bytes;
            T.flops = tfl;
            L.flops -= tfl;
            N.sched.push_back(L);
            N.sched.push_back(T);
            return;
        }
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
    // recv_strm: the stream that consumes what the step receives (it waits for the step;
    // the main stream by default)
    auto emit_step = [&](int32_t id, int send_ev = -1, int recv_strm = 0) {
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
            // copy tiles pack the column offset in 16 bits and the row chunk above it
            // (j | rc << 16, copy2d_kernel): a block wider than COPY_MAX_COLS goes as several
            // descriptors, each staging its columns at their packed position in the slot
            if ((int64_t)rows > (int64_t)COPY_ROWS * 32767) {
                N.err = "comm plan: block too tall for the copy tiles";
                return false;
            }
            for (int c0 = 0; c0 < cols; c0 += COPY_MAX_COLS) {
                Copy2D c {};
                c.a = a + (int64_t)c0 * ld;
                c.lda = ld;
                c.rows = rows;
                c.cols = std::min(COPY_MAX_COLS, cols - c0);
                (pack ? pack_d : unpack_d).push_back((int32_t)cbld.copies.size());
                cbld.copies.push_back(c);
                cbld.copy_slot.push_back(slot + (int64_t)c0 * rows);
            }
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
                for (int j = 0; j < cbld.copies[d].cols; j += COPY_COLS)
                    for (int rc = 0; rc * COPY_ROWS < cbld.copies[d].rows; ++rc)
                        cbld.ctiles.push_back(make_int2(d, j | (rc << 16)));
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
        if (any_recv) push_wait(recv_strm, push_record(2));
    };
    // the step of piece p of slab k of front s (-1: none), and all pieces of slab k
    auto slab_piece = [&](int32_t s, int k, int p) -> int32_t {
        if (!multi || k >= (int)slab_step[s].size() || p >= (int)slab_step[s][k].size()) return -1;
        return slab_step[s][k][p];
    };
    auto emit_slab = [&](int32_t s, int k, int recv_strm = 0) {
        if (!multi || k >= (int)slab_step[s].size()) return;
        for (int32_t id : slab_step[s][k]) emit_step(id, -1, recv_strm);
    };
    // the extend-add gather's segment table of front s on hosted rank v (GSeg): per 64 x 64
    // block of its CB, every child with CB rows and columns in the block, in child order
    // (the order the entries are added in); returns the task's offset in B.gblk
    auto gather_segments = [&](int32_t s, int v) -> int64_t {
        const int w = S.w(s), mb = S.mb(s), nb = (mb + 63) / 64;
        const int64_t gb = (int64_t)B.gblk.size();
        const RankMem& R = N.R[v];
        for (int rb = 0; rb < nb; ++rb)
            for (int cbk = 0; cbk <= rb; ++cbk) {
                B.gblk.push_back((int64_t)B.gseg.size());
                for (int32_t q = S.child_ptr[s]; q < S.child_ptr[s + 1]; ++q) {
                    const int32_t c = S.child_list[q];
                    const int32_t* rel = S.relind.data() + S.rel_ptr[c];
                    const int mbc = (int)(S.rel_ptr[c + 1] - S.rel_ptr[c]);
                    auto at = [&](int x) { return (int)(std::lower_bound(rel, rel + mbc, w + x) - rel); };
                    GSeg g {};
                    g.ilo = at(64 * rb);
                    g.ihi = at(std::min(mb, 64 * rb + 64));
                    g.jlo = at(64 * cbk);
                    g.jhi = at(std::min(mb, 64 * cbk + 64));
                    if (g.ilo >= g.ihi || g.jlo >= g.jhi) continue;
                    if (R.cb_off[c] < 0) {  // the memory plan keeps every gathered child's CB here
                        N.err = "schedule: gathered child CB not resident on its parent's rank";
                        continue;
                    }
                    g.cb = R.P.cb_pool + R.cb_base(S, c);
                    g.rel = R.P.relind + S.rel_ptr[c];
                    g.mbc = mbc;
                    B.gseg.push_back(g);
                }
            }
        B.gblk.push_back((int64_t)B.gseg.size());
        return gb;
    };
    auto is_early_sender = [&](int32_t s, int v) {
        return multi && D.early[s] && D.owner[s] == N.R[v].rank;
    };
    auto is_dasm = [&](int32_t s) { return multi && D.dasm[s]; };
    // panel_prefactor: the recursive inner update after a chain step also factors the next
    // step's diagonal block when that block is a full 64-column block of the same slab and
    // the update runs on 64 x 64 tiles (span <= 128; K = 64 or 128)
    auto prefactor_ok = [&](int span, int k1, int slab1) {
        return S.opt.panel_prefactor && S.opt.inner_order == 1 && S.opt.syrk_tile != 128 && span <= 2 * PNB &&
               k1 + PNB <= slab1;
    };
    // distributed assembly: one write-once tile-assembly launch of the front columns of
    // s that hosted rank v owns (its panel slabs and CB column blocks, D.col_owner), in
    // 16-column blocks; a block straddling another rank's columns computes those too,
    // into this rank's private copy, where nothing reads them
    auto emit_region_asm = [&](int32_t lev, int32_t s, int v) {
        const int who = N.R[v].rank, m = S.sn_m[s];
        Launch L {};
        L.kind = L_ASM;
        L.level = lev;
        L.vr = v;
        L.big = 1;
        L.epi = 1;  // the tasks carry column limits (B.asml)
        L.off = (int64_t)asmv.size();
        for (int cb = 0; cb * ASM_COLS < m; ++cb) {
            const int c1 = std::min(m, (cb + 1) * ASM_COLS);
            for (int a = cb * ASM_COLS; a < c1;) {  // each run of owned columns of the block
                if (D.col_owner(S, s, a) != who) {
                    ++a;
                    continue;
                }
                int b = a + 1;
                while (b < c1 && D.col_owner(S, s, b) == who) ++b;
                for (int k = cb * ASM_COLS / ASM_ROWS; k * ASM_ROWS < m; ++k) {
                    asmv.push_back(make_int2(s, (k << 16) | cb));
                    B.asml.resize(asmv.size(), make_int2(0, INT32_MAX));
                    B.asml.back() = make_int2(a, b);
                }
                a = b;
            }
        }
        L.count = (int32_t)((int64_t)asmv.size() - L.off);
        if (L.count > 0) N.sched.push_back(L);
    };
    // CB rank (hosted index v) of split front s: per final panel slab, CB -= L21_k
    // L21_k^T on the column blocks it owns (K = slab width), from its R_LAND copy
    auto emit_cb_rank = [&](int32_t lev, int32_t s, int v) {
        const int who = N.R[v].rank;
        const std::vector<int32_t>& cbr = D.cb_rank[D.split[s]];
        const int w = S.w(s), m = S.sn_m[s], mb = m - w;
        if (is_dasm(s))
            emit_region_asm(lev, s, v);  // its own CB blocks, from the children's columns it received
        else
            emit_step(init_step[s]);
        for (int k0 = 0, k = 0; k0 < w; k0 += D.nbo, ++k) {
            const int k1 = std::min(w, k0 + D.nbo);
            emit_slab(s, k);
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
        // small fronts: one launch sized for the level's largest front when the level
        // fits one workgroup per CU (fewer dependent launches on thin levels), else one
        // launch per LDS bucket (small fronts keep their occupancy on wide levels)
        int nsmall = 0, bmax = 0;
        for (int32_t s : nodes)
            if (S.fclass[s] == FRONT_SMALL) {
                ++nsmall;
                bmax = std::max(bmax, bucket_of(S.sn_m[s]));
            }
        for (int b : {32, 64, 88, 96, 128}) {
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
        auto gather = [&](int32_t s) {
            return S.opt.cb_gather && S.mb(s) > 0 && !is_split(s) && !is_early_sender(s, v);
        };
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
                if ((m >= tile_min_m) != (tiled == 1) || is_dasm(s)) continue;
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
        // distributed assembly of a split front: the owner assembles its panel columns,
        // the CB ranks their blocks (emit_cb_rank)
        for (int32_t s : large)
            if (is_dasm(s)) emit_region_asm(lev, s, v);
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
        // fronts whose block at the current step was pre-factored by the previous step's
        // inner update (panel_prefactor): their TRSM loads L11 (trsm_panel_g_kernel<2>)
        std::vector<char> pre((size_t)S.ns, 0);
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
            std::vector<TrsmTask> trsm_part;   // partial last blocks: own launch (big = 1)
            std::vector<TrsmTask> trsm_split;  // full blocks factored by the POTRF launch (own launch)
            // a step whose fused launch would exceed trsm_split_wg workgroups (more than the GPU
            // holds at once) factors each diagonal block once, in the POTRF launch, instead of
            // in every workgroup of every round
            int64_t step_wg = 0;
            for (int32_t s : large) {
                if (S.w(s) < k0 + PNB) continue;
                step_wg += (std::max(S.sn_m[s], k0 + PNB + 1) - (k0 + PNB) + TRSM_ROWS - 1) / TRSM_ROWS;
            }
            const bool split_step = S.opt.trsm_split_wg > 0 && step_wg > S.opt.trsm_split_wg;
            double uflops = 0.0, afl = 0.0, bfl = 0.0;
            for (int32_t s : large) {
                const int w = S.w(s), m = S.sn_m[s];
                if (w <= k0) continue;
                const int nb = std::min(PNB, w - k0);
                const int k1 = k0 + nb;
                const int slab0 = (k0 / NBO) * NBO;
                const int slab1 = std::min(w, slab0 + NBO);
                if (nb < PNB) {
                    potrf.push_back(make_int2(s, k0));
                    for (int r0 = k1; r0 < m; r0 += TRSM_ROWS) trsm_part.push_back(TrsmTask {s, k0, r0, m, 0});
                } else if (pre[s]) {  // L11 in place: the rows below only
                    for (int r0 = k1; r0 < m; r0 += TRSM_ROWS) trsm_split.push_back(TrsmTask {s, k0, r0, m, 0});
                } else if (split_step) {
                    potrf.push_back(make_int2(s, k0));
                    for (int r0 = k1; r0 < m; r0 += TRSM_ROWS) trsm_split.push_back(TrsmTask {s, k0, r0, m, 0});
                } else {  // fused POTRF (one task if no rows below); ctr - 1: arrival counter
                    const int ctr = (int)trsm.size() + 1;
                    for (int r0 = k1; r0 < std::max(m, k1 + 1); r0 += TRSM_ROWS) trsm.push_back(TrsmTask {s, k0, r0, m, ctr});
                }
                double* pan = panel_pool + poff[s];
                pre[s] = 0;
                if (k1 < slab1 && S.opt.inner_order == 1) {
                    // recursive order: block b of the slab closes a run of 2^t blocks
                    // (t = trailing zeros of b + 1); that run updates the next 2^t
                    // blocks (K = 64 * 2^t).  Same flops and dependencies as
                    // right-looking, 768 instead of 1792 C columns rewritten per slab.
                    const int b = (k0 - slab0) / PNB;
                    const int span = PNB << __builtin_ctz((unsigned)(b + 1));
                    add_update(upd, uflops, pan, m, m, k1, std::min(slab1, k1 + span), k1 - span, k1);
                    if (prefactor_ok(span, k1, slab1)) {
                        upd.back().pf = S.sn_start[s] + k1;
                        pre[s] = 1;
                    }
                } else if (k1 < slab1) {
                    add_update(upd, uflops, pan, m, m, k1, slab1, k0, k1);
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
            if (!trsm_split.empty()) {
                Launch Ls = Lt;
                Ls.off = (int64_t)trsm.size();
                Ls.count = (int32_t)trsm_split.size();
                Ls.epi = 2;  // the prefactored-block kernel instance
                trsm.insert(trsm.end(), trsm_split.begin(), trsm_split.end());
                N.sched.push_back(Ls);
            }
            if (!trsm_part.empty()) {
                Launch Lq = Lt;
                Lq.off = (int64_t)trsm.size();
                Lq.count = (int32_t)trsm_part.size();
                Lq.big = 1;
                trsm.insert(trsm.end(), trsm_part.begin(), trsm_part.end());
                N.sched.push_back(Lq);
            }
            push_gemm_launch(L_PANEL, lev, upd, 0, uflops);
            // split fronts: a slab is final after the TRSM of its last block; at a slab end
            // no inner update is pending
            for (int32_t s : large) {
                const int w = S.w(s);
                if (!is_split(s) || w <= k0) continue;
                const int k1 = std::min(w, k0 + PNB);
                if (k1 == w || k1 % D.nbo == 0) emit_slab(s, k0 / D.nbo);
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
                t.C = cb_pool + N.R[v].cb_base(S, s) + (int64_t)j0 * mb + j0;
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
                t.C = cb_pool + N.R[v].cb_base(S, s);
                t.A = panel_pool + poff[s] + w;
                t.ldc = mb;
                t.lda = m;
                t.M = mb;
                t.N = mb;
                t.K = w;
                if (gather(s)) {
                    t.gs = s;
                    t.gv = v;
                    t.gb = gather_segments(s, v);
                    t.gw = w;
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
        if (is_dasm(s)) {  // every holder assembles its own slabs and CB blocks
            for (int v : vs) emit_region_asm(lev, s, v);
        } else if (vo >= 0) {  // the owner assembles the whole front (tiled or column-streaming)
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
        int local_ev = -1;  // dist_local_pieces: event after the last local piece update
        for (int k = 0; k < nsl; ++k) {
            const int k0s = slab_c0(k), k1s = slab_c1(k);
            const int vk = hosted_of[sr[k]];
            local_ev = -1;
            if (vk >= 0) {
                // factor slab k: per 64 columns POTRF, TRSM of the rows below, and the
                // update of the slab's next columns (recursive order, as emit_level)
                const int e = last_ev1(vk, k - 2);
                if (e >= 0) push_wait(0, e);
                double* pan = pan_of(vk);
                bool pre_blk = false;  // this block was pre-factored by the previous inner update
                // dist_local_pieces: when this rank also owns the next slab, its update by each
                // finished piece of this slab goes on the lookahead stream while the chain goes on
                const bool local_next = S.opt.dist_local_pieces && k + 1 < nsl && sr[k + 1] == sr[k];
                local_ev = -1;
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
                    Lt.epi = pre_blk ? 2 : 0;  // L11 already in place: load it
                    const int ctr = (nb < PNB || pre_blk) ? 0 : (int)trsm.size() + 1;  // fused POTRF: arrival counter
                    for (int r0 = k1; r0 < ((nb < PNB || pre_blk) ? m : std::max(m, k1 + 1)); r0 += TRSM_ROWS)
                        trsm.push_back(TrsmTask {s, k0, r0, m, ctr});
                    pre_blk = false;
                    Lt.count = (int32_t)((int64_t)trsm.size() - Lt.off);
                    if (Lt.count > 0) N.sched.push_back(Lt);
                    // a finished piece of the slab leaves now (dist_pieces)
                    if (k1 == k1s || (k1 - k0s) % D.pw == 0) {
                        const int pc = (k1 - 1 - k0s) / D.pw;
                        emit_step(slab_piece(s, k, pc));
                        if (local_next) {  // dist_local_pieces: this rank's next slab, by this piece, now
                            const int j0 = slab_c0(k + 1), j1 = slab_c1(k + 1), c0 = k0s + pc * D.pw;
                            std::vector<GemmTask> t0;
                            double fl = 0.0;
                            upd_task(t0, fl, pan + (int64_t)j0 * m + j0, m, pan + (int64_t)c0 * m + j0, m, m - j0,
                                     j1 - j0, std::min(k1s, c0 + D.pw) - c0);
                            push_wait(1, push_record(0));
                            push_gemm_launch(L_PANEL, lev, t0, 0, fl, 1);
                            local_ev = push_record(1);
                        }
                    }
                    if (k1 < k1s) {
                        std::vector<GemmTask> upd;
                        double fl = 0.0;
                        if (S.opt.inner_order == 1) {
                            const int b = (k0 - k0s) / PNB;
                            const int span = PNB << __builtin_ctz((unsigned)(b + 1));
                            const int c1 = std::min(k1s, k1 + span);
                            upd_task(upd, fl, pan + (int64_t)k1 * m + k1, m, pan + (int64_t)(k1 - span) * m + k1, m,
                                     m - k1, c1 - k1, span);
                            if (!upd.empty() && prefactor_ok(span, k1, k1s)) {
                                upd.back().pf = S.sn_start[s] + k1;
                                pre_blk = true;
                            }
                        } else {
                            upd_task(upd, fl, pan + (int64_t)k1 * m + k1, m, pan + (int64_t)k0 * m + k1, m, m - k1,
                                     k1s - k1, nb);
                        }
                        push_gemm_launch(L_PANEL, lev, upd, 0, fl);
                    }
                }
            }
            // slab k's update on every hosted rank that needs it
            for (int v : vs) {
                const int r = N.R[v].rank;
                if (D.need_row(S, s, k, r) >= m) continue;
                double* pan = pan_of(v);
                const double* Lk = pan + (int64_t)k0s * m;  // column k0s of the slab, row 0
                const int K = k1s - k0s;
                if (k + 1 < nsl && sr[k + 1] == r && v == vk && local_ev >= 0) {  // done during the chain
                    push_wait(0, local_ev);
                } else if (k + 1 < nsl && sr[k + 1] == r) {  // the next slab: critical path, piece by piece
                    const int e = last_ev1(v, k - 1);
                    if (e >= 0) push_wait(0, e);
                    const int j0 = slab_c0(k + 1), j1 = slab_c1(k + 1);
                    for (int p = 0, c0 = k0s; c0 < k1s; ++p, c0 += D.pw) {
                        emit_step(slab_piece(s, k, p));
                        std::vector<GemmTask> t0;
                        double fl = 0.0;
                        upd_task(t0, fl, pan + (int64_t)j0 * m + j0, m, pan + (int64_t)c0 * m + j0, m, m - j0,
                                 j1 - j0, std::min(k1s, c0 + D.pw) - c0);
                        push_gemm_launch(L_PANEL, lev, t0, 0, fl);
                    }
                }
                // the rest of slab k feeds only the lookahead stream's updates here: that
                // stream waits for it, the main stream (this rank's chain) does not
                emit_slab(s, k, 1);
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
    // single device, n <= TINY_DENSE_N (and the tiny_dense option): the whole matrix as
    // one dense lower triangle in one wave (kernels.hip tiny_dense_kernel); the plan is
    // one (Ax index, panel position) pair per dense entry (column c, row r) at c * 64 + r,
    // -1 where the entry has no A value / is not stored (internal numbering: the factor
    // of the postordered matrix is the postordered factor, so the dense image is the
    // multifrontal result)
    // (A value and panel byte offsets stay inside the kernel's 32-bit buffer ranges)
    const bool dense = !multi && S.opt.tiny_dense && S.n > 0 && S.n <= TINY_DENSE_N && S.nnzA_in < (1 << 27);
    if (dense) {
        for (int32_t s = 0; s < S.ns; ++s) {
            const int m = S.sn_m[s], w = S.w(s), c0 = S.sn_start[s];
            const int32_t* rows = S.rows.data() + S.rows_ptr[s];
            if (B.ta.empty()) B.ta.assign((size_t)tiny_dense_np((int)S.n) * 64, make_int2(-1, -1));
            for (int lc = 0; lc < w; ++lc)
                for (int64_t q = S.a_ptr[c0 + lc]; q < S.a_ptr[c0 + lc + 1]; ++q)
                    B.ta[(size_t)(c0 + lc) * 64 + rows[S.a_pos[q]]].x = (int32_t)S.a_src[q];
            const int64_t off = N.R[0].panel_off[s];
            for (int j = 0; j < w; ++j)
                for (int i = j; i < m; ++i) B.ta[(size_t)(c0 + j) * 64 + rows[i]].y = (int32_t)(off + (int64_t)j * m + i);
        }
        Launch L {};
        L.kind = L_SMALL;
        L.level = 0;
        L.maxm = (int32_t)S.n;
        L.big = 3;  // tiny dense
        L.count = 1;
        N.sched.push_back(L);
    }
    bool tiny = !dense && !multi && S.ns > 1 && S.ns <= TINY_MAX_FRONTS;
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
    for (int32_t lev = (tiny || dense) ? S.nlevels : 0; lev < S.nlevels; ++lev) {
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
            if (!D.early[c] || early_step[c].empty()) continue;
            const int ng = (S.mb(c) + D.early_gw - 1) / D.early_gw;
            const int vs = hosted_of[D.owner[c]];
            for (int g = 0; g < ng; ++g)
                if (g < (int)early_step[c].size())
                    emit_step(early_step[c][g], vs >= 0 && !early_ev[c].empty() ? early_ev[c][g] : -1);
        }
        emit_step(deliver_step[lev]);
        comm_done[lev] = push_record(2);
    }
    if (multi) push_wait(0, push_record(2));  // join the comm stream (its last sends)
    if (!N.err.empty()) return SC_ERR_ARG;
    return SC_OK;
}

}  // namespace sc
