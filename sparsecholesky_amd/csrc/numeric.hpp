// Device numeric factorization driver: memory plan, level schedule, launches, export.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "kernels.hpp"
#include "symbolic.hpp"

namespace sc {

enum LaunchKind : int32_t {
    L_SMALL = 0,
    L_ASM = 1,
    L_POTRF = 2,
    L_TRSM = 3,
    L_PANEL = 4,
    L_CB = 5,
    L_COMM = 6,    // one comm step of the hosted ranks (pack, transfer group, unpack)
    L_RECORD = 11, // record sync event `count` on stream `strm`
    L_WAIT = 12,   // stream `strm` waits for sync event `count`
    L_KINDS = 13
};

// ---------------- multi-GPU plan (dist.cpp) ----------------
// Comm steps, in one global order every rank follows (each rank posts exactly its
// part of every step it takes part in, as one transfer group, on its comm stream):
//   STEP_INIT(s)    split front s: the owner sends the assembled CB column blocks to
//                   the ranks that compute them
//   STEP_SLAB(s,k)  split front s: the owner sends rows [w, m) of panel slab k (final)
//                   to every CB rank
//   STEP_DELIVER(l) after level l: every contribution block (column block) whose
//                   producer is not the executing rank of the parent goes there; one
//                   sub-step (s = child, k = group) per column group of an early child
//                   first, then one (s = -1) with the rest
enum StepKind : int32_t { STEP_INIT = 0, STEP_SLAB = 1, STEP_DELIVER = 2 };
struct DistStep {
    int32_t kind, level, s, k;
    int32_t p = 0;  // STEP_SLAB of a distributed panel: the column piece of slab k (dist_pieces)
};

// Device memory regions of a rank (memplan.cpp).  Messages and tasks name a region
// by kind, supernode and LOGICAL coordinates; every rank maps them to its own
// physical layout, so sender and receiver may store a block differently.
//   R_PANEL  the L panel of s: m x w, row = front row (owner only; permanent)
//   R_CB     the contribution block of s: mb x mb, row/col = front row - w, held as a
//            full square (ld = mb) on every rank that computes or receives part of it
//            (only those parts are valid there)
//   R_LAND   a split front's L21 (rows [w, m) of its panel) on a CB rank: mb x w
enum RegionKind : int32_t { R_PANEL = 0, R_CB = 1, R_LAND = 2 };

// One 2D block transfer: rows x cols doubles from (skind, s, srow, scol) on src to
// (dkind, s, drow, dcol) on dst, moved packed (column-contiguous) through staging.
struct DistMsg {
    int32_t step;
    int32_t src, dst;
    int32_t skind, dkind;
    int32_t s;
    int32_t srow, scol, drow, dcol;
    int32_t rows, cols;
};
struct DistPlan {
    int nranks = 1;
    int cbb = 1024;  // CB column-block width
    int nbo = 1024;  // panel slab width (panel_nb_outer)
    int pw = 1024;   // distributed panels: columns per STEP_SLAB piece (nbo / dist_pieces, 64-aligned)
    std::vector<int32_t> owner;    // rank executing each supernode's assembly + panel
    std::vector<int32_t> gsize;    // rank-group size of each supernode (1 = inside a subtree)
    std::vector<int32_t> split;    // index into split_s / cb_rank, or -1
    std::vector<int32_t> split_s;
    std::vector<std::vector<int32_t>> cb_rank;  // per split front: rank of CB column block jb
    // distributed panels (dist_panel): a shared front wider than one slab has panel slab
    // k (columns [k nbo, (k+1) nbo)) factored by slab_rank[pd[s]][k] (slab 0 on the
    // owner, the rest cyclic over the group); every rank in holders[pd[s]] (slab owners
    // and CB ranks, ascending) keeps a full m x w panel copy
    std::vector<int32_t> pd;       // per supernode: index into pd_s / slab_rank / holders, or -1
    std::vector<int32_t> pd_s;
    std::vector<std::vector<int32_t>> slab_rank;
    std::vector<std::vector<int32_t>> holders;
    // first front row rank r needs of final slab k of distributed front s: the start of
    // its first own slab after k, or w for a CB rank; m = not needed
    int need_row(const Symbolic& S, int32_t s, int k, int r) const;
    bool holds(int32_t s, int r) const;  // r keeps a panel copy of s (owner included)
    // distributed assembly (dist_asm): a shared front with a distributed panel or a split
    // CB is assembled where its columns live -- every rank assembles the panel slabs and
    // CB column blocks it owns, and each child's CB columns go straight to the rank
    // owning the parent columns they map into (no STEP_INIT)
    std::vector<char> dasm;
    int col_owner(const Symbolic& S, int32_t p, int col) const;  // rank assembling front column col of p
    // rank r assembles a parent column that child c's CB maps into (holds CB(c) until then)
    bool receives(const Symbolic& S, int32_t c, int r) const;
    // rank r computes column blocks of s's CB (holds the full-square CB(s) from level(s))
    bool produces_cb(const Symbolic& S, int32_t s, int r) const;
    // early delivery: a large, unsplit child whose parent runs on another rank has its
    // CB SYRK in column groups of early_gw, each group sent as soon as it is computed
    int early_gw = 4096;
    std::vector<char> early;
    std::vector<DistStep> steps;
    std::vector<DistMsg> msgs;     // ascending step
    std::vector<double> work;      // estimated flops per rank
};
int64_t dist_plan(const Symbolic& S, int nranks, DistPlan& D);

// Memory of one rank (a process hosts one rank, or every rank when emulated).
//   panel arena  the L panels of the supernodes this rank owns, back to back
//   work arena   transient regions (contribution blocks, landing slabs), each live
//                over a closed interval of assembly-tree levels; offsets from an
//                interval plan (memplan.cpp), so a region is reused once dead
struct RankMem {
    int32_t rank = 0;
    std::vector<int64_t> panel_off;  // per supernode: doubles into the panel arena, -1 = not here
    std::vector<int64_t> cb_off;     // per supernode: the CB region in the work arena, -1 = not here
    // per supernode: first CB column the region holds (columns [cb_col0, ...) of the mb x mb
    // square, ld = mb): a rank computing or receiving only some column blocks of a shared
    // front's CB keeps just their column range; cb_base() is the square's (virtual) origin
    std::vector<int32_t> cb_col0;
    int64_t cb_base(const Symbolic& S, int32_t s) const { return cb_off[s] - (int64_t)cb_col0[s] * S.mb(s); }
    std::vector<int64_t> land_off;   // per supernode: R_LAND slab (ld = mb) in the work arena, -1
    int64_t panel_total = 0;     // doubles (incl. the PNB tail the TRSM reads past)
    int64_t work_total = 0;      // doubles: high-water mark of the interval plan
    int64_t work_live_max = 0;   // doubles: max over levels of the live region sizes (lower bound)
    DevPlan P {};                // pools + device copies of panel_off / cb_off
};
// Plan rank `rank`'s regions (D == nullptr: single device, every front here);
// `placed` (optional) receives every work-arena region with its lifetime.
struct PlacedRegion {
    int64_t off, size;
    int32_t t0, t1;
};
int64_t plan_rank_memory(const Symbolic& S, const DistPlan* D, int rank, RankMem& R,
                         std::vector<PlacedRegion>* placed = nullptr);
// Panel arena of `rank` alone: panel_off per supernode (-1 = no copy here); returns
// the arena size in doubles (incl. the PNB tail the TRSM reads past)
int64_t plan_rank_panels(const Symbolic& S, const DistPlan* D, int rank, std::vector<int64_t>& panel_off);
int64_t plan_check(const Symbolic& S, int nranks);
// Physical location of logical element (row, col) of region (kind, s) on R: arena
// (0 panel, 1 work), offset in doubles and leading dimension.  false: not on R.
bool region_addr(const Symbolic& S, const DistPlan* D, const RankMem& R, int kind, int s, int row, int col,
                 int& arena, int64_t& off, int64_t& ld);
// Region lifetimes of the plan, in assembly-tree levels (exposed for tests):
// fills the peak and the lower bound of the work arena of every rank.
int64_t plan_memory_stats(const Symbolic& S, int nranks, int64_t* panel_doubles, int64_t* work_doubles,
                          int64_t* work_lower_bound);

// transport argument of numeric_create_dist selecting the dry mode
#define DIST_DRY ((int32_t(*)(void*, int32_t, int32_t, void*, int64_t))1)

// One transfer of a comm step, device addresses resolved.
enum MsgOp : int32_t { MSG_SEND = 0, MSG_RECV = 1, MSG_COPY = 2 };
struct Msg {
    double* buf;      // staging slot (packed rows x cols), or the region itself when contiguous
    double* src_buf;  // MSG_COPY (both ends hosted, device-copy transport): the sender's slot
    int64_t count;    // doubles
    int32_t peer;     // communicator rank of the other end
    int32_t op;       // MsgOp
};

struct Launch {
    int32_t kind;
    int32_t level;
    int64_t off;      // first task in the kind's task array
    int64_t toff;     // first tile in the SYRK tile list
    int32_t count;    // grid size (tiles for SYRK launches)
    int32_t ntasks;   // tasks (SYRK launches)
    int32_t maxm;     // small-front LDS edge
    int32_t big;      // CB launch covering fronts with w >= 256
    int32_t bt;       // SYRK tile edge (64 or 128)
    int32_t epi;      // SYRK instance tag: critical-path panel updates and short-K CB launches (profiles)
    int32_t lean;     // SYRK on 64 x 64 tiles with half the LDS (deepest K <= syrk_lean_kmax)
    int32_t pf;       // panel update carrying pre-factor workgroups (GemmTask.pf; 64 x 64 tiles)
    int32_t strm;     // 0 = main stream, 1 = lookahead stream, 2 = comm stream
    int32_t vr;       // hosted rank whose DevPlan the kernel uses
    double flops;     // algorithmic SYRK flops (CB launches: mb*(mb+1)*w)
    double bytes;     // algorithmic HBM bytes of a SYRK launch (numeric_syrk_bytes)
    // L_COMM: copy tiles [poff, poff + pcount) pack the sends, [uoff, uoff + ucount)
    // unpack the receives (Numeric::d_ctiles)
    int64_t poff, uoff;
    int32_t pcount, ucount;
    int32_t step;
};

struct Numeric {
    const Symbolic* S = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;  // trailing panel updates overlapped with the next slab
    hipStream_t stream3 = nullptr;  // multi-rank: comm stream (pack, transfer group, unpack), strm == 2
    std::vector<hipEvent_t> sync_ev;
    int32_t n_sync_events = 0;
    std::vector<RankMem> R;          // hosted ranks
    std::vector<int64_t> rank_base;  // gathered panel layout: first double of each rank's arena
    std::vector<void*> allocs;
    int64_t dev_bytes = 0;           // device memory held (pools, plan, staging)
    std::vector<Launch> sched;
    int32_t* d_small = nullptr;
    ChainPlan CP {};                 // chain launches (runs of single small-front levels)
    TinyPlan TP {};                  // tiny trees: the whole factorization in one workgroup
    int64_t n_chain = 0;             // chained fronts (descriptors)
    int2* d_asm = nullptr;
    int2* d_asml = nullptr;  // per assembly task: owned front columns (distributed-assembly launches)
    int2* d_potrf = nullptr;
    TrsmTask* d_trsm = nullptr;
    int32_t* d_arrive = nullptr;  // fused POTRF + TRSM: per-block arrival counters
    GemmTask* d_gemm = nullptr;
    int2* d_tiles = nullptr;
    GatherTab gtab;              // the CB SYRK extend-add gather's segment tables (schedule.cpp)
    int32_t* d_info = nullptr;       // shared by the hosted ranks' DevPlans
    int32_t* h_info = nullptr;       // pinned host copy, written at the end of each factorization
    static constexpr int32_t STATUS_PENDING = -2;  // h_info before the status kernel's store
    // single-rank handles: device view of h_info; the last launch of a factorization stores
    // the status word there (and re-arms d_info), the host polls it (no memset / copy)
    int32_t* status_dp = nullptr;
    double* d_Ax_owned = nullptr;
    const double* last_Ax = nullptr;
    bool factored = false;
    int64_t factor_gen = 0;          // factorizations enqueued
    int64_t status = 0;
    bool status_valid = false;

    // profiling: 1 = HIP events around every launch (eager runs); 2 = timestamp
    // kernels around the CB SYRK launches only (works inside hipGraph replay)
    int profile = 0;
    uint64_t* d_stamps = nullptr;
    std::vector<int32_t> stamp_of;  // launch -> stamp pair index, -1 = none
    std::vector<hipEvent_t> ev;
    double phase_ms[8] = {0};
    // hipGraph replay
    bool use_graph = false;
    hipGraphExec_t gexec = nullptr;
    hipGraph_t graph = nullptr;
    const double* graph_Ax = nullptr;
    int graph_profiled = 0;

    // multi-rank: this process hosts R (one rank of nranks, or all of them when
    // emulated on one device with private per-rank memory)
    int rank = 0, nranks = 1;
    bool emulated = false;
    int emul_rccl = 0;  // emulated: 1 = hosted-to-hosted transfers as RCCL self send/recv
    std::vector<int32_t> owner;  // empty = single device
    DistPlan D;
    std::vector<Msg> msgs;
    Copy2D* d_copy = nullptr;     // pack / unpack descriptors
    int2* d_ctiles = nullptr;     // (descriptor, first column) per copy workgroup
    double* staging = nullptr;    // packed slots of the hosted ranks' messages
    void* comm = nullptr;  // ncclComm_t
    // host-staged transport (tests: several processes on one GPU, no RCCL):
    // op 0 post send, 1 post recv, 2 complete everything posted
    int32_t (*xport)(void* ctx, int32_t op, int32_t peer, void* buf, int64_t bytes) = nullptr;
    void* xport_ctx = nullptr;
    bool dry_comm = false;  // comm steps pack / unpack but move nothing (one-rank timing projection)

    // gathered factor (every supernode's panel in the rank_base layout): the panel
    // arena itself for single-device and emulated handles, else gathered on demand
    double* gpanel = nullptr;
    bool gpanel_owned = false;
    int64_t gather_gen = -1;         // factor_gen the gathered copy belongs to
    std::vector<int64_t> gpo;        // per supernode: offset in gpanel
    int64_t* d_gpo = nullptr;
    struct SlabFix {                 // gathered copy of a slab another rank factored
        int64_t src, dst, ld;        // doubles into gpanel
        int32_t rows, cols;
    };
    std::vector<SlabFix> fix;

    // triangular solves (built at the first solve)
    struct SolveStep {
        int64_t doff, goff, foff, gaoff;
        int32_t dcount, gcount, fcount, gacount;  // gacount: forward-gather fronts (level's first step)
    };
    std::vector<SolveStep> solve_steps;  // forward order (levels up, k0 up)
    bool solve_ready = false;
    SolvePlan SP {};
    int4* d_sdiag = nullptr;         // 128-column diagonal blocks (s, k0, first GEMV task, GEMV tasks)
    int32_t* d_sgather = nullptr;    // forward gather: fronts with children, per level
    int64_t u_total = 0;             // doubles of SP.u (sum of the fronts' mb)
    int2* d_sinv = nullptr;          // 64-column blocks (s, k0): inverse preparation
    int2* d_sinv2 = nullptr;         // 128-column blocks wider than 64: off-diagonal inverse quadrant
    int32_t n_sinv = 0, n_sinv2 = 0;
    int64_t inv_gen = -1;            // factor_gen whose diagonal-block inverses are in place
    int4* d_sgemv = nullptr;         // backward GEMV tasks (s, k0, r0)
    int4* d_sfwd = nullptr;  // fused forward steps (s, k0, r0, writer)
    int32_t* d_post = nullptr;
    double* d_sbuf = nullptr;  // host-interface staging (b in, x out)
    bool solve_eager = false;          // debug: launch the sweeps directly instead of the graph
    hipGraph_t solve_graph = nullptr;  // both sweeps captured once (b in / x out through d_sbuf)
    hipGraphExec_t solve_gexec = nullptr;

    std::string err;
};

// Builds the memory plan, pools and schedule of the hosted ranks.
int64_t numeric_init(Numeric& N, const Symbolic& S, int device);

int64_t numeric_create(const Symbolic& S, int device, Numeric*& out, std::string& err);
int64_t numeric_factor(Numeric& N, const double* d_Ax, bool sync);
int64_t numeric_status(Numeric& N);
// Makes gpanel / gpo hold the whole factor of the last factorization (multi-rank
// handles: a collective exchange of every rank's panel arena; all ranks call it).
int64_t numeric_gather(Numeric& N);
int64_t numeric_export(Numeric& N, int64_t* Lp, int32_t* Li, double* Lx);
// Natural columns [j0, j1) in front-row form (count only when ri == NULL): column j
// holds the rows of its supernode's front from its own position down (natural
// numbering, front order; relaxed zeros included) with their values.  cp[j1-j0+1].
int64_t numeric_export_cols(Numeric& N, int64_t j0, int64_t j1, int64_t* cp, int32_t* ri, double* rx);
int64_t numeric_timing(Numeric& N, double* t, int nt);
int64_t numeric_level_times(Numeric& N, double* ms, int nl);
int64_t numeric_launch_trace(Numeric& N, int32_t* kind, int32_t* level, int32_t* strm, double* ms, double* flops,
                             int64_t cap);
int64_t numeric_syrk_stats(Numeric& N, int wmin, double* flops, double* ms, int64_t* launches);
int64_t numeric_syrk_bytes(Numeric& N, int wmin, double* bytes);
int64_t numeric_launch_times(Numeric& N, double* t0, double* t1, int32_t* kind, int32_t* step, int32_t* strm,
                             int64_t cap);
void numeric_free(Numeric* N);
// x = A^{-1} b with the factor: device vectors of length n (may alias), on the
// library stream, synchronous.  Multi-rank handles gather the factor first
// (collective) and every rank solves with the whole factor.
int64_t numeric_solve_device(Numeric& N, const double* d_b, double* d_x);
int64_t numeric_solve_host(Numeric& N, const double* b, double* x);
int64_t debug_syrk(double* dC, int ldc, const double* dA, int lda, int M, int N, int K);
int64_t numeric_chain_stamps(Numeric& N, int enable, uint64_t* out, int64_t cap);
int64_t debug_bench(int which, int M, int K, int reps, int arg, double* tflops);
int64_t debug_contention(int M, int K, int chain_rows, int nchain, int mode, int mask_stride, double* out);

}  // namespace sc
