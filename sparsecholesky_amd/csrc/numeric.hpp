// Device numeric factorization driver: pools, level schedule, launches, export.
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
    L_COMM = 6,    // CB send/recv group after a level (multi-GPU)
    L_RECORD = 7,  // record sync event `count` on stream `strm`
    L_WAIT = 8,    // stream `strm` waits for sync event `count`
    L_KINDS = 9
};

// ---------------- multi-GPU plan (dist.cpp) ----------------
// Comm steps, in one global order every rank follows (each rank posts exactly its
// part of every step it takes part in, as one RCCL group, on its comm stream):
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
};
// One 2D block transfer: rows x cols doubles at pool + off, leading dimension ld,
// moved packed (rows-contiguous) through a staging slot.
struct DistMsg {
    int32_t step;
    int32_t src, dst;
    int32_t pool;  // 0 = panel pool, 1 = CB pool
    int64_t off;
    int64_t ld;
    int32_t rows, cols;
    int32_t s;     // supernode the block belongs to
};
struct DistPlan {
    int nranks = 1;
    int cbb = 1024;  // CB column-block width
    int nbo = 1024;  // panel slab width (panel_nb_outer)
    std::vector<int32_t> owner;    // rank executing each supernode's assembly + panel
    std::vector<int32_t> gsize;    // rank-group size of each supernode (1 = inside a subtree)
    std::vector<int32_t> split;    // index into split_s / cb_rank, or -1
    std::vector<int32_t> split_s;
    std::vector<std::vector<int32_t>> cb_rank;  // per split front: rank of CB column block jb
    // early delivery: a large, unsplit child whose parent runs on another rank has its
    // CB SYRK in column groups of early_gw, each group sent as soon as it is computed
    int early_gw = 4096;
    std::vector<char> early;
    std::vector<DistStep> steps;
    std::vector<DistMsg> msgs;     // ascending step
    std::vector<double> work;      // estimated flops per rank
};
int64_t dist_plan(const Symbolic& S, int nranks, DistPlan& D);
// transport argument of numeric_create_dist selecting the dry mode
#define DIST_DRY ((int32_t(*)(void*, int32_t, int32_t, void*, int64_t))1)

// One point-to-point block transfer of this rank (device addresses resolved).
struct Msg {
    double* buf;      // staging slot (packed rows x cols)
    int64_t count;    // doubles
    int32_t peer;
    int32_t is_send;
    int32_t child;    // supernode whose data moves
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
    int32_t strm;     // 0 = main stream, 1 = lookahead stream
    double flops;     // algorithmic SYRK flops (CB launches: mb*(mb+1)*w)
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
    hipStream_t stream3 = nullptr;  // multi-GPU: comm stream (pack, RCCL group, unpack), strm == 2
    std::vector<hipEvent_t> sync_ev;
    int32_t n_sync_events = 0;
    DevPlan P {};
    std::vector<void*> allocs;
    std::vector<Launch> sched;
    int32_t* d_small = nullptr;
    int2* d_asm = nullptr;
    int2* d_potrf = nullptr;
    int4* d_trsm = nullptr;
    GemmTask* d_gemm = nullptr;
    int2* d_tiles = nullptr;
    double* d_Ax_owned = nullptr;
    const double* last_Ax = nullptr;
    bool factored = false;
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

    // multi-GPU: owner rank per supernode (empty = single GPU).  virt_ranks > 1
    // runs the partitioned schedule of all ranks in this one process (shared
    // pools, no transfers) to validate the partition on one device.
    int rank = 0, nranks = 1, virt_ranks = 0;
    std::vector<int32_t> owner;
    DistPlan D;
    std::vector<Msg> msgs;
    Copy2D* d_copy = nullptr;     // pack / unpack descriptors
    int2* d_ctiles = nullptr;     // (descriptor, first column) per copy workgroup
    double* staging = nullptr;    // one packed slot per message of this rank
    void* comm = nullptr;  // ncclComm_t
    // host-staged transport (tests: several processes on one GPU, no RCCL):
    // op 0 post send, 1 post recv, 2 complete everything posted
    int32_t (*xport)(void* ctx, int32_t op, int32_t peer, void* buf, int64_t bytes) = nullptr;
    void* xport_ctx = nullptr;
    bool dry_comm = false;  // comm steps pack / unpack but move nothing (one-rank timing projection)
    double comm_ms = 0.0;

    // triangular solves (built at the first solve)
    struct SolveStep {
        int64_t doff, goff, foff;
        int32_t dcount, gcount, fcount;
    };
    std::vector<SolveStep> solve_steps;  // forward order (levels up, k0 up)
    bool solve_ready = false;
    SolvePlan SP {};
    int2* d_sdiag = nullptr;
    int4* d_sgemv = nullptr;
    int4* d_sfwd = nullptr;  // fused forward steps (s, k0, r0, writer)
    int32_t* d_post = nullptr;
    double* d_sbuf = nullptr;  // host-interface staging (b in, x out)
    hipGraph_t solve_graph = nullptr;  // both sweeps captured once per (b, x) pair
    hipGraphExec_t solve_gexec = nullptr;
    const double* solve_b = nullptr;
    double* solve_x = nullptr;

    std::string err;
};

// Builds pools + schedule; owner/rank restrict the schedule to one rank's fronts.
int64_t numeric_init(Numeric& N, const Symbolic& S, int device);

int64_t numeric_create(const Symbolic& S, int device, Numeric*& out, std::string& err);
int64_t numeric_factor(Numeric& N, const double* d_Ax, bool sync);
int64_t numeric_status(Numeric& N);
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
void numeric_free(Numeric* N);
// x = A^{-1} b with the factor: device vectors of length n (may alias), on the
// library stream, synchronous.  Single-device factors only.
int64_t numeric_solve_device(Numeric& N, const double* d_b, double* d_x);
int64_t numeric_solve_host(Numeric& N, const double* b, double* x);
int64_t debug_syrk(double* dC, int ldc, const double* dA, int lda, int M, int N, int K);
int64_t debug_bench(int which, int M, int K, int reps, int arg, double* tflops);

}  // namespace sc
