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

// One point-to-point contribution-block transfer (multi-GPU).
struct Msg {
    double* buf;
    int64_t count;  // doubles
    int32_t peer;
    int32_t is_send;
    int32_t child;  // supernode whose CB moves
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
    int32_t fuse;     // panel launch whose tasks may factor the next diagonal block (potrf_col)
    double flops;     // algorithmic SYRK flops (CB launches: mb*(mb+1)*w)
};

struct Numeric {
    const Symbolic* S = nullptr;
    int device = 0;
    int panel_variant = PANEL_VARIANT;  // large-front POTRF/TRSM kernels (kernels.hpp)
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;  // trailing panel updates overlapped with the next slab
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
    std::vector<Msg> msgs;
    void* comm = nullptr;  // ncclComm_t
    double comm_ms = 0.0;

    std::string err;
};

// Builds pools + schedule; owner/rank restrict the schedule to one rank's fronts.
int64_t numeric_init(Numeric& N, const Symbolic& S, int device);

int64_t numeric_create(const Symbolic& S, int device, Numeric*& out, std::string& err);
int64_t numeric_factor(Numeric& N, const double* d_Ax, bool sync);
int64_t numeric_status(Numeric& N);
int64_t numeric_export(Numeric& N, int64_t* Lp, int32_t* Li, double* Lx);
int64_t numeric_timing(Numeric& N, double* t, int nt);
int64_t numeric_level_times(Numeric& N, double* ms, int nl);
int64_t numeric_launch_trace(Numeric& N, int32_t* kind, int32_t* level, int32_t* strm, double* ms, double* flops,
                             int64_t cap);
int64_t numeric_syrk_stats(Numeric& N, int wmin, double* flops, double* ms, int64_t* launches);
void numeric_free(Numeric* N);
int64_t debug_syrk(double* dC, int ldc, const double* dA, int lda, int M, int N, int K);
int64_t debug_bench(int which, int M, int K, int reps, int arg, double* tflops);

}  // namespace sc
