// Device-side plan layout and kernel launch wrappers (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace sc {

// Inner panel width (POTRF/TRSM block); the diagonal block lives in LDS.
constexpr int PNB = 64;
// Rows per TRSM workgroup (one lane per row).
constexpr int TRSM_ROWS = 256;
// Columns owned by one assembly workgroup (one wave per column at a time).
constexpr int ASM_COLS = 16;
constexpr int ASM_ROWS = 256;  // rows per LDS tile of the write-once assembly
constexpr int ASM_TILE_MIN_M = 512;   // fronts at least this tall use the write-once tile kernel
// Output tile edges of the MFMA SYRK kernel (per launch).
constexpr int SYRK_BT_SMALL = 64;
constexpr int SYRK_BT_LARGE = 128;

// C/D register map of v_mfma_f64_16x16x4_f64 on gfx950 (cdna_hip_programming.md
// section 3): col = lane & 15, row = (lane >> 4) + 4 * reg.
#define MFMA_F64_ROW(lane, r) (((lane) >> 4) + 4 * (r))

// child columns per batch of loads in the CB SYRK's extend-add gather
#ifndef SC_GATHER_Q
#define SC_GATHER_Q 4
#endif

// All device arrays of the numeric plan (internal numbering).
struct DevPlan {
    const int32_t* sn_start;    // ns+1
    const int32_t* sn_m;        // ns
    const int64_t* panel_off;   // ns+1
    const int64_t* cb_off;      // ns+1
    const int32_t* child_ptr;   // ns+1
    const int32_t* child_list;
    const int64_t* rel_ptr;     // ns+1
    const int32_t* relind;
    const int64_t* rb_ptr;      // ns+1
    const int32_t* rel_bnd;     // per child: CB row bounds of the parent's ASM_ROWS row tiles
    const int64_t* cbk_ptr;     // ns+1
    const int32_t* col_bnd;     // per child: CB row bounds of the parent's ASM_COLS column blocks
    const int64_t* tb_ptr;      // ns+1
    const int32_t* tile_bnd;    // per child: CB row bounds of the parent's 64-row CB blocks (symbolic.hpp)
    const int64_t* a_ptr;       // n+1 (internal columns)
    const int32_t* a_pos;       // row position in the column's front
    const int64_t* a_src;       // index into the input value array
    double* panel_pool;
    double* cb_pool;
    int32_t* info;              // min failing internal column + 1
};

// One child's share of one 64 x 64 block (rb, cb) of a parent's contribution block
// (the CB SYRK's extend-add gather): its CB rows [ilo, ihi) map into the parent's CB
// rows [64 rb, 64 rb + 64) and its CB columns [jlo, jhi) into the parent's CB columns
// [64 cb, 64 cb + 64); cb / rel: the child's CB (ld mbc) and relative indices (parent
// front positions).  Host-built per gathering task (schedule.cpp gather_segments).
struct GSeg {
    const double* cb;
    const int32_t* rel;
    int32_t mbc, ilo, ihi, jlo, jhi, pad;
};

// The schedule's gather tables (device), kernel arguments of the CB SYRK launches.
struct GatherTab {
    const int64_t* blk = nullptr;
    const GSeg* seg = nullptr;
    int32_t* info = nullptr;  // status word (pivot failures of the panel pre-factor workgroups)
};

// One lower-trapezoid SYRK update: C[i,j] -= sum_k A[i,k] A[j,k], j < N, j <= i < M.
// gs >= 0 (CB updates only): C is front gs's whole contribution block and is not read;
// the children's CB entries that fall into it are gathered instead (the extend-add of
// the reference's apply_update, chol.hpp:1196) and C = sum(children) - A A^T is written.
// gv: the hosted rank that holds the children.  gb: the task's offset in the gather
// table's block list (GatherTab.blk: per 64 x 64 block (rb, cb <= rb) of the CB, at
// gb + rb (rb + 1) / 2 + cb, the block's first segment in GatherTab.seg; the next entry
// ends it).
struct GemmTask {
    double* C;
    const double* A;
    int64_t ldc;
    int64_t lda;
    int32_t M, N, K;
    int32_t gs = -1, gv = 0;
    int64_t gb = -1;
    int32_t gw = 0;  // gathering tasks: the front's width (the CB starts at front row gw; K may be one slab)
    // panel updates (launches with pf = 1): >= 0 = the internal column of the 64 x 64 diagonal
    // block at C's origin, which this task's pre-factor workgroup (tile marker y = -1) updates
    // and factors in registers, so the next chain step's TRSM loads L11 instead of factoring it
    int32_t pf = -1;
};
// Strided <-> packed copy of a rows x cols block (pack: a -> b; unpack: b -> a).
struct Copy2D {
    double* a;  // strided, leading dimension lda
    double* b;  // packed, leading dimension rows
    int64_t lda;
    int32_t rows, cols;
};

constexpr int COPY_COLS = 16;    // columns per copy workgroup
constexpr int COPY_ROWS = 2048;  // rows per copy workgroup
// copy tiles encode (column offset | row chunk << 16): the host cuts wider blocks into
// descriptors of at most this many columns (schedule.cpp emit_step)
constexpr int COPY_MAX_COLS = 32768;
static_assert(COPY_MAX_COLS + COPY_COLS <= 65536, "column offsets fit the tile's 16 low bits");
// tiles: (descriptor, first column | row chunk << 16) per workgroup
hipError_t launch_copy2d(const Copy2D* descs, const int2* tiles, int count, bool unpack, hipStream_t st);

// ---- triangular solves with the supernodal factor ----
struct SolvePlan {
    const int32_t* sn_start;
    const int32_t* sn_m;
    const int64_t* panel_off;
    const int64_t* rows_ptr;  // ns+1
    const int32_t* rows;      // front rows (internal numbering), first w = the pivots
    const double* panel_pool;
    double* c;                // right-hand side / solution, internal numbering
    double* y;                // forward result (fused steps write here; copied to c after the sweep)
    // deterministic accumulation (no atomics): the forward sweep leaves each front's
    // updates of its contribution-block rows in u (u + u_off[s], mb entries, multifrontal
    // style), and the parent's gather (solve_fwd_gather_kernel) adds its children's u in
    // child order; the backward GEMV leaves one partial column sum per workgroup in part
    // (SOLVE_NB per task of the launch), summed in task order by the diagonal kernel
    double* u;
    const int64_t* u_off;     // per supernode
    const int32_t* child_ptr; // ns+1
    const int32_t* child_list;
    const int64_t* rel_ptr;   // ns+1: child c's CB rows -> parent front rows
    const int32_t* relind;
    double* part;
};
constexpr int SOLVE_ROWS = 256;  // front rows per GEMV workgroup
constexpr int SOLVE_NB = 128;    // columns per solve step (two 64-blocks)
// X = inv(L11) of the 64 x 64 diagonal blocks (s, k0) (tasks) into their strict upper
// triangles, then (tasks2: 128-column blocks wider than 64) the off-diagonal quadrant
// E = -Xb B Xa of the 128-block inverse into the block's upper-right square; the
// factor's lower part is untouched.  Once per factorization, before the first solve.
hipError_t launch_solve_inv(const SolvePlan& P, const int2* tasks, int count, const int2* tasks2, int count2,
                            hipStream_t st);
// Forward step: tasks (s, k0, r0, writer) of 128-column blocks; every workgroup forms
// y = X128 c_blk and applies -L[r, blk] y for its SOLVE_ROWS rows: to c for the front's
// own later pivot rows, to u for its contribution-block rows (no atomics: each row has
// one writer per step); r0 < 0 = the diagonal block only.
hipError_t launch_solve_fwd(const SolvePlan& P, const int4* tasks, int count, hipStream_t st);
// Forward gather, before a level's first step: per front s of the list, its children's
// u in child order -- entries at s's pivot rows into c, the rest into u of s.
hipError_t launch_solve_fwd_gather(const SolvePlan& P, const int32_t* fronts, int count, hipStream_t st);
// Backward step: tasks (s, k0, r0): partial -L[rows, blk]^T x[rows] per workgroup into
// part, then tasks (s, k0, g0, ng): c_blk plus the block's ng partials (launch-relative
// GEMV tasks g0..) in order, x_blk = X128^T c_blk.
hipError_t launch_solve_gemv(const SolvePlan& P, const int4* tasks, int count, hipStream_t st);
hipError_t launch_solve_diag(const SolvePlan& P, const int4* tasks, int count, hipStream_t st);
// c[i] = b[perm[i]] (gather) or x[perm[i]] = c[i] (scatter)
hipError_t launch_permute(double* dst, const double* src, const int32_t* perm, int64_t n, bool scatter,
                          hipStream_t st);

// Small fronts (m <= maxm <= 128): one workgroup per front, factored in registers
// (4 x 4 tiles per thread); seq: one workgroup runs the fronts in order (a whole
// small tree in postorder, CBs through HBM).
hipError_t launch_front_small(const DevPlan& P, const int32_t* nodes, int count, int maxm, bool seq,
                              const double* Ax, hipStream_t st);

// Chain launches (a run of >= 2 single-front levels; each front the parent of the one
// before).  chain_init_kernel assembles every chained front's A entries and its
// children other than the chain child (all computed by earlier launches) into a
// packed image in HBM, all fronts in parallel; front_chain_kernel (one workgroup)
// then runs the chain, front i + 1's image streaming into registers while front i
// is factored and front i's CB added into front i + 1 straight from registers.
struct ChainDesc {
    int32_t s, c0, w, m;
    int32_t sp;      // the chain child (previous chained front), -1 for the first
    int32_t pad;
    int64_t panel_off, cb_off;
    int64_t init_off;  // doubles into ChainPlan::init (packed image, m (m + 1) / 2)
    int64_t relp_off;  // words into ChainPlan::relp: per tile row, the parent rows of its 4 rows
};
struct ChainPlan {
    const ChainDesc* desc;
    double* init;
    const uint32_t* relp;  // four 8-bit parent rows per word (relind < parent m <= 128)
    uint64_t* stamps;  // debug: per front 5 shader-clock stamps (thread 0; stride 8), or null
};
constexpr int CHAIN_NT = 768;        // threads of the chain workgroup (>= 528 tiles of m = 128; 3 waves per SIMD)
constexpr int CHAIN_MAXF = 256;      // chained fronts whose descriptors are staged in LDS
// Tiny trees (every front small, few of them, everything fits LDS): one workgroup
// runs the whole factorization with every front image and contribution block in
// LDS.  Host-built lists: the A stores (Ax index -> LDS), and per front and child the
// extend-add pairs (LDS CB entry -> LDS image entry), child by child.
struct TinyFront {
    int32_t s, c0, w, m;
    int32_t img, cb;  // LDS offsets (doubles) of the image (packed m x m lower) and the CB (packed)
    int32_t e0, np;   // the front's extend-add phases: ph[e0 .. e0 + np)
    int64_t panel_off;
};
struct TinyPlan {
    const TinyFront* fr;
    const int2* a;    // (Ax index, LDS image index)
    const int2* ph;   // (first pair, end pair) per phase
    const int2* pr;   // (LDS CB index, LDS image index)
    int32_t nf, na, nph, npr;
    int32_t lds;      // doubles of images + CBs
    int32_t* host_info;  // device view of the handle's pinned status word: the kernel owns the status
                         // (no reset / copy launches around it), or null
    int32_t nax = 0;     // tiny dense: A values (the range of the lane map's Ax indices)
    int32_t npan = 0;    // tiny dense: panel-pool doubles (the range of its panel offsets)
};
constexpr int TINY_MAX_FRONTS = 16;
constexpr int TINY_MAX_LDS = 12288;  // doubles of images + CBs (96 KB)
constexpr int TINY_PR_LDS = 2048;    // extend-add pairs staged in LDS with the A loads (the rest from HBM)
hipError_t launch_tiny_tree(const DevPlan& P, const TinyPlan& T, int maxm, const double* Ax, hipStream_t st);
// Tiny dense (n <= TINY_DENSE_N, one device): the whole matrix as one dense lower
// triangle in one wave, lane i holding row i in registers, four pivots per step.  The
// TinyPlan list a is reused as the lane map: a[c * 64 + r] = (Ax index of entry (r, c)
// or -1, its panel-pool offset or -1) for the kernel's padded order NP; na = NP * 64.
constexpr int TINY_DENSE_N = 64;
inline int tiny_dense_np(int n) { return n <= 16 ? 16 : n <= 32 ? 32 : n <= 48 ? 48 : 64; }
hipError_t launch_tiny_dense(const DevPlan& P, const TinyPlan& T, int n, const double* Ax, hipStream_t st);

hipError_t launch_front_chain(const DevPlan& P, const ChainPlan& C, int first, int count, int maxm,
                              const double* Ax, hipStream_t st);
// tiled: tasks are (front, (row tile << 16) | 16-column block) for the write-once
// tile kernel (fronts with m >= ASM_TILE_MIN_M), else (front, column block); lim (tiled
// only, may be null): per task the front columns [x, y) to assemble (distributed assembly)
hipError_t launch_assemble_large(const DevPlan& P, const int2* tasks, int count, const double* Ax,
                                 hipStream_t st, bool tiled, const int2* lim = nullptr);
// Large-front panel kernels (generated straight-line code, panel_gen.inc): the
// 64 x 64 diagonal POTRF (one wave per block) and the TRSM of the rows below it
// (TRSM_ROWS rows per task).  partial: every task is a partial last block (nb < 64).
hipError_t launch_potrf_diag(const DevPlan& P, const int2* tasks, int count, hipStream_t st);
// One workgroup of the panel TRSM of block k0 (columns k0 .. k0 + 64) of front s: rows
// [r0, min(r0 + TRSM_ROWS, r1)); ctr - 1 indexes the block's arrival counter (fused POTRF).
struct TrsmTask {
    int32_t s, k0, r0, r1, ctr;
};
// partial: blocks with nb < 64; else full blocks with the POTRF fused (arrive: the
// per-block arrival counters, zeroed)
// pre: 0 fused POTRF, 2 the diagonal blocks already factored by their own launch
// (trsm_split_wg)
hipError_t launch_trsm_panel(const DevPlan& P, const TrsmTask* tasks, int count, hipStream_t st, bool partial,
                             int32_t* arrive, int pre = 0);
// gt: the gather tables (CB tasks with gs >= 0 gather their children's entries)
// lean: 64 x 64 tiles with half the LDS (BK = 8; short-K launches, syrk_lean_kmax)
hipError_t launch_syrk(const GemmTask* tasks, const int2* tiles, int total_tiles, int bt, int tag, hipStream_t st,
                       int epi = 0, GatherTab gt = {}, bool lean = false, bool pf = false);
hipError_t launch_stamp(uint64_t* slot, hipStream_t st);
// the factorization's status word (d_info) to the pinned host word, d_info re-armed
hipError_t launch_status_publish(int32_t* info, int32_t* host, hipStream_t st);

hipError_t launch_hwid(uint32_t* out, int nwg, int threads, int spin, hipStream_t st);
hipError_t launch_fill_random(double* p, int64_t n, hipStream_t st);
hipError_t launch_mfma_peak(double* out, int blocks, int iters, int nacc, hipStream_t st);

// tiles of an M x N lower trapezoid with square BT tiles
inline int64_t syrk_tiles(int64_t M, int64_t N, int bt) {
    const int64_t TM = (M + bt - 1) / bt, TN = (N + bt - 1) / bt;
    return TN * TM - TN * (TN - 1) / 2;
}

// Append the lower-trapezoid tiles of `task` as {task, ti<<16 | tj}, walking
// G x G super-tiles so that consecutive tiles share row and column panels.
void append_tiles(std::vector<int2>& out, int task, int M, int N, int bt, int G = 8);
// Permute a launch's tile run so block b (XCD b % 8 under round-robin dispatch)
// takes a contiguous chunk: neighbouring tiles share one XCD's L2.
void xcd_order(int2* tiles, int64_t n);

}  // namespace sc
