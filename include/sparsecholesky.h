/*
 * sparsecholesky.h -- C-ABI of the MI355X-native supernodal sparse Cholesky.
 *
 * This is the drop-in boundary for the numeric path of evanwporter/SparseCholesky.
 * The reference has no FFI: its API is header-only C++ templates
 * (include/chol.hpp).  Each entry point below names the reference interface it
 * replaces (file:line in the reference).  The C++ drop-in header
 * include/sparsecholesky/chol.hpp rebuilds the reference's templates
 * (csc_matrix, SChol, schol, chol, chol_sn, ...) on top of these calls.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Column pointers are int64 (the reference's
 *     int overflows past 2^31-1 nonzeros, chol.hpp:52,765); row indices int32.
 *   - Matrices are CSC.  "A upper" means the reference's csc_matrix<T,sym::upper>
 *     (chol.hpp:134): entries with row > col are ignored, exactly as the
 *     reference's etree/ereach/col_count ignore them (chol.hpp:392,696,539).
 *   - Status: 0 = OK; >0 = 1-based global (natural) column whose pivot was not
 *     positive ("A is not positive definite.", chol.hpp:849-850; LAPACK info
 *     style); <0 = an sc_status error code below.
 *   - The caller owns every host array it passes; the library owns device memory.
 *     One handle per host thread; all device work runs on the stream given at
 *     numeric creation (or the library's own stream).
 */
#ifndef SPARSECHOLESKY_H
#define SPARSECHOLESKY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

#define SC_VERSION 121 /* 1.2.1: small merged fronts amalgamated past relax_wmax (different supernode partition of some inputs, same L); 1.2.0: persistent slab chain options removed; panel_prefactor, dist_local_pieces and SC_ORDER_AMD added; out-of-range lookahead / inner_order / ordering rejected */

enum sc_status {
    SC_OK = 0,
    SC_ERR_ARG = -1,      /* bad argument / malformed CSC */
    SC_ERR_NOMEM = -2,    /* host allocation failed */
    SC_ERR_HIP = -3,      /* HIP runtime error (device missing, launch failure) */
    SC_ERR_DEVMEM = -4,   /* device allocation failed */
    SC_ERR_STATE = -5,    /* call out of order (e.g. export before factor) */
    SC_ERR_COMM = -6,     /* RCCL / transport error */
    SC_ERR_NOTIMPL = -7,
    SC_ERR_NOTSYM = -8,   /* MatrixMarket input that is not symmetric (general / skew-symmetric) */
    SC_ERR_IO = -9        /* file could not be opened */
};

typedef struct sc_symbolic sc_symbolic;
typedef struct sc_numeric sc_numeric;

/* Analysis options.  Defaults: sc_default_options(), which also sets struct_size;
 * sc_analyze rejects (SC_ERR_ARG) options whose struct_size is not this header's
 * sizeof(sc_options), so a caller built against another layout fails loudly instead
 * of misreading fields. */
typedef struct sc_options {
    int32_t struct_size;     /* sizeof(sc_options) of the caller's header (set by sc_default_options) */
    int32_t relax;           /* 1 = relaxed supernode amalgamation (CHOLMOD-style) */
    int32_t nrelax[3];       /* width thresholds for amalgamation */
    double zrelax[3];        /* zero-fraction thresholds for amalgamation */
    int32_t small_front_max; /* fronts with m <= this run in the fused one-workgroup kernel (clamped to [0, 128]) */
    int32_t panel_nb;        /* inner panel block (potrf/trsm width), 64 */
    int32_t panel_nb_outer;  /* slab width NBO: rank-NBO outer panel updates at slab ends (default 1024) */
    int32_t use_graph;       /* capture the level schedule into a hipGraph and replay it */
    int32_t relax_wmax;      /* a child and its parent that are both wider than this are not amalgamated when
                                the parent has other children (chains still merge; 0 = no limit; default 1) */
    int32_t syrk_tile;       /* 0 = auto (128x128/8 waves for wide, deep updates, else 64x64/4 waves); 64; 128 */
    int32_t lookahead;       /* 0 or 1 (other values: SC_ERR_ARG); 1 (default): at a slab end the next slab's columns are updated on the main stream
                                and every later column on a second stream, overlapping the next slab's
                                POTRF/TRSM chain; 0: the whole trailing update on the main stream */
    int32_t inner_order;     /* updates inside a slab: 0 right-looking (K = 64), 1 recursive (K = 64..NBO/2);
                                other values: SC_ERR_ARG */
    int32_t asm_tile_min_m;  /* fronts with m >= this use the write-once tiled assembly (0 = default 8192) */
    int32_t dist_split;      /* multi-GPU: a shared front with a contribution block keeps its panel on one rank and
                                has its contribution block computed by the other ranks of its group, slab-streamed
                                (1, default); 0: every front on one rank */
    int32_t dist_cbb;        /* multi-GPU: column-block width of contribution-block ownership and transfers (1024) */
    int32_t ordering;        /* SC_ORDER_NATURAL (default: the given order, as the reference), SC_ORDER_ND or
                                SC_ORDER_AMD: factor P A P^T with a nested-dissection / approximate-minimum-degree
                                P (sc_symbolic_perm); L, the pattern and the statistics are then those of P A P^T,
                                solves take and return A's order; other values: SC_ERR_ARG */
    int32_t dist_early;      /* multi-GPU: a large child whose parent runs on another rank computes its CB in
                                4-block column groups and sends each group as soon as it is done (1, default) */
    int32_t dist_panel;      /* multi-GPU: a shared front wider than one slab (panel_nb_outer) has its panel
                                factored 1D slab-cyclic over its rank group, each final slab sent to the ranks
                                that update later slabs or its contribution block (1, default); 0: the panel
                                on the front's owner */
    int32_t cb_gather;       /* 1 (default): a large front's contribution block is not assembled; its CB SYRK
                                gathers the children's entries into each output tile (C = sum - L21 L21^T,
                                written once); 0: assembly writes the whole front, the SYRK updates it */
    int32_t dist_slab_block; /* multi-GPU distributed panels: consecutive slabs per rank in the cyclic deal
                                (default 2: every other slab hand-over is rank-local, off the critical path;
                                capped at slabs / ranks so that every rank of the group gets a block) */
    int32_t trsm_split_wg;   /* a 64-column chain step whose TRSM launch spans more than this many 256-row
                                workgroups (more than the GPU holds at once) factors its diagonal blocks in a
                                launch of their own (one workgroup per block) and the TRSM workgroups load the
                                factored blocks instead of each refactoring them (default 1024; 0: always fused) */
    int32_t syrk_lean_kmax;  /* SYRK launches on 64 x 64 tiles whose deepest K is at most this use the lean
                                kernel instance (K staged 8 deep, 32-row extend-add chunks: half the LDS, six
                                workgroups per CU instead of four); default 128, 0: never */
    int32_t cb_tail_split;   /* 1 (default): the last, partial round of a deep-K CB launch on 128 x 128 tiles
                                runs as 64 x 64 tiles in a launch of its own (a shorter tail); 0: one launch */
    int32_t tiny_dense;      /* 1 (default): on one device, a matrix with n <= 64 factors as one dense n x n
                                lower triangle in a single wave (the symbolic pattern is exact: entries outside
                                it come out as exact zeros and are not exported); 0: the tiny-tree launch */
    int32_t dist_asm;        /* multi-GPU: 1 (default): a shared front with a distributed panel or split CB is
                                assembled where its columns live (each rank its own slabs / CB blocks; child CB
                                columns go straight to the rank owning the parent columns they map into, no
                                assembled-front hand-out); 0: its owner assembles it and sends the pieces */
    int32_t dist_pieces;     /* multi-GPU distributed panels: each final slab is handed over in this many column
                                pieces (default 4: 256 of a 1024-column slab), each sent as soon as the chain has
                                finished it, so the next slab's owner starts updating before the slab is done */
    int32_t dist_local_pieces; /* multi-GPU distributed panels: when a rank owns two consecutive slabs, its update of
                                the second by each finished piece of the first runs on the lookahead stream while
                                the first slab's chain goes on (1, default), instead of after the chain on the
                                main stream (0) */
    int32_t panel_prefactor; /* 1 (default): in the 64-column panel chain, the recursive inner update after a step
                                (K = 64 or 128) also forms and factors the NEXT step's 64 x 64 diagonal block in one
                                extra workgroup, so that step's TRSM loads L11 instead of every TRSM workgroup
                                factoring it (the POTRF runs beside the update's tiles, off the chain's critical
                                path; bitwise-identical factor); 0: every full step fuses its POTRF */
} sc_options;

enum { SC_ORDER_NATURAL = 0, SC_ORDER_ND = 1, SC_ORDER_AMD = 2 };

/* Symbolic statistics (host analysis). */
typedef struct sc_symbolic_stats {
    int64_t n;
    int64_t nnz_A;            /* stored upper entries used */
    int64_t nnz_L;            /* sum of column counts (reference L pattern) */
    double flops;             /* F = sum_j colcount[j]^2 */
    int64_t etree_depth;
    int64_t n_fundamental;    /* supernodes by the reference rule, in postorder */
    int64_t n_supernodes;     /* after relaxed amalgamation */
    int64_t n_levels;         /* assembly-tree height + 1 */
    int64_t max_front_m;
    int64_t max_front_w;
    int64_t panel_entries;    /* sum m*w (L storage incl. relaxed zeros) */
    int64_t cb_entries;       /* sum (m-w)^2 (contribution-block storage) */
    double flops_executed;    /* dense flops the fronts actually execute */
    double flops_syrk_w256;   /* SYRK flops mb*(mb+1)*w of fronts with w >= 256 */
    int64_t n_small_fronts;
    int64_t n_large_fronts;
} sc_symbolic_stats;

/* Version / status text. */
int32_t sc_version(void);
const char* sc_status_string(int64_t status);
void sc_default_options(sc_options* opt);

/* ---------------- host symbolic analysis ----------------
 * Replaces: schol(A)            chol.hpp:873-946  (pattern of L)
 *           etree/post_order/col_count inside chol() and schol()
 *           compute_supernodes / atree / compute_levels  src/chol.cpp:7-136
 * The supernode partition used numerically is the reference rule
 * (src/chol.cpp:75-85) applied in etree postorder, plus relaxed amalgamation.
 */
int64_t sc_analyze(int64_t n, const int64_t* Ap, const int32_t* Ai, const sc_options* opt,
                   sc_symbolic** out);
int64_t sc_symbolic_get_stats(const sc_symbolic* sym, sc_symbolic_stats* stats);
int64_t sc_nnz_L(const sc_symbolic* sym);
double sc_flops(const sc_symbolic* sym);
/* Pattern of L in the reference layout (schol(A).p()/i(), chol.hpp:873-946):
 * Lp[n+1], Li[nnz_L]; lower, diagonal first, rows ascending. */
int64_t sc_symbolic_pattern(const sc_symbolic* sym, int64_t* Lp, int32_t* Li);
/* etree parent (chol.hpp:377) and postorder (chol.hpp:466), natural numbering. */
int64_t sc_symbolic_etree(const sc_symbolic* sym, int32_t* parent, int32_t* post);
/* The relaxed supernode partition used on the device (internal = postorder
 * numbering): sn_start[ns+1] first internal column, sn_m[ns] front rows,
 * sn_parent[ns] assembly-tree parent (-1 = root), level[ns] height.  Any may be NULL. */
int64_t sc_symbolic_supernodes(const sc_symbolic* sym, int32_t* sn_start, int32_t* sn_m, int32_t* sn_parent,
                               int32_t* level);
/* The ordering used: perm[new] = old (identity for SC_ORDER_NATURAL); returns 1
 * when a fill-reducing permutation is in effect, else 0. */
int64_t sc_symbolic_perm(const sc_symbolic* sym, int32_t* perm);
void sc_free_symbolic(sc_symbolic* sym);

/* ---------------- device numeric factorization ----------------
 * Replaces: chol(A)     chol.hpp:749-863  (simplicial, the parity oracle)
 *           chol_sn(A)  chol.hpp:1406-1446 (supernodal: dpotrf_ 1263,
 *                       cblas_dtrsm 1292, cblas_dsyrk 1322, apply_update 1196)
 * sc_numeric_create allocates the device pools for L panels and contribution
 * blocks on HIP device `device` (-1 = current) and builds the level schedule.
 */
int64_t sc_numeric_create(const sc_symbolic* sym, int32_t device, sc_numeric** out);
/* Factor with host values Ax[nnz(A)] (same order as Ai).  Includes H2D copy. */
int64_t sc_factor(sc_numeric* num, const double* Ax);
/* Factor with device-resident values d_Ax (HBM).  Asynchronous on the library
 * stream unless sync != 0; sc_numeric_status() syncs and returns the status. */
int64_t sc_factor_device(sc_numeric* num, const double* d_Ax, int32_t sync);
/* Status of the last factorization: 0, or the 1-based natural column of the failing
 * pivot (not positive definite).  COLLECTIVE on a one-rank-per-process handle
 * (sc_numeric_create_dist / _dist_host): the first call after each factorization
 * reduces the minimum failing column over all ranks, so every rank must make it, in
 * the same order relative to the handle's other collective calls -- and so must
 * sc_factor, sc_factor_device(sync != 0), sc_export_L, sc_export_L_cols(rx != NULL)
 * and the solves, which read the status.  A rank that skips it leaves the others
 * waiting.  Later calls before the next factorization are local. */
int64_t sc_numeric_status(sc_numeric* num);
/* Export L in the reference CSC layout (chol() output, chol.hpp:749-863):
 * Lp[n+1], Li[nnz_L], Lx[nnz_L]; any of the three may be NULL.  On a multi-rank
 * handle the call is collective (every rank calls it): the ranks exchange their
 * panels and every rank receives the whole L, as the reference's chol() returns it
 * (chol.hpp:858-862). */
int64_t sc_export_L(sc_numeric* num, int64_t* Lp, int32_t* Li, double* Lx);
/* Columns [j0, j1) of L straight from the supernodal panels (no pattern pass; for
 * factors too large for sc_export_L): column j holds its front's rows from j down
 * (row indices in the same numbering as Lp/Li, relaxed zeros included), values
 * in rx.  cp[j1-j0+1] offsets; ri / rx may be NULL to query the count.  Returns
 * the entry count (>= 0) or an error.  Collective on multi-rank handles when rx != NULL. */
int64_t sc_export_L_cols(sc_numeric* num, int64_t j0, int64_t j1, int64_t* cp, int32_t* ri, double* rx);
/* Device pointer of the library stream (hipStream_t) for event timing. */
void* sc_numeric_stream(sc_numeric* num);
/* Per-phase timing of the last factorization, milliseconds (HIP events):
 * t[0]=total, t[1]=CB transfers (multi-GPU), t[2]=small fronts, t[3]=assembly, t[4]=potrf,
 * t[5]=trsm, t[6]=panel update, t[7]=CB syrk.  sc_numeric_set_profile(num, 1): HIP
 * events around every launch (eager runs; sets use_graph aside); 2: timestamp
 * kernels around the CB SYRK launches only, which also works under hipGraph
 * replay (feeds sc_numeric_syrk_stats). */
int64_t sc_numeric_set_profile(sc_numeric* num, int32_t on);
int64_t sc_numeric_timing(sc_numeric* num, double* t, int32_t nt);
/* Wall time (ms) of each assembly-tree level of the last profiled factorization;
 * returns the number of levels. */
int64_t sc_numeric_level_times(sc_numeric* num, double* ms, int32_t nl);
/* Per-launch trace of the last profiled factorization (kind: 0 small fronts,
 * 1 assembly, 2 potrf, 3 trsm, 4 panel SYRK, 5 CB SYRK, 6 CB transfer); returns
 * the launch count; arrays may be NULL to query it. */
int64_t sc_numeric_launch_trace(sc_numeric* num, int32_t* kind, int32_t* level, int32_t* stream, double* ms,
                                double* flops, int64_t cap);
/* SYRK flops and kernel time (ms) of the last factorization restricted to
 * fronts with w >= wmin (north-star gate: wmin = 256); wmin = 0: every CB launch;
 * wmin = -1: the panel-update launches; wmin = -2: the CB launches on 128 x 128
 * tiles (one kernel instance, comparable with a kernel trace). */
int64_t sc_numeric_syrk_stats(sc_numeric* num, int32_t wmin, double* flops, double* ms,
                              int64_t* launches);
/* Algorithmic HBM bytes of the same launch selection as sc_numeric_syrk_stats: the
 * operand rows read once (8 M K per task), C written once (gathered CB) or read and
 * written (assembled C), and every gathered child's CB entries read once.  A launch
 * whose tail tiles are re-cut into a launch of their own splits its bytes in
 * proportion to the flops. */
int64_t sc_numeric_syrk_bytes(sc_numeric* num, int32_t wmin, double* bytes);
/* Timeline of the last profiled (sc_numeric_set_profile(num, 1)) factorization: per
 * launch its start and end (ms from the first main-stream launch), its kind (the
 * launch-trace kinds; 6 = a comm step), for comm steps the step index of the plan
 * (sc_dist_steps, else -1) and its stream (0 main, 1 lookahead, 2 comm).  Returns the
 * number of launches (t0 == NULL: count only). */
int64_t sc_numeric_launch_times(sc_numeric* num, double* t0, double* t1, int32_t* kind, int32_t* step,
                                int32_t* stream, int64_t cap);
/* Device memory of the handle, bytes: info[0] everything allocated (pools, plan,
 * staging, a gathered factor), info[1] panel arenas (L), info[2] work arenas (the
 * interval-planned contribution blocks), info[3] the work arenas' lower bound (the
 * largest sum of regions live at one level).  n = entries wanted (<= 4). */
int64_t sc_numeric_memory(sc_numeric* num, int64_t* info, int32_t n);
/* The memory plan without a device: per rank (nranks entries each) the panel arena,
 * the work arena and its lower bound, bytes.  nranks = 1: the single-device plan. */
int64_t sc_memory_plan(const sc_symbolic* sym, int32_t nranks, int64_t* panel_bytes, int64_t* work_bytes,
                       int64_t* work_lower_bound_bytes);
/* Test hook: checks the memory plan of every rank (no two regions overlap while both
 * are live, all inside the arena); returns the number of violations (0 = sound). */
int64_t sc_memory_plan_check(const sc_symbolic* sym, int32_t nranks);
void sc_free_numeric(sc_numeric* num);

/* Solve A x = b with the factor on the GPU (not in the reference):
 * level-scheduled supernodal forward (L y = P b) and backward (L^T z = y) sweeps,
 * x = P^T z.  sc_solve_host: host vectors b, x (length n; copies over PCIe);
 * sc_solve_device: device vectors (may alias), synchronous; d_b must be complete
 * on the device when the call is made (the library's stream does not order against
 * the caller's).  Returns the factor's status (> 0: not positive definite, nothing
 * solved).  Multi-rank handles: collective; the first solve after a factorization
 * gathers the whole factor onto every rank, then every rank solves. */
int64_t sc_solve_host(sc_numeric* num, const double* b, double* x);
int64_t sc_solve_device(sc_numeric* num, const double* d_b, double* d_x);

/* ---------------- reference-API helpers (host) ----------------
 * Each mirrors one reference function, with int64 column pointers. */
/* etree(A)  chol.hpp:377-410 */
int64_t sc_etree(int64_t n, const int64_t* Ap, const int32_t* Ai, int32_t* parent);
/* post_order(parent)  chol.hpp:466-499 */
int64_t sc_post_order(int64_t n, const int32_t* parent, int32_t* post);
/* col_count(A, parent, post)  chol.hpp:567-622 */
int64_t sc_col_count(int64_t n, const int64_t* Ap, const int32_t* Ai, const int32_t* parent,
                     const int32_t* post, int64_t* colcount);
/* ereach(A, k, parent, s, w[, x])  chol.hpp:680-739; returns top. Ax/x may be NULL. */
int64_t sc_ereach(int64_t n, const int64_t* Ap, const int32_t* Ai, const double* Ax, int64_t k,
                  const int32_t* parent, int32_t* s, int32_t* w, double* x);
/* compute_levels(parent)  src/chol.cpp:7-40: level_of[n] (0 = deepest level
 * processed first) ; returns number of levels. */
int64_t sc_compute_levels(int64_t n, const int32_t* parent, int32_t* level_of);
/* compute_supernodes(S, supernodes)  src/chol.cpp:42-100 on the reference
 * pattern (natural order): sn_id[n], supernodes[ns+1]; returns ns. */
int64_t sc_compute_supernodes(int64_t n, const int32_t* parent, const int64_t* Lp,
                              int32_t* sn_id, int64_t* supernodes);
/* atree(S, sn_id, supernodes)  src/chol.cpp:102-136 */
int64_t sc_atree(int64_t n, const int64_t* Lp, const int32_t* Li, const int32_t* sn_id,
                 const int64_t* supernodes, int64_t ns, int32_t* super_parent);
/* triplet_to_csc_matrix(ti, tj, tx, n)  chol.hpp:308-369: swaps to row<=col,
 * sorts by (col,row), sums duplicates.  Two-phase: call with Ap only to size,
 * then with Ai/Ax.  Returns nnz. */
int64_t sc_triplet_to_csc(int64_t n, int64_t nt, const int32_t* ti, const int32_t* tj,
                          const double* tx, int64_t* Ap, int32_t* Ai, double* Ax);
/* load_matrix_market_to_csc(filename)  include/mtx_reader.hpp:16-62, with the
 * banner honoured: coordinate real / integer / pattern (value 1); symmetric,
 * hermitian or no banner as the reference; general must hold a symmetric matrix
 * (both triangles, equal after summing duplicates; else SC_ERR_NOTSYM) and keeps
 * its upper entries; skew-symmetric SC_ERR_NOTSYM; array / complex
 * SC_ERR_NOTIMPL; out-of-range indices SC_ERR_ARG.  Two-phase like above:
 * first call with Ai==NULL returns n in *n and nnz; second fills. */
int64_t sc_read_mtx(const char* path, int64_t* n, int64_t* Ap, int32_t* Ai, double* Ax);
/* Synthetic 3D 7-point Laplacian on a k^3 grid in deterministic geometric
 * nested-dissection order.  n=k^3, nnz=n+3k^2(k-1).
 * Ap[n+1], Ai[nnz], Ax[nnz] (upper CSC); perm (new->old) may be NULL. */
int64_t sc_laplacian3d(int64_t k, int32_t nd_order, int64_t* Ap, int32_t* Ai, double* Ax,
                       int32_t* perm);

/* ---------------- multi-GPU (subtree partition over RCCL) ----------------
 * Proportional subtree-to-GPU mapping of the assembly tree; contribution
 * blocks cross GPUs only at subtree-merge fronts. */
/* RCCL unique id (128 bytes), created on rank 0 and broadcast by the caller. */
int64_t sc_dist_unique_id(void* id128);
int64_t sc_dist_owner_map(const sc_symbolic* sym, int32_t nranks, int32_t* owner_of_supernode,
                          double* work_per_rank);
/* This process is `rank` of `nranks` (one GPU each); it factors only the
 * supernodes it owns and exchanges contribution blocks with ncclSend/ncclRecv
 * after each assembly-tree level.  id128 == NULL: emulate all nranks ranks inside
 * this process on one device (sc_numeric_create_dist_emulated, device copies). */
int64_t sc_numeric_create_dist(const sc_symbolic* sym, int32_t device, int32_t rank,
                               int32_t nranks, const void* id128, sc_numeric** out);
/* Every rank of an nranks-rank plan in this process on one device, each with its
 * own memory plan and arenas; every message of the plan moves between them, as
 * device copies (use_rccl = 0) or as ncclSend / ncclRecv to self inside one
 * ncclGroupStart / ncclGroupEnd per comm step on a 1-rank RCCL communicator
 * (use_rccl = 1).  Validation of the partition and of the message plan. */
int64_t sc_numeric_create_dist_emulated(const sc_symbolic* sym, int32_t device, int32_t nranks, int32_t use_rccl,
                                        sc_numeric** out);
/* Per-rank message schedule for tests: returns number of messages; if the
 * arrays are non-NULL fills (comm step, peer, bytes, is_send) per message, in
 * posting order (comm steps ascending; all ranks follow one global step order). */
int64_t sc_dist_schedule(const sc_symbolic* sym, int32_t nranks, int32_t rank, int32_t* step,
                         int32_t* peer, int64_t* bytes, int32_t* is_send, int64_t cap);
/* The plan's comm steps in their global order: kind (0 INIT: assembled columns to
 * the ranks that factor / update them, 1 SLAB: a final panel slab to its users,
 * 2 DELIVER: contribution blocks to the parent's owner), assembly-tree level, front
 * (-1: a level's collective delivery), k (SLAB: the slab; DELIVER of an early child:
 * its column group) and p (SLAB: the column piece of the slab).  Any array may be
 * NULL.  Returns the step count. */
int64_t sc_dist_steps(const sc_symbolic* sym, int32_t nranks, int32_t* kind, int32_t* level, int32_t* front,
                      int32_t* k, int32_t* p, int64_t cap);
/* Plan summary: per supernode the rank-group size (1 = inside one rank's subtree),
 * for split fronts the number of ranks computing its contribution block (0 = not
 * split), for distributed panels the number of ranks factoring its slabs (0 = the
 * panel on one rank); *n_steps = comm steps.  Returns the total message count. */
int64_t sc_dist_plan_info(const sc_symbolic* sym, int32_t nranks, int32_t* gsize, int32_t* split_cb_ranks,
                          int32_t* slab_ranks, int64_t* n_steps);
/* Host-staged transport (tests / debugging without RCCL: several processes may
 * share one GPU).  The library calls fn(ctx, op, peer, buf, bytes) with op 0 =
 * post a send of host buffer buf, 1 = post a receive into buf, 2 = complete every
 * posted operation (buffers stay valid until then); nonzero return = failure. */
typedef int32_t (*sc_transport_fn)(void* ctx, int32_t op, int32_t peer, void* buf, int64_t bytes);
int64_t sc_numeric_create_dist_host(const sc_symbolic* sym, int32_t device, int32_t rank,
                                    int32_t nranks, sc_transport_fn fn, void* ctx, sc_numeric** out);
/* Timing projection: rank `rank`'s part of an nranks-GPU factorization alone on
 * this device; comm steps pack and unpack but move nothing (received blocks hold
 * stale values, so the numbers are not a factor). */
int64_t sc_numeric_create_dist_dry(const sc_symbolic* sym, int32_t device, int32_t rank, int32_t nranks,
                                   sc_numeric** out);

int64_t sc_device_count(void);
/* Message of the last failing call on this thread. */
const char* sc_last_error(void);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif

#endif /* SPARSECHOLESKY_H */
