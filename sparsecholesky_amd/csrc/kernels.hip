// CDNA4 (gfx950) kernels of the supernodal multifrontal numeric factorization.
//
// One front per supernode s: an m x m symmetric dense matrix whose first w
// columns (the L panel, m x w, column-major, ld = m) become L and whose trailing
// (m-w) x (m-w) lower block is the contribution block CB (ld = mb) handed to the
// parent.  Replaces the reference's per-supernode dense calls:
//   dpotrf_     include/chol.hpp:1263   -> front_small_kernel / potrf_diag_kernel
//   cblas_dtrsm include/chol.hpp:1292   -> front_small_kernel / trsm_panel_kernel
//   cblas_dsyrk include/chol.hpp:1322   -> front_small_kernel / syrk_mfma_kernel
//   apply_update include/chol.hpp:1196  -> extend-add gather in front_small_kernel /
//                                          assemble_large_kernel
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace sc {

typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void report_fail(int32_t* info, int32_t col_internal) {
    atomicMin(info, col_internal + 1);
}

// ---------------------------------------------------------------------------
// Large fronts, assembly: one workgroup per (front, 64-column block).  Zeroes its
// panel / CB columns, stores the A entries, then adds every child's CB entries
// whose parent column falls in the block (children in fixed order: deterministic).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lower_bound_i32(const int32_t* a, int n, int v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Column-streaming assembly (fronts with m < ASM_TILE_MIN_M): one workgroup per
// (front, 16-column block), one wave per column.  Zeroes its columns, stores the A
// entries, then adds every child's CB entries whose parent column falls in the
// block (children in fixed order: deterministic).
__global__ __launch_bounds__(256) void assemble_cols_kernel(DevPlan P, const int2* __restrict__ tasks,
                                                              const double* __restrict__ Ax) {
    const int2 t = tasks[blockIdx.x];
    const int s = t.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int j0 = t.y * ASM_COLS;
    const int j1 = min(m, j0 + ASM_COLS);
    double* panel = P.panel_pool + P.panel_off[s];
    double* cbs = P.cb_pool + P.cb_off[s];
    // zero the lower part of the owned columns: one wave per column
    for (int j = j0 + wid; j < j1; j += 4) {
        double* col = (j < w) ? panel + (int64_t)j * m : cbs + (int64_t)(j - w) * mb - w;
#pragma unroll 4
        for (int r = j + lane; r < m; r += 64) col[r] = 0.0;
    }
    __syncthreads();
    for (int j = j0 + wid; j < min(j1, w); j += 4) {
        const int64_t a0 = P.a_ptr[c0 + j], a1 = P.a_ptr[c0 + j + 1];
        for (int64_t q = a0 + lane; q < a1; q += 64) panel[(int64_t)j * m + P.a_pos[q]] = Ax[P.a_src[q]];
    }
    __syncthreads();
    // extend-add: children in fixed order; within a child, one wave per child
    // column (relative indices are injective, so columns never collide)
    for (int ci = P.child_ptr[s]; ci < P.child_ptr[s + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        const int32_t* __restrict__ rel = P.relind + P.rel_ptr[c];
        const double* __restrict__ cb = P.cb_pool + P.cb_off[c];
        const int jlo = lower_bound_i32(rel, mbc, j0);
        const int jhi = lower_bound_i32(rel, mbc, j1);
        for (int jc = jlo + wid; jc < jhi; jc += 4) {
            const int pj = rel[jc];
            const double* __restrict__ src = cb + (int64_t)jc * mbc;
            double* dst = (pj < w) ? panel + (int64_t)pj * m : cbs + (int64_t)(pj - w) * mb - w;
#pragma unroll 4
            for (int ic = jc + lane; ic < mbc; ic += 64) dst[rel[ic]] += src[ic];
        }
        __syncthreads();
    }
}

// Write-once assembly, one workgroup per (front, 16 columns, 256-row tile): the
// tile is built in LDS (zero, A entries, then each child's rows that map into it,
// children in fixed order; relative indices are injective and increasing, so a
// child's rows for the tile are one contiguous run, precomputed on the host in
// rel_bnd) and its lower part is stored once.  HBM traffic: one write per front
// entry plus one read per child entry (zero-then-add paid 8 + 24 B).
__global__ __launch_bounds__(256) void assemble_tile_kernel(DevPlan P, const int2* __restrict__ tasks,
                                                             const double* __restrict__ Ax) {
    __shared__ double T[ASM_COLS * ASM_ROWS];  // T[(j - j0) * ASM_ROWS + (r - r0)]
    const int2 t = tasks[blockIdx.x];
    const int s = t.x;
    const int k = t.y >> 16;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int j0 = (t.y & 0xffff) * ASM_COLS;
    const int j1 = min(m, j0 + ASM_COLS);
    const int r0 = k * ASM_ROWS, r1 = min(m, r0 + ASM_ROWS);
    double* panel = P.panel_pool + P.panel_off[s];
    double* cbs = P.cb_pool + P.cb_off[s];
    for (int idx = tid; idx < ASM_COLS * ASM_ROWS; idx += 256) T[idx] = 0.0;
    __syncthreads();
    for (int j = j0 + wid; j < min(j1, w); j += 4) {
        const int64_t a0 = P.a_ptr[c0 + j], a1 = P.a_ptr[c0 + j + 1];
        for (int64_t q = a0 + lane; q < a1; q += 64) {
            const int p = P.a_pos[q];
            if (p >= r0 && p < r1) T[(j - j0) * ASM_ROWS + (p - r0)] = Ax[P.a_src[q]];
        }
    }
    __syncthreads();
    for (int ci = P.child_ptr[s]; ci < P.child_ptr[s + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        const int32_t* __restrict__ rel = P.relind + P.rel_ptr[c];
        const int32_t* __restrict__ bnd = P.rel_bnd + P.rb_ptr[c];
        const int ilo = bnd[k], ihi = bnd[k + 1];
        if (ilo < ihi) {
            // child columns landing in [j0, j1) lie in row tile j0 / ASM_ROWS
            const int u0 = bnd[j0 / ASM_ROWS], u1 = bnd[j0 / ASM_ROWS + 1];
            const int jlo = u0 + lower_bound_i32(rel + u0, u1 - u0, j0);
            const int jhi = u0 + lower_bound_i32(rel + u0, u1 - u0, j1);
            const double* __restrict__ cb = P.cb_pool + P.cb_off[c];
            for (int jc = jlo + wid; jc < jhi; jc += 4) {
                const double* __restrict__ src = cb + (int64_t)jc * mbc;
                double* Tc = T + (rel[jc] - j0) * ASM_ROWS - r0;
                for (int ic = max(jc, ilo) + lane; ic < ihi; ic += 64) Tc[rel[ic]] += src[ic];
            }
        }
        __syncthreads();
    }
    for (int j = j0 + wid; j < j1; j += 4) {
        double* col = (j < w) ? panel + (int64_t)j * m : cbs + (int64_t)(j - w) * mb - w;
        const double* Tc = T + (j - j0) * ASM_ROWS - r0;
        for (int r = max(r0, j) + lane; r < r1; r += 64) col[r] = Tc[r];
    }
}

// Wave-uniform broadcast of lane `src`'s double (two v_readlane_b32).
__device__ __forceinline__ double readlane_f64(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Step J of the register-resident right-looking Cholesky of a <= 64 x 64 block
// (lane = row).  Template recursion forces full unrolling so r[] keeps static
// register indices (a rolled loop turns them into select chains).
template <int J>
__device__ __forceinline__ void potrf_steps(double (&r)[PNB], double* colj, int lane, int nb, int32_t* info,
                                            int col0) {
    if constexpr (J < PNB) {
        if (J < nb) {
            const double d = readlane_f64(r[J], J);
            if (lane == 0 && !(d > 0.0)) report_fail(info, col0 + J);
            const double piv = sqrt(d);
            const double inv = 1.0 / piv;
            const double rj = (lane == J) ? piv : r[J] * inv;
            r[J] = rj;
            colj[lane] = rj;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = J + 1; q < PNB; ++q) r[q] = fma(-rj, colj[q], r[q]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            potrf_steps<J + 1>(r, colj, lane, nb, info, col0);
        }
    }
}

// One wave factors the nb x nb (nb <= 64) lower block at `blk` (ld) in place.
__device__ __forceinline__ void potrf_block_wave(double* blk, int64_t ld, int nb, int lane, double* colj,
                                                 int32_t* info, int col0) {
    const bool live = lane < nb;
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = (live && c <= lane) ? blk[(int64_t)c * ld + lane] : 0.0;
    potrf_steps<0>(r, colj, lane, nb, info, col0);
    if (live) {
#pragma unroll
        for (int c = 0; c < PNB; ++c)
            if (c < nb && c <= lane) blk[(int64_t)c * ld + lane] = r[c];
    }
}

// Forward substitution steps of one row against L11 (column-major in LDS).
template <int J>
__device__ __forceinline__ void trsm_steps(double (&r)[PNB], const double* Lc, const double* invd, int nb) {
    constexpr int LD = PNB + 2;
    if constexpr (J < PNB) {
        if (J < nb) {
            const double rj = r[J] * invd[J];
            r[J] = rj;
#pragma unroll
            for (int q = J + 1; q < PNB; ++q) r[q] = fma(-rj, Lc[J * LD + q], r[q]);
            trsm_steps<J + 1>(r, Lc, invd, nb);
        }
    }
}

// ---------------------------------------------------------------------------
// Small fronts (m <= 128): the whole front in LDS, one 256-thread workgroup per
// front, the lower triangle packed by columns (column j holds rows j..m-1 at
// j m - j (j - 1) / 2): 64.5 KB at m = 128, two workgroups per CU.
//   1. assemble: zero, A entries of the pivot columns, the children's CBs
//      (extend-add, one wave per child column, children in a fixed order:
//      deterministic, no atomics);
//   2. POTRF of the w x w diagonal block by one wave in registers (w <= 64);
//   3. TRSM: one thread per row of L21 (independent rows);
//   4. the panel and CB = F22 - L21 L21^T (the SYRK, one wave per CB column,
//      w-long dot products from LDS) written straight to HBM.
// Fronts wider than 64 take a right-looking loop over the panel columns instead.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int pk_col(int m, int j) { return j * m - ((j * (j - 1)) >> 1); }

__device__ __forceinline__ void small_front(const DevPlan& P, const int s, const double* __restrict__ Ax,
                                            double* F, double* colj) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int tot = (m * (m + 1)) >> 1;
    for (int idx = tid; idx < tot; idx += 256) F[idx] = 0.0;
    __syncthreads();
    for (int lc = wid; lc < w; lc += 4) {
        const int64_t a0 = P.a_ptr[c0 + lc], a1 = P.a_ptr[c0 + lc + 1];
        double* Fc = F + pk_col(m, lc) - lc;
        for (int64_t q = a0 + lane; q < a1; q += 64) Fc[P.a_pos[q]] = Ax[P.a_src[q]];
    }
    __syncthreads();
    for (int ci = P.child_ptr[s]; ci < P.child_ptr[s + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        const int32_t* __restrict__ rel = P.relind + P.rel_ptr[c];
        const double* __restrict__ cb = P.cb_pool + P.cb_off[c];
        for (int jc = wid; jc < mbc; jc += 4) {
            const int pj = rel[jc];
            double* Fc = F + pk_col(m, pj) - pj;
            const double* __restrict__ src = cb + (int64_t)jc * mbc;
            for (int ic = jc + lane; ic < mbc; ic += 64) Fc[rel[ic]] += src[ic];
        }
        __syncthreads();
    }
    if (w <= PNB) {
        if (wid == 0) {  // 2. POTRF, lane = row of the diagonal block
            const bool live = lane < w;
            double r[PNB];
#pragma unroll
            for (int c = 0; c < PNB; ++c) r[c] = (live && c <= lane && c < w) ? F[pk_col(m, c) + lane - c] : 0.0;
            potrf_steps<0>(r, colj, lane, w, P.info, c0);
            if (live) {
#pragma unroll
                for (int c = 0; c < PNB; ++c)
                    if (c < w && c <= lane) F[pk_col(m, c) + lane - c] = r[c];
            }
        }
        __syncthreads();
        if (tid < mb) {  // 3. TRSM, thread = row w + tid: x_j = (F_ij - sum_t<j x_t L_jt) / L_jj
            const int i = w + tid;
            int oj = 0;  // pk_col(m, j)
            for (int j = 0; j < w; ++j) {
                double acc = F[oj + i - j];
                int ot = 0;
                for (int t = 0; t < j; ++t) {
                    acc -= F[ot + i - t] * F[ot + j - t];
                    ot += m - t;
                }
                F[oj + i - j] = acc / F[oj];
                oj += m - j;
            }
        }
    } else {
        for (int k = 0; k < w; ++k) {  // right-looking over the panel columns
            double* Fk = F + pk_col(m, k) - k;
            if (tid == 0) {
                const double d = Fk[k];
                if (!(d > 0.0)) report_fail(P.info, c0 + k);
                Fk[k] = sqrt(d);
            }
            __syncthreads();
            const double inv = 1.0 / Fk[k];
            for (int r = k + 1 + tid; r < m; r += 256) Fk[r] *= inv;
            __syncthreads();
            for (int j = k + 1 + wid; j < w; j += 4) {
                double* Fj = F + pk_col(m, j) - j;
                const double ljk = Fk[j];
                for (int r = j + lane; r < m; r += 64) Fj[r] -= Fk[r] * ljk;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    double* panel = P.panel_pool + P.panel_off[s];
    for (int j = wid; j < w; j += 4) {
        const double* Fj = F + pk_col(m, j) - j;
        for (int i = j + lane; i < m; i += 64) panel[(int64_t)j * m + i] = Fj[i];
    }
    if (mb > 0) {  // 4. CB(ic, jc) = F22(ic, jc) - sum_t L21(ic, t) L21(jc, t)
        double* cb = P.cb_pool + P.cb_off[s];
        for (int jc = wid; jc < mb; jc += 4) {
            const int jj = w + jc;
            for (int ic = jc + lane; ic < mb; ic += 64) {
                const int ii = w + ic;
                double v = F[pk_col(m, jj) + ii - jj];
                int ot = 0;
                for (int t = 0; t < w; ++t) {
                    v -= F[ot + ii - t] * F[ot + jj - t];
                    ot += m - t;
                }
                cb[(int64_t)jc * mb + ic] = v;
            }
        }
    }
}

// maxm: LDS edge of the launch (the packed front plus the POTRF column buffer)
__global__ __launch_bounds__(256) void front_small_kernel(DevPlan P, const int32_t* __restrict__ nodes,
                                                           const double* __restrict__ Ax) {
    extern __shared__ double F[];
    __shared__ double colj[PNB];
    small_front(P, nodes[blockIdx.x], Ax, F, colj);
}

// ---------------------------------------------------------------------------
// Pipelined variants (default).  A full 64-column block runs generated
// straight-line code (panel_gen.inc, gen_panel.py) that keeps ~24 LDS operands
// in flight per wave; a partial last block (nb < 64) uses the template path.
// ---------------------------------------------------------------------------
// Buffer-resource access for the panel kernels: one VGPR lane offset plus an
// SGPR column offset per access, so 64 column addresses never occupy VGPRs.
// Raw buffers (stride 0) drop stores and zero loads at offsets >= nbytes, so a
// dead lane is masked by giving it an out-of-range lane offset (BUF_DEAD).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const double* base, uint32_t nbytes = 0xffffffffu) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, (int)nbytes, 0x00020000);
}
constexpr int BUF_DEAD = 0x7ffffff0;
__device__ __forceinline__ double buf_ld(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
__device__ __forceinline__ void buf_st(double v, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0)), v), rs, voff, soff, 0);
}

// 1/sqrt(d): v_rsq_f64 seed plus two Newton steps (~1 ulp; NaN/inf for d <= 0,
// which the callers flag separately).
__device__ __forceinline__ double rsqrt_f64(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

#include "panel_gen.inc"

__global__ __launch_bounds__(64) void potrf_diag_g_kernel(DevPlan P, const int2* __restrict__ tasks) {
    __shared__ double C[2 * PNB];
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    double* blk = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + k0;
    const int lane = threadIdx.x;
    if (nb < PNB) {
        potrf_block_wave(blk, m, nb, lane, C, P.info, c0 + k0);
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(blk);
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = buf_ld(rs, lane * 8, c * m * 8);
    const int bad = potrf64_full(r, C, lane);
    if (bad >= 0 && lane == 0) report_fail(P.info, c0 + k0 + bad);
#pragma unroll
    for (int c = 0; c < PNB; ++c)
        if (c <= lane) buf_st(r[c], rs, lane * 8, c * m * 8);
}

// Partial last block (nb < 64) of the panel TRSM: template path, kept out of
// line so its registers do not constrain the generated full-block code.
// Rows [r0, r0 + nrows).
__device__ __forceinline__ void trsm_partial(double* pan, int m, int k0, int nb, int r0, int nrows, double* Lc,
                                             double* invd) {
    constexpr int LD = PNB + 2;
    const int tid = threadIdx.x;
    const double* blk = pan + (int64_t)k0 * m + k0;
    for (int idx = tid; idx < PNB * PNB; idx += 256) {
        const int q = idx % PNB, j = idx / PNB;
        const double v = (q < nb && j < nb && j <= q) ? blk[(int64_t)j * m + q] : 0.0;
        Lc[j * LD + q] = v;
        if (q == j) invd[j] = (j < nb) ? 1.0 / v : 0.0;
    }
    __syncthreads();
    const int row = r0 + tid;
    const bool live = row < m && tid < nrows;
    double* xs = pan + (int64_t)k0 * m + (live ? row : r0);
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = (live && c < nb) ? xs[(int64_t)c * m] : 0.0;
    trsm_steps<0>(r, Lc, invd, nb);
    if (live) {
#pragma unroll
        for (int c = 0; c < PNB; ++c)
            if (c < nb) xs[(int64_t)c * m] = r[c];
    }
}

// Partial last blocks (nb < 64) of the panel TRSM, launched separately so the
// full-block kernels keep their own register budgets.  Rows [r0, r0 + nrows).
__global__ __launch_bounds__(256) void trsm_partial_kernel(DevPlan P, const int4* __restrict__ tasks, int nrows) {
    __shared__ double Lc[PNB * (PNB + 2)];
    __shared__ double invd[PNB];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    trsm_partial(P.panel_pool + P.panel_off[s], m, k0, min(PNB, w - k0), r0, nrows, Lc, invd);
}

// Panel TRSM, rows [r0, r0 + 256): L11 operands packed into an LDS stream in the
// order the generated solve consumes them (1/L(J,J), then L(J+1..63, J)).
__global__ __launch_bounds__(256) void trsm_panel_g_kernel(DevPlan P, const int4* __restrict__ tasks) {
    __shared__ double2 S[TRSM64_STREAM / 2];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    double* pan = P.panel_pool + P.panel_off[s];
    if (nb < PNB) return;  // partial blocks: trsm_partial_kernel
    const double* blk = pan + (int64_t)k0 * m + k0;
    const int row = r0 + tid;
    // the 64 block columns, m rows each (< 2^31 bytes for m < 4M); dead lanes masked
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan + (int64_t)k0 * m, (uint32_t)m * PNB * 8u);
    const int voff = row < m ? row * 8 : BUF_DEAD;
    double* Sd = reinterpret_cast<double*>(S);
    for (int e = tid; e < PNB * PNB; e += 256) {
        const int j = e / PNB, q = e % PNB;
        if (q >= j) {
            const double v = blk[(int64_t)j * m + q];
            Sd[PNB * j - j * (j - 1) / 2 + (q - j)] = (q == j) ? 1.0 / v : v;
        }
    }
    __syncthreads();
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = buf_ld(rs, voff, c * m * 8);
    trsm64_full(r, S);
#pragma unroll
    for (int c = 0; c < PNB; ++c) buf_st(r[c], rs, voff, c * m * 8);
}

// ---------------------------------------------------------------------------
// fp64 MFMA SYRK on a lower trapezoid: C[i,j] -= sum_k A[i,k] * A[j,k] for
// 0 <= j < N, j <= i < M.  BT x BT output tiles (ti >= tj) on WM x WN waves, each
// wave (BT/WM) x (BT/WN) = RTM x RTN tiles of v_mfma_f64_16x16x4_f64.  A (M x K)
// and the B operand (its first N rows) share one column-major array.  K is
// staged through double-buffered LDS (register staging, BK = 16).
// (BK = 8 and 32, and a 4-wave 128 x 128 instance, were measured slower on every
// shape: DESIGN.md section 5.)
// ---------------------------------------------------------------------------
template <int BT, int WM, int WN, int TAG>
__global__ __launch_bounds__(64 * WM * WN) void syrk_mfma_kernel(const GemmTask* __restrict__ tasks,
                                                                  const int2* __restrict__ tiles) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BK = 16;
    constexpr int LDT = BT + 16;  // +128 B row pad: the two k-rows read by a half-wave hit disjoint banks
    constexpr int RTM = BT / WM / 16, RTN = BT / WN / 16;
    __shared__ double smem[2 * 2 * BK * LDT];  // A and B stages
    double(*As)[BK * LDT] = reinterpret_cast<double(*)[BK * LDT]>(smem);
    double(*Bs)[BK * LDT] = reinterpret_cast<double(*)[BK * LDT]>(smem + 2 * BK * LDT);

    // host-ordered tile list: blocks sharing an XCD walk a contiguous, L2-blocked run of tiles
    const int2 tl = tiles[blockIdx.x];
    const GemmTask T = tasks[tl.x];
    const int ti = tl.y >> 16, tj = tl.y & 0xffff;
    const int row0 = ti * BT, col0 = tj * BT;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid / WN, wc = wid % WN;
    const double* __restrict__ A = T.A;
    const int64_t lda = T.lda;

    double4_t acc[RTM][RTN];
#pragma unroll
    for (int a = 0; a < RTM; ++a)
#pragma unroll
        for (int b = 0; b < RTN; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};

    // staging: BK x BT doubles per operand over NT threads
    constexpr int PER = BT * BK / NT;
    // Operands through a per-stage buffer resource (columns k0 .. k0 + BK of A):
    // K past the end and rows past M / N fall outside it and load 0 -- no branches,
    // and buffer loads count only vmcnt, so the LDS waits of the MFMA loop do not
    // also wait for the next stage's prefetch (flat loads count both).
    double ra[PER], rb[PER];
    auto gload = [&](int k0) {
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(A + (int64_t)k0 * lda, (uint32_t)(min(BK, T.K - k0) * lda * 8));
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + q * NT;
            const int r = e % BT, kk = e / BT;
            const int gr = row0 + r, gc = col0 + r;
            ra[q] = buf_ld(rs, gr < T.M ? (int)((gr + kk * lda) * 8) : BUF_DEAD, 0);
            rb[q] = buf_ld(rs, gc < T.N ? (int)((gc + kk * lda) * 8) : BUF_DEAD, 0);
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + q * NT;
            const int r = e % BT, kk = e / BT;
            As[buf][kk * LDT + r] = ra[q];
            Bs[buf][kk * LDT + r] = rb[q];
        }
    };

    const int nk = (T.K + BK - 1) / BK;
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * BK);
        // LDS operand fragments double-buffered across the 4-deep k sub-steps: the
        // reads of sub-step kk + 1 are in flight while sub-step kk's MFMAs issue
        double av[2][RTM], bv[2][RTN];
        auto lread = [&](int kk, int slot) {
            const int krow = kk + (lane >> 4);
#pragma unroll
            for (int a = 0; a < RTM; ++a)
                av[slot][a] = As[cur][krow * LDT + wr * (BT / WM) + a * 16 + (lane & 15)];
#pragma unroll
            for (int b = 0; b < RTN; ++b)
                bv[slot][b] = Bs[cur][krow * LDT + wc * (BT / WN) + b * 16 + (lane & 15)];
        };
        lread(0, 0);
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const int slot = (kk / 4) & 1;
            if (kk + 4 < BK) lread(kk + 4, slot ^ 1);
#pragma unroll
            for (int a = 0; a < RTM; ++a)
#pragma unroll
                for (int b = 0; b < RTN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[slot][a], bv[slot][b], acc[a][b], 0, 0, 0);
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

    // epilogue: f64 16x16x4 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg.
    // C read-modify-write through a buffer resource over the tile's columns (dead
    // elements -- above the diagonal, past M / N -- masked by range, no branches).
    double* __restrict__ C = T.C;
    const int64_t ldc = T.ldc;
    const __amdgpu_buffer_rsrc_t rc =
        buf_rsrc(C + (int64_t)col0 * ldc, (uint32_t)(min(BT, T.N - col0) * ldc * 8));
#pragma unroll
    for (int a = 0; a < RTM; ++a)
#pragma unroll
        for (int b = 0; b < RTN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = row0 + wr * (BT / WM) + a * 16 + MFMA_F64_ROW(lane, r);
                const int gj = col0 + wc * (BT / WN) + b * 16 + (lane & 15);
                const bool live = gi < T.M && gi >= gj;
                const int off = live ? (int)((gi + (int64_t)(gj - col0) * ldc) * 8) : BUF_DEAD;
                buf_st(buf_ld(rc, off, 0) - acc[a][b][r], rc, off, 0);
            }
}

// ---------------------------------------------------------------------------
// Launch wrappers
// ---------------------------------------------------------------------------
hipError_t launch_front_small(const DevPlan& P, const int32_t* nodes, int count, int maxm, const double* Ax,
                              hipStream_t st) {
    if (count <= 0) return hipSuccess;
    const size_t lds = (size_t)maxm * (maxm + 1) / 2 * sizeof(double);
    hipLaunchKernelGGL(front_small_kernel, dim3(count), dim3(256), lds, st, P, nodes, Ax);
    return hipGetLastError();
}

hipError_t launch_assemble_large(const DevPlan& P, const int2* tasks, int count, const double* Ax,
                                 hipStream_t st, bool tiled) {
    if (count <= 0) return hipSuccess;
    if (tiled)
        hipLaunchKernelGGL(assemble_tile_kernel, dim3(count), dim3(256), 0, st, P, tasks, Ax);
    else
        hipLaunchKernelGGL(assemble_cols_kernel, dim3(count), dim3(256), 0, st, P, tasks, Ax);
    return hipGetLastError();
}

hipError_t launch_potrf_diag(const DevPlan& P, const int2* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(potrf_diag_g_kernel, dim3(count), dim3(64), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_trsm_panel(const DevPlan& P, const int4* tasks, int count, hipStream_t st, bool partial) {
    if (count <= 0) return hipSuccess;
    if (partial)
        hipLaunchKernelGGL(trsm_partial_kernel, dim3(count), dim3(256), 0, st, P, tasks, TRSM_ROWS);
    else
        hipLaunchKernelGGL(trsm_panel_g_kernel, dim3(count), dim3(TRSM_ROWS), 0, st, P, tasks);
    return hipGetLastError();
}

// TAG only separates the launches in profiles: 0 = panel update, 1 = CB update.
// bt = 64: 64x64 tiles on 4 waves (2x2); bt = 128: 128x128 tiles on 8 waves (2x4).
template <int TAG>
static void launch_syrk_t(const GemmTask* tasks, const int2* tiles, int n, int bt, hipStream_t st) {
    if (bt == 128)
        hipLaunchKernelGGL((syrk_mfma_kernel<128, 2, 4, TAG>), dim3(n), dim3(512), 0, st, tasks, tiles);
    else
        hipLaunchKernelGGL((syrk_mfma_kernel<64, 2, 2, TAG>), dim3(n), dim3(256), 0, st, tasks, tiles);
}

hipError_t launch_syrk(const GemmTask* tasks, const int2* tiles, int total_tiles, int bt, int tag, hipStream_t st) {
    if (total_tiles <= 0) return hipSuccess;
    if (tag)
        launch_syrk_t<1>(tasks, tiles, total_tiles, bt, st);
    else
        launch_syrk_t<0>(tasks, tiles, total_tiles, bt, st);
    return hipGetLastError();
}

// Fills n doubles with a deterministic pseudo-random pattern in [-1, 1) (microbenchmarks:
// zero operands run the MFMA at a higher clock than real data).
__global__ void fill_random_kernel(double* p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        p[i] = (double)(x >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    }
}

hipError_t launch_fill_random(double* p, int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(fill_random_kernel, dim3(1024), dim3(256), 0, st, p, n);
    return hipGetLastError();
}

// Timestamp probe for graph-captured timing (s_memrealtime: constant 100 MHz).
__global__ void stamp_kernel(uint64_t* slot) { *slot = __builtin_amdgcn_s_memrealtime(); }

hipError_t launch_stamp(uint64_t* slot, hipStream_t st) {
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, st, slot);
    return hipGetLastError();
}

// Multi-GPU staging: strided <-> packed copy of contribution-block / panel column
// blocks around the RCCL transfers.  One workgroup per COPY_COLS columns of one
// block, one wave per column, 64 consecutive doubles per wave access (HBM-bound).
__global__ __launch_bounds__(256) void copy2d_kernel(const Copy2D* __restrict__ descs, const int2* __restrict__ tiles,
                                                     int unpack) {
    const int2 t = tiles[blockIdx.x];
    const Copy2D d = descs[t.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int j1 = min(d.cols, t.y + COPY_COLS);
    for (int j = t.y + wid; j < j1; j += 4) {
        double* a = d.a + (int64_t)j * d.lda;
        double* b = d.b + (int64_t)j * d.rows;
        if (unpack) {
            for (int r = lane; r < d.rows; r += 64) a[r] = b[r];
        } else {
            for (int r = lane; r < d.rows; r += 64) b[r] = a[r];
        }
    }
}

hipError_t launch_copy2d(const Copy2D* descs, const int2* tiles, int count, bool unpack, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(copy2d_kernel, dim3(count), dim3(256), 0, st, descs, tiles, unpack ? 1 : 0);
    return hipGetLastError();
}

// Peak probe: independent fp64 MFMA chains, operands in registers.
template <int NACC>
__global__ __launch_bounds__(256) void mfma_peak_kernel(double* out, int iters) {
    double4_t acc[NACC];
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = (double4_t){0.0, 0.0, 0.0, 0.0};
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - blockIdx.x * 1e-9;
    // 16 MFMAs per accumulator per trip: the compiler moves the accumulators between
    // VGPRs and AGPRs at the loop edge, which a short body would not amortise
    for (int i = 0; i < iters; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    if (s == 1234.5) out[blockIdx.x] = s;  // keep the chain live
}

hipError_t launch_mfma_peak(double* out, int blocks, int iters, int nacc, hipStream_t st) {
    if (nacc == 16)
        hipLaunchKernelGGL((mfma_peak_kernel<16>), dim3(blocks), dim3(256), 0, st, out, iters);
    else if (nacc == 8)
        hipLaunchKernelGGL((mfma_peak_kernel<8>), dim3(blocks), dim3(256), 0, st, out, iters);
    else if (nacc == 2)
        hipLaunchKernelGGL((mfma_peak_kernel<2>), dim3(blocks), dim3(256), 0, st, out, iters);
    else
        hipLaunchKernelGGL((mfma_peak_kernel<4>), dim3(blocks), dim3(256), 0, st, out, iters);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Triangular solves with the supernodal factor (the
// reference has no solve).  Level-scheduled like the factorization.  Forward:
// one fused launch per 64-column step (solve_fwd_kernel).  Backward, per step in
// reverse: the transposed GEMV over the rows below each 64-column block
// (solve_gemv_kernel), then the one-wave diagonal solve L11^T x = c
// (solve_diag_kernel).  HBM-bound: L is read once per sweep.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void solve_diag_kernel(SolvePlan P, const int2* __restrict__ tasks) {
    __shared__ double Lb[PNB * (PNB + 1)];  // Lb[j * (PNB + 1) + i] = L(k0 + i, k0 + j)
    __shared__ double dinv[PNB];
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    const double* __restrict__ pan = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + k0;
    // stage the block: 16 independent loads per thread, one column per wave access
#pragma unroll
    for (int q = 0; q < PNB * PNB / 256; ++q) {
        const int e = tid + 256 * q, j = e >> 6, i = e & 63;
        Lb[j * (PNB + 1) + i] = (i < nb && j < nb) ? pan[(int64_t)j * m + i] : 0.0;
    }
    if (tid < PNB) dinv[tid] = 0.0;
    __syncthreads();
    if (tid < nb) dinv[tid] = 1.0 / Lb[tid * (PNB + 1) + tid];
    __syncthreads();
    if (tid >= 64) return;
    // lane i keeps column i of the block (L(j, i)) in registers; all 64 steps run
    // (zero padding past nb is inert), fully unrolled so the pivot and its
    // reciprocal come from readlane, not LDS
    double r[PNB];
#pragma unroll
    for (int j = 0; j < PNB; ++j) r[j] = Lb[lane * (PNB + 1) + j];
    const double d = dinv[lane];
    double v = lane < nb ? P.c[c0 + k0 + lane] : 0.0;
#pragma unroll
    for (int j = PNB - 1; j >= 0; --j) {  // x_j = v_j / L_jj; v_i -= L_ji x_j (i < j)
        const double xj = readlane_f64(v, j) * readlane_f64(d, j);
        v = lane == j ? xj : (lane < j ? v - r[j] * xj : v);
    }
    if (lane < nb) P.c[c0 + k0 + lane] = v;
}

// c[blk] -= L[rows, blk]^T x[rows].  Per 64-row chunk: coalesced column loads into
// LDS, then thread (column j, quarter g) sums 16 rows of column j.
__global__ __launch_bounds__(SOLVE_ROWS) void solve_gemv_kernel(SolvePlan P, const int4* __restrict__ tasks) {
    __shared__ double vb[SOLVE_ROWS];             // x of the rows
    __shared__ double T[PNB * (PNB + 1)];         // 64-row chunk, T[j * (PNB + 1) + i]
    __shared__ double part[SOLVE_ROWS / 64][PNB];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    const double* __restrict__ pan = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m;
    const int32_t* __restrict__ rows = P.rows + P.rows_ptr[s];
    const int r = r0 + tid;
    const bool live = r < m;
    vb[tid] = live ? P.c[rows[r]] : 0.0;
    const int j = tid & 63, g = tid >> 6;
    double acc = 0.0;
    for (int ch = 0; ch < SOLVE_ROWS && r0 + ch < m; ch += 64) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PNB * 64 / SOLVE_ROWS; ++q) {
            const int e = tid + SOLVE_ROWS * q, jj = e >> 6, ii = e & 63;
            const int rr = r0 + ch + ii;
            T[jj * (PNB + 1) + ii] = (rr < m && jj < nb) ? pan[(int64_t)jj * m + rr] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += T[j * (PNB + 1) + g * 16 + q] * vb[ch + g * 16 + q];
    }
    part[g][j] = acc;
    __syncthreads();
    if (tid < nb) {
        double a = 0.0;
#pragma unroll
        for (int q = 0; q < SOLVE_ROWS / 64; ++q) a += part[q][tid];
        unsafeAtomicAdd(P.c + c0 + k0 + tid, -a);
    }
}

// Fused forward step (one launch per 64-column step instead of two): every GEMV
// workgroup of block (s, k0) solves L11 y = c_blk itself from the 64 x 64 block
// (32 KB, L2-resident across the step's workgroups) and applies its rows.  The
// block's writer (t.w = 1) stores y to P.y, not to c, which the step's other
// workgroups still read.  r0 < 0: a block with no rows below (diagonal only).
__global__ __launch_bounds__(SOLVE_ROWS) void solve_fwd_kernel(SolvePlan P, const int4* __restrict__ tasks) {
    __shared__ double Lb[PNB * (PNB + 1)];  // Lb[j * (PNB + 1) + i] = L(k0 + i, k0 + j)
    __shared__ double vb[PNB];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x, lane = tid & 63;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    const double* __restrict__ pan = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m;
#pragma unroll
    for (int q = 0; q < PNB * PNB / SOLVE_ROWS; ++q) {
        const int e = tid + SOLVE_ROWS * q, j = e >> 6, i = e & 63;
        Lb[j * (PNB + 1) + i] = (i < nb && j < nb) ? pan[(int64_t)j * m + k0 + i] : 0.0;
    }
    __syncthreads();
    if (tid < 64) {
        double r[PNB];
#pragma unroll
        for (int j = 0; j < PNB; ++j) r[j] = Lb[j * (PNB + 1) + lane];
        const double d = lane < nb ? 1.0 / Lb[lane * (PNB + 1) + lane] : 0.0;
        double v = lane < nb ? P.c[c0 + k0 + lane] : 0.0;
#pragma unroll
        for (int j = 0; j < PNB; ++j) {  // y_j = v_j / L_jj; v_i -= L_ij y_j (i > j)
            const double yj = readlane_f64(v, j) * readlane_f64(d, j);
            v = lane == j ? yj : (lane > j ? v - r[j] * yj : v);
        }
        vb[lane] = v;
        if (t.w && lane < nb) P.y[c0 + k0 + lane] = v;
    }
    __syncthreads();
    if (r0 < 0) return;
    const int32_t* __restrict__ rows = P.rows + P.rows_ptr[s];
    const int r = r0 + tid;
    const bool live = r < m;
    double acc = 0.0;
#pragma unroll
    for (int jc = 0; jc < PNB; jc += 16) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = (live && jc + q < nb) ? pan[(int64_t)(jc + q) * m + r] : 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += v[q] * vb[jc + q];
    }
    if (live) unsafeAtomicAdd(P.c + rows[r], -acc);
}

hipError_t launch_solve_fwd(const SolvePlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_fwd_kernel, dim3(count), dim3(SOLVE_ROWS), 0, st, P, tasks);
    return hipGetLastError();
}

__global__ void permute_kernel(double* __restrict__ dst, const double* __restrict__ src,
                               const int32_t* __restrict__ perm, int64_t n, int scatter) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (scatter)
        dst[perm[i]] = src[i];
    else
        dst[i] = src[perm[i]];
}

hipError_t launch_solve_diag(const SolvePlan& P, const int2* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_diag_kernel, dim3(count), dim3(256), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_solve_gemv(const SolvePlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_gemv_kernel, dim3(count), dim3(SOLVE_ROWS), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_permute(double* dst, const double* src, const int32_t* perm, int64_t n, bool scatter,
                          hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(permute_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, src, perm, n,
                       scatter ? 1 : 0);
    return hipGetLastError();
}

}  // namespace sc
