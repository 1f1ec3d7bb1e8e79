// CDNA4 (gfx950) kernels of the supernodal multifrontal numeric factorization.
//
// One front per supernode s: an m x m symmetric dense matrix whose first w
// columns (the L panel, m x w, column-major, ld = m) become L and whose trailing
// (m-w) x (m-w) lower block is the contribution block CB (ld = mb) handed to the
// parent.  Replaces the reference's per-supernode dense calls:
//   dpotrf_     include/chol.hpp:1263   -> front_small_kernel / trsm_panel_g_kernel (fused)
//   cblas_dtrsm include/chol.hpp:1292   -> front_small_kernel / trsm_panel_g_kernel
//   cblas_dsyrk include/chol.hpp:1322   -> front_small_kernel / syrk_mfma_kernel
//   apply_update include/chol.hpp:1196  -> extend-add gather in front_small_kernel /
//                                          assemble_large_kernel
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "kernels.hpp"

namespace sc {

typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void report_fail(int32_t* info, int32_t col_internal) {
    atomicMin(info, col_internal + 1);
}

// g(k) of a child's compact block bounds (symbolic.cpp bounds()): [k_lo, k_hi, g(k_lo),
// g(k_lo + 1) .. g(k_hi - 1)]; g = g(k_lo) at or below k_lo, mbc at or above k_hi
__device__ __forceinline__ int bnd_at(const int32_t* b, int k, int mbc) {
    const int klo = b[0], khi = b[1];
    return k <= klo ? b[2] : (k >= khi ? mbc : b[2 + k - klo]);
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
        const int32_t* __restrict__ cbnd = P.col_bnd + P.cbk_ptr[c];  // j0 = t.y * ASM_COLS
        const int jlo = bnd_at(cbnd, t.y, mbc), jhi = bnd_at(cbnd, t.y + 1, mbc);
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
// rel_bnd / col_bnd) and its lower part is stored once.  HBM traffic: one write
// per front entry plus one read per child entry (zero-then-add paid 8 + 24 B).
// Wave w owns the tile columns j0 + w + 4q, so after one prologue that stages up
// to ASM_CCH children's bounds in LDS the waves never synchronise: each child's
// entries for a wave's columns (<= 4 columns x 256 rows) are loaded with all
// loads in flight before the adds (the kernel is latency-bound otherwise).
constexpr int ASM_CCH = 32;  // children staged per prologue
// lim (distributed assembly, or null): per task the front columns [x, y) this rank
// assembles; the tile's other columns are neither gathered nor stored (their children's
// columns went to another rank, and this rank may hold no copy of them)
__global__ __launch_bounds__(256) void assemble_tile_kernel(DevPlan P, const int2* __restrict__ tasks,
                                                             const double* __restrict__ Ax,
                                                             const int2* __restrict__ lim) {
    __shared__ double T[ASM_COLS * ASM_ROWS];  // T[(j - j0) * ASM_ROWS + (r - r0)]
    __shared__ const double* s_src[ASM_CCH];
    __shared__ const int32_t* s_rel[ASM_CCH];
    __shared__ int s_mbc[ASM_CCH], s_ilo[ASM_CCH], s_ihi[ASM_CCH], s_jlo[ASM_CCH];
    __shared__ int8_t s_pj[ASM_CCH][ASM_COLS];  // parent tile column of child column jlo + l, or -1
    const int2 t = tasks[blockIdx.x];
    const int s = t.x;
    const int k = t.y >> 16;
    const int jb = t.y & 0xffff;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int j0 = jb * ASM_COLS;
    const int j1 = min(m, j0 + ASM_COLS);
    const int r0 = k * ASM_ROWS, r1 = min(m, r0 + ASM_ROWS);
    const int2 cl = lim ? lim[blockIdx.x] : make_int2(0, m);  // owned front columns
    double* panel = P.panel_pool + P.panel_off[s];
    double* cbs = P.cb_pool + P.cb_off[s];
    const int cp0 = P.child_ptr[s], cp1 = P.child_ptr[s + 1];
    // own columns: zero, then A entries (program order within the wave)
#pragma unroll
    for (int q = 0; q < ASM_COLS / 4; ++q)
#pragma unroll
        for (int r = lane; r < ASM_ROWS; r += 64) T[(wid + 4 * q) * ASM_ROWS + r] = 0.0;
    for (int j = j0 + wid; j < min(j1, w); j += 4) {
        const int64_t a0 = P.a_ptr[c0 + j], a1 = P.a_ptr[c0 + j + 1];
        for (int64_t q = a0 + lane; q < a1; q += 64) {
            const int p = P.a_pos[q];
            if (p >= r0 && p < r1) T[(j - j0) * ASM_ROWS + (p - r0)] = Ax[P.a_src[q]];
        }
    }
    for (int cb = cp0; cb < cp1; cb += ASM_CCH) {
        const int nc = min(ASM_CCH, cp1 - cb);
        if (cb > cp0) __syncthreads();  // previous chunk's staging fully read
        if (tid < nc) {
            const int c = P.child_list[cb + tid];
            const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
            const int32_t* rel = P.relind + P.rel_ptr[c];
            const int32_t* bnd = P.rel_bnd + P.rb_ptr[c];
            const int32_t* cbnd = P.col_bnd + P.cbk_ptr[c];
            const int ilo = bnd_at(bnd, k, mbc), ihi = bnd_at(bnd, k + 1, mbc);
            const int jlo = bnd_at(cbnd, jb, mbc), jhi = bnd_at(cbnd, jb + 1, mbc);
            int pj[ASM_COLS];
#pragma unroll
            for (int l = 0; l < ASM_COLS; ++l) {
                const int pc = (jlo + l < jhi && ilo < ihi) ? rel[jlo + l] : -1;
                pj[l] = (pc >= cl.x && pc < cl.y) ? pc - j0 : -1;
            }
#pragma unroll
            for (int l = 0; l < ASM_COLS; ++l) s_pj[tid][l] = (int8_t)pj[l];
            s_src[tid] = P.cb_pool + P.cb_off[c];
            s_rel[tid] = rel;
            s_mbc[tid] = mbc;
            s_ilo[tid] = ilo;
            s_ihi[tid] = ihi;
            s_jlo[tid] = jlo;
        }
        __syncthreads();
        for (int i = 0; i < nc; ++i) {
            const int pjl = lane < ASM_COLS ? (int)s_pj[i][lane] : -1;
            uint64_t mask = __ballot(pjl >= 0 && (pjl & 3) == wid);
            if (!mask) continue;
            const int mbc = s_mbc[i], ilo = s_ilo[i], ihi = s_ihi[i], jlo = s_jlo[i];
            const double* __restrict__ src = s_src[i];
            const int32_t* __restrict__ rel = s_rel[i];
            // up to 4 child columns for this wave, each <= ASM_ROWS rows: all loads first
            int jc[4], tc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int b = mask ? __builtin_ctzll(mask) : -1;
                jc[q] = b < 0 ? -1 : jlo + b;
                tc[q] = b < 0 ? 0 : __shfl(pjl, b);
                mask &= mask - 1;
            }
            double v[4][ASM_ROWS / 64];
            int rr[4][ASM_ROWS / 64];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lo = max(jc[q], ilo) + lane;
#pragma unroll
                for (int ch = 0; ch < ASM_ROWS / 64; ++ch) {
                    const int ic = lo + 64 * ch;
                    const bool ok = jc[q] >= 0 && ic < ihi;
                    rr[q][ch] = ok ? rel[ic] : -1;
                    v[q][ch] = ok ? src[(int64_t)jc[q] * mbc + ic] : 0.0;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int ch = 0; ch < ASM_ROWS / 64; ++ch)
                    if (rr[q][ch] >= 0) T[tc[q] * ASM_ROWS + rr[q][ch] - r0] += v[q][ch];
        }
    }
    // own columns: store the lower part once
    for (int j = j0 + wid; j < j1; j += 4) {
        if (j < cl.x || j >= cl.y) continue;
        double* col = (j < w) ? panel + (int64_t)j * m : cbs + (int64_t)(j - w) * mb - w;
        const double* Tc = T + (j - j0) * ASM_ROWS - r0;
        for (int r = max(r0, j) + lane; r < r1; r += 64) col[r] = Tc[r];
    }
}

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

// Wave-uniform broadcast of lane `src`'s double (two v_readlane_b32).
__device__ __forceinline__ double readlane_f64(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
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
// Small fronts (m <= 128).  The front is assembled in LDS (lower triangle packed by
// columns: column j holds rows j..m-1 at j m - j (j - 1) / 2) -- zero, the A entries
// of the pivot columns, then the children's CBs in a fixed order (extend-add,
// deterministic, no atomics) -- and then factored in REGISTERS: the 256 threads
// hold 4 x 4 tiles of the lower front (KT tiles each), and the w pivot steps run
// right-looking over the whole front at once, so POTRF, TRSM and the CB update
// (the reference's dpotrf_ / cblas_dtrsm / cblas_dsyrk, chol.hpp:1263-1322) are
// one loop.  Step J: the owners of column J publish it to LDS (double-buffered,
// one barrier per step), every thread takes the pivot's 1/sqrt and updates its
// tiles right of J.  The panel (columns < w) and the CB leave straight from the
// registers: to HBM, or -- chain launches -- added into the parent's LDS front.
// ---------------------------------------------------------------------------
// 1/sqrt(d): v_rsq_f64 seed plus two Newton steps (~1 ulp; NaN/inf for d <= 0,
// which the callers flag separately).
__device__ __forceinline__ double rsqrt_f64(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

__device__ __forceinline__ int pk_col(int m, int j) { return j * m - ((j * (j - 1)) >> 1); }

// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not
// for its global stores (the panel / CB stores stay in flight across it).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Tile q -> (bi, bj), bi >= bj, for T tile rows of which the first WT tile columns
// hold pivot columns: the WT * T - WT (WT - 1) / 2 panel tiles first, column by
// column (neighbouring threads share a tile column, so the masked pivot-column work
// stays wave-coherent), then the CB tiles row by row.
__device__ __forceinline__ void tile_map(int q, int T, int WT, int& bi, int& bj) {
    const int np = WT * T - WT * (WT - 1) / 2;
    if (q < np) {
        int c = 0, rem = q;
        while (rem >= T - c) {
            rem -= T - c;
            ++c;
        }
        bi = c + rem;
        bj = c;
        return;
    }
    const int r = q - np;
    int b = (int)((sqrtf(8.0f * (float)r + 1.0f) - 1.0f) * 0.5f);
    while (b * (b + 1) / 2 > r) --b;
    while ((b + 1) * (b + 2) / 2 <= r) ++b;
    bi = WT + b;
    bj = WT + r - b * (b + 1) / 2;
}

constexpr int COLB = 132;  // column buffer stride (128 rows + a tile of slack)

template <int KT>
struct SmallRegs {
    double v[KT][16];  // v[k][r * 4 + c] = F(4 bi_k + r, 4 bj_k + c)
    int bi[KT], bj[KT];  // bi < 0: no tile
};

template <int KT, int NT = 256>
__device__ __forceinline__ void small_tiles(SmallRegs<KT>& R, int m, int w) {
    const int T = (m + 3) >> 2, WT = (w + 3) >> 2, ntile = T * (T + 1) / 2;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        const int q = threadIdx.x + NT * k;
        int bi = -1, bj = -1;
        if (q < ntile) tile_map(q, T, WT, bi, bj);
        R.bi[k] = bi;
        R.bj[k] = bj;
    }
}

// Load the tiles of the assembled packed front F (entries above the diagonal or
// past m read as 0; they are never stored).
template <int KT>
__device__ __forceinline__ void small_load(SmallRegs<KT>& R, const double* F, int m) {
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[k] + r, j = 4 * R.bj[k] + c;
                R.v[k][r * 4 + c] = (R.bi[k] >= 0 && i < m && i >= j) ? F[pk_col(m, j) + i - j] : 0.0;
            }
}

// The w pivot steps, right-looking over the whole front, four pivots (one tile
// column) per step.  Step b (pivots J = 4b .. J + nb - 1, nb = min(4, w - J)): the
// owners of tile column b publish its four columns (colbuf row-major, [row][4],
// double-buffered: one barrier per step); every thread factors the 4 x 4 diagonal
// block D itself (L_D), solves its rows i against it (l_i = c_i L_D^-T, l_i = L(i,
// J..J+3)) and updates its tiles right of the block with the rank-nb product; tiles
// in column b take l_i in the pivot columns (and the update in any CB column).
// colbuf: 2 x 4 * COLB doubles.
template <int KT>
__device__ __forceinline__ void small_steps(SmallRegs<KT>& R, double* colbuf, int w, int32_t* info, int c0) {
    for (int J = 0, b = 0; J < w; J += 4, ++b) {
        double* cb = colbuf + (b & 1) * 4 * COLB;
        const int nb = min(4, w - J);
#pragma unroll
        for (int k = 0; k < KT; ++k)  // publish tile column b
            if (R.bj[k] == b) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double* row = cb + 4 * (4 * R.bi[k] + r);
                    *reinterpret_cast<double2*>(row) = make_double2(R.v[k][r * 4], R.v[k][r * 4 + 1]);
                    *reinterpret_cast<double2*>(row + 2) = make_double2(R.v[k][r * 4 + 2], R.v[k][r * 4 + 3]);
                }
            }
        lds_barrier();
        // L_D = chol(D), D = rows J..J+3 of the published columns; rc[k] = 1 / L_D(k, k)
        double D[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double2 x01 = *reinterpret_cast<const double2*>(cb + 4 * (J + r));
            const double2 x23 = *reinterpret_cast<const double2*>(cb + 4 * (J + r) + 2);
            D[r][0] = x01.x;
            D[r][1] = x01.y;
            D[r][2] = x23.x;
            D[r][3] = x23.y;
        }
        double Ld[4][4], rc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double dd = D[c][c];
#pragma unroll
            for (int t = 0; t < c; ++t) dd = fma(-Ld[c][t], Ld[c][t], dd);
            if (c < nb && threadIdx.x == 0 && !(dd > 0.0)) report_fail(info, c0 + J + c);
            rc[c] = c < nb ? rsqrt_f64(dd) : 0.0;
            Ld[c][c] = dd * rc[c];
#pragma unroll
            for (int r = c + 1; r < 4; ++r) {
                double x = D[r][c];
#pragma unroll
                for (int t = 0; t < c; ++t) x = fma(-Ld[r][t], Ld[c][t], x);
                Ld[r][c] = x * rc[c];
            }
        }
        // l of one row: l[k] = (c[k] - sum_t<k l[t] L_D(k, t)) / L_D(k, k) (0 past nb)
        auto solve_row = [&](int row, double (&l)[4]) {
            const double2 x01 = *reinterpret_cast<const double2*>(cb + 4 * row);
            const double2 x23 = *reinterpret_cast<const double2*>(cb + 4 * row + 2);
            const double cr[4] = {x01.x, x01.y, x23.x, x23.y};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                double x = cr[k];
#pragma unroll
                for (int t = 0; t < k; ++t) x = fma(-l[t], Ld[k][t], x);
                l[k] = x * rc[k];
            }
        };
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            const int bi = R.bi[k], bj = R.bj[k];
            if (bi < 0 || bj < b) continue;  // no tile, or left of the block
            double lj[4][4];
#pragma unroll
            for (int c = 0; c < 4; ++c) solve_row(4 * bj + c, lj[c]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double li[4];
                solve_row(4 * bi + r, li);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    double x = R.v[k][r * 4 + c];
                    if (bj == b && c < nb) {  // tile column b: the pivot columns take l
                        x = li[c];
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; ++t) x = fma(-li[t], lj[c][t], x);
                    }
                    R.v[k][r * 4 + c] = x;
                }
            }
        }
    }
}

#ifndef SC_POTRF_FAST
#define SC_POTRF_FAST 1
#endif
// small_steps<1> restated for latency (the 64 x 64 diagonal blocks of the panel chain,
// and the tiny tree): one tile per thread, and after each step's barrier every LDS read
// of the step -- the 4 x 4 block D and this tile's 4 column rows and 4 row rows -- is in
// flight at once, before the serial L_D factorization; the pivot checks are folded into
// one report per step.  Same arithmetic in the same order as small_steps (bitwise equal).
__device__ __forceinline__ void small_steps1_fast(SmallRegs<1>& R, double* colbuf, int w, int32_t* info, int c0) {
    const int bi = R.bi[0], bj = R.bj[0];
    for (int J = 0, b = 0; J < w; J += 4, ++b) {
        double* cb = colbuf + (b & 1) * 4 * COLB;
        const int nb = min(4, w - J);
        if (bj == b) {  // publish tile column b
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double* row = cb + 4 * (4 * bi + r);
                *reinterpret_cast<double2*>(row) = make_double2(R.v[0][r * 4], R.v[0][r * 4 + 1]);
                *reinterpret_cast<double2*>(row + 2) = make_double2(R.v[0][r * 4 + 2], R.v[0][r * 4 + 3]);
            }
        }
        lds_barrier();
        const bool act = bi >= 0 && bj >= b;
        const int rj = act ? 4 * bj : J, ri = act ? 4 * bi : J;
        double2 d01[4], d23[4], j01[4], j23[4], i01[4], i23[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            d01[r] = *reinterpret_cast<const double2*>(cb + 4 * (J + r));
            d23[r] = *reinterpret_cast<const double2*>(cb + 4 * (J + r) + 2);
            j01[r] = *reinterpret_cast<const double2*>(cb + 4 * (rj + r));
            j23[r] = *reinterpret_cast<const double2*>(cb + 4 * (rj + r) + 2);
            i01[r] = *reinterpret_cast<const double2*>(cb + 4 * (ri + r));
            i23[r] = *reinterpret_cast<const double2*>(cb + 4 * (ri + r) + 2);
        }
        double D[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            D[r][0] = d01[r].x;
            D[r][1] = d01[r].y;
            D[r][2] = d23[r].x;
            D[r][3] = d23[r].y;
        }
        double Ld[4][4], rc[4];
        int bad = 4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double dd = D[c][c];
#pragma unroll
            for (int t = 0; t < c; ++t) dd = fma(-Ld[c][t], Ld[c][t], dd);
            if (c < nb && !(dd > 0.0)) bad = min(bad, c);
            rc[c] = c < nb ? rsqrt_f64(dd) : 0.0;
            Ld[c][c] = dd * rc[c];
#pragma unroll
            for (int r = c + 1; r < 4; ++r) {
                double x = D[r][c];
#pragma unroll
                for (int t = 0; t < c; ++t) x = fma(-Ld[r][t], Ld[c][t], x);
                Ld[r][c] = x * rc[c];
            }
        }
        if (bad < 4 && threadIdx.x == 0) report_fail(info, c0 + J + bad);
        if (!act) continue;
        auto solve = [&](const double2& x01, const double2& x23, double (&l)[4]) {
            const double cr[4] = {x01.x, x01.y, x23.x, x23.y};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                double x = cr[k];
#pragma unroll
                for (int t = 0; t < k; ++t) x = fma(-l[t], Ld[k][t], x);
                l[k] = x * rc[k];
            }
        };
        double lj[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c) solve(j01[c], j23[c], lj[c]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double li[4];
            solve(i01[r], i23[r], li);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                double x = R.v[0][r * 4 + c];
                if (bj == b && c < nb) {
                    x = li[c];
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t) x = fma(-li[t], lj[c][t], x);
                }
                R.v[0][r * 4 + c] = x;
            }
        }
    }
}

// The panel (columns < w, rows >= the column) to HBM.
template <int KT>
__device__ __forceinline__ void small_store_panel(const SmallRegs<KT>& R, double* __restrict__ panel, int m, int w) {
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        if (R.bi[k] < 0 || 4 * R.bj[k] >= w) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[k] + r, j = 4 * R.bj[k] + c;
                if (j < w && i >= j && i < m) panel[(int64_t)j * m + i] = R.v[k][r * 4 + c];
            }
    }
}

// The CB (rows / cols >= w) to HBM, column-major, ld = mb.
template <int KT>
__device__ __forceinline__ void small_store_cb(const SmallRegs<KT>& R, double* __restrict__ cb, int m, int w) {
    const int mb = m - w;
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        if (R.bi[k] < 0 || 4 * R.bi[k] + 3 < w) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[k] + r, j = 4 * R.bj[k] + c;
                if (j >= w && i >= j && i < m) cb[(int64_t)(j - w) * mb + (i - w)] = R.v[k][r * 4 + c];
            }
    }
}

// Zero, A entries, children's CBs from HBM (children in child-list order; skip: a
// child left out, the chain child of a chained front).  Latency-bound (a few entries
// per lane, several dependent global loads each), so every wave issues the loads of
// SA_U of its columns before the LDS stores / adds, and the next child's metadata is
// loaded while the current child is added.  SA_U = 4 where registers allow (the
// register-tile kernels with KT = 1 stay at 4 waves per SIMD only with SA_U = 1).
template <int SA_U = 4>
__device__ __forceinline__ void small_assemble(const DevPlan& P, int s, int c0, int w, int m,
                                               const double* __restrict__ Ax, double* F, int skip = -1) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int tot = (m * (m + 1)) >> 1;
    for (int idx = tid; idx < tot; idx += 256) F[idx] = 0.0;
    lds_barrier();
    for (int l0 = wid; l0 < w; l0 += 4 * SA_U) {  // A entries of the pivot columns
        int64_t q[SA_U];
        bool ok[SA_U];
        int pos[SA_U];
        int64_t src[SA_U];
#pragma unroll
        for (int u = 0; u < SA_U; ++u) {
            const int lc = l0 + 4 * u;
            const int64_t a0 = lc < w ? P.a_ptr[c0 + lc] : 0, a1 = lc < w ? P.a_ptr[c0 + lc + 1] : 0;
            q[u] = a0 + lane;
            ok[u] = q[u] < a1;
        }
#pragma unroll
        for (int u = 0; u < SA_U; ++u) {
            pos[u] = ok[u] ? P.a_pos[q[u]] : 0;
            src[u] = ok[u] ? P.a_src[q[u]] : 0;
        }
        double v[SA_U];
#pragma unroll
        for (int u = 0; u < SA_U; ++u) v[u] = ok[u] ? Ax[src[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < SA_U; ++u) {
            const int lc = l0 + 4 * u;
            if (ok[u]) F[pk_col(m, lc) - lc + pos[u]] = v[u];
        }
        // rare long columns (more than 64 entries): the rest one column at a time
#pragma unroll 1
        for (int u = 0; u < SA_U; ++u) {
            const int lc = l0 + 4 * u;
            if (lc >= w) break;
            const int64_t a1 = P.a_ptr[c0 + lc + 1];
            double* Fcol = F + pk_col(m, lc) - lc;
            for (int64_t qq = P.a_ptr[c0 + lc] + 64 + lane; qq < a1; qq += 64) Fcol[P.a_pos[qq]] = Ax[P.a_src[qq]];
        }
    }
    lds_barrier();
    const int cp0 = P.child_ptr[s], cp1 = P.child_ptr[s + 1];
    auto meta = [&](int ci, int& c, int& mbc, const int32_t*& rel, const double*& cb) {
        c = ci < cp1 ? P.child_list[ci] : -1;
        if (c < 0) return;
        mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        rel = P.relind + P.rel_ptr[c];
        cb = P.cb_pool + P.cb_off[c];
    };
    int c = -1, mbc = 0;
    const int32_t* rel = nullptr;
    const double* cb = nullptr;
    meta(cp0, c, mbc, rel, cb);
    for (int ci = cp0; ci < cp1; ++ci) {
        int cn = -1, mbn = 0;
        const int32_t* reln = nullptr;
        const double* cbn = nullptr;
        meta(ci + 1, cn, mbn, reln, cbn);  // in flight under this child's adds
        if (c != skip) {
            for (int j0 = wid; j0 < mbc; j0 += 4 * SA_U) {
                // SA_U columns jc = j0 + 4u of the child's CB, rows jc + lane (+ 64):
                // parent column, parent rows and values, all loads in flight first
                int pj[SA_U], r0[SA_U], r1[SA_U];
                double v0[SA_U], v1[SA_U];
#pragma unroll
                for (int u = 0; u < SA_U; ++u) {
                    const int jc = j0 + 4 * u;
                    const int i0 = jc + lane, i1 = i0 + 64;
                    pj[u] = jc < mbc ? rel[jc] : 0;
                    const bool k0 = jc < mbc && i0 < mbc, k1 = jc < mbc && i1 < mbc;
                    r0[u] = k0 ? rel[i0] : -1;
                    r1[u] = k1 ? rel[i1] : -1;
                    v0[u] = k0 ? cb[(int64_t)jc * mbc + i0] : 0.0;
                    v1[u] = k1 ? cb[(int64_t)jc * mbc + i1] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < SA_U; ++u) {
                    double* Fcol = F + pk_col(m, pj[u]) - pj[u];
                    if (r0[u] >= 0) Fcol[r0[u]] += v0[u];
                    if (r1[u] >= 0) Fcol[r1[u]] += v1[u];
                }
            }
            lds_barrier();
        }
        c = cn;
        mbc = mbn;
        rel = reln;
        cb = cbn;
    }
}

// Level launch: one workgroup per front; LDS = the packed front (maxm) + colbuf.
// seq > 0: one workgroup runs nodes[0 .. seq) in order (a whole small tree in
// postorder): each front's children were stored by earlier iterations, and the
// workgroup barrier between fronts makes those CB stores visible (one CU, one L1).
template <int KT>
__global__ __launch_bounds__(256) void front_small_kernel(DevPlan P, const int32_t* __restrict__ nodes,
                                                           const double* __restrict__ Ax, int seq) {
    extern __shared__ double F[];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    const int n = seq > 0 ? seq : 1;
    for (int f = 0; f < n; ++f) {
        const int s = nodes[seq > 0 ? f : blockIdx.x];
        const int c0 = P.sn_start[s];
        const int w = P.sn_start[s + 1] - c0;
        const int m = P.sn_m[s];
        SmallRegs<KT> R;
        small_tiles<KT>(R, m, w);
        small_assemble<KT == 1 ? 1 : 4>(P, s, c0, w, m, Ax, F);
        small_load<KT>(R, F, m);
        small_steps<KT>(R, colbuf, w, P.info, c0);
        small_store_panel<KT>(R, P.panel_pool + P.panel_off[s], m, w);
        if (m > w) small_store_cb<KT>(R, P.cb_pool + P.cb_off[s], m, w);
        if (seq > 0) __syncthreads();  // global CB stores visible to the next front's loads
    }
}

// Tiny tree: one workgroup, every image and CB in LDS (see TinyPlan).  The A stores
// of all fronts go in parallel first; then per front (postorder): its children's
// CB entries (one phase per child), the register factorization, the panel to HBM and
// the CB (packed lower, column j - w at pk_col(mb, j - w)) to LDS.
__global__ __launch_bounds__(256) void tiny_tree_kernel(DevPlan P, TinyPlan T, const double* __restrict__ Ax) {
    extern __shared__ double Lm[];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    __shared__ TinyFront fr[TINY_MAX_FRONTS];
    __shared__ int2 s_ph[TINY_MAX_FRONTS * TINY_MAX_FRONTS];
    __shared__ int2 s_pr[TINY_PR_LDS];
    __shared__ int32_t s_info;
    const int tid = threadIdx.x;
    // every plan word this workgroup will read, and the A values, loaded in one pass:
    // one global latency instead of one per extend-add phase
    if (tid < T.nf) fr[tid] = T.fr[tid];
    for (int e = tid; e < T.nph; e += 256) s_ph[e] = T.ph[e];
    for (int e = tid; e < min(T.npr, TINY_PR_LDS); e += 256) s_pr[e] = T.pr[e];
    if (tid == 0) s_info = 0x7f7f7f7f;
    for (int i = tid; i < T.lds; i += 256) Lm[i] = 0.0;
    lds_barrier();
    for (int e = tid; e < T.na; e += 256) {
        const int2 a = T.a[e];
        Lm[a.y] = Ax[a.x];
    }
    lds_barrier();
    int32_t* info = T.host_info ? &s_info : P.info;
    for (int f = 0; f < T.nf; ++f) {
        const TinyFront d = fr[f];
        for (int p = 0; p < d.np; ++p) {
            const int2 q = s_ph[d.e0 + p];
            for (int e = q.x + tid; e < q.y; e += 256) {
                const int2 pr = e < TINY_PR_LDS ? s_pr[e] : T.pr[e];
                Lm[pr.y] += Lm[pr.x];
            }
            lds_barrier();
        }
        SmallRegs<1> R;
        small_tiles<1>(R, d.m, d.w);
        small_load<1>(R, Lm + d.img, d.m);
        if (SC_POTRF_FAST)
            small_steps1_fast(R, colbuf, d.w, info, d.c0);
        else
            small_steps<1>(R, colbuf, d.w, info, d.c0);
        small_store_panel<1>(R, P.panel_pool + d.panel_off, d.m, d.w);
        if (d.m > d.w && R.bi[0] >= 0) {
            const int mb = d.m - d.w;
            double* cb = Lm + d.cb;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * R.bi[0] + r - d.w, j = 4 * R.bj[0] + c - d.w;
                    if (j >= 0 && i >= j && i < mb) cb[pk_col(mb, j) + i - j] = R.v[0][r * 4 + c];
                }
        }
        lds_barrier();
    }
    if (T.host_info) __syncthreads();  // every wave's panel stores done before the status word
    if (T.host_info && tid == 0) {  // the status word straight to the pinned host copy
        P.info[0] = s_info;
        __hip_atomic_store(T.host_info, s_info, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_tiny_tree(const DevPlan& P, const TinyPlan& T, int maxm, const double* Ax, hipStream_t st) {
    if (T.nf <= 0) return hipSuccess;
    if (T.nf > TINY_MAX_FRONTS || T.lds > TINY_MAX_LDS || maxm > 64 || T.nph > TINY_MAX_FRONTS * TINY_MAX_FRONTS)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(tiny_tree_kernel, dim3(1), dim3(256), (size_t)T.lds * sizeof(double), st, P, T, Ax);
    return hipGetLastError();
}

// Tiny dense: a matrix with n <= 64 as one dense lower triangle, factored right-looking
// by a single wave (no workgroup barriers: one wave's LDS operations complete in issue
// order).  Lane i holds row i in registers; the matrix is padded to NP = n rounded up
// to 16 with identity rows, so every loop is straight-line code.  Four pivots per step:
// the rows publish their four step columns to LDS, every lane factors the 4 x 4 diagonal
// block D redundantly, solves its own row of the step panel and publishes it, updates
// the next step's four columns first, publishes them and factors the next D, and only
// then applies the rest of the rank-4 update -- so the next step's serial chain (LDS
// round trip, four pivots) overlaps this step's bulk FMAs.  Entries outside the
// symbolic pattern come out as exact zeros (every product of the update has a
// structurally zero factor) and are not stored: a host-built lane map names, per dense
// entry, its A value and its panel-pool offset.  Status as tiny_tree_kernel.
#ifndef SC_TD_LA
#define SC_TD_LA 1  // 1: the next step's D factored under this step's bulk update
#endif
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "tiny_dense_kernel exchanges rows between the lanes of ONE 64-wide wave"
#endif
// Cross-lane LDS hand-over inside one wave: the lanes' stores must be ordered before the
// other lanes' loads (and earlier loads before later stores).  The hardware keeps one
// wave's LDS operations in issue order; the fence and the wave barrier keep the compiler
// from moving the lane-indexed stores and the constant-indexed loads across each other
// (they may alias).  Neither emits an instruction on gfx950.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
#ifndef SC_TD_BUF
#define SC_TD_BUF 1  // 1: the A loads and panel stores as range-checked buffer accesses (no branches)
#endif
#ifndef SC_TD_PROBE
#define SC_TD_PROBE 0  // timing probe (scripts/tiny_probe.py): 1 = loads and stores only, no factorization
#endif
// raw[4 * r .. 4 * r + 3] = step columns of row r (published) -> D and its factor
__device__ __forceinline__ void td_factor_d(const double* raw, int J, double (&Ld)[4][4], double (&rc)[4], int& bad) {
    double D[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double2 x01 = *reinterpret_cast<const double2*>(raw + 4 * (J + r));
        const double2 x23 = *reinterpret_cast<const double2*>(raw + 4 * (J + r) + 2);
        D[r][0] = x01.x;
        D[r][1] = x01.y;
        D[r][2] = x23.x;
        D[r][3] = x23.y;
    }
    bad = 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        double dd = D[c][c];
#pragma unroll
        for (int t = 0; t < c; ++t) dd = fma(-Ld[c][t], Ld[c][t], dd);
        if (!(dd > 0.0)) bad = min(bad, c);
        rc[c] = rsqrt_f64(dd);
        Ld[c][c] = dd * rc[c];
#pragma unroll
        for (int r = c + 1; r < 4; ++r) {
            double x = D[r][c];
#pragma unroll
            for (int t = 0; t < c; ++t) x = fma(-Ld[r][t], Ld[c][t], x);
            Ld[r][c] = x * rc[c];
        }
    }
}

// One four-pivot step of tiny_dense_kernel at compile-time column J (recursive over
// the steps, so that every register index is a constant).
template <int NP, int J>
__device__ __forceinline__ void td_steps(double (&a)[NP], double (&Ld)[4][4], double (&rc)[4], int& bad, int& fail,
                                         double* raw, double* lv, int i) {
    if constexpr (J < NP) {
        __builtin_amdgcn_sched_barrier(0);  // one step's live registers at a time
        if (bad < 4) fail = min(fail, J + bad);
        // this row's part of the step panel: l = a[J..J+3] L_D^-T
        const bool below = i >= J + 4;
        double l[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double x = below ? a[J + k] : 0.0;
#pragma unroll
            for (int t = 0; t < k; ++t) x = fma(-l[t], Ld[k][t], x);
            l[k] = x * rc[k];
        }
        wave_lds_sync();  // the previous step's lv reads are done
        *reinterpret_cast<double2*>(lv + 4 * i) = make_double2(l[0], l[1]);
        *reinterpret_cast<double2*>(lv + 4 * i + 2) = make_double2(l[2], l[3]);
        wave_lds_sync();  // every lane's l published before update() reads them
        // the step's columns of this row become final: L_D rows (the diagonal block's
        // rows) or l (below it); selects, not branches, so that a[] stays in registers
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double v = below ? l[c] : a[J + c];
#pragma unroll
            for (int r = c; r < 4; ++r) v = i == J + r ? Ld[r][c] : v;
            a[J + c] = v;
        }
        auto update = [&](int jj) {  // rank-4 update of column jj of this row
            const double2 x01 = *reinterpret_cast<const double2*>(lv + 4 * jj);
            const double2 x23 = *reinterpret_cast<const double2*>(lv + 4 * jj + 2);
            double x = a[jj];
            x = fma(-l[0], x01.x, x);
            x = fma(-l[1], x01.y, x);
            x = fma(-l[2], x23.x, x);
            x = fma(-l[3], x23.y, x);
            a[jj] = x;
        };
        if constexpr (J + 4 < NP && !SC_TD_LA) {  // no lookahead: the whole update, then the next D
#pragma unroll
            for (int jj = J + 4; jj < NP; ++jj) update(jj);
            wave_lds_sync();
            *reinterpret_cast<double2*>(raw + 4 * i) = make_double2(a[J + 4], a[J + 5]);
            *reinterpret_cast<double2*>(raw + 4 * i + 2) = make_double2(a[J + 6], a[J + 7]);
            wave_lds_sync();
            td_factor_d(raw, J + 4, Ld, rc, bad);
        }
        if constexpr (J + 4 < NP && SC_TD_LA) {
            // the next step's columns first, published, and its D loaded ...
#pragma unroll
            for (int jj = J + 4; jj < J + 8; ++jj) update(jj);
            wave_lds_sync();
            *reinterpret_cast<double2*>(raw + 4 * i) = make_double2(a[J + 4], a[J + 5]);
            *reinterpret_cast<double2*>(raw + 4 * i + 2) = make_double2(a[J + 6], a[J + 7]);
            wave_lds_sync();
            double Dn[4][4], Ln[4][4], rn[4];
            int bn = 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double2 x01 = *reinterpret_cast<const double2*>(raw + 4 * (J + 4 + r));
                const double2 x23 = *reinterpret_cast<const double2*>(raw + 4 * (J + 4 + r) + 2);
                Dn[r][0] = x01.x;
                Dn[r][1] = x01.y;
                Dn[r][2] = x23.x;
                Dn[r][3] = x23.y;
            }
            auto pivot = [&](int c) {  // pivot c of the next D (td_factor_d, one column)
                double dd = Dn[c][c];
#pragma unroll
                for (int t = 0; t < c; ++t) dd = fma(-Ln[c][t], Ln[c][t], dd);
                if (!(dd > 0.0)) bn = min(bn, c);
                rn[c] = rsqrt_f64(dd);
                Ln[c][c] = dd * rn[c];
#pragma unroll
                for (int r = c + 1; r < 4; ++r) {
                    double x = Dn[r][c];
#pragma unroll
                    for (int t = 0; t < c; ++t) x = fma(-Ln[r][t], Ln[c][t], x);
                    Ln[r][c] = x * rn[c];
                }
            };
            // ... and factored under the rest of this step's update, in groups of GW
            // columns with one pivot of the next D per group (the scheduling barriers
            // bound the registers the compiler's load hoisting takes; entries above the
            // diagonal are computed too and never read)
            constexpr int GW = NP > 48 ? 4 : 8;  // columns per group (registers: a[] is 2 NP VGPRs)
            constexpr int NG = (NP - J - 8 + GW - 1) / GW;
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if (g < 4) pivot(g);
#pragma unroll
                for (int u = 0; u < GW; ++u)
                    if (J + 8 + GW * g + u < NP) update(J + 8 + GW * g + u);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int c = NG; c < 4; ++c) pivot(c);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                rc[r] = rn[r];
#pragma unroll
                for (int c = 0; c < 4; ++c) Ld[r][c] = Ln[r][c];
            }
            bad = bn;
        }
        td_steps<NP, J + 4>(a, Ld, rc, bad, fail, raw, lv, i);
    }
}

template <int NP>
__global__ __launch_bounds__(64) void tiny_dense_kernel(DevPlan P, TinyPlan T, int n, const double* __restrict__ Ax) {
    __shared__ __attribute__((aligned(16))) double raw[NP * 4];
    __shared__ __attribute__((aligned(16))) double lv[NP * 4];
    __shared__ int po[NP * 64];  // the panel offsets of the lane map, parked for the end
    const int i = threadIdx.x;
    // the lane map: entry (row i, column j) comes from Ax[q[j].x] and goes to panel
    // offset q[j].y (-1: none) -- one coalesced 512-byte load per column, then every A
    // value straight into its register (no LDS image, no barriers); the panel offsets
    // wait in LDS (lane-private slots) for the stores at the end
    int2 q[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) q[j] = T.a[j * 64 + i];
#pragma unroll
    for (int j = 0; j < NP; ++j) po[j * 64 + i] = q[j].y;
    double a[NP];
    int fail = n;
    double Ld[4][4], rc[4];
    int bad;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
#if SC_TD_BUF  // branch-free: a missing entry reads 0 through the buffer's range check
        a[j] = buf_ld(buf_rsrc(Ax, (uint32_t)T.nax * 8u), q[j].x >= 0 ? q[j].x * 8 : BUF_DEAD, 0);
#else
        a[j] = q[j].x >= 0 ? Ax[q[j].x] : 0.0;
#endif
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) a[j] = (i == j && i >= n) ? 1.0 : a[j];  // identity padding
    if (SC_TD_PROBE != 1) {
        wave_lds_sync();
        *reinterpret_cast<double2*>(raw + 4 * i) = make_double2(a[0], a[1]);
        *reinterpret_cast<double2*>(raw + 4 * i + 2) = make_double2(a[2], a[3]);
        wave_lds_sync();
        td_factor_d(raw, 0, Ld, rc, bad);
        td_steps<NP, 0>(a, Ld, rc, bad, fail, raw, lv, i);
    }
    if (fail > n) fail = n;  // padding pivots never fail; a failure at or past n is none
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int o = po[j * 64 + i];
#if SC_TD_BUF  // branch-free: an entry that is not stored goes out of the buffer's range
        buf_st(a[j], buf_rsrc(P.panel_pool, (uint32_t)T.npan * 8u), o >= 0 ? o * 8 : BUF_DEAD, 0);
#else
        if (o >= 0) P.panel_pool[o] = a[j];
#endif
    }
    // one wave: lane 0's system-scope release store below waits for the wave's panel
    // stores, so the status word is seen after the factor
    if (i == 0) {
        if (T.host_info) {  // the status word straight to the pinned host copy
            const int32_t st = fail < n ? fail + 1 : 0x7f7f7f7f;
            P.info[0] = st;
            __hip_atomic_store(T.host_info, st, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (fail < n) {
            report_fail(P.info, fail);
        }
    }
}

hipError_t launch_tiny_dense(const DevPlan& P, const TinyPlan& T, int n, const double* Ax, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (n > TINY_DENSE_N || T.na != tiny_dense_np(n) * 64) return hipErrorInvalidValue;  // the lane map's shape
    // every A / panel byte offset in range, and the dead offset out of it
    if ((int64_t)T.nax * 8 >= BUF_DEAD || (int64_t)T.npan * 8 >= BUF_DEAD) return hipErrorInvalidValue;
    if (n <= 16)
        hipLaunchKernelGGL(tiny_dense_kernel<16>, dim3(1), dim3(64), 0, st, P, T, n, Ax);
    else if (n <= 32)
        hipLaunchKernelGGL(tiny_dense_kernel<32>, dim3(1), dim3(64), 0, st, P, T, n, Ax);
    else if (n <= 48)
        hipLaunchKernelGGL(tiny_dense_kernel<48>, dim3(1), dim3(64), 0, st, P, T, n, Ax);
    else
        hipLaunchKernelGGL(tiny_dense_kernel<64>, dim3(1), dim3(64), 0, st, P, T, n, Ax);
    return hipGetLastError();
}

// Chain, part 1 (one workgroup per chained front, all in parallel): the packed image
// of A entries and the children other than the chain child, to HBM.
__global__ __launch_bounds__(256) void chain_init_kernel(DevPlan P, ChainPlan C, int first,
                                                          const double* __restrict__ Ax) {
    extern __shared__ double F[];
    const ChainDesc d = C.desc[first + blockIdx.x];
    small_assemble(P, d.s, d.c0, d.w, d.m, Ax, F, d.sp);
    const int tot = (d.m * (d.m + 1)) >> 1;
    double* out = C.init + d.init_off;
    for (int idx = threadIdx.x; idx < tot; idx += 256) out[idx] = F[idx];
}

#ifndef SC_CHAIN_DB
#define SC_CHAIN_DB 1
#endif
// Chain, part 2 (one workgroup of CHAIN_NT threads, one tile each): iteration i loads
// front i's tiles from the LDS front buffer, writes front i + 1's image (held in
// registers since iteration i - 1) into the buffer, issues the loads of front i + 2's
// image and CB relind, factors front i, stores its panel, and adds its CB into the
// buffer at the parent's positions (the last front's CB goes to HBM).
constexpr int CHAIN_IMG = (128 * 129 / 2 + CHAIN_NT - 1) / CHAIN_NT;  // image doubles per thread
__global__ __launch_bounds__(CHAIN_NT) void front_chain_kernel(DevPlan P, ChainPlan C, int first, int count, int fsz) {
    extern __shared__ double F[];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    __shared__ ChainDesc ds[CHAIN_MAXF];
    const int tid = threadIdx.x;
    for (int i = tid; i < count; i += CHAIN_NT) ds[i] = C.desc[first + i];
    lds_barrier();
    // the next front's prefetched image slice, tile and its CB relind (rows, cols;
    // four 8-bit parent rows packed per word: relind < m <= 128)
    double img[CHAIN_IMG];
    int nbi, nbj;
    uint32_t nrr, nrc;
    auto prefetch = [&](int f) {
        const ChainDesc& d = ds[f];
        const int tot = (d.m * (d.m + 1)) >> 1;
        const double* src = C.init + d.init_off;
#pragma unroll
        for (int q = 0; q < CHAIN_IMG; ++q) {
            const int idx = tid + CHAIN_NT * q;
            img[q] = idx < tot ? src[idx] : 0.0;
        }
        const int T = (d.m + 3) >> 2;
        nbi = nbj = -1;
        if (tid < T * (T + 1) / 2) tile_map(tid, T, (d.w + 3) >> 2, nbi, nbj);
        // parent rows of the tile's CB rows / columns: one packed word per tile row
        // (host-built, 0 where the chain ends or rows are pivots)
        nrr = nbi >= 0 ? C.relp[d.relp_off + nbi] : 0u;
        nrc = nbi >= 0 ? C.relp[d.relp_off + nbj] : 0u;
    };
    // two front buffers (SC_CHAIN_DB): front i + 1's image goes into the other buffer
    // while front i loads its tiles, with no barrier between
    auto Fb = [&](int f) { return SC_CHAIN_DB ? F + (f & 1) * fsz : F; };
    auto put = [&](int f) {  // image slice -> the LDS buffer
        const int tot = (ds[f].m * (ds[f].m + 1)) >> 1;
        double* Fd = Fb(f);
#pragma unroll
        for (int q = 0; q < CHAIN_IMG; ++q) {
            const int idx = tid + CHAIN_NT * q;
            if (idx < tot) Fd[idx] = img[q];
        }
    };
    int cbi, cbj;
    uint32_t crr, crc;
    auto take = [&]() {
        cbi = nbi;
        cbj = nbj;
        crr = nrr;
        crc = nrc;
    };
    prefetch(0);
    put(0);
    take();
    if (count > 1) prefetch(1);
    lds_barrier();
    for (int i = 0; i < count; ++i) {
        uint64_t* stamp = C.stamps ? C.stamps + 8 * (first + i) : nullptr;
        if (stamp && tid == 0) stamp[0] = __builtin_amdgcn_s_memtime();
        const ChainDesc d = ds[i];
        const int m = d.m, w = d.w;
        SmallRegs<1> R;
        R.bi[0] = cbi;
        R.bj[0] = cbj;
        const uint32_t rr = crr, rc = crc;
        small_load<1>(R, Fb(i), m);
        if (!SC_CHAIN_DB) lds_barrier();  // every thread has its tile: the buffer is free
        if (stamp && tid == 0) stamp[1] = __builtin_amdgcn_s_memtime();
        const bool has_parent = i + 1 < count;
        if (has_parent) {
            put(i + 1);  // ordered before the CB adds below by the steps' barriers
            take();
            if (i + 2 < count) prefetch(i + 2);
        }
        if (stamp && tid == 0) stamp[2] = __builtin_amdgcn_s_memtime();
        small_steps<1>(R, colbuf, w, P.info, d.c0);
        if (w == 0) lds_barrier();
        if (stamp && tid == 0) stamp[3] = __builtin_amdgcn_s_memtime();
        small_store_panel<1>(R, P.panel_pool + d.panel_off, m, w);
        if (m > w && R.bi[0] >= 0 && 4 * R.bi[0] + 3 >= w) {
            if (!has_parent) {
                small_store_cb<1>(R, P.cb_pool + d.cb_off, m, w);
            } else {  // CB entries into the parent's front (relind injective: no collisions)
                const int mp = ds[i + 1].m;
                double* Fp = Fb(i + 1);
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int ii = 4 * R.bi[0] + r, jj = 4 * R.bj[0] + c;
                        const int pr = (rr >> (8 * r)) & 255, pc = (rc >> (8 * c)) & 255;
                        if (jj >= w && ii >= jj && ii < m) Fp[pk_col(mp, pc) + pr - pc] += R.v[0][r * 4 + c];
                    }
            }
        }
        lds_barrier();
        if (stamp && tid == 0) stamp[4] = __builtin_amdgcn_s_memtime();
    }
}

// ---------------------------------------------------------------------------
// Pipelined variants (default).  A full 64-column block runs generated
// straight-line code (panel_gen.inc, gen_panel.py) that keeps ~24 LDS operands
// in flight per wave; a partial last block (nb < 64) uses the template path.
// ---------------------------------------------------------------------------
#include "panel_gen.inc"

// Diagonal block (nb <= 64) of a large front's panel: 256 threads hold its 4 x 4
// tiles in registers (the small-front machinery with m = w = nb: 16 four-pivot
// steps, one LDS barrier each) instead of one wave walking 64 pivots.
__global__ __launch_bounds__(256) void potrf_tiles_kernel(DevPlan P, const int2* __restrict__ tasks) {
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    double* blk = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + k0;
    SmallRegs<1> R;
    small_tiles<1>(R, nb, nb);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
            R.v[0][r * 4 + c] = (R.bi[0] >= 0 && i < nb && i >= j) ? blk[(int64_t)j * m + i] : 0.0;
        }
    if (SC_POTRF_FAST)
        small_steps1_fast(R, colbuf, nb, P.info, c0 + k0);
    else
        small_steps<1>(R, colbuf, nb, P.info, c0 + k0);
    if (R.bi[0] < 0) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
            if (i < nb && i >= j) blk[(int64_t)j * m + i] = R.v[0][r * 4 + c];
        }
}

// Partial last block (nb < 64) of the panel TRSM: template path, kept out of
// line so its registers do not constrain the generated full-block code.
// Rows [r0, r0 + nrows).
__device__ __forceinline__ void trsm_partial(double* pan, int m, int k0, int nb, int r0, int nrows, double* Lc,
                                             double* invd) {
    constexpr int LD = PNB + 2;
    const int tid = threadIdx.x;
    const double* blk = pan + (int64_t)k0 * m + k0;
    for (int idx = tid; idx < PNB * PNB; idx += TRSM_ROWS) {
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
__global__ __launch_bounds__(TRSM_ROWS) void trsm_partial_kernel(DevPlan P, const TrsmTask* __restrict__ tasks) {
    __shared__ double Lc[PNB * (PNB + 2)];
    __shared__ double invd[PNB];
    const TrsmTask t = tasks[blockIdx.x];
    const int s = t.s, k0 = t.k0, r0 = t.r0;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    trsm_partial(P.panel_pool + P.panel_off[s], m, k0, min(PNB, w - k0), r0, min(TRSM_ROWS, t.r1 - r0), Lc, invd);
}

// Diagonal block POTRF fused with the panel TRSM, rows [r0, r0 + TRSM_ROWS): every
// workgroup loads the 64 x 64 diagonal block, factors it in registers (4 x 4 tiles,
// 16 four-pivot steps: a few microseconds) and packs L11 into an LDS stream in the
// order the generated solve consumes it (1/L(J,J), then L(J+1..63, J)).  One launch
// per 64-column step instead of two: on the panel chain every kernel boundary costs
// more than this redundant factorization.  L11 overwrites the block in HBM only once
// every workgroup of the block has read it: t.w - 1 indexes the block's arrival
// counter, and the last workgroup to arrive stores L11 and rearms the counter.  A
// block with no rows below gets one task with r0 >= m (factor and store only).
template <int PRE>
__global__ __launch_bounds__(TRSM_ROWS) void trsm_panel_g_kernel(DevPlan P, const TrsmTask* __restrict__ tasks,
                                                                 int32_t* __restrict__ arrive) {
    static_assert(TRSM_ROWS == 256, "the fused POTRF maps 4 x 4 tiles onto 256 threads");
    __shared__ double2 S[TRSM64_STREAM / 2];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    __shared__ int s_last;
    const TrsmTask t = tasks[blockIdx.x];
    const int s = t.s, k0 = t.k0, r0 = t.r0, r1 = t.r1;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    double* pan = P.panel_pool + P.panel_off[s];
    if (nb < PNB) return;  // partial blocks: potrf_tiles_kernel + trsm_partial_kernel
    double* blk = pan + (int64_t)k0 * m + k0;
    double* Sd = reinterpret_cast<double*>(S);
    SmallRegs<1> R;
    small_tiles<1>(R, PNB, PNB);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
            R.v[0][r * 4 + c] = (R.bi[0] >= 0 && i >= j) ? blk[(int64_t)j * m + i] : 0.0;
        }
    if constexpr (PRE == 2) {  // the block is L11 already (its own launch): stream it, solve the rows
        if (R.bi[0] >= 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
                    if (i >= j) Sd[PNB * j - j * (j - 1) / 2 + (i - j)] = (i == j) ? 1.0 / R.v[0][r * 4 + c] : R.v[0][r * 4 + c];
                }
        }
        const int row = r0 + tid;
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan + (int64_t)k0 * m, (uint32_t)m * PNB * 8u);
        const int voff = row < r1 ? row * 8 : BUF_DEAD;
        double r[PNB];
#pragma unroll
        for (int c = 0; c < PNB; ++c) r[c] = buf_ld(rs, voff, c * m * 8);
        __syncthreads();
        trsm64_full(r, S);
#pragma unroll
        for (int c = 0; c < PNB; ++c) buf_st(r[c], rs, voff, c * m * 8);
        return;
    }
    if (SC_POTRF_FAST)  // every block load has returned
        small_steps1_fast(R, colbuf, PNB, P.info, c0 + k0);
    else
        small_steps<1>(R, colbuf, PNB, P.info, c0 + k0);
    if (R.bi[0] >= 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
                if (i >= j) Sd[PNB * j - j * (j - 1) / 2 + (i - j)] = (i == j) ? 1.0 / R.v[0][r * 4 + c] : R.v[0][r * 4 + c];
            }
    }
    const int row = r0 + tid;
    // the 64 block columns, m rows each (< 2^31 bytes for m < 4M); dead lanes masked
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan + (int64_t)k0 * m, (uint32_t)m * PNB * 8u);
    const int voff = row < r1 ? row * 8 : BUF_DEAD;
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = buf_ld(rs, voff, c * m * 8);
    __syncthreads();
    if (tid == 0) {
        const int k1 = k0 + PNB;
        const int nwg = (max(r1, k1 + 1) - k1 + TRSM_ROWS - 1) / TRSM_ROWS;
        const int old = __hip_atomic_fetch_add(arrive + (t.ctr - 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == nwg - 1;
        if (old == nwg - 1) __hip_atomic_store(arrive + (t.ctr - 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_last && R.bi[0] >= 0) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[0] + rr, j = 4 * R.bj[0] + c;
                if (i >= j) blk[(int64_t)j * m + i] = R.v[0][rr * 4 + c];
            }
    }
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
// Extend-add fused into the CB update (fronts whose contribution block is not
// assembled): C = sum over children of their CB entries that map into the tile, minus
// the tile's A A^T.  Replaces the assembly's zero + add of the CB region and the
// SYRK's read of it (two of the four HBM passes over every CB entry).  The tile is
// built in LDS in 64-row chunks (G[col * GLD + row], GLD odd: the epilogue's 16
// columns x 4 rows per load hit distinct banks); wave w owns the chunk's columns
// c = w (mod waves), so children add in their fixed order with no atomics and no
// barrier per child (deterministic).  A child's CB rows that land in a 64-row block
// of the parent's CB are one contiguous run (relind is increasing), and so are its
// columns in a 64-column block: the host's segment table (GSeg) lists, per 64 x 64
// block of the CB, each child's runs and base pointers -- one uniform (scalar) load
// per child instead of the child-list / plan / bounds lookup chain.
// timing probes of the gathering CB launches (results wrong by construction):
// SC_PROBE_NOGATHER = 1 leaves the children's entries out, SC_PROBE_NOK = 1 the K loop
#ifndef SC_PROBE_NOGATHER
#define SC_PROBE_NOGATHER 0
#endif
#ifndef SC_PROBE_NOK
#define SC_PROBE_NOK 0
#endif
template <int BT, int WM, int WN, int BK = 16, int GR = 64>
__device__ __forceinline__ void syrk_gather_epilogue(const GemmTask& T, const int64_t* __restrict__ gblk,
                                                     const GSeg* __restrict__ gseg, int row0, int col0,
                                                     double4_t (&acc)[BT / WM / 16][BT / WN / 16], double* smem) {
    constexpr int NW = WM * WN, NT = 64 * NW;
    constexpr int RTM = BT / WM / 16, RTN = BT / WN / 16;
    // GR: rows per chunk (64, or 32 for the lean instance), GLD: LDS column stride (doubles)
    constexpr int GLD = GR + 1;
    // child columns per batch of loads: all of a wave's <= 64 / NW columns per child for
    // 64-tiles; 4 for 128-tiles (VGPR budget: 4 waves / SIMD)
    constexpr int GQ = BT == 64 ? (GR == 32 ? 8 : 64 / NW) : SC_GATHER_Q;
    // segments whose relative indices are loaded together (VGPR budget: 128-tiles keep
    // four workgroups per CU with one)
    constexpr int SB = BT == 64 ? 4 : 1;
    constexpr int OPS = 2 * 2 * BK * (BT + 16);  // the operand stages' doubles (smem)
    static_assert(BT * GLD <= OPS, "gather chunk fits the operand LDS");
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid / WN, wc = wid % WN;
    const int w = T.gw;
    const int mb = T.M;
    const int nb = (mb + 63) >> 6;
    const int64_t* __restrict__ blk = gblk + T.gb;
    const GSeg* __restrict__ seg = gseg;
    double* G = smem;
    double* __restrict__ C = T.C;
    const int64_t ldc = T.ldc;
    const __amdgpu_buffer_rsrc_t rc = buf_rsrc(C + (int64_t)col0 * ldc, (uint32_t)(min(BT, T.N - col0) * ldc * 8));
#pragma unroll 1
    for (int h = 0; h < BT / GR; ++h) {
        const int r0 = row0 + h * GR;  // CB rows of this chunk: [r0, r0 + GR)
        const int rb = r0 >> 6;        // its 64-row block of the CB
        if (h) __syncthreads();        // previous chunk's G fully read
        for (int e = tid; e < BT * GLD; e += NT) G[e] = 0.0;
        __syncthreads();
        // the segments of the chunk's blocks (rb, cb), cb over the tile's 64-column
        // blocks on or below the diagonal, in the host table's (child) order: each G
        // entry gets its children's adds in child order (deterministic, no atomics)
        const int cb1 = min(min(nb, rb + 1), (col0 + BT) >> 6);
        for (int cbk = col0 >> 6; !SC_PROBE_NOGATHER && r0 < mb && cbk < cb1; ++cbk) {
            const int64_t bi = (int64_t)rb * (rb + 1) / 2 + cbk;
            const int64_t p0 = blk[bi], p1 = blk[bi + 1];
            for (int64_t pb = p0; pb < p1; pb += SB) {
                // this lane's chunk row and tile column of SB segments, loads in flight together
                int prw[SB], pcl[SB];
#pragma unroll
                for (int q = 0; q < SB; ++q) {
                    prw[q] = -1;
                    pcl[q] = -1;
                    if (pb + q < p1) {
                        const GSeg& g = seg[pb + q];
                        const int ic = g.ilo + lane, jl = g.jlo + lane;
                        if (ic < g.ihi) prw[q] = g.rel[ic] - w - r0;
                        if (jl < g.jhi) pcl[q] = g.rel[jl] - w - col0;
                    }
                }
#pragma unroll
                for (int q = 0; q < SB; ++q) {
                    if (pb + q >= p1) break;
                    const GSeg& g = seg[pb + q];
                    const int ic = g.ilo + lane;
                    const int prow = prw[q] < GR ? prw[q] : -1;  // 32-row chunks: the other half of the block
                    const int mbc = g.mbc;
                    const double* __restrict__ cb = g.cb;
                    uint64_t mask = __ballot(pcl[q] >= 0 && pcl[q] % NW == wid);
                    while (mask) {  // up to GQ owned child columns (uniform), all loads in flight first
                        int jc[GQ], pc[GQ];
#pragma unroll
                        for (int u = 0; u < GQ; ++u) {
                            const int b = mask ? __builtin_ctzll(mask) : -1;
                            jc[u] = b < 0 ? -1 : g.jlo + b;
                            pc[u] = b < 0 ? 0 : __builtin_amdgcn_readlane(pcl[q], b);
                            mask &= mask - 1;
                        }
                        double v[GQ];
                        bool ok[GQ];
#pragma unroll
                        for (int u = 0; u < GQ; ++u) {  // column jc of the child's CB, rows >= jc
                            ok[u] = jc[u] >= 0 && prow >= 0 && ic >= jc[u];
                            const __amdgpu_buffer_rsrc_t rs = buf_rsrc(cb + (int64_t)max(jc[u], 0) * mbc, (uint32_t)mbc * 8u);
                            v[u] = buf_ld(rs, ok[u] ? ic * 8 : BUF_DEAD, 0);
                        }
#pragma unroll
                        for (int u = 0; u < GQ; ++u)
                            if (ok[u]) G[pc[u] * GLD + prow] += v[u];
                    }
                }
            }
        }
        __syncthreads();
        // the waves whose MFMA rows lie in this chunk (a wave's BT / WM <= 64 rows sit in
        // one chunk) form C = G - acc (no C read)
        static_assert(GR % (BT / WM) == 0, "a wave's rows lie in one chunk");
        // ... in G (each entry by its one owner lane), then the chunk leaves column by
        // column: GR consecutive rows of a column per wave-wide store, where the MFMA
        // layout stores 16 runs of 32 bytes per instruction (502.7 / 503.5 -> 499.0 /
        // 499.2 ms at 128^3)
        if ((wr * (BT / WM)) / GR == h) {
#pragma unroll
            for (int a = 0; a < RTM; ++a)
#pragma unroll
                for (int b = 0; b < RTN; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int lr = wr * (BT / WM) + a * 16 + MFMA_F64_ROW(lane, r);
                        const int lc = wc * (BT / WN) + b * 16 + (lane & 15);
                        G[lc * GLD + (lr - h * GR)] -= acc[a][b][r];
                    }
        }
        __syncthreads();
#pragma unroll 4
        for (int e = tid; e < BT * GR; e += NT) {
            const int lr = e % GR, lc = e / GR;
            const int gi = r0 + lr, gj = col0 + lc;
            const bool live = gi < T.M && gi >= gj && gj < T.N;
            buf_st(G[lc * GLD + lr], rc, live ? (int)((gi + (int64_t)(gj - col0) * ldc) * 8) : BUF_DEAD, 0);
        }
    }
}

// C -= acc through LDS (C read-modify-write launches: panel updates, assembled CBs), in
// GR-row chunks: the chunk's C loaded column by column (GR consecutive rows per wave-wide
// load), the owner lanes subtract their MFMA entries in LDS, the chunk stored column by
// column -- where the MFMA layout reads and writes 16 runs of 32 bytes per instruction.
template <int BT, int WM, int WN, int BK = 16, int GR = 64>
__device__ __forceinline__ void syrk_rmw_epilogue(const GemmTask& T, int row0, int col0,
                                                  double4_t (&acc)[BT / WM / 16][BT / WN / 16], double* smem) {
    constexpr int NW = WM * WN, NT = 64 * NW;
    constexpr int RTM = BT / WM / 16, RTN = BT / WN / 16;
    constexpr int GLD = GR + 1;
    constexpr int OPS = 2 * 2 * BK * (BT + 16);
    static_assert(BT * GLD <= OPS, "chunk fits the operand LDS");
    static_assert(GR % (BT / WM) == 0, "a wave's rows lie in one chunk");
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid / WN, wc = wid % WN;
    double* G = smem;
    const int64_t ldc = T.ldc;
    const __amdgpu_buffer_rsrc_t rc = buf_rsrc(T.C + (int64_t)col0 * ldc, (uint32_t)(min(BT, T.N - col0) * ldc * 8));
#pragma unroll 1
    for (int h = 0; h < BT / GR; ++h) {
        const int r0 = row0 + h * GR;
        if (h) __syncthreads();  // the previous chunk's stores have read G
#pragma unroll 4
        for (int e = tid; e < BT * GR; e += NT) {
            const int lr = e % GR, lc = e / GR;
            const int gi = r0 + lr, gj = col0 + lc;
            const bool live = gi < T.M && gi >= gj && gj < T.N;
            G[lc * GLD + lr] = buf_ld(rc, live ? (int)((gi + (int64_t)(gj - col0) * ldc) * 8) : BUF_DEAD, 0);
        }
        __syncthreads();
        if ((wr * (BT / WM)) / GR == h) {
#pragma unroll
            for (int a = 0; a < RTM; ++a)
#pragma unroll
                for (int b = 0; b < RTN; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int lr = wr * (BT / WM) + a * 16 + MFMA_F64_ROW(lane, r);
                        const int lc = wc * (BT / WN) + b * 16 + (lane & 15);
                        G[lc * GLD + (lr - h * GR)] -= acc[a][b][r];
                    }
        }
        __syncthreads();
#pragma unroll 4
        for (int e = tid; e < BT * GR; e += NT) {
            const int lr = e % GR, lc = e / GR;
            const int gi = r0 + lr, gj = col0 + lc;
            const bool live = gi < T.M && gi >= gj && gj < T.N;
            buf_st(G[lc * GLD + lr], rc, live ? (int)((gi + (int64_t)(gj - col0) * ldc) * 8) : BUF_DEAD, 0);
        }
    }
}

// The MFMA K loop of one BT x BT output tile: acc += A[row0 + i, :] A[col0 + j, :]^T
// over k < K (A column-major, ld lda; rows past M (i) / N (j) read as 0).  BK = 16,
// register-staged double-buffered LDS (As / Bs: 2 stages of BK x (BT + 16) doubles
// each, +128 B row pad: the two k-rows read by a half-wave hit disjoint banks).
// The last K stage is peeled out of the loop (no prefetch, no next-stage stores): 503.8 /
// 504.5 -> 502.7 / 502.5 ms at 128^3, interleaved (profiles/r06/ab_kloop.txt).  Skipping
// work there was measured too and dropped: the last stage's sub-steps past K (w = 16q + 1
// is common) and, on tiles on the diagonal of C, the MFMAs of 16 x 16 tiles above it
// (discarded by every epilogue) gained 1-2 ms with the old epilogues and nothing with the
// staged ones (493.7 ms without, 493.4 with the K skip, 494.7 with both), while the tiles'
// changed timing raised the CB SYRK's L2-miss fetches 34 -> 42 / 59 GB per launch
// (profiles/r06/ab_kskip.txt); as branches inside the K loop they lost outright (513 ms).
template <int BT, int WM, int WN, int BK = 16>
__device__ __forceinline__ void mfma_kloop(const double* __restrict__ A, int64_t lda, int K, int M, int N, int row0,
                                           int col0, double4_t (&acc)[BT / WM / 16][BT / WN / 16], double* smem) {
    static_assert(BK == 16 || BK == 8, "four-deep k sub-steps of the MFMA");
    constexpr int NT = 64 * WM * WN;
    constexpr int LDT = BT + 16;
    constexpr int RTM = BT / WM / 16, RTN = BT / WN / 16;
    double(*As)[BK * LDT] = reinterpret_cast<double(*)[BK * LDT]>(smem);
    double(*Bs)[BK * LDT] = reinterpret_cast<double(*)[BK * LDT]>(smem + 2 * BK * LDT);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid / WN, wc = wid % WN;
    // staging: BK x BT doubles per operand over NT threads
    constexpr int PER = BT * BK / NT;
    // Operands through a per-stage buffer resource (columns k0 .. k0 + BK of A):
    // K past the end and rows past M / N fall outside it and load 0 -- no branches,
    // and buffer loads count only vmcnt, so the LDS waits of the MFMA loop do not
    // also wait for the next stage's prefetch (flat loads count both).
    double ra[PER], rb[PER];
    auto gload = [&](int k0) {
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(A + (int64_t)k0 * lda, (uint32_t)(min(BK, K - k0) * lda * 8));
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + q * NT;
            const int r = e % BT, kk = e / BT;
            const int gr = row0 + r, gc = col0 + r;
            ra[q] = buf_ld(rs, gr < M ? (int)((gr + kk * lda) * 8) : BUF_DEAD, 0);
            rb[q] = buf_ld(rs, gc < N ? (int)((gc + kk * lda) * 8) : BUF_DEAD, 0);
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

    const int nk = (K + BK - 1) / BK;
    // one K stage; LAST: no prefetch of a next stage
    auto stage = [&](int kt, auto last) {
        constexpr bool LAST = decltype(last)::value;
        const int cur = kt & 1;
        if (!LAST) gload((kt + 1) * BK);
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
            // the next stage's LDS stores go out under the last sub-step's MFMAs, not
            // between them and the barrier: 547 -> 532 ms at 128^3 (stores after sub-step
            // 1: 535.8; A after 1 and B after 2: 533.0; the loads issued after sub-step 0
            // instead: 533.3, both: 536.8)
            if (!LAST && kk == BK - 8) sstore(cur ^ 1);
        }
        __syncthreads();
    };
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt + 1 < nk; ++kt) stage(kt, std::false_type {});
    if (nk > 0) stage(nk - 1, std::true_type {});
}

// Panel chain lookahead (the pre-factor workgroup of an inner panel update, tile marker
// y = -1): the update's tile (0, 0) is the NEXT chain step's 64 x 64 diagonal block.  This
// workgroup forms it (C - A A^T, the same MFMA sums as the regular tile), keeps it in LDS
// (packed lower triangle), factors it in registers (the fused TRSM kernel's POTRF,
// small_steps1_fast) and stores L11, so the next step's TRSM launch only loads L11
// (trsm_panel_g_kernel<2>): the 64-pivot POTRF leaves the chain's critical path and runs
// beside the update's other tiles.  Same arithmetic in the same order: bitwise identical.
template <int BK>
__device__ __forceinline__ void panel_prefactor(const GemmTask& T, int32_t* info, double* smem) {
    static_assert(2 * 2 * BK * (64 + 16) >= 64 * 65 / 2, "the packed diagonal block fits the operand LDS");
    double4_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    mfma_kloop<64, 2, 2, BK>(T.A, T.lda, T.K, T.M, T.N, 0, 0, acc, smem);  // ends with a barrier
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int64_t ldc = T.ldc;
    double* __restrict__ F = smem;  // column j at pk_col(64, j), rows j..63
    const __amdgpu_buffer_rsrc_t rc = buf_rsrc(T.C, (uint32_t)(64 * ldc * 8));
    double cv[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = wr * 32 + a * 16 + MFMA_F64_ROW(lane, r), gj = wc * 32 + b * 16 + (lane & 15);
                cv[a][b][r] = buf_ld(rc, gi >= gj ? (int)((gi + (int64_t)gj * ldc) * 8) : BUF_DEAD, 0);
            }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = wr * 32 + a * 16 + MFMA_F64_ROW(lane, r), gj = wc * 32 + b * 16 + (lane & 15);
                if (gi >= gj) F[pk_col(64, gj) + gi - gj] = cv[a][b][r] - acc[a][b][r];
            }
    __syncthreads();
    SmallRegs<1> R;
    small_tiles<1>(R, PNB, PNB);
    small_load<1>(R, F, PNB);
    __syncthreads();  // F is read: the column buffer overlays it
    small_steps1_fast(R, smem, PNB, info, T.pf);
    if (R.bi[0] < 0) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
            if (i >= j) T.C[(int64_t)j * ldc + i] = R.v[0][r * 4 + c];
        }
}

// LEAN (short-K launches on 64 x 64 tiles): BK = 8 and 32-row gather chunks halve the
// LDS (20 KB), so six workgroups fit a CU instead of four -- these launches are latency-
// bound (a few K stages, then the C traffic), not MFMA-bound
// PF: panel-update launch carrying pre-factor workgroups (panel_prefactor)
template <int BT, int WM, int WN, int TAG, int EPI, int LEAN = 0, int PF = 0>
__device__ __forceinline__ void syrk_tile_body(const GemmTask* __restrict__ tasks, const int2* __restrict__ tiles,
                                               int bidx, const int64_t* __restrict__ gblk,
                                               const GSeg* __restrict__ gseg, int32_t* info = nullptr) {
    constexpr int BK = LEAN ? 8 : 16;
    constexpr int LDT = BT + 16;
    constexpr int RTM = BT / WM / 16, RTN = BT / WN / 16;
    __shared__ __attribute__((aligned(16))) double smem[2 * 2 * BK * LDT];  // A and B stages

    // host-ordered tile list: blocks sharing an XCD walk a contiguous, L2-blocked run of tiles
    const int2 tl = tiles[bidx];
    const GemmTask T = tasks[tl.x];
    if constexpr (PF) {
        static_assert(BT == 64 && WM == 2 && WN == 2 && TAG == 0, "pre-factor on 64 x 64 panel-update tiles");
        if (tl.y < 0) {
            panel_prefactor<BK>(T, info, smem);
            return;
        }
    }
    const int ti = tl.y >> 16, tj = tl.y & 0xffff;
    const int row0 = ti * BT, col0 = tj * BT;

    const int wid = threadIdx.x >> 6;
    // static priority for the second-dispatched half of the waves (the arbitration loser
    // on every segment of two co-resident waves per SIMD): 547.8-548.5 -> 544.6-546.0 ms
    if (wid >= WM * WN / 2) __builtin_amdgcn_s_setprio(1);

    double4_t acc[RTM][RTN];
#pragma unroll
    for (int a = 0; a < RTM; ++a)
#pragma unroll
        for (int b = 0; b < RTN; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    // (operand stages by LDS-DMA, buffer_load_dwordx4 ... lds per 1-KB k-row, measured
    // slower: 510.5 ms with two 16-deep stages, 521.5 with four 8-deep, vs 505.7-507.3)
    if (!(SC_PROBE_NOK && TAG == 1 && T.gs >= 0)) mfma_kloop<BT, WM, WN, BK>(T.A, T.lda, T.K, T.M, T.N, row0, col0, acc, smem);

    if constexpr (TAG == 1) {
        if (T.gs >= 0) {  // the front's CB is not assembled: gather the children's entries
            syrk_gather_epilogue<BT, WM, WN, BK, LEAN ? 32 : 64>(T, gblk, gseg, row0, col0, acc, smem);
            return;
        }
    }
    syrk_rmw_epilogue<BT, WM, WN, BK, LEAN ? 32 : 64>(T, row0, col0, acc, smem);
}

template <int BT, int WM, int WN, int TAG, int EPI, int LEAN = 0, int PF = 0>
__global__ __launch_bounds__(64 * WM * WN, LEAN ? (TAG ? 5 : 6) : 1) void syrk_mfma_kernel(const GemmTask* __restrict__ tasks,
                                                                  const int2* __restrict__ tiles,
                                                                  const int64_t* __restrict__ gblk,
                                                                  const GSeg* __restrict__ gseg, int32_t* info) {
    syrk_tile_body<BT, WM, WN, TAG, EPI, LEAN, PF>(tasks, tiles, blockIdx.x, gblk, gseg, info);
}

// ---------------------------------------------------------------------------
// Launch wrappers
// ---------------------------------------------------------------------------
// KT: 4 x 4 register tiles per thread for fronts up to maxm (ceil(tiles / 256))
static int small_kt(int maxm) {
    const int T = (maxm + 3) / 4;
    return (T * (T + 1) / 2 + 255) / 256;
}

hipError_t launch_front_small(const DevPlan& P, const int32_t* nodes, int count, int maxm, bool seq,
                              const double* Ax, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    const size_t lds = (size_t)maxm * (maxm + 1) / 2 * sizeof(double);
    const int kt = small_kt(maxm);
    const dim3 grid(seq ? 1 : count);
    const int sq = seq ? count : 0;
    if (kt <= 1)
        hipLaunchKernelGGL(front_small_kernel<1>, grid, dim3(256), lds, st, P, nodes, Ax, sq);
    else if (kt == 2)
        hipLaunchKernelGGL(front_small_kernel<2>, grid, dim3(256), lds, st, P, nodes, Ax, sq);
    else
        hipLaunchKernelGGL(front_small_kernel<3>, grid, dim3(256), lds, st, P, nodes, Ax, sq);
    return hipGetLastError();
}

hipError_t launch_front_chain(const DevPlan& P, const ChainPlan& C, int first, int count, int maxm,
                              const double* Ax, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    if (count > CHAIN_MAXF || maxm > 128) return hipErrorInvalidValue;  // the host splits longer chains
    const int fsz = maxm * (maxm + 1) / 2;
    const size_t lds = (size_t)fsz * sizeof(double);
    hipLaunchKernelGGL(chain_init_kernel, dim3(count), dim3(256), lds, st, P, C, first, Ax);
    hipLaunchKernelGGL(front_chain_kernel, dim3(1), dim3(CHAIN_NT), (SC_CHAIN_DB ? 2 : 1) * lds, st, P, C, first, count,
                       fsz);
    return hipGetLastError();
}

hipError_t launch_assemble_large(const DevPlan& P, const int2* tasks, int count, const double* Ax,
                                 hipStream_t st, bool tiled, const int2* lim) {
    if (count <= 0) return hipSuccess;
    if (tiled)
        hipLaunchKernelGGL(assemble_tile_kernel, dim3(count), dim3(256), 0, st, P, tasks, Ax, lim);
    else
        hipLaunchKernelGGL(assemble_cols_kernel, dim3(count), dim3(256), 0, st, P, tasks, Ax);
    return hipGetLastError();
}

hipError_t launch_potrf_diag(const DevPlan& P, const int2* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(potrf_tiles_kernel, dim3(count), dim3(256), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_trsm_panel(const DevPlan& P, const TrsmTask* tasks, int count, hipStream_t st, bool partial,
                             int32_t* arrive, int pre) {
    if (count <= 0) return hipSuccess;
    if (partial)
        hipLaunchKernelGGL(trsm_partial_kernel, dim3(count), dim3(TRSM_ROWS), 0, st, P, tasks);
    else if (pre == 2)
        hipLaunchKernelGGL(trsm_panel_g_kernel<2>, dim3(count), dim3(TRSM_ROWS), 0, st, P, tasks, arrive);
    else
        hipLaunchKernelGGL(trsm_panel_g_kernel<0>, dim3(count), dim3(TRSM_ROWS), 0, st, P, tasks, arrive);
    return hipGetLastError();
}

// TAG and EPI only separate the launches in profiles: TAG 0 = panel update, 1 = CB update;
// EPI 1 = the main-stream (critical-path) panel updates and the short-K CB launches, 0 =
// the lookahead stream and the deep-K CB (round 6: every instance stages its epilogue
// through LDS; until then EPI chose a batched or a trickled C read-modify-write).
// bt = 64: 64x64 tiles on 4 waves (2x2); bt = 128: 128x128 tiles on 8 waves (2x4).
template <int TAG, int EPI>
static void launch_syrk_t(const GemmTask* tasks, const int2* tiles, int n, int bt, hipStream_t st, GatherTab gt,
                          bool lean) {
    if (bt == 64 && lean)
        hipLaunchKernelGGL((syrk_mfma_kernel<64, 2, 2, TAG, EPI, 1>), dim3(n), dim3(256), 0, st, tasks, tiles, gt.blk,
                           gt.seg, gt.info);
    else if (bt == 128)
        hipLaunchKernelGGL((syrk_mfma_kernel<128, 2, 4, TAG, EPI>), dim3(n), dim3(512), 0, st, tasks, tiles, gt.blk,
                           gt.seg, gt.info);
    else
        hipLaunchKernelGGL((syrk_mfma_kernel<64, 2, 2, TAG, EPI>), dim3(n), dim3(256), 0, st, tasks, tiles, gt.blk,
                           gt.seg, gt.info);
}

hipError_t launch_syrk(const GemmTask* tasks, const int2* tiles, int total_tiles, int bt, int tag, hipStream_t st,
                       int epi, GatherTab gt, bool lean, bool pf) {
    if (total_tiles <= 0) return hipSuccess;
    if (pf) {  // panel update with pre-factor workgroups: 64 x 64 tiles, batched epilogue
        if (bt != 64 || tag) return hipErrorInvalidValue;
        hipLaunchKernelGGL((syrk_mfma_kernel<64, 2, 2, 0, 1, 0, 1>), dim3(total_tiles), dim3(256), 0, st, tasks, tiles,
                           gt.blk, gt.seg, gt.info);
        return hipGetLastError();
    }
    if (tag)
        epi ? launch_syrk_t<1, 1>(tasks, tiles, total_tiles, bt, st, gt, lean)
            : launch_syrk_t<1, 0>(tasks, tiles, total_tiles, bt, st, gt, lean);
    else
        epi ? launch_syrk_t<0, 1>(tasks, tiles, total_tiles, bt, st, gt, lean)
            : launch_syrk_t<0, 0>(tasks, tiles, total_tiles, bt, st, gt, lean);
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

// Last launch of a single-rank factorization (main stream, which every other stream has
// joined): the status word to pinned host memory by a system-scope release store, and
// d_info re-armed for the next factorization.
__global__ void status_publish_kernel(int32_t* info, int32_t* host) {
    const int32_t v = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(info, 0x7f7f7f7f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(host, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_status_publish(int32_t* info, int32_t* host, hipStream_t st) {
    hipLaunchKernelGGL(status_publish_kernel, dim3(1), dim3(1), 0, st, info, host);
    return hipGetLastError();
}

// Hardware placement probe: per workgroup its HW_ID (wave/SIMD/CU/SH/SE fields) and XCC_ID.
__global__ void hwid_kernel(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
        out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_hwid(uint32_t* out, int nwg, int threads, int spin, hipStream_t st) {
    hipLaunchKernelGGL(hwid_kernel, dim3(nwg), dim3(threads), 0, st, out, spin);
    return hipGetLastError();
}

hipError_t launch_stamp(uint64_t* slot, hipStream_t st) {
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, st, slot);
    return hipGetLastError();
}

// Multi-GPU staging: strided <-> packed copy of contribution-block / panel column
// blocks around the RCCL transfers.  One workgroup per (COPY_COLS columns, COPY_ROWS
// rows) of one block, one wave per column; every lane keeps 8 loads in flight before
// its stores (HBM-bound; round 4's one-load-then-one-store loop over whole columns was
// latency-bound: 0.74 ms per launch, 35 ms of a dry 8-rank step at 128^3).
__global__ __launch_bounds__(256) void copy2d_kernel(const Copy2D* __restrict__ descs, const int2* __restrict__ tiles,
                                                     int unpack) {
    const int2 t = tiles[blockIdx.x];
    const Copy2D d = descs[t.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int j0 = t.y & 0xffff, r0 = (t.y >> 16) * COPY_ROWS;
    const int j1 = min(d.cols, j0 + COPY_COLS), r1 = min(d.rows, r0 + COPY_ROWS);
    for (int j = j0 + wid; j < j1; j += 4) {
        const double* __restrict__ src = unpack ? d.b + (int64_t)j * d.rows : d.a + (int64_t)j * d.lda;
        double* __restrict__ dst = unpack ? d.a + (int64_t)j * d.lda : d.b + (int64_t)j * d.rows;
        for (int r = r0 + lane; r < r1; r += 64 * 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = r + 64 * u < r1 ? src[r + 64 * u] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (r + 64 * u < r1) dst[r + 64 * u] = v[u];
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
// reference has no solve).  Level-scheduled like the factorization, one launch per
// 64-column step in each sweep.  Before the first solve of a factorization,
// solve_inv_kernel stores X = inv(L11) of every 64 x 64 diagonal block in the
// block's unused upper triangle (X(i, k), k < i, at panel row k, column i; the
// diagonal 1 / L(i, i) is recomputed), so no step runs a serial substitution:
//   forward  (solve_fwd_kernel): every workgroup of a block forms y = X c_blk (a
//            64 x 64 product) and applies its rows, c[rows[r]] -= L(r, blk) y;
//   backward (solve_gemv_kernel, then solve_diag_kernel): every workgroup adds its
//            rows' share -L(rows, blk)^T x(rows) into c_blk, then one workgroup per
//            block forms x_blk = X^T c_blk (a kernel boundary between them: a
//            device-scope fence per workgroup would write back the XCD's L2).
// HBM-bound in principle: L is read once per sweep.
// ---------------------------------------------------------------------------
// One wave per diagonal block (s, k0): lane j solves e_j L11^-T (the panel TRSM's
// row solve with the identity row), which is column j of X = inv(L11), and stores its
// strict lower part transposed into the strict upper triangle.
__global__ __launch_bounds__(64) void solve_inv_kernel(SolvePlan P, const int2* __restrict__ tasks) {
    __shared__ double2 S[TRSM64_STREAM / 2];
    __shared__ double Lc[PNB * (PNB + 2)];
    __shared__ double invd[PNB];
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int lane = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    double* blk = const_cast<double*>(P.panel_pool) + P.panel_off[s] + (int64_t)k0 * m + k0;
    double r[PNB];
    {  // row `lane` of the block, all loads in flight first (lane = row: coalesced per column)
#pragma unroll
        for (int j = 0; j < PNB; ++j) r[j] = (j < nb && lane < nb && lane >= j) ? blk[(int64_t)j * m + lane] : 0.0;
    }
    if (nb == PNB) {
        double* Sd = reinterpret_cast<double*>(S);
#pragma unroll
        for (int j = 0; j < PNB; ++j)  // the packed stream: 1 / L(j, j), then L(j+1..63, j)
            if (lane >= j) Sd[PNB * j - j * (j - 1) / 2 + (lane - j)] = lane == j ? 1.0 / r[j] : r[j];
    } else {
        constexpr int LD = PNB + 2;
#pragma unroll
        for (int j = 0; j < PNB; ++j) {
            Lc[j * LD + lane] = r[j];
            if (lane == j) invd[j] = j < nb ? 1.0 / r[j] : 0.0;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = c == lane ? 1.0 : 0.0;
    if (nb == PNB)
        trsm64_full(r, S);
    else
        trsm_steps<0>(r, Lc, invd, nb);
#pragma unroll
    for (int c = 0; c < PNB; ++c)
        if (lane < c && c < nb) blk[(int64_t)c * m + lane] = r[c];
}

// Off-diagonal quadrant of the 128-column block inverse: for the block at blk
// (columns k0 .. k0 + nb, 64 < nb <= 128), X128 = [Xa 0; E Xb] with Xa, Xb the 64-block
// inverses (solve_inv_kernel) and E = -Xb B Xa, B = L(k0+64 .., k0 .. k0+64).  E(i, k)
// goes to row k, column 64 + i of the block -- its unused upper triangle, like Xa and
// Xb -- so X128(i, k) sits at (row k, column i) for every k < i.  256 threads, once per
// factorization.
__global__ __launch_bounds__(256) void solve_inv2_kernel(SolvePlan P, const int2* __restrict__ tasks) {
    __shared__ double Xa[PNB][PNB + 1], Bm[PNB][PNB + 1], Xb[PNB][PNB + 1];
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nbb = min(SOLVE_NB, w - k0) - PNB;  // > 0
    double* blk = const_cast<double*>(P.panel_pool) + P.panel_off[s] + (int64_t)k0 * m + k0;
    const double* blkb = blk + (int64_t)PNB * m + PNB;
#pragma unroll
    for (int q = 0; q < PNB * PNB / 256; ++q) {
        const int e = tid + 256 * q, i = e >> 6, k = e & 63;  // lanes along k: coalesced in column i
        Xa[i][k] = k < i ? blk[(int64_t)i * m + k] : (k == i ? 1.0 / blk[(int64_t)i * m + i] : 0.0);
        Xb[i][k] = (i < nbb && k < i) ? blkb[(int64_t)i * m + k] : ((i < nbb && k == i) ? 1.0 / blkb[(int64_t)i * m + i] : 0.0);
        Bm[k][i] = k < nbb ? blk[(int64_t)i * m + PNB + k] : 0.0;  // B(k, i) = L(k0 + 64 + k, k0 + i)
    }
    __syncthreads();
    // thread: row i = tid >> 2, columns j = (tid & 3) + 4 q
    const int i = tid >> 2, jg = tid & 3;
    double acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0;
    for (int k = 0; k < PNB; ++k) {
        const double bik = Bm[i][k];
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = fma(bik, Xa[k][jg + 4 * q], acc[q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) Bm[i][jg + 4 * q] = acc[q];  // T = B Xa
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0;
    for (int k = 0; k <= i; ++k) {
        const double xik = Xb[i][k];
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = fma(xik, Bm[k][jg + 4 * q], acc[q]);
    }
    if (i < nbb) {
#pragma unroll
        for (int q = 0; q < 16; ++q) blk[(int64_t)(PNB + i) * m + jg + 4 * q] = -acc[q];
    }
}

// out[i] (+)= sum_k X128(64 I + i, 64 K + k) cb[64 K + k] for the block at blk (nb
// columns): the quadrant is staged through LDS with coalesced loads (X128(gi, gk) at
// row gk, column gi; the diagonal as 1 / L), then thread (row i = tid & 63, quarter
// g) sums 16 k.  256 threads.
__device__ __forceinline__ void quad_apply(const double* __restrict__ blk, int64_t m, int nb, int I, int K,
                                           const double* cb, double* out, bool add, double (*part)[PNB],
                                           double (*Xs)[PNB + 1]) {
    const int tid = threadIdx.x;
    // branch-free: dead elements read 0 through the buffer's range check, all loads in flight
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(blk, (uint32_t)(((int64_t)(nb - 1) * m + nb) * 8));
    double v[PNB * PNB / 256];
#pragma unroll
    for (int q = 0; q < PNB * PNB / 256; ++q) {
        const int e = tid + 256 * q, i = e >> 6, k = e & 63;  // lanes along k: coalesced in column gi
        const int gi = PNB * I + i, gk = PNB * K + k;
        v[q] = buf_ld(rs, (gi < nb && gk <= gi) ? (int)(((int64_t)gi * m + gk) * 8) : BUF_DEAD, 0);
    }
#pragma unroll
    for (int q = 0; q < PNB * PNB / 256; ++q) {
        const int e = tid + 256 * q, i = e >> 6, k = e & 63;
        Xs[i][k] = (PNB * I + i == PNB * K + k && PNB * I + i < nb) ? 1.0 / v[q] : v[q];  // dead: 0, not 1/0
    }
    __syncthreads();
    const int i = tid & 63, g = tid >> 6;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = fma(Xs[i][g * 16 + q], cb[PNB * K + g * 16 + q], acc);
    part[g][i] = acc;
    __syncthreads();
    if (tid < PNB) {
        const double v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
        out[tid] = add ? out[tid] + v : v;
    }
    __syncthreads();
}

// Forward step (128-column blocks): every workgroup of block (s, k0) forms y = X128
// c_blk (quadrants Xa, E, Xb) and applies its rows [r0, r0 + SOLVE_ROWS) below the
// block, c[rows[r]] -= L(r, blk) y; the writer (t.w = 1) stores y to P.y (not c, which
// the step's other workgroups still read).  r0 < 0: the diagonal block only.
__global__ __launch_bounds__(SOLVE_ROWS) void solve_fwd_kernel(SolvePlan P, const int4* __restrict__ tasks) {
    __shared__ double vb[SOLVE_NB], cb[SOLVE_NB];
    __shared__ double part[4][PNB];
    __shared__ double Xs[PNB][PNB + 1];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(SOLVE_NB, w - k0);
    const double* __restrict__ pan = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m;
    // this thread's row below the block: its first 64 loads go out first, overlapping y
    const int r = r0 + tid;
    const bool live = r0 >= 0 && r < m;
    // the block's columns; the whole offset in the VGPR so the range check masks dead
    // rows and columns past nb
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan, (uint32_t)((int64_t)nb * m * 8));
    double v[PNB];
#pragma unroll
    for (int q = 0; q < PNB; ++q) v[q] = buf_ld(rs, (live && q < nb) ? (q * m + r) * 8 : BUF_DEAD, 0);
    if (tid < SOLVE_NB) cb[tid] = tid < nb ? P.c[c0 + k0 + tid] : 0.0;
    __syncthreads();
    quad_apply(pan + k0, m, nb, 0, 0, cb, vb, false, part, Xs);
    if (nb > PNB) {
        quad_apply(pan + k0, m, nb, 1, 0, cb, vb + PNB, false, part, Xs);
        quad_apply(pan + k0, m, nb, 1, 1, cb, vb + PNB, true, part, Xs);
    }
    if (t.w && tid < nb) P.y[c0 + k0 + tid] = vb[tid];
    if (r0 < 0) return;
    const int32_t* __restrict__ rows = P.rows + P.rows_ptr[s];
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < PNB; ++q) acc = fma(v[q], vb[q], acc);
    if (nb > PNB) {
#pragma unroll
        for (int q = 0; q < PNB; ++q) v[q] = buf_ld(rs, (live && PNB + q < nb) ? ((PNB + q) * m + r) * 8 : BUF_DEAD, 0);
#pragma unroll
        for (int q = 0; q < PNB; ++q) acc = fma(v[q], vb[PNB + q], acc);
    }
    // rows < w: this front's own later pivots (no other front of the level has them);
    // rows >= w: its contribution block's entry of u, gathered by the parent in child order
    if (live) {
        if (r < w)
            P.c[rows[r]] -= acc;
        else
            P.u[P.u_off[s] + (r - w)] -= acc;
    }
}

// Forward gather (deterministic extend-add of the solve): front s = fronts[blockIdx.x]
// takes its children's u in child order; an entry mapping to one of s's pivot rows goes
// to c, the rest to u of s (zeroed by the sweep's memset).  Within a child relind is
// injective, so a barrier per child orders the adds.
__global__ __launch_bounds__(256) void solve_fwd_gather_kernel(SolvePlan P, const int32_t* __restrict__ fronts) {
    const int s = fronts[blockIdx.x];
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int32_t* __restrict__ rows = P.rows + P.rows_ptr[s];
    double* __restrict__ us = P.u + P.u_off[s];
    for (int q = P.child_ptr[s]; q < P.child_ptr[s + 1]; ++q) {
        const int ch = P.child_list[q];
        const int64_t r0 = P.rel_ptr[ch];
        const int mbc = (int)(P.rel_ptr[ch + 1] - r0);
        const double* __restrict__ uc = P.u + P.u_off[ch];
        const int32_t* __restrict__ rel = P.relind + r0;
        __syncthreads();  // the previous child's adds are done
        for (int i = tid; i < mbc; i += 256) {
            const int t = rel[i];
            const double v = uc[i];
            if (t < w)
                P.c[rows[t]] += v;
            else
                us[t - w] += v;
        }
    }
}

// Backward step, part 1: workgroup (s, k0, r0) adds -L(rows, blk)^T x(rows) into
// c_blk for rows [r0, r0 + SOLVE_ROWS) below the 128-column block (fp64 atomics), in
// two 64-column halves.  Thread t owns row r0 + t: it loads its 64 entries of the half
// (coalesced per column, all in flight), scales them by x of its row and leaves them
// in LDS; then thread (column j, quarter g) sums a quarter of column j.
__global__ __launch_bounds__(SOLVE_ROWS) void solve_gemv_kernel(SolvePlan P, const int4* __restrict__ tasks) {
    __shared__ double T[PNB][SOLVE_ROWS + 1];     // T[j][row] = L(row, j) x(row)
    __shared__ double part[SOLVE_ROWS / 64][PNB];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(SOLVE_NB, w - k0);
    const double* __restrict__ pan = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m;
    const int32_t* __restrict__ rows = P.rows + P.rows_ptr[s];
    const int r = r0 + tid;
    const bool live = r < m;
    const double xr = live ? P.c[rows[r]] : 0.0;
    // the block's columns; the whole offset in the VGPR (range check masks dead rows / columns)
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan, (uint32_t)((int64_t)nb * m * 8));
    for (int h = 0; h * PNB < nb; ++h) {
        if (h) __syncthreads();  // the previous half's T fully read
        double v[PNB];
#pragma unroll
        for (int q = 0; q < PNB; ++q) {
            const int col = h * PNB + q;
            v[q] = buf_ld(rs, (live && col < nb) ? (col * m + r) * 8 : BUF_DEAD, 0);
        }
#pragma unroll
        for (int q = 0; q < PNB; ++q) T[q][tid] = v[q] * xr;
        __syncthreads();
        const int j = tid & 63, g = tid >> 6;
        double acc = 0.0;
#pragma unroll 8
        for (int q = 0; q < SOLVE_ROWS / 4; ++q) acc += T[j][g * (SOLVE_ROWS / 4) + q];
        part[g][j] = acc;
        __syncthreads();
        if (tid < PNB)  // this workgroup's partial, summed by the diagonal kernel in task order
            P.part[(int64_t)blockIdx.x * SOLVE_NB + h * PNB + tid] =
                -(part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]);
    }
}

// Backward step, part 2: x_blk = X128^T c_blk for every block (s, k0) of the step:
// thread (column k = tid & 127, half g) sums X128(i, k) c_i over i in its half
// (X128(i, k) at row k, column i of the block: lanes along k read coalesced).
__global__ __launch_bounds__(256) void solve_diag_kernel(SolvePlan P, const int4* __restrict__ tasks) {
    __shared__ double cb[SOLVE_NB];
    __shared__ double part[2][SOLVE_NB];
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int tid = threadIdx.x, k = tid & (SOLVE_NB - 1), g = tid >> 7;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(SOLVE_NB, w - k0);
    const double* __restrict__ blk = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + k0;
    if (tid < SOLVE_NB) {
        double v = 0.0;
        if (tid < nb) {  // columns past nb: no partials written (dead entries must stay 0, not NaN)
            v = P.c[c0 + k0 + tid];
            for (int g2 = 0; g2 < t.w; ++g2) v += P.part[(int64_t)(t.z + g2) * SOLVE_NB + tid];  // GEMV partials, in order
        }
        cb[tid] = v;
    }
    __syncthreads();
    // branch-free: dead elements read 0 through the buffer's range check, all loads in flight
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(blk, (uint32_t)(((int64_t)(nb - 1) * m + nb) * 8));
    double xv[PNB];
#pragma unroll
    for (int q = 0; q < PNB; ++q) {
        const int i = g * PNB + q;
        xv[q] = buf_ld(rs, (i < nb && k <= i) ? (int)(((int64_t)i * m + k) * 8) : BUF_DEAD, 0);
    }
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < PNB; ++q) {
        const int i = g * PNB + q;
        acc = fma((k == i && i < nb) ? 1.0 / xv[q] : xv[q], cb[i], acc);  // dead: 0, not 1/0
    }
    part[g][k] = acc;
    __syncthreads();
    if (tid < nb) P.c[c0 + k0 + tid] = part[0][tid] + part[1][tid];
}

hipError_t launch_solve_fwd(const SolvePlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_fwd_kernel, dim3(count), dim3(SOLVE_ROWS), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_solve_gemv(const SolvePlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_gemv_kernel, dim3(count), dim3(SOLVE_ROWS), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_solve_fwd_gather(const SolvePlan& P, const int32_t* fronts, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_fwd_gather_kernel, dim3(count), dim3(256), 0, st, P, fronts);
    return hipGetLastError();
}

hipError_t launch_solve_diag(const SolvePlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(solve_diag_kernel, dim3(count), dim3(256), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_solve_inv(const SolvePlan& P, const int2* tasks, int count, const int2* tasks2, int count2,
                            hipStream_t st) {
    if (count > 0) hipLaunchKernelGGL(solve_inv_kernel, dim3(count), dim3(64), 0, st, P, tasks);
    if (count2 > 0) hipLaunchKernelGGL(solve_inv2_kernel, dim3(count2), dim3(256), 0, st, P, tasks2);
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

hipError_t launch_permute(double* dst, const double* src, const int32_t* perm, int64_t n, bool scatter,
                          hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(permute_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, src, perm, n,
                       scatter ? 1 : 0);
    return hipGetLastError();
}

}  // namespace sc
