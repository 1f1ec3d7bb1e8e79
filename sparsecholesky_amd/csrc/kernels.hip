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
// Small fronts: whole front in LDS, one 256-thread workgroup per front.
// Assemble A columns + children CBs (extend-add, children in a fixed order:
// deterministic, no atomics), right-looking partial Cholesky of the w pivots
// (the CB is updated in place = the SYRK), write L panel and CB.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void front_small_kernel(DevPlan P, const int32_t* __restrict__ nodes,
                                                           const double* __restrict__ Ax) {
    extern __shared__ double F[];
    __shared__ double s_piv;
    const int s = nodes[blockIdx.x];
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int mm = m * m;

    for (int idx = tid; idx < mm; idx += 256) F[idx] = 0.0;
    __syncthreads();
    // A entries of the pivot columns
    for (int lc = 0; lc < w; ++lc) {
        const int64_t a0 = P.a_ptr[c0 + lc], a1 = P.a_ptr[c0 + lc + 1];
        for (int64_t q = a0 + tid; q < a1; q += 256) F[lc * m + P.a_pos[q]] = Ax[P.a_src[q]];
    }
    __syncthreads();
    // extend-add of the children's contribution blocks
    for (int ci = P.child_ptr[s]; ci < P.child_ptr[s + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        const int32_t* rel = P.relind + P.rel_ptr[c];
        const double* cb = P.cb_pool + P.cb_off[c];
        const int tot = mbc * mbc;
        for (int idx = tid; idx < tot; idx += 256) {
            const int ic = idx % mbc, jc = idx / mbc;
            if (ic >= jc) F[rel[jc] * m + rel[ic]] += cb[idx];
        }
        __syncthreads();
    }
    // right-looking partial factorization
    const int G = (m <= 256) ? (256 / m) : 1;  // column groups
    const int i = tid % m;
    const int g = tid / m;
    for (int k = 0; k < w; ++k) {
        if (tid == 0) {
            double d = F[k * m + k];
            if (!(d > 0.0)) report_fail(P.info, c0 + k);
            s_piv = sqrt(d);
            F[k * m + k] = s_piv;
        }
        __syncthreads();
        const double dk = s_piv;
        for (int r = k + 1 + tid; r < m; r += 256) F[k * m + r] = F[k * m + r] / dk;
        __syncthreads();
        if (g < G && i > k) {
            const double lik = F[k * m + i];
            for (int j = k + 1 + g; j <= i; j += G) F[j * m + i] -= lik * F[k * m + j];
        }
        __syncthreads();
    }
    // write back the L panel (contiguous m*w) and the CB (lower)
    double* panel = P.panel_pool + P.panel_off[s];
    for (int idx = tid; idx < m * w; idx += 256) panel[idx] = F[idx];
    if (mb > 0) {
        double* cb = P.cb_pool + P.cb_off[s];
        const int tot = mb * mb;
        for (int idx = tid; idx < tot; idx += 256) {
            const int ic = idx % mb, jc = idx / mb;
            if (ic >= jc) cb[idx] = F[(jc + w) * m + (ic + w)];
        }
    }
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

__global__ __launch_bounds__(256) void assemble_large_kernel(DevPlan P, const int2* __restrict__ tasks,
                                                              const double* __restrict__ Ax) {
    const int2 t = tasks[blockIdx.x];
    const int s = t.x;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int mb = m - w;
    const int j0 = t.y * ASM_COLS;
    const int j1 = min(m, j0 + ASM_COLS);
    double* panel = P.panel_pool + P.panel_off[s];
    double* cbs = P.cb_pool + P.cb_off[s];
    // zero the lower part of the owned columns
    for (int j = j0; j < j1; ++j) {
        if (j < w) {
            for (int r = j + tid; r < m; r += 256) panel[(int64_t)j * m + r] = 0.0;
        } else {
            const int jj = j - w;
            for (int r = jj + tid; r < mb; r += 256) cbs[(int64_t)jj * mb + r] = 0.0;
        }
    }
    __syncthreads();
    for (int j = j0; j < min(j1, w); ++j) {
        const int64_t a0 = P.a_ptr[c0 + j], a1 = P.a_ptr[c0 + j + 1];
        for (int64_t q = a0 + tid; q < a1; q += 256) panel[(int64_t)j * m + P.a_pos[q]] = Ax[P.a_src[q]];
    }
    __syncthreads();
    for (int ci = P.child_ptr[s]; ci < P.child_ptr[s + 1]; ++ci) {
        const int c = P.child_list[ci];
        const int mbc = P.sn_m[c] - (P.sn_start[c + 1] - P.sn_start[c]);
        const int32_t* rel = P.relind + P.rel_ptr[c];
        const double* cb = P.cb_pool + P.cb_off[c];
        const int jlo = lower_bound_i32(rel, mbc, j0);
        const int jhi = lower_bound_i32(rel, mbc, j1);
        for (int jc = jlo; jc < jhi; ++jc) {
            const int pj = rel[jc];
            const double* src = cb + (int64_t)jc * mbc;
            if (pj < w) {
                double* dst = panel + (int64_t)pj * m;
                for (int ic = jc + tid; ic < mbc; ic += 256) dst[rel[ic]] += src[ic];
            } else {
                double* dst = cbs + (int64_t)(pj - w) * mb - w;
                for (int ic = jc + tid; ic < mbc; ic += 256) dst[rel[ic]] += src[ic];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Large fronts, diagonal block POTRF (nb <= 64): one workgroup per front.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void potrf_diag_kernel(DevPlan P, const int2* __restrict__ tasks) {
    __shared__ double D[PNB * (PNB + 1)];
    __shared__ double s_piv;
    const int2 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    constexpr int LD = PNB + 1;
    double* blk = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + k0;
    for (int idx = tid; idx < nb * nb; idx += 256) {
        const int r = idx % nb, c = idx / nb;
        D[c * LD + r] = (r >= c) ? blk[(int64_t)c * m + r] : 0.0;
    }
    __syncthreads();
    const int i = tid % PNB, g = tid / PNB;  // 4 column groups
    for (int k = 0; k < nb; ++k) {
        if (tid == 0) {
            double d = D[k * LD + k];
            if (!(d > 0.0)) report_fail(P.info, c0 + k0 + k);
            s_piv = sqrt(d);
            D[k * LD + k] = s_piv;
        }
        __syncthreads();
        const double dk = s_piv;
        if (tid > k && tid < nb) D[k * LD + tid] = D[k * LD + tid] / dk;
        __syncthreads();
        if (i > k && i < nb) {
            const double lik = D[k * LD + i];
            for (int j = k + 1 + g; j <= i; j += 4) D[j * LD + i] -= lik * D[k * LD + j];
        }
        __syncthreads();
    }
    for (int idx = tid; idx < nb * nb; idx += 256) {
        const int r = idx % nb, c = idx / nb;
        if (r >= c) blk[(int64_t)c * m + r] = D[c * LD + r];
    }
}

// ---------------------------------------------------------------------------
// Large fronts, panel TRSM: X := X * L11^{-T} for a 64-row block below the
// diagonal block.  tasks = (s, k0, r0): rows [r0, min(m, r0+64)).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void trsm_panel_kernel(DevPlan P, const int4* __restrict__ tasks) {
    constexpr int LD = PNB + 1;
    __shared__ double L[PNB * LD];
    __shared__ double X[PNB * LD];  // X[col * LD + row]
    const int4 t = tasks[blockIdx.x];
    const int s = t.x, k0 = t.y, r0 = t.z;
    const int tid = threadIdx.x;
    const int c0 = P.sn_start[s];
    const int w = P.sn_start[s + 1] - c0;
    const int m = P.sn_m[s];
    const int nb = min(PNB, w - k0);
    const int nr = min(TRSM_ROWS, m - r0);
    const double* pan = P.panel_pool + P.panel_off[s];
    const double* blk = pan + (int64_t)k0 * m + k0;
    for (int idx = tid; idx < nb * nb; idx += 256) {
        const int r = idx % nb, c = idx / nb;
        L[c * LD + r] = (r >= c) ? blk[(int64_t)c * m + r] : 0.0;
    }
    const double* xs = pan + (int64_t)k0 * m + r0;
    for (int idx = tid; idx < nb * TRSM_ROWS; idx += 256) {
        const int r = idx % TRSM_ROWS, c = idx / TRSM_ROWS;
        X[c * LD + r] = (r < nr) ? xs[(int64_t)c * m + r] : 0.0;
    }
    __syncthreads();
    const int r = tid % TRSM_ROWS, g = tid / TRSM_ROWS;
    for (int j = 0; j < nb; ++j) {
        if (g == 0) X[j * LD + r] = X[j * LD + r] / L[j * LD + j];
        __syncthreads();
        const double xj = X[j * LD + r];
        for (int jj = j + 1 + g; jj < nb; jj += 4) X[jj * LD + r] -= xj * L[j * LD + jj];
        __syncthreads();
    }
    double* xd = P.panel_pool + P.panel_off[s] + (int64_t)k0 * m + r0;
    for (int idx = tid; idx < nb * TRSM_ROWS; idx += 256) {
        const int rr = idx % TRSM_ROWS, c = idx / TRSM_ROWS;
        if (rr < nr) xd[(int64_t)c * m + rr] = X[c * LD + rr];
    }
}

// ---------------------------------------------------------------------------
// fp64 MFMA SYRK on a lower trapezoid: C[i,j] -= sum_k A[i,k] * A[j,k] for
// 0 <= j < N, j <= i < M.  Tiles BT x BT with ti >= tj; 256 threads = 4 waves
// (2 x 2), each wave (BT/2) x (BT/2) = RT x RT tiles of v_mfma_f64_16x16x4_f64.
// A (M x K) and the B operand (its first N rows) share one column-major array.
// ---------------------------------------------------------------------------
template <int BT, int TAG>
__global__ __launch_bounds__(256) void syrk_mfma_kernel(const GemmTask* __restrict__ tasks, int ntasks) {
    constexpr int BK = 16;
    constexpr int LDT = BT + 16;  // +128 B row pad: the two k-rows read by a half-wave hit disjoint banks
    constexpr int RT = BT / 32;   // 16x16 MFMA tiles per wave per dimension
    __shared__ double As[2][BK * LDT];
    __shared__ double Bs[2][BK * LDT];

    // locate the task (tasks sorted by tile_base)
    const int bid = blockIdx.x;
    int lo = 0, hi = ntasks - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (tasks[mid].tile_base <= bid)
            lo = mid;
        else
            hi = mid - 1;
    }
    const GemmTask T = tasks[lo];
    int idx = bid - T.tile_base;
    // lower-trapezoid enumeration, column-major over tile columns: column tj has (TM - tj) tiles
    const int TM = (T.M + BT - 1) / BT;
    int tj = 0;
    {
        // closed form then fix-up: S(tj) = tj*TM - tj*(tj-1)/2
        const double a = 2.0 * TM + 1.0;
        double disc = a * a - 8.0 * (double)idx;
        int guess = (int)floor((a - sqrt(disc > 0 ? disc : 0.0)) * 0.5);
        if (guess < 0) guess = 0;
        auto S = [&](int c) { return (int64_t)c * TM - (int64_t)c * (c - 1) / 2; };
        while (guess > 0 && S(guess) > idx) --guess;
        while (S(guess + 1) <= idx) ++guess;
        tj = guess;
        idx -= (int)S(tj);
    }
    const int ti = tj + idx;
    const int row0 = ti * BT, col0 = tj * BT;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const double* __restrict__ A = T.A;
    const int64_t lda = T.lda;

    double4_t acc[RT][RT];
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
        for (int b = 0; b < RT; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};

    // staging: BK x BT doubles per operand; 256 threads -> (BT*BK/256) each
    constexpr int PER = BT * BK / 256;
    double ra[PER], rb[PER];
    auto gload = [&](int k0) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + q * 256;
            const int r = e % BT, kk = e / BT;
            const int gk = k0 + kk;
            const int gr = row0 + r, gc = col0 + r;
            ra[q] = (gr < T.M && gk < T.K) ? A[gr + gk * lda] : 0.0;
            rb[q] = (gc < T.N && gk < T.K) ? A[gc + gk * lda] : 0.0;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + q * 256;
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
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            double av[RT], bv[RT];
            const int krow = kk + (lane >> 4);
#pragma unroll
            for (int a = 0; a < RT; ++a) av[a] = As[cur][krow * LDT + wr * (BT / 2) + a * 16 + (lane & 15)];
#pragma unroll
            for (int b = 0; b < RT; ++b) bv[b] = Bs[cur][krow * LDT + wc * (BT / 2) + b * 16 + (lane & 15)];
#pragma unroll
            for (int a = 0; a < RT; ++a)
#pragma unroll
                for (int b = 0; b < RT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

    // epilogue: f64 16x16x4 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
    double* __restrict__ C = T.C;
    const int64_t ldc = T.ldc;
#pragma unroll
    for (int a = 0; a < RT; ++a)
#pragma unroll
        for (int b = 0; b < RT; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = row0 + wr * (BT / 2) + a * 16 + MFMA_F64_ROW(lane, r);
                const int gj = col0 + wc * (BT / 2) + b * 16 + (lane & 15);
                if (gi < T.M && gj < T.N && gi >= gj) C[gi + gj * ldc] -= acc[a][b][r];
            }
}

// ---------------------------------------------------------------------------
// Launch wrappers
// ---------------------------------------------------------------------------
hipError_t launch_front_small(const DevPlan& P, const int32_t* nodes, int count, int maxm, const double* Ax,
                              hipStream_t st) {
    if (count <= 0) return hipSuccess;
    size_t lds = (size_t)maxm * maxm * sizeof(double);
    hipLaunchKernelGGL(front_small_kernel, dim3(count), dim3(256), lds, st, P, nodes, Ax);
    return hipGetLastError();
}

hipError_t launch_assemble_large(const DevPlan& P, const int2* tasks, int count, const double* Ax,
                                 hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(assemble_large_kernel, dim3(count), dim3(256), 0, st, P, tasks, Ax);
    return hipGetLastError();
}

hipError_t launch_potrf_diag(const DevPlan& P, const int2* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(potrf_diag_kernel, dim3(count), dim3(256), 0, st, P, tasks);
    return hipGetLastError();
}

hipError_t launch_trsm_panel(const DevPlan& P, const int4* tasks, int count, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(trsm_panel_kernel, dim3(count), dim3(256), 0, st, P, tasks);
    return hipGetLastError();
}

// TAG only separates the launches in profiles: 0 = panel update, 1 = CB update.
hipError_t launch_syrk(const GemmTask* tasks, int ntasks, int total_tiles, int bt, int tag, hipStream_t st) {
    if (total_tiles <= 0) return hipSuccess;
    if (bt == 128) {
        if (tag)
            hipLaunchKernelGGL((syrk_mfma_kernel<128, 1>), dim3(total_tiles), dim3(256), 0, st, tasks, ntasks);
        else
            hipLaunchKernelGGL((syrk_mfma_kernel<128, 0>), dim3(total_tiles), dim3(256), 0, st, tasks, ntasks);
    } else {
        if (tag)
            hipLaunchKernelGGL((syrk_mfma_kernel<64, 1>), dim3(total_tiles), dim3(256), 0, st, tasks, ntasks);
        else
            hipLaunchKernelGGL((syrk_mfma_kernel<64, 0>), dim3(total_tiles), dim3(256), 0, st, tasks, ntasks);
    }
    return hipGetLastError();
}

}  // namespace sc
