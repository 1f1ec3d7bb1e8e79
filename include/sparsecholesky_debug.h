/*
 * sparsecholesky_debug.h -- debug, probe and microbenchmark hooks of the library.
 *
 * Not part of the drop-in boundary (include/sparsecholesky.h): these entry points
 * have no counterpart in the reference.  They exist for the tests (the MFMA SYRK
 * kernel against numpy), for C-level timing of small configurations, and for the
 * measurement scripts under scripts/ (microbenchmarks, placement and contention
 * probes).  Same conventions as sparsecholesky.h.
 */
#ifndef SPARSECHOLESKY_DEBUG_H
#define SPARSECHOLESKY_DEBUG_H

#include "sparsecholesky.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* C[i,j] -= sum_k A[i,k] A[j,k] for i>=j over an M x N trapezoid (device
 * pointers, column-major) through the fp64 MFMA SYRK kernel. */
int64_t sc_debug_syrk(double* dC, int32_t ldc, const double* dA, int32_t lda, int32_t M, int32_t N,
                      int32_t K);
/* Best wall time (ms) of reps synchronous factorizations from device values
 * (sc_factor_device(num, d_Ax, 1): launch, run, status read-back), timed in C. */
int64_t sc_debug_time_factor(sc_numeric* num, const double* d_Ax, int32_t reps, double* best_ms);
/* Debug: eager = 1 launches the solve sweeps directly instead of replaying their graph. */
int64_t sc_debug_solve_eager(sc_numeric* num, int32_t eager);
/* Chain launches (runs of single small-front levels): enable = 1 makes the next
 * eager factorizations record 8 shader-clock stamps per chained front (phase
 * boundaries); enable = 0 copies up to cap of them to out.  Returns the count. */
int64_t sc_debug_chain_stamps(sc_numeric* num, int32_t enable, uint64_t* out, int64_t cap);
/* Microbenchmarks: which=0 register-only fp64 MFMA probe (TFLOP/s; M blocks of
 * 4 waves, K iterations, arg accumulators); which=1/5 the SYRK kernel on an M x M
 * triangle with depth K, tile arg (64/128), with / without the XCD tile order
 * (TFLOP/s); which=2/3 the panel POTRF / TRSM kernel on an M x 64 front
 * (microseconds per launch). */
int64_t sc_debug_bench(int32_t which, int32_t M, int32_t K, int32_t reps, int32_t arg, double* tflops);
/* Placement probe: nwg workgroups of `threads` threads, each spinning spin_ticks of the
 * 100 MHz clock; out[2 i] = HW_ID, out[2 i + 1] = XCC_ID of workgroup i. */
int64_t sc_debug_hwid(int32_t nwg, int32_t threads, int32_t spin_ticks, uint32_t* out);
/* Dispatch-contention probe: a panel-update SYRK "hog" (M x M triangle, K deep) on a
 * low-priority stream against a chain of nchain fused POTRF + TRSM launches (chain_rows
 * x 64 front) on the high-priority stream.  mode bit 0: hog stream CU-masked (every
 * mask_stride-th CU off), bit 1: hog replayed from a hipGraph, bit 2: chain from a
 * hipGraph.  out[8]: chain alone, hog alone, chain under hog, hog under chain, both
 * (ms), CUs available to the hog. */
int64_t sc_debug_contention(int32_t M, int32_t K, int32_t chain_rows, int32_t nchain, int32_t mode,
                            int32_t mask_stride, double* out);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif

#endif /* SPARSECHOLESKY_DEBUG_H */
