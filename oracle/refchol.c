/*
 * oracle/refchol.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's simplicial path (evanwporter/SparseCholesky,
 * include/chol.hpp).  It is the parity CHECKER for the HIP numeric path and the
 * `cpu_baseline` leg of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load it; the product library never links it.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference cannot be built in this image
 * without stand-in headers (cblas.h, <expected>, Eigen, pcg), so the oracle is
 * pinned by the reference's own known answers (tests/test_chol.cpp:21,38,59-97,
 * README.md:6-37) and by reference outputs recorded by the survey (SURVEY.md
 * §8c checksums, Appendix B symbolic table), all committed under tests/golden/.
 *
 * Differences from the reference that do not change results:
 *   - 64-bit column pointers (reference: int, overflows past 2^31-1 nnz,
 *     chol.hpp:52,765);
 *   - rows are processed in natural order instead of etree depth levels
 *     (chol.hpp:789-796).  Every row's etree descendants are processed before
 *     it in both orders, and the per-row arithmetic (reach order, axpy order)
 *     is identical, so L is bit-identical.  Rows are appended in ascending
 *     order in both cases.
 *   - `faithful_workspace` keeps the reference's per-row O(n) allocation of
 *     s, w, x (chol.hpp:801-803) so the CPU baseline is timing-faithful; 0
 *     hoists it (O(n) once).
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define EXPORT __attribute__((visibility("default")))

/* etree with ancestor path compression -- chol.hpp:377-410 */
EXPORT void oracle_etree(int64_t n, const int64_t* Ap, const int32_t* Ai, int32_t* parent) {
    int32_t* ancestor = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t k = 0; k < n; k++) {
        parent[k] = -1;
        ancestor[k] = -1;
        for (int64_t p = Ap[k]; p < Ap[k + 1]; p++) {
            int32_t i = Ai[p];
            if (i > k) continue; /* upper triangle only */
            while (i != -1 && i < k) {
                int32_t inext = ancestor[i];
                ancestor[i] = (int32_t)k;
                if (inext == -1) {
                    parent[i] = (int32_t)k;
                    break;
                }
                i = inext;
            }
        }
    }
    free(ancestor);
}

/* iterative DFS -- chol.hpp:445-463 */
static int64_t tdfs(int32_t root, int64_t k, int32_t* head, const int32_t* next, int32_t* post,
                    int32_t* stack) {
    int64_t top = 0;
    stack[0] = root;
    while (top >= 0) {
        int32_t p = stack[top];
        int32_t child = head[p];
        if (child == -1) {
            top--;
            post[k++] = p;
        } else {
            head[p] = next[child];
            stack[++top] = child;
        }
    }
    return k;
}

/* postorder of the etree forest -- chol.hpp:466-499 */
EXPORT void oracle_post_order(int64_t n, const int32_t* parent, int32_t* post) {
    size_t sz = sizeof(int32_t) * (size_t)(n > 0 ? n : 1);
    int32_t* head = (int32_t*)malloc(sz);
    int32_t* next = (int32_t*)malloc(sz);
    int32_t* stack = (int32_t*)malloc(sz);
    for (int64_t j = 0; j < n; j++) {
        head[j] = -1;
        next[j] = -1;
        post[j] = -1;
    }
    for (int64_t j = n - 1; j >= 0; --j) {
        int32_t p = parent[j];
        if (p == -1) continue;
        next[j] = head[p];
        head[p] = (int32_t)j;
    }
    int64_t k = 0;
    for (int64_t j = 0; j < n; ++j) {
        if (parent[j] != -1) continue;
        k = tdfs((int32_t)j, k, head, next, post, stack);
    }
    free(head);
    free(next);
    free(stack);
}

/* column counts, cs_counts skeleton/LCA -- chol.hpp:506-622 */
EXPORT void oracle_col_count(int64_t n, const int64_t* Ap, const int32_t* Ai, const int32_t* parent,
                             const int32_t* post, int64_t* colcount) {
    size_t sz = sizeof(int32_t) * (size_t)(n > 0 ? n : 1);
    int64_t nnz = Ap[n];
    /* transpose_pattern (chol.hpp:507-535) */
    int64_t* ATp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int32_t* ATi = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t p = Ap[j]; p < Ap[j + 1]; ++p) ATp[Ai[p] + 1]++;
    for (int64_t j = 0; j < n; ++j) ATp[j + 1] += ATp[j];
    int64_t* nxt = (int64_t*)malloc(sizeof(int64_t) * ((size_t)n + 1));
    memcpy(nxt, ATp, sizeof(int64_t) * ((size_t)n + 1));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t p = Ap[j]; p < Ap[j + 1]; ++p) ATi[nxt[Ai[p]]++] = (int32_t)j;
    free(nxt);

    int32_t* first = (int32_t*)malloc(sz);
    int32_t* maxfirst = (int32_t*)malloc(sz);
    int32_t* prevleaf = (int32_t*)malloc(sz);
    int32_t* ancestor = (int32_t*)malloc(sz);
    int64_t* delta = (int64_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) {
        first[i] = -1;
        maxfirst[i] = -1;
        prevleaf[i] = -1;
        ancestor[i] = (int32_t)i;
    }
    for (int64_t k = 0; k < n; ++k) {
        int32_t j = post[k];
        delta[j] = (first[j] == -1) ? 1 : 0;
        for (; j != -1 && first[j] == -1; j = parent[j]) first[j] = (int32_t)k;
    }
    for (int64_t k = 0; k < n; ++k) {
        int32_t j = post[k];
        if (parent[j] != -1) delta[parent[j]]--;
        for (int64_t p = ATp[j]; p < ATp[j + 1]; ++p) {
            int32_t i = ATi[p];
            /* process_edge, chol.hpp:537-561 */
            if (i <= j || first[j] <= maxfirst[i]) continue;
            maxfirst[i] = first[j];
            int32_t jprev = prevleaf[i];
            delta[j]++;
            if (jprev != -1) {
                int32_t q = jprev;
                while (q != ancestor[q]) q = ancestor[q];
                for (int32_t s = jprev; s != q;) {
                    int32_t sp = ancestor[s];
                    ancestor[s] = q;
                    s = sp;
                }
                delta[q]--;
            }
            prevleaf[i] = j;
        }
        if (parent[j] != -1) ancestor[j] = parent[j];
    }
    for (int64_t j = 0; j < n; ++j) colcount[j] = delta[j];
    for (int64_t j = 0; j < n; ++j) {
        int32_t pj = parent[j];
        if (pj != -1) colcount[pj] += colcount[j];
    }
    free(ATp);
    free(ATi);
    free(first);
    free(maxfirst);
    free(prevleaf);
    free(ancestor);
    free(delta);
}

/*
 * ereach of row k -- chol.hpp:680-739 (ereach_impl).  s[top..n) receives the
 * reach in topological order; w is the mark array (caller pre-marks w[k]=k to
 * stop at k, as chol() does at chol.hpp:806; the gtest ColumnReach at
 * tests/test_chol.cpp:27-57 does not, and the reach then climbs to the root).
 * If x != NULL, A(:,k) is scattered into x.  The reference allocates a
 * std::vector path per nonzero (chol.hpp:701); `path` here is caller scratch.
 */
static int64_t ereach_impl(const int64_t* Ap, const int32_t* Ai, const double* Ax, int64_t k,
                           const int32_t* parent, int32_t* s, int32_t* w, double* x, int64_t top,
                           int32_t* path) {
    for (int64_t p = Ap[k]; p < Ap[k + 1]; ++p) {
        int32_t i = Ai[p];
        if (i > k) continue;
        if (x) x[i] = Ax[p];
        int64_t len = 0;
        while (i != -1 && w[i] != k) {
            path[len++] = i;
            w[i] = (int32_t)k;
            i = parent[i];
        }
        while (len > 0) s[--top] = path[--len];
    }
    return top;
}

EXPORT int64_t oracle_ereach(int64_t n, const int64_t* Ap, const int32_t* Ai, const double* Ax,
                             int64_t k, const int32_t* parent, int32_t* s, int32_t* w, double* x) {
    int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int64_t top = ereach_impl(Ap, Ai, Ax, k, parent, s, w, x, n, path);
    free(path);
    return top;
}

/* nnz(L) = sum of column counts (chol.hpp:762-771, int64 here) */
EXPORT int64_t oracle_symbolic(int64_t n, const int64_t* Ap, const int32_t* Ai, int32_t* parent,
                               int32_t* post, int64_t* colcount, int64_t* Lp, double* flops) {
    oracle_etree(n, Ap, Ai, parent);
    oracle_post_order(n, parent, post);
    oracle_col_count(n, Ap, Ai, parent, post, colcount);
    int64_t nz = 0;
    double f = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        if (Lp) Lp[j] = nz;
        nz += colcount[j];
        f += (double)colcount[j] * (double)colcount[j];
    }
    if (Lp) Lp[n] = nz;
    if (flops) *flops = f;
    return nz;
}

/*
 * Up-looking simplicial Cholesky -- chol.hpp:749-863.
 * Inputs: A upper CSC (entries with row > col are ignored, chol.hpp:696);
 * Lp from oracle_symbolic.  Outputs Li/Lx in the reference layout (diagonal
 * first, rows ascending).  Returns 0 on success, or k+1 for the first row k
 * (natural order) whose pivot d <= 0 ("A is not positive definite.",
 * chol.hpp:849-850).
 */
/* Rows finished by the running oracle_chol (every 4096 rows), for monitors of
 * long runs such as tests/golden/make_lap128_sketch.py.  Not part of the result. */
EXPORT volatile int64_t oracle_chol_rows_done = 0;

EXPORT int64_t oracle_chol(int64_t n, const int64_t* Ap, const int32_t* Ai, const double* Ax,
                           const int32_t* parent, const int64_t* Lp, int32_t* Li, double* Lx,
                           int faithful_workspace) {
    size_t sz = (size_t)(n > 0 ? n : 1);
    int64_t* c = (int64_t*)malloc(sizeof(int64_t) * sz);
    int32_t* path = (int32_t*)malloc(sizeof(int32_t) * sz);
    int32_t* s = NULL;
    int32_t* w = NULL;
    double* x = NULL;
    if (!faithful_workspace) {
        s = (int32_t*)malloc(sizeof(int32_t) * sz);
        w = (int32_t*)malloc(sizeof(int32_t) * sz);
        x = (double*)calloc(sz, sizeof(double));
        for (int64_t j = 0; j < n; ++j) w[j] = -1;
    }
    for (int64_t j = 0; j < n; ++j) c[j] = Lp[j];
    int64_t status = 0;
    for (int64_t k = 0; k < n; ++k) {
        if ((k & 4095) == 0) oracle_chol_rows_done = k;
        if (faithful_workspace) {
            /* chol.hpp:801-803: three length-n vectors per row */
            s = (int32_t*)malloc(sizeof(int32_t) * sz);
            w = (int32_t*)malloc(sizeof(int32_t) * sz);
            x = (double*)calloc(sz, sizeof(double));
            for (int64_t j = 0; j < n; ++j) {
                s[j] = -1;
                w[j] = -1;
            }
        }
        x[k] = 0.0;
        w[k] = (int32_t)k;
        int64_t top = ereach_impl(Ap, Ai, Ax, k, parent, s, w, x, n, path);
        double d = x[k];
        x[k] = 0.0;
        for (int64_t t = top; t < n; t++) {
            int32_t i = s[t];
            double Lii = Lx[Lp[i]];
            double lki = x[i] / Lii;
            x[i] = 0.0;
            for (int64_t p = Lp[i] + 1; p < c[i]; ++p) x[Li[p]] -= Lx[p] * lki;
            d -= lki * lki;
            int64_t q = c[i]++;
            Li[q] = (int32_t)k;
            Lx[q] = lki;
        }
        if (faithful_workspace) {
            free(s);
            free(w);
            free(x);
        }
        if (d <= 0.0) {
            status = k + 1;
            break;
        }
        int64_t q = c[k]++;
        Li[q] = (int32_t)k;
        Lx[q] = sqrt(d);
    }
    if (!faithful_workspace) {
        free(s);
        free(w);
        free(x);
    }
    oracle_chol_rows_done = n;
    free(c);
    free(path);
    return status;
}

/* Symbolic pattern of L, as schol() builds it -- chol.hpp:873-946 */
EXPORT void oracle_schol(int64_t n, const int64_t* Ap, const int32_t* Ai, const int32_t* parent,
                         const int64_t* Lp, int32_t* Li) {
    size_t sz = (size_t)(n > 0 ? n : 1);
    int64_t* c = (int64_t*)malloc(sizeof(int64_t) * sz);
    int32_t* s = (int32_t*)malloc(sizeof(int32_t) * sz);
    int32_t* w = (int32_t*)malloc(sizeof(int32_t) * sz);
    int32_t* path = (int32_t*)malloc(sizeof(int32_t) * sz);
    for (int64_t j = 0; j < n; ++j) {
        c[j] = Lp[j];
        w[j] = -1;
    }
    for (int64_t j = 0; j < n; ++j) {
        w[j] = (int32_t)j;
        int64_t top = ereach_impl(Ap, Ai, NULL, j, parent, s, w, NULL, n, path);
        for (int64_t t = top; t < n; ++t) Li[c[s[t]]++] = (int32_t)j;
        Li[c[j]++] = (int32_t)j;
    }
    free(c);
    free(s);
    free(w);
    free(path);
}

/*
 * Timing of the whole reference chol() call (chol.hpp:750-863: etree, post_order,
 * col_count, column pointers, L allocation, numeric rows) in C, best of `reps`,
 * so that small matrices are not timed through the ctypes wrapper.  Returns the
 * factorization status; *best_seconds = the fastest repetition.
 */
EXPORT int64_t oracle_time_chol(int64_t n, const int64_t* Ap, const int32_t* Ai, const double* Ax, int reps,
                                int faithful_workspace, double* best_seconds) {
    size_t sz = (size_t)(n > 0 ? n : 1);
    int64_t status = 0;
    double best = -1.0;
    for (int r = 0; r < reps; ++r) {
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        int32_t* parent = (int32_t*)malloc(sizeof(int32_t) * sz);
        int32_t* post = (int32_t*)malloc(sizeof(int32_t) * sz);
        int64_t* cc = (int64_t*)malloc(sizeof(int64_t) * sz);
        int64_t* Lp = (int64_t*)malloc(sizeof(int64_t) * (sz + 1));
        int64_t nz = oracle_symbolic(n, Ap, Ai, parent, post, cc, Lp, NULL);
        int32_t* Li = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nz > 0 ? nz : 1));
        double* Lx = (double*)malloc(sizeof(double) * (size_t)(nz > 0 ? nz : 1));
        status = oracle_chol(n, Ap, Ai, Ax, parent, Lp, Li, Lx, faithful_workspace);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        free(parent);
        free(post);
        free(cc);
        free(Lp);
        free(Li);
        free(Lx);
        const double dt = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        if (best < 0 || dt < best) best = dt;
    }
    if (best_seconds) *best_seconds = best;
    return status;
}
