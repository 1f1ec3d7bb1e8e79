// extern "C" boundary (include/sparsecholesky.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/sparsecholesky.h"
#include "../../include/sparsecholesky_debug.h"
#include "numeric.hpp"
#include "symbolic.hpp"

namespace sc {
i64 triplet_to_csc(i64 n, i64 nt, const i32* ti, const i32* tj, const double* tx, i64* Ap, i32* Ai,
                   double* Ax);
i64 read_mtx(const char* path, i64* n_out, i64* Ap, i32* Ai, double* Ax);
i64 compute_supernodes_ref(i64 n, const i32* parent, const i64* cp, i32* sn_id, i64* supernodes);
i64 atree_ref(i64 n, const i64* Lp, const i32* Li, const i32* sn_id, const i64* supernodes, i64 ns,
              i32* super_parent);
i64 laplacian3d(i64 k, int nd, i64* Ap, i32* Ai, double* Ax, i32* perm_out);
i64 dist_owner_map(const Symbolic& S, int nranks, i32* owner, double* work);
i64 dist_schedule(const Symbolic& S, int nranks, int rank, i32* level, i32* peer, i64* bytes, i32* is_send,
                  i64 cap);
i64 numeric_create_dist(const Symbolic& S, int device, int rank, int nranks, const void* id128,
                        int32_t (*xport)(void*, int32_t, int32_t, void*, int64_t), void* xport_ctx, int emulate,
                        Numeric*& out, std::string& err);
i64 dist_unique_id(void* id128);
}  // namespace sc

struct sc_symbolic {
    sc::Symbolic S;
};
struct sc_numeric {
    sc::Numeric* N = nullptr;
    const sc_symbolic* sym = nullptr;
};

static thread_local std::string g_last_error;

extern "C" {

int32_t sc_version(void) { return SC_VERSION; }

const char* sc_status_string(int64_t st) {
    if (st > 0) return "A is not positive definite.";  // chol.hpp:850
    switch (st) {
        case SC_OK: return "ok";
        case SC_ERR_ARG: return "invalid argument";
        case SC_ERR_NOMEM: return "host allocation failed";
        case SC_ERR_HIP: return "HIP runtime error";
        case SC_ERR_DEVMEM: return "device allocation failed";
        case SC_ERR_STATE: return "call out of order";
        case SC_ERR_COMM: return "communication error";
        case SC_ERR_NOTIMPL: return "not implemented";
        case SC_ERR_NOTSYM: return "matrix is not symmetric";
        case SC_ERR_IO: return "file could not be opened";
    }
    return "unknown status";
}

const char* sc_last_error(void) { return g_last_error.c_str(); }

void sc_default_options(sc_options* opt) {
    if (!opt) return;
    std::memset(opt, 0, sizeof(*opt));
    opt->struct_size = (int32_t)sizeof(sc_options);
    opt->relax = 1;
    opt->nrelax[0] = 4;
    opt->nrelax[1] = 16;
    opt->nrelax[2] = 48;
    opt->zrelax[0] = 0.8;
    opt->zrelax[1] = 0.1;
    opt->zrelax[2] = 0.05;
    opt->small_front_max = 128;
    opt->panel_nb = 64;
    opt->panel_nb_outer = 1024;
    opt->use_graph = 0;
    opt->relax_wmax = 1;
    opt->syrk_tile = 0;
    opt->lookahead = 1;
    opt->inner_order = 1;
    opt->asm_tile_min_m = 0;
    opt->dist_split = 1;
    opt->dist_cbb = 1024;
    opt->dist_early = 1;
    opt->dist_panel = 1;
    opt->cb_gather = 1;
    opt->dist_slab_block = 2;
    opt->trsm_split_wg = 1024;
    opt->syrk_lean_kmax = 128;
    opt->cb_tail_split = 1;
    opt->tiny_dense = 1;
    opt->dist_asm = 1;
    opt->dist_pieces = 4;
    opt->dist_local_pieces = 1;
    opt->panel_prefactor = 1;
}

int64_t sc_analyze(int64_t n, const int64_t* Ap, const int32_t* Ai, const sc_options* opt,
                   sc_symbolic** out) {
    if (!out) return SC_ERR_ARG;
    *out = nullptr;
    sc_options o;
    if (opt) {
        if (opt->struct_size != (int32_t)sizeof(sc_options)) {
            g_last_error = "sc_options.struct_size does not match this library's sizeof(sc_options): "
                           "initialise the options with sc_default_options() from the matching header";
            return SC_ERR_ARG;
        }
        o = *opt;
    } else {
        sc_default_options(&o);
    }
    if (o.small_front_max > 128) o.small_front_max = 128;
    if (o.small_front_max < 0) o.small_front_max = 0;
    if (o.lookahead != 0 && o.lookahead != 1) {
        g_last_error = "sc_options.lookahead must be 0 or 1";
        return SC_ERR_ARG;
    }
    if (o.inner_order != 0 && o.inner_order != 1) {
        g_last_error = "sc_options.inner_order must be 0 or 1";
        return SC_ERR_ARG;
    }
    sc_symbolic* h = new (std::nothrow) sc_symbolic();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc;
    try {
        if (o.ordering != SC_ORDER_NATURAL && o.ordering != SC_ORDER_ND && o.ordering != SC_ORDER_AMD) {
            rc = SC_ERR_ARG;
            err = "sc_options.ordering must be SC_ORDER_NATURAL, SC_ORDER_ND or SC_ORDER_AMD";
        } else if (o.ordering != SC_ORDER_NATURAL && n > 0 && Ap && (Ai || Ap[n] == 0)) {
            // factor B = P A P^T; numeric values still come from A's arrays (a_src remapped)
            std::vector<int32_t> perm((size_t)n);
            std::vector<int64_t> Bp, src;
            std::vector<int32_t> Bi;
            // the CSC checks analyze() makes, before the ordering walks the arrays
            rc = Ap[0] == 0 ? SC_OK : SC_ERR_ARG;
            for (int64_t j = 0; rc == SC_OK && j < n; ++j)
                if (Ap[j + 1] < Ap[j]) rc = SC_ERR_ARG;
            for (int64_t p = 0; rc == SC_OK && p < Ap[n]; ++p)
                if (Ai[p] < 0 || Ai[p] >= n) rc = SC_ERR_ARG;
            if (rc != SC_OK) err = "malformed CSC";
            if (rc == SC_OK) {
                rc = o.ordering == SC_ORDER_AMD ? sc::amd_order(n, Ap, Ai, perm.data())
                                                : sc::nd_order(n, Ap, Ai, perm.data());
                if (rc != SC_OK) err = "ordering failed";
            }
            if (rc == SC_OK) {
                sc::permute_upper(n, Ap, Ai, perm.data(), Bp, Bi, src);
                rc = sc::analyze(n, Bp.data(), Bi.data(), o, h->S, err);
            }
            if (rc == SC_OK) {
                auto& S = h->S;
                for (int64_t q = 0; q < S.nnzA_used; ++q) S.a_src[q] = src[S.a_src[q]];
                S.nnzA_in = Ap[n];
                S.perm = std::move(perm);
            }
        } else {
            rc = sc::analyze(n, Ap, Ai, o, h->S, err);
        }
    } catch (const std::bad_alloc&) {
        rc = SC_ERR_NOMEM;
        err = "out of host memory";
    }
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    *out = h;
    return SC_OK;
}

int64_t sc_symbolic_get_stats(const sc_symbolic* sym, sc_symbolic_stats* st) {
    if (!sym || !st) return SC_ERR_ARG;
    *st = sym->S.stats;
    return SC_OK;
}

int64_t sc_nnz_L(const sc_symbolic* sym) { return sym ? sym->S.nnzL : SC_ERR_ARG; }
double sc_flops(const sc_symbolic* sym) { return sym ? sym->S.flops : -1.0; }

int64_t sc_symbolic_pattern(const sc_symbolic* sym, int64_t* Lp, int32_t* Li) {
    if (!sym || !Lp) return SC_ERR_ARG;
    sc::pattern_L(sym->S, Lp, Li);
    return SC_OK;
}

int64_t sc_symbolic_etree(const sc_symbolic* sym, int32_t* parent, int32_t* post) {
    if (!sym) return SC_ERR_ARG;
    const auto& S = sym->S;
    if (parent) std::memcpy(parent, S.parent.data(), sizeof(int32_t) * (size_t)S.n);
    if (post) std::memcpy(post, S.post.data(), sizeof(int32_t) * (size_t)S.n);
    return SC_OK;
}

int64_t sc_symbolic_supernodes(const sc_symbolic* sym, int32_t* sn_start, int32_t* sn_m, int32_t* sn_parent,
                               int32_t* level) {
    if (!sym) return SC_ERR_ARG;
    const auto& S = sym->S;
    const size_t ns = (size_t)S.ns;
    if (sn_start) std::memcpy(sn_start, S.sn_start.data(), sizeof(int32_t) * (ns + 1));
    if (sn_m && ns) std::memcpy(sn_m, S.sn_m.data(), sizeof(int32_t) * ns);
    if (sn_parent && ns) std::memcpy(sn_parent, S.sn_parent.data(), sizeof(int32_t) * ns);
    if (level && ns) std::memcpy(level, S.level.data(), sizeof(int32_t) * ns);
    return S.ns;
}

int64_t sc_symbolic_perm(const sc_symbolic* sym, int32_t* perm) {
    if (!sym) return SC_ERR_ARG;
    const auto& S = sym->S;
    if (perm) {
        if (S.perm.empty())
            for (int64_t i = 0; i < S.n; ++i) perm[i] = (int32_t)i;
        else
            std::memcpy(perm, S.perm.data(), sizeof(int32_t) * (size_t)S.n);
    }
    return S.perm.empty() ? 0 : 1;
}

void sc_free_symbolic(sc_symbolic* sym) { delete sym; }

int64_t sc_numeric_create(const sc_symbolic* sym, int32_t device, sc_numeric** out) {
    if (!sym || !out) return SC_ERR_ARG;
    *out = nullptr;
    sc_numeric* h = new (std::nothrow) sc_numeric();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc = sc::numeric_create(sym->S, device, h->N, err);
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    h->sym = sym;
    *out = h;
    return SC_OK;
}

int64_t sc_factor_device(sc_numeric* num, const double* d_Ax, int32_t sync) {
    if (!num || !num->N || (!d_Ax && num->sym->S.nnzA_in > 0)) return SC_ERR_ARG;
    int64_t rc = sc::numeric_factor(*num->N, d_Ax, sync != 0);
    if (rc < 0) g_last_error = num->N->err;
    return rc;
}

int64_t sc_debug_time_factor(sc_numeric* num, const double* d_Ax, int32_t reps, double* best_ms) {
    if (!num || !num->N || reps < 1 || !best_ms) return SC_ERR_ARG;
    double best = 1e30;
    for (int r = 0; r <= reps; ++r) {  // the first call captures / warms up
        const auto t0 = std::chrono::steady_clock::now();
        const int64_t rc = sc::numeric_factor(*num->N, d_Ax, true);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc < 0) {
            g_last_error = num->N->err;
            return rc;
        }
        if (r > 0) best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    *best_ms = best;
    return SC_OK;
}

int64_t sc_debug_solve_eager(sc_numeric* num, int32_t eager) {
    if (!num || !num->N) return SC_ERR_ARG;
    num->N->solve_eager = eager != 0;
    return SC_OK;
}

int64_t sc_factor(sc_numeric* num, const double* Ax) {
    if (!num || !num->N) return SC_ERR_ARG;
    sc::Numeric& N = *num->N;
    const int64_t nnz = num->sym->S.nnzA_in;
    if (nnz > 0 && !Ax) return SC_ERR_ARG;
    if (hipSetDevice(N.device) != hipSuccess) return SC_ERR_HIP;
    if (!N.d_Ax_owned) {
        if (hipMalloc(&N.d_Ax_owned, (size_t)std::max<int64_t>(nnz, 1) * sizeof(double)) != hipSuccess) {
            N.d_Ax_owned = nullptr;
            return SC_ERR_DEVMEM;
        }
    }
    if (nnz > 0 && hipMemcpyAsync(N.d_Ax_owned, Ax, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice,
                                  N.stream) != hipSuccess)
        return SC_ERR_HIP;
    return sc_factor_device(num, N.d_Ax_owned, 1);
}

int64_t sc_numeric_status(sc_numeric* num) {
    if (!num || !num->N) return SC_ERR_ARG;
    return sc::numeric_status(*num->N);
}

int64_t sc_export_L(sc_numeric* num, int64_t* Lp, int32_t* Li, double* Lx) {
    if (!num || !num->N) return SC_ERR_ARG;
    try {
        return sc::numeric_export(*num->N, Lp, Li, Lx);
    } catch (const std::bad_alloc&) {
        return SC_ERR_NOMEM;
    }
}

int64_t sc_export_L_cols(sc_numeric* num, int64_t j0, int64_t j1, int64_t* cp, int32_t* ri, double* rx) {
    if (!num || !num->N || !cp) return SC_ERR_ARG;
    try {
        const int64_t rc = sc::numeric_export_cols(*num->N, j0, j1, cp, ri, rx);
        if (rc < 0) g_last_error = num->N->err;
        return rc;
    } catch (const std::bad_alloc&) {
        return SC_ERR_NOMEM;
    }
}

void* sc_numeric_stream(sc_numeric* num) { return (num && num->N) ? (void*)num->N->stream : nullptr; }

int64_t sc_numeric_set_profile(sc_numeric* num, int32_t on) {
    if (!num || !num->N) return SC_ERR_ARG;
    num->N->profile = (on == 1 || on == 2) ? on : 0;
    return SC_OK;
}

int64_t sc_numeric_timing(sc_numeric* num, double* t, int32_t nt) {
    if (!num || !num->N || !t) return SC_ERR_ARG;
    return sc::numeric_timing(*num->N, t, nt);
}

int64_t sc_numeric_level_times(sc_numeric* num, double* ms, int32_t nl) {
    if (!num || !num->N || !ms) return SC_ERR_ARG;
    return sc::numeric_level_times(*num->N, ms, nl);
}

int64_t sc_numeric_launch_trace(sc_numeric* num, int32_t* kind, int32_t* level, int32_t* strm, double* ms,
                                double* flops, int64_t cap) {
    if (!num || !num->N) return SC_ERR_ARG;
    return sc::numeric_launch_trace(*num->N, kind, level, strm, ms, flops, cap);
}

int64_t sc_numeric_syrk_stats(sc_numeric* num, int32_t wmin, double* flops, double* ms, int64_t* launches) {
    if (!num || !num->N) return SC_ERR_ARG;
    return sc::numeric_syrk_stats(*num->N, wmin, flops, ms, launches);
}

int64_t sc_numeric_launch_times(sc_numeric* num, double* t0, double* t1, int32_t* kind, int32_t* step,
                                int32_t* stream, int64_t cap) {
    if (!num || !num->N) return SC_ERR_ARG;
    if (t0 && (!t1 || !kind || !step || !stream)) return SC_ERR_ARG;
    return sc::numeric_launch_times(*num->N, t0, t1, kind, step, stream, cap);
}

int64_t sc_numeric_syrk_bytes(sc_numeric* num, int32_t wmin, double* bytes) {
    if (!num || !num->N || !bytes) return SC_ERR_ARG;
    return sc::numeric_syrk_bytes(*num->N, wmin, bytes);
}

int64_t sc_debug_chain_stamps(sc_numeric* num, int32_t enable, uint64_t* out, int64_t cap) {
    if (!num || !num->N) return SC_ERR_ARG;
    return sc::numeric_chain_stamps(*num->N, enable, out, cap);
}

void sc_free_numeric(sc_numeric* num) {
    if (!num) return;
    sc::numeric_free(num->N);
    delete num;
}

int64_t sc_solve_host(sc_numeric* num, const double* b, double* x) {
    if (!num || !num->N || !b || !x) return SC_ERR_ARG;
    int64_t rc = sc::numeric_solve_host(*num->N, b, x);
    if (rc < 0) g_last_error = num->N->err;
    return rc;
}

int64_t sc_solve_device(sc_numeric* num, const double* d_b, double* d_x) {
    if (!num || !num->N || !d_b || !d_x) return SC_ERR_ARG;
    int64_t rc = sc::numeric_solve_device(*num->N, d_b, d_x);
    if (rc < 0) g_last_error = num->N->err;
    return rc;
}

// ---- reference-API helpers ----
int64_t sc_etree(int64_t n, const int64_t* Ap, const int32_t* Ai, int32_t* parent) {
    if (n < 0 || !Ap || !parent) return SC_ERR_ARG;
    sc::etree(n, Ap, Ai, parent);
    return SC_OK;
}

int64_t sc_post_order(int64_t n, const int32_t* parent, int32_t* post) {
    if (n < 0 || !parent || !post) return SC_ERR_ARG;
    sc::post_order(n, parent, post);
    return SC_OK;
}

int64_t sc_col_count(int64_t n, const int64_t* Ap, const int32_t* Ai, const int32_t* parent,
                     const int32_t* post, int64_t* colcount) {
    if (n < 0 || !Ap || !parent || !post || !colcount) return SC_ERR_ARG;
    sc::col_count(n, Ap, Ai, parent, post, colcount);
    return SC_OK;
}

int64_t sc_ereach(int64_t n, const int64_t* Ap, const int32_t* Ai, const double* Ax, int64_t k,
                  const int32_t* parent, int32_t* s, int32_t* w, double* x) {
    if (n < 0 || k < 0 || k >= n || !Ap || !parent || !s || !w) return SC_ERR_ARG;
    std::vector<int32_t> path((size_t)n);
    return sc::ereach(n, Ap, Ai, Ax, k, parent, s, w, x, path);
}

int64_t sc_compute_levels(int64_t n, const int32_t* parent, int32_t* level_of) {
    if (n < 0 || !parent) return SC_ERR_ARG;
    return sc::compute_levels(n, parent, level_of);
}

int64_t sc_compute_supernodes(int64_t n, const int32_t* parent, const int64_t* Lp, int32_t* sn_id,
                              int64_t* supernodes) {
    if (n < 0 || !parent || !Lp) return SC_ERR_ARG;
    return sc::compute_supernodes_ref(n, parent, Lp, sn_id, supernodes);
}

int64_t sc_atree(int64_t n, const int64_t* Lp, const int32_t* Li, const int32_t* sn_id,
                 const int64_t* supernodes, int64_t ns, int32_t* super_parent) {
    if (n < 0 || !Lp || !Li || !sn_id || !supernodes || !super_parent) return SC_ERR_ARG;
    return sc::atree_ref(n, Lp, Li, sn_id, supernodes, ns, super_parent);
}

int64_t sc_triplet_to_csc(int64_t n, int64_t nt, const int32_t* ti, const int32_t* tj, const double* tx,
                          int64_t* Ap, int32_t* Ai, double* Ax) {
    if (n < 0 || nt < 0 || (nt > 0 && (!ti || !tj))) return SC_ERR_ARG;
    return sc::triplet_to_csc(n, nt, ti, tj, tx, Ap, Ai, Ax);
}

int64_t sc_read_mtx(const char* path, int64_t* n, int64_t* Ap, int32_t* Ai, double* Ax) {
    if (!path || !n) return SC_ERR_ARG;
    return sc::read_mtx(path, n, Ap, Ai, Ax);
}

int64_t sc_laplacian3d(int64_t k, int32_t nd_order, int64_t* Ap, int32_t* Ai, double* Ax, int32_t* perm) {
    return sc::laplacian3d(k, nd_order, Ap, Ai, Ax, perm);
}

// ---- multi-GPU ----
int64_t sc_dist_unique_id(void* id128) { return sc::dist_unique_id(id128); }

int64_t sc_dist_owner_map(const sc_symbolic* sym, int32_t nranks, int32_t* owner, double* work) {
    if (!sym || nranks <= 0) return SC_ERR_ARG;
    return sc::dist_owner_map(sym->S, nranks, owner, work);
}

int64_t sc_dist_schedule(const sc_symbolic* sym, int32_t nranks, int32_t rank, int32_t* level, int32_t* peer,
                         int64_t* bytes, int32_t* is_send, int64_t cap) {
    if (!sym || nranks <= 0 || rank < 0 || rank >= nranks) return SC_ERR_ARG;
    return sc::dist_schedule(sym->S, nranks, rank, level, peer, bytes, is_send, cap);
}

int64_t sc_numeric_create_dist(const sc_symbolic* sym, int32_t device, int32_t rank, int32_t nranks,
                               const void* id128, sc_numeric** out) {
    if (!sym || !out || nranks <= 0 || rank < 0 || rank >= nranks) return SC_ERR_ARG;
    *out = nullptr;
    sc_numeric* h = new (std::nothrow) sc_numeric();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc = sc::numeric_create_dist(sym->S, device, rank, nranks, id128, nullptr, nullptr, id128 ? 0 : 1, h->N,
                                         err);
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    h->sym = sym;
    *out = h;
    return SC_OK;
}

int64_t sc_numeric_create_dist_host(const sc_symbolic* sym, int32_t device, int32_t rank, int32_t nranks,
                                    sc_transport_fn fn, void* ctx, sc_numeric** out) {
    if (!sym || !out || !fn || nranks <= 0 || rank < 0 || rank >= nranks) return SC_ERR_ARG;
    *out = nullptr;
    sc_numeric* h = new (std::nothrow) sc_numeric();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc = sc::numeric_create_dist(sym->S, device, rank, nranks, nullptr, fn, ctx, 0, h->N, err);
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    h->sym = sym;
    *out = h;
    return SC_OK;
}

int64_t sc_numeric_create_dist_dry(const sc_symbolic* sym, int32_t device, int32_t rank, int32_t nranks,
                                   sc_numeric** out) {
    if (!sym || !out || nranks <= 0 || rank < 0 || rank >= nranks) return SC_ERR_ARG;
    *out = nullptr;
    sc_numeric* h = new (std::nothrow) sc_numeric();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc = sc::numeric_create_dist(sym->S, device, rank, nranks, nullptr, DIST_DRY, nullptr, 0, h->N, err);
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    h->sym = sym;
    *out = h;
    return SC_OK;
}

int64_t sc_numeric_create_dist_emulated(const sc_symbolic* sym, int32_t device, int32_t nranks, int32_t use_rccl,
                                        sc_numeric** out) {
    if (!sym || !out || nranks <= 0) return SC_ERR_ARG;
    *out = nullptr;
    sc_numeric* h = new (std::nothrow) sc_numeric();
    if (!h) return SC_ERR_NOMEM;
    std::string err;
    int64_t rc = sc::numeric_create_dist(sym->S, device, 0, nranks, nullptr, nullptr, nullptr, use_rccl ? 2 : 1, h->N,
                                         err);
    if (rc != SC_OK) {
        g_last_error = err;
        delete h;
        return rc;
    }
    h->sym = sym;
    *out = h;
    return SC_OK;
}

int64_t sc_memory_plan(const sc_symbolic* sym, int32_t nranks, int64_t* panel_bytes, int64_t* work_bytes,
                       int64_t* work_lower_bound_bytes) {
    if (!sym || nranks <= 0) return SC_ERR_ARG;
    std::vector<int64_t> p((size_t)nranks), w((size_t)nranks), l((size_t)nranks);
    const int64_t rc = sc::plan_memory_stats(sym->S, nranks, p.data(), w.data(), l.data());
    if (rc != SC_OK) return rc;
    for (int32_t r = 0; r < nranks; ++r) {
        if (panel_bytes) panel_bytes[r] = p[r] * (int64_t)sizeof(double);
        if (work_bytes) work_bytes[r] = w[r] * (int64_t)sizeof(double);
        if (work_lower_bound_bytes) work_lower_bound_bytes[r] = l[r] * (int64_t)sizeof(double);
    }
    return SC_OK;
}

int64_t sc_memory_plan_check(const sc_symbolic* sym, int32_t nranks) {
    if (!sym || nranks <= 0) return SC_ERR_ARG;
    return sc::plan_check(sym->S, nranks);
}

int64_t sc_numeric_memory(sc_numeric* num, int64_t* info, int32_t n) {
    if (!num || !num->N || !info) return SC_ERR_ARG;
    const sc::Numeric& N = *num->N;
    int64_t v[4] = {N.dev_bytes, 0, 0, 0};
    for (const sc::RankMem& R : N.R) {
        v[1] += R.panel_total * (int64_t)sizeof(double);
        v[2] += R.work_total * (int64_t)sizeof(double);
        v[3] += R.work_live_max * (int64_t)sizeof(double);
    }
    for (int32_t i = 0; i < n && i < 4; ++i) info[i] = v[i];
    return SC_OK;
}

int64_t sc_dist_steps(const sc_symbolic* sym, int32_t nranks, int32_t* kind, int32_t* level, int32_t* front,
                      int32_t* k, int32_t* p, int64_t cap) {
    if (!sym || nranks <= 0) return SC_ERR_ARG;
    sc::DistPlan D;
    int64_t rc = sc::dist_plan(sym->S, nranks, D);
    if (rc != SC_OK) return rc;
    for (size_t i = 0; i < D.steps.size() && (int64_t)i < cap; ++i) {
        if (kind) kind[i] = D.steps[i].kind;
        if (level) level[i] = D.steps[i].level;
        if (front) front[i] = D.steps[i].s;
        if (k) k[i] = D.steps[i].k;
        if (p) p[i] = D.steps[i].p;
    }
    return (int64_t)D.steps.size();
}

int64_t sc_dist_plan_info(const sc_symbolic* sym, int32_t nranks, int32_t* gsize, int32_t* split_cb_ranks,
                          int32_t* slab_ranks, int64_t* n_steps) {
    if (!sym || nranks <= 0) return SC_ERR_ARG;
    sc::DistPlan D;
    int64_t rc = sc::dist_plan(sym->S, nranks, D);
    if (rc != SC_OK) return rc;
    for (int32_t s = 0; s < sym->S.ns; ++s) {
        if (gsize) gsize[s] = D.gsize[s];
        if (split_cb_ranks) {
            int32_t v = 0;
            if (D.split[s] >= 0) {
                std::vector<int32_t> r = D.cb_rank[D.split[s]];
                std::sort(r.begin(), r.end());
                v = (int32_t)(std::unique(r.begin(), r.end()) - r.begin());
            }
            split_cb_ranks[s] = v;
        }
        if (slab_ranks) {
            int32_t v = 0;
            if (D.pd[s] >= 0) {
                std::vector<int32_t> r = D.slab_rank[D.pd[s]];
                std::sort(r.begin(), r.end());
                v = (int32_t)(std::unique(r.begin(), r.end()) - r.begin());
            }
            slab_ranks[s] = v;
        }
    }
    if (n_steps) *n_steps = (int64_t)D.steps.size();
    return (int64_t)D.msgs.size();
}

// ---- debug hooks ----
int64_t sc_debug_syrk(double* dC, int32_t ldc, const double* dA, int32_t lda, int32_t M, int32_t N,
                      int32_t K) {
    if (!dC || !dA || M < 0 || N < 0 || K < 0 || N > M) return SC_ERR_ARG;
    return sc::debug_syrk(dC, ldc, dA, lda, M, N, K);
}

int64_t sc_debug_bench(int32_t which, int32_t M, int32_t K, int32_t reps, int32_t arg, double* tflops) {
    if (!tflops || M <= 0 || K <= 0 || reps <= 0) return SC_ERR_ARG;
    return sc::debug_bench(which, M, K, reps, arg, tflops);
}

int64_t sc_debug_contention(int32_t M, int32_t K, int32_t chain_rows, int32_t nchain, int32_t mode,
                            int32_t mask_stride, double* out) {
    if (!out) return SC_ERR_ARG;
    return sc::debug_contention(M, K, chain_rows, nchain, mode, mask_stride, out);
}

int64_t sc_debug_hwid(int32_t nwg, int32_t threads, int32_t spin_ticks, uint32_t* out) {
    // spin_ticks is compared unsigned in the kernel: a negative value would spin ~forever,
    // and more than ~1 s (1e8 ticks of the 100 MHz clock) is never a placement probe
    if (!out || nwg <= 0 || threads <= 0 || threads > 1024 || spin_ticks < 0 || spin_ticks > 100000000)
        return SC_ERR_ARG;
    void* d = nullptr;
    if (hipMalloc(&d, (size_t)nwg * 8) != hipSuccess) return SC_ERR_DEVMEM;
    hipError_t e = sc::launch_hwid((uint32_t*)d, nwg, threads, spin_ticks, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d, (size_t)nwg * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? SC_OK : SC_ERR_HIP;
}

int64_t sc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
