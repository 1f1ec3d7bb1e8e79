// Internal helpers shared by the numeric units (numeric.cpp: handle, plan upload,
// launch / replay; schedule.cpp: the static launch schedule; solve.cpp: export and
// triangular solves; debug.cpp: microbenchmark hooks).
#pragma once

#include <algorithm>
#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "numeric.hpp"

namespace sc {

// CB launches with every K below this use the batched SYRK epilogue (measured per
// level at 128^3: K <= 121 gains, K = 226 loses)
#ifndef SC_LA_EPI
#define SC_LA_EPI 0  // 1: lookahead-stream panel updates with the batched epilogue too
#endif
#ifndef SC_EPI_KMAX
#define SC_EPI_KMAX 192
#endif

#define HIP_TRY(x)                                                                \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            N.err = std::string(#x) + ": " + hipGetErrorString(e_);               \
            return SC_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

template <class T>
inline int64_t upload(Numeric& N, const std::vector<T>& v, T*& dptr) {
    dptr = nullptr;
    size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(T);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        N.err = std::string("hipMalloc(plan): ") + hipGetErrorString(e);
        return SC_ERR_DEVMEM;
    }
    N.allocs.push_back(p);
    N.dev_bytes += (int64_t)bytes;
    if (!v.empty()) {
        e = hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            N.err = std::string("hipMemcpy(plan): ") + hipGetErrorString(e);
            return SC_ERR_HIP;
        }
    }
    dptr = (T*)p;
    return SC_OK;
}

// device allocation owned by the handle (freed by numeric_free)
int64_t dalloc(Numeric& N, size_t bytes, void*& p);

#define TRY(x)                        \
    do {                              \
        int64_t r_ = (x);             \
        if (r_ != SC_OK) return r_;   \
    } while (0)


// Staging slots of the hosted ranks' messages (patched to device addresses once
// the staging pool is allocated): slot < 0 = the buffer is the region itself.
struct CommBuild {
    std::vector<Copy2D> copies;
    std::vector<int64_t> copy_slot;
    std::vector<int2> ctiles;
    std::vector<int64_t> msg_slot, msg_src_slot;
    int64_t stage_total = 0;
};

struct SchedBuild {
    std::vector<ChainDesc> cdesc;
    std::vector<uint32_t> crelp;
    int64_t chain_init = 0;  // doubles of the chained fronts' packed images
    std::vector<TinyFront> tfr;  // tiny-tree plan
    std::vector<int2> ta, tph, tpr;
    int32_t tiny_lds = 0;
    std::vector<int32_t> small;
    std::vector<int2> asmv, potrf, inv;
    std::vector<int2> asml;  // parallel to asmv: owned front columns [x, y) of a task
    std::vector<TrsmTask> trsm;
    std::vector<int4> tall;
    std::vector<XinvTask> xinv;
    std::vector<GemmTask> gemm;
    std::vector<int2> tiles;
    std::vector<int64_t> gblk;  // CB gather: per task, per 64 x 64 CB block, its first segment
    std::vector<GSeg> gseg;
    CommBuild cb;
};

// The static launch schedule of a handle (schedule.cpp): N.sched plus the task arrays
// in B, final device addresses of the hosted ranks' pools.
int64_t build_schedule(Numeric& N, SchedBuild& B);

// Tall-TRSM-by-inverse panel mode (panel_tall = 2, schedule.cpp).  A front in the mode
// factors each slab's diagonal block with the 64-column chain on the block's rows only,
// forms X = inv(L11) (64-block inverses, then log2 doubling products), and solves the
// rows below the slab as one MFMA product L21 = A21 X^T, A21 staged out of place.  Per
// front, in the handle's tall pool (doubles, 64-aligned pieces):
//   S   (m - nbs0 - skip) x nbs0, ld m - nbs0 - skip: the current slab's rows below its
//       diagonal block (panel_tall = 3: below its near rows)
//   X, XT  nbs0 x nbs0, ld nbs0: inv(L11) and its transpose
//   U   nbs0 x nbs0: the doubling steps' intermediate products (transposed)
struct TallLayout {
    int32_t nbs0 = 0;     // first slab width = min(w, NBO)
    int32_t skip = 0;     // panel_tall = 3: the NBO "near" rows below each slab stay in the panel (S holds
                          // the rows from slab end + skip on)
    int64_t lds = 0;      // ld of S
    int64_t x = 0, xt = 0, u = 0, total = 0;  // offsets from the front's base, size
};
TallLayout tall_layout(const Symbolic& S, int32_t s, int nbo);
bool tallx_front(const Symbolic& S, const DistPlan* D, int rank, int32_t s);
// the hosted rank's per-front bases (level-local: fronts of one level side by side,
// every level from 0); returns the pool size it needs, doubles
int64_t plan_tall_scratch(const Symbolic& S, const DistPlan* D, int rank, std::vector<int64_t>& off);

// dist.cpp
hipError_t comm_launch(Numeric& N, const Launch& L);
int64_t dist_min_info(Numeric& N, int32_t& info);
int64_t dist_gather_panels(Numeric& N);
void comm_destroy(Numeric& N);

}  // namespace sc
