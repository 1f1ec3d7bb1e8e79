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
    std::vector<int2> asmv, potrf;
    std::vector<int2> asml;  // parallel to asmv: owned front columns [x, y) of a task
    std::vector<TrsmTask> trsm;
    std::vector<GemmTask> gemm;
    std::vector<int2> tiles;
    std::vector<int64_t> gblk;  // CB gather: per task, per 64 x 64 CB block, its first segment
    std::vector<GSeg> gseg;
    CommBuild cb;
};

// The static launch schedule of a handle (schedule.cpp): N.sched plus the task arrays
// in B, final device addresses of the hosted ranks' pools.
int64_t build_schedule(Numeric& N, SchedBuild& B);

// dist.cpp
hipError_t comm_launch(Numeric& N, const Launch& L);
int64_t dist_min_info(Numeric& N, int32_t& info);
int64_t dist_gather_panels(Numeric& N);
void comm_destroy(Numeric& N);

}  // namespace sc
