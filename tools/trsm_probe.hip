// Microbenchmark of the fused POTRF + panel TRSM kernel's parts (tools/, not shipped):
// variants on one m x 64 panel, 200 back-to-back launches each, us per launch.
//   0 fused kernel (as shipped)     1 POTRF part only      2 row loads + stores only
//   3 solve only (stream built from the block without factoring)
//   4 POTRF part only, small_steps1_fast      5 fused kernel with small_steps1_fast
#include "../sparsecholesky_amd/csrc/kernels.hip"

#include <cstdio>
#include <vector>

namespace sc {
template <int V>
__global__ __launch_bounds__(TRSM_ROWS) void probe_kernel(double* pan, int m, int32_t* info) {
    __shared__ double2 S[TRSM64_STREAM / 2];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * 4 * COLB];
    const int tid = threadIdx.x;
    const int r0 = PNB + blockIdx.x * TRSM_ROWS;
    double* blk = pan;
    double* Sd = reinterpret_cast<double*>(S);
    SmallRegs<1> R;
    small_tiles<1>(R, PNB, PNB);
    if (V != 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
                R.v[0][r * 4 + c] = (R.bi[0] >= 0 && i >= j) ? blk[(int64_t)j * m + i] : 0.0;
            }
        if (V == 4 || V == 5)
            small_steps1_fast(R, colbuf, PNB, info, 0);
        else if (V != 3)
            small_steps<1>(R, colbuf, PNB, info, 0);
        if (R.bi[0] >= 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 4 * R.bi[0] + r, j = 4 * R.bj[0] + c;
                    if (i >= j) Sd[PNB * j - j * (j - 1) / 2 + (i - j)] = (i == j) ? 1.0 / R.v[0][r * 4 + c] : R.v[0][r * 4 + c];
                }
        }
    }
    if (V == 1 || V == 4) {
        if (R.bi[0] >= 0 && blockIdx.x == 0) pan[(int64_t)m * PNB + tid] = R.v[0][0] + Sd[tid];
        return;
    }
    const int row = r0 + tid;
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pan, (uint32_t)m * PNB * 8u);
    const int voff = row < m ? row * 8 : BUF_DEAD;
    double r[PNB];
#pragma unroll
    for (int c = 0; c < PNB; ++c) r[c] = buf_ld(rs, voff, c * m * 8);
    __syncthreads();
    if (V != 2) trsm64_full(r, S);
#pragma unroll
    for (int c = 0; c < PNB; ++c) buf_st(r[c], rs, voff, c * m * 8);
}
}  // namespace sc

int main(int argc, char** argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 16448;
    const int reps = 200;
    std::vector<double> h((size_t)m * 64 + 256, 0.0);
    for (int j = 0; j < 64; ++j)
        for (int i = 0; i < m; ++i) h[(size_t)j * m + i] = (i == j) ? 64.0 : 0.001 * ((i * 7 + j * 13) % 17);
    double *d, *dref;
    int32_t* info;
    hipMalloc(&d, h.size() * 8);
    hipMalloc(&dref, h.size() * 8);
    hipMalloc(&info, 4);
    hipMemcpy(dref, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int nwg = (m - 64 + sc::TRSM_ROWS - 1) / sc::TRSM_ROWS;
    for (int v = 0; v < 6; ++v) {
        for (int pass = 0; pass < 2; ++pass) {
            hipMemcpy(d, dref, h.size() * 8, hipMemcpyDeviceToDevice);
            hipEventRecord(e0, nullptr);
            for (int r = 0; r < reps; ++r) {
                if (v == 0) hipLaunchKernelGGL(sc::probe_kernel<0>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
                if (v == 1) hipLaunchKernelGGL(sc::probe_kernel<1>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
                if (v == 2) hipLaunchKernelGGL(sc::probe_kernel<2>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
                if (v == 3) hipLaunchKernelGGL(sc::probe_kernel<3>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
                if (v == 4) hipLaunchKernelGGL(sc::probe_kernel<4>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
                if (v == 5) hipLaunchKernelGGL(sc::probe_kernel<5>, dim3(nwg), dim3(256), 0, nullptr, d, m, info);
            }
            hipEventRecord(e1, nullptr);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            if (pass == 1) printf("m %d variant %d: %.2f us per launch (%d workgroups)\n", m, v, 1e3 * ms / reps, nwg);
        }
    }
    hipLaunchKernelGGL(sc::stamp_kernel, dim3(1), dim3(1), 0, nullptr, (uint64_t*)info);
    hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(sc::stamp_kernel, dim3(1), dim3(1), 0, nullptr, (uint64_t*)d);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("empty kernel: %.2f us per launch\n", 1e3 * ms / reps);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
