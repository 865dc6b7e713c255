// exp_slow.hip -- experiment (GPU box): WHERE a "slow" north-star pool loses its time.
//
// K pools (32 slots of 256 MiB + output, the ctx layout) are allocated one after another and kept.
// Per pool, interleaved over rounds, it times:
//   full     the product reduction (fa_reduce_device, 33 streams)
//   noout    the same 32 loads + FMAs per lane, no store (one lane-conditional store of a value
//            that is never true, so the loads are not dead code)
//   half0    the product reduction over slots 0..15 only      half1   over slots 16..31
//   single   one slot read alone by the whole grid (slots 0, 15, 31), GB/s
//   wonly    write-only stream over the output region
// If slow pools read single slots slower too, the slowness belongs to where the allocation sits
// (nothing a layout inside it can change); if single reads match and only the 33-stream mix is
// slow, it is an interaction of the streams (a layout inside the pool could change it).
//
//   ./exp_slow [n_log2] [K] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fedavg/fa.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

static const int D = 32;
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Ptrs {
    const float* p[D];
};

__global__ __launch_bounds__(128) void noout_kernel(Ptrs t, int nc, float* out, int64_t nvec) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvec) return;
    f32x4 acc = {0, 0, 0, 0};
#pragma unroll 16
    for (int k = 0; k < nc; ++k) acc += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(t.p[k]) + v);
    if (acc.x == 1234.5f && acc.y == -3.25f) out[v] = acc.z;  // never true for the fill data
}

__global__ __launch_bounds__(128) void read_kernel(const float* p, float* out, int64_t nvec) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvec) return;
    f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + v);
    if (x.x == 1234.5f && x.y == -3.25f) out[v] = x.z;
}

__global__ __launch_bounds__(128) void write_kernel(float* out, int64_t nvec) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvec) return;
    f32x4 z = {1.0f, 2.0f, 3.0f, (float)v};
    __builtin_nontemporal_store(z, reinterpret_cast<f32x4*>(out) + v);
}

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int K = argc > 2 ? atoi(argv[2]) : 6;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 512;
    const int64_t nvec = (int64_t)(n / 4);
    const unsigned grid = (unsigned)((nvec + 127) / 128);
    std::vector<char*> pools(K);
    for (int p = 0; p < K; ++p) {
        CK(hipMalloc((void**)&pools[p], stride * (D + 1)));
        for (int k = 0; k < D; ++k)
            if (fa_fill_uniform(pools[p] + k * stride, n, FA_F32, 0x5EED, k, 0, nullptr) != FA_OK) return 1;
    }
    CK(hipDeviceSynchronize());
    std::vector<float> w(D, 1.0f / D);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const std::vector<std::string> tests = {"full", "noout", "half0", "half1", "single0", "single15", "single31", "wonly"};
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(tests.size()));
    for (int r = 0; r < rounds; ++r)
        for (int p = 0; p < K; ++p) {
            const void* cl[D];
            Ptrs pt;
            for (int k = 0; k < D; ++k) {
                cl[k] = pools[p] + k * stride;
                pt.p[k] = (const float*)cl[k];
            }
            float* out = (float*)(pools[p] + D * stride);
            for (size_t ti = 0; ti < tests.size(); ++ti) {
                for (int it = 0; it < 4; ++it) {
                    CK(hipEventRecord(a, st));
                    const std::string& tn = tests[ti];
                    if (tn == "full" || tn == "half0" || tn == "half1") {
                        const int k0 = tn == "half1" ? 16 : 0, nc = tn == "full" ? D : 16;
                        if (fa_reduce_device(nullptr, 0, cl + k0, w.data(), nc, n, FA_F32, out, FA_F32, FA_FEDAVG,
                                             nullptr, st) != FA_OK)
                            return 1;
                    } else if (tn == "noout") {
                        hipLaunchKernelGGL(noout_kernel, dim3(grid), dim3(128), 0, st, pt, D, out, nvec);
                    } else if (tn.rfind("single", 0) == 0) {
                        const int k = atoi(tn.c_str() + 6);
                        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(128), 0, st, pt.p[k], out, nvec);
                    } else {
                        hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(128), 0, st, out, nvec);
                    }
                    CK(hipGetLastError());
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float t;
                    CK(hipEventElapsedTime(&t, a, b));
                    if (it > 0) ms[p][ti].push_back(t);
                }
            }
        }
    for (int p = 0; p < K; ++p) {
        printf("{\"pool\": %d", p);
        for (size_t ti = 0; ti < tests.size(); ++ti) {
            auto v = ms[p][ti];
            std::sort(v.begin(), v.end());
            const double med = v[v.size() / 2];
            const std::string& tn = tests[ti];
            double bytes = 0;
            if (tn == "full") bytes = (D + 1.0) * n * 4;
            else if (tn == "noout") bytes = (double)D * n * 4;
            else if (tn == "half0" || tn == "half1") bytes = 17.0 * n * 4;
            else bytes = (double)n * 4;
            printf(", \"%s_ms\": %.4f, \"%s_GBs\": %.0f", tn.c_str(), med, tn.c_str(), bytes / (med * 1e-3) / 1e9);
        }
        printf("}\n");
    }
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
