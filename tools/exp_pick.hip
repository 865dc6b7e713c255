// exp_pick.hip -- experiment (GPU box): reduce time of K pools allocated one after another
// (hipMalloc, ctx layout: 32 slots + output, 4 KiB-aligned stride + 512 B skew), all kept alive, timed
// in interleaved rounds.  Shows how often a north-star-sized allocation lands in "fast" memory and
// whether that is stable per allocation (the basis for a probe-and-keep placement policy).
//
//   ./exp_pick [n_log2] [K] [rounds] [spacer_GiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int K = argc > 2 ? atoi(argv[2]) : 8;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t spacer = (size_t)(argc > 4 ? atof(argv[4]) : 0.0) * (1ull << 30);
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 512;
    void* sp = nullptr;
    if (spacer) CK(hipMalloc(&sp, spacer));
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
    std::vector<std::vector<float>> ms(K);
    for (int r = 0; r < rounds; ++r)
        for (int p = 0; p < K; ++p) {
            const void* cl[D];
            for (int k = 0; k < D; ++k) cl[k] = pools[p] + k * stride;
            for (int it = 0; it < 5; ++it) {
                CK(hipEventRecord(a, st));
                if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, pools[p] + D * stride, FA_F32, FA_FEDAVG,
                                     nullptr, st) != FA_OK)
                    return 1;
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                if (it > 0) ms[p].push_back(t);
            }
        }
    const double algo = (double)(D + 1) * n * 4;
    for (int p = 0; p < K; ++p) {
        auto v = ms[p];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("{\"pool\": %d, \"n\": %zu, \"spacer_GiB\": %.0f, \"median_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, "
               "\"GBs\": %.0f}\n",
               p, n, spacer / double(1ull << 30), med, v[0], v.back(), algo / (med * 1e-3) / 1e9);
    }
    for (auto p : pools) CK(hipFree(p));
    if (sp) CK(hipFree(sp));
    return 0;
}
