// exp_skew.hip -- experiment (GPU box): can a layout INSIDE a slow pool make it fast?
//
// tools/exp_slow.hip showed that slow and fast pools read alike (32 streams without the output:
// 1.21 ms in every pool) and differ only once the output stream joins (1.30 vs 1.41 ms).  Here each
// of K pools is allocated with slack, and the product reduction is timed with the slots laid out
// inside the SAME allocation at different per-slot skews (slot k at k * (align4K(bytes) + skew),
// output after the last slot).  Values do not matter for timing (tools/exp_data.py), so the fill
// is done once.  A skew that is fast in every pool would make placement probing unnecessary; a
// per-pool best skew would make it a cheap in-place probe.
//
//   ./exp_skew [n_log2] [K] [rounds]
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
    const int K = argc > 2 ? atoi(argv[2]) : 4;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t al = (n * 4 + 4095) / 4096 * 4096;
    const std::vector<size_t> skews = {0, 256, 512, 768, 1024, 1536, 2048, 3072, 4096 + 512, 8192 + 512,
                                       65536 + 512, 1048576 + 512, 2097152 + 512};
    const size_t maxskew = *std::max_element(skews.begin(), skews.end());
    const size_t bytes = (al + maxskew) * (D + 1);
    std::vector<char*> pools(K);
    for (int p = 0; p < K; ++p) {
        CK(hipMalloc((void**)&pools[p], bytes));
        for (int k = 0; k < D; ++k)
            if (fa_fill_uniform(pools[p] + k * (al + 512), n, FA_F32, 0x5EED, k, 0, nullptr) != FA_OK) return 1;
    }
    CK(hipDeviceSynchronize());
    std::vector<float> w(D, 1.0f / D);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(skews.size()));
    for (int r = 0; r < rounds; ++r)
        for (int p = 0; p < K; ++p)
            for (size_t si = 0; si < skews.size(); ++si) {
                const size_t stride = al + skews[si];
                const void* cl[D];
                for (int k = 0; k < D; ++k) cl[k] = pools[p] + k * stride;
                void* out = pools[p] + D * stride;
                for (int it = 0; it < 4; ++it) {
                    CK(hipEventRecord(a, st));
                    if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out, FA_F32, FA_FEDAVG, nullptr,
                                         st) != FA_OK)
                        return 1;
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float t;
                    CK(hipEventElapsedTime(&t, a, b));
                    if (it > 0) ms[p][si].push_back(t);
                }
            }
    for (int p = 0; p < K; ++p) {
        printf("{\"pool\": %d, \"ms_by_skew\": {", p);
        for (size_t si = 0; si < skews.size(); ++si) {
            auto v = ms[p][si];
            std::sort(v.begin(), v.end());
            printf("%s\"%zu\": %.4f", si ? ", " : "", skews[si], v[v.size() / 2]);
        }
        printf("}}\n");
    }
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
