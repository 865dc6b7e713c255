// exp_cross.hip -- experiment (GPU box): is a pool's slowness owned by its INPUTS or by the OUTPUT?
//
// Slow and fast pools read alike without the output stream (tools/exp_slow.hip), and a skew inside a
// pool does not turn a slow pool fast (tools/exp_skew.hip).  K pools (32 slots + output each) are
// timed crosswise: the inputs of pool p reduced into the output region of pool q, for every (p, q).
// Rows that are uniformly slow or fast -> the inputs decide; columns -> the output decides.
//
//   ./exp_cross [n_log2] [K] [rounds]
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
    const int K = argc > 2 ? atoi(argv[2]) : 5;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 512;
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
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(K));
    for (int r = 0; r < rounds; ++r)
        for (int p = 0; p < K; ++p)
            for (int q = 0; q < K; ++q) {
                const void* cl[D];
                for (int k = 0; k < D; ++k) cl[k] = pools[p] + k * stride;
                void* out = pools[q] + D * stride;
                for (int it = 0; it < 4; ++it) {
                    CK(hipEventRecord(a, st));
                    if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out, FA_F32, FA_FEDAVG, nullptr,
                                         st) != FA_OK)
                        return 1;
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float t;
                    CK(hipEventElapsedTime(&t, a, b));
                    if (it > 0) ms[p][q].push_back(t);
                }
            }
    for (int p = 0; p < K; ++p) {
        printf("{\"inputs_pool\": %d, \"ms_by_output_pool\": [", p);
        for (int q = 0; q < K; ++q) {
            auto v = ms[p][q];
            std::sort(v.begin(), v.end());
            printf("%s%.4f", q ? ", " : "", v[v.size() / 2]);
        }
        printf("]}\n");
    }
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
