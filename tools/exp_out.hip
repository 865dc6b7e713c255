// exp_out.hip -- experiment (GPU box): north-star reduce time vs WHERE the output is written.
//
// One client pool laid out like the ctx's (32 slots of n fp32, stride = align(4 KiB) + 512 B skew,
// one hipMalloc); the output goes to
//   tail        the pool's output slot after the last client (what the ctx does)
//   separate    its own hipMalloc
//   inplace_last  over client D-1's slot (the last bucket the wave read)
//   inplace_first over client 0's slot
//   tail_1M     the output slot moved 1 MiB further
// The read:write mix hits HBM's read->write turnaround; an output row that was just opened by a read
// may be cheaper to write.  Timed in rounds interleaved over the variants.
//
//   ./exp_out [n_log2] [rounds]
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

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int rounds = argc > 2 ? atoi(argv[2]) : 4;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 512;
    char* pool = nullptr;
    CK(hipMalloc((void**)&pool, stride * (D + 1) + (1u << 20)));
    char* sep = nullptr;
    CK(hipMalloc((void**)&sep, n * 4));
    auto refill = [&]() {
        for (int k = 0; k < D; ++k)
            if (fa_fill_uniform(pool + k * stride, n, FA_F32, 0x5EED, k, 0, nullptr) != FA_OK) exit(1);
    };
    refill();
    CK(hipDeviceSynchronize());
    const void* cl[D];
    for (int k = 0; k < D; ++k) cl[k] = pool + k * stride;
    struct V {
        const char* name;
        void* out;
    };
    std::vector<V> vs = {{"tail", pool + D * stride},
                         {"separate", sep},
                         {"inplace_last", pool + (D - 1) * stride},
                         {"inplace_first", pool},
                         {"tail_1M", pool + D * stride + (1u << 20)}};
    std::vector<float> w(D, 1.0f / D);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            for (int it = 0; it < 6; ++it) {
                CK(hipEventRecord(a, st));
                if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, vs[i].out, FA_F32, FA_FEDAVG, nullptr,
                                     st) != FA_OK) {
                    fprintf(stderr, "reduce: %s\n", fa_last_error());
                    return 1;
                }
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                if (it > 0) ms[i].push_back(t);
            }
        }
    const double algo = (double)(D + 1) * n * 4;
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = ms[i];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("{\"out\": \"%s\", \"n\": %zu, \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBs\": %.0f}\n", vs[i].name, n,
               med, v[0], algo / (med * 1e-3) / 1e9);
    }
    CK(hipFree(pool));
    CK(hipFree(sep));
    return 0;
}
