// exp_order.hip -- experiment (GPU box): does the ORDER in which the grid walks the buckets change the
// slow-pool penalty?
//
// Slow pools are slow only when the output stream joins the 32 input streams, and the inputs' pool
// decides it (tools/exp_slow.hip, tools/exp_cross.hip).  The product kernel walks the buckets in one
// narrow window: workgroup b owns vectors [b*128, b*128+128) and the whole chip works near the same
// offset of every bucket.  Variants of the same f32 chain (16 loads in flight, sc1 stores), each on
// K pools:
//   linear   the product's mapping (reference point, fa_reduce_device)
//   xcd      workgroups of one XCD (b % 8) own one contiguous eighth of the bucket: 8 windows
//   chunk    a persistent grid of P workgroups, each walking its own contiguous chunk: P windows
//   rev      linear, but odd XCDs walk their eighth backwards (read/write phases de-correlated)
//
//   ./exp_order [n_log2] [K] [rounds]
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
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Tab {
    const float* p[D];
    float w[D];
};

__device__ __forceinline__ void do_vec(const Tab& t, float* out, int64_t v) {
    float acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < D; g += 16) {
        u32x4 raw[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            raw[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t.p[g + u]) + v);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float w = t.w[g + u];
            acc[0] = __builtin_fmaf(__uint_as_float(raw[u].x), w, acc[0]);
            acc[1] = __builtin_fmaf(__uint_as_float(raw[u].y), w, acc[1]);
            acc[2] = __builtin_fmaf(__uint_as_float(raw[u].z), w, acc[2]);
            acc[3] = __builtin_fmaf(__uint_as_float(raw[u].w), w, acc[3]);
        }
    }
    u32x4 r = {__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
    void* p = reinterpret_cast<u32x4*>(out) + v;
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(r) : "memory");
}

// mode 1: XCD-partitioned (blocks with equal b % 8 own one contiguous eighth); mode 3: same, odd
// eighths walked backwards.  nblk = gridDim.x, a multiple of 8.
template <int MODE>
__global__ __launch_bounds__(128) void xcd_kernel(Tab t, float* out, int64_t nvec) {
    const int64_t per = nvec / 8;  // nvec is a multiple of 8 * 128 here
    const int x = blockIdx.x % 8;
    const int64_t bl = blockIdx.x / 8, nb = gridDim.x / 8;
    for (int64_t j = bl; j * 128 < per; j += nb) {
        int64_t jj = j;
        if (MODE == 3 && (x & 1)) jj = per / 128 - 1 - j;
        do_vec(t, out, (int64_t)x * per + jj * 128 + threadIdx.x);
    }
}

// persistent chunks: block b owns [b*chunk, (b+1)*chunk) vectors
__global__ __launch_bounds__(128) void chunk_kernel(Tab t, float* out, int64_t nvec) {
    const int64_t chunk = nvec / gridDim.x;
    const int64_t base = (int64_t)blockIdx.x * chunk;
    for (int64_t j = threadIdx.x; j < chunk; j += 128) do_vec(t, out, base + j);
}

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int K = argc > 2 ? atoi(argv[2]) : 5;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 512;
    const int64_t nvec = (int64_t)(n / 4);
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
    const std::vector<std::string> modes = {"linear", "xcd", "rev", "chunk2048", "chunk4096", "xcd_grid16k"};
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(modes.size()));
    for (int r = 0; r < rounds; ++r)
        for (int p = 0; p < K; ++p) {
            Tab t;
            const void* cl[D];
            for (int k = 0; k < D; ++k) {
                cl[k] = pools[p] + k * stride;
                t.p[k] = (const float*)cl[k];
                t.w[k] = w[k];
            }
            float* out = (float*)(pools[p] + D * stride);
            for (size_t mi = 0; mi < modes.size(); ++mi) {
                for (int it = 0; it < 4; ++it) {
                    CK(hipEventRecord(a, st));
                    const std::string& m = modes[mi];
                    if (m == "linear") {
                        if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out, FA_F32, FA_FEDAVG, nullptr,
                                             st) != FA_OK)
                            return 1;
                    } else if (m == "xcd") {
                        hipLaunchKernelGGL(xcd_kernel<1>, dim3((unsigned)(nvec / 128)), dim3(128), 0, st, t, out, nvec);
                    } else if (m == "rev") {
                        hipLaunchKernelGGL(xcd_kernel<3>, dim3((unsigned)(nvec / 128)), dim3(128), 0, st, t, out, nvec);
                    } else if (m == "xcd_grid16k") {
                        hipLaunchKernelGGL(xcd_kernel<1>, dim3(16384), dim3(128), 0, st, t, out, nvec);
                    } else {
                        const unsigned g = m == "chunk2048" ? 2048 : 4096;
                        hipLaunchKernelGGL(chunk_kernel, dim3(g), dim3(128), 0, st, t, out, nvec);
                    }
                    CK(hipGetLastError());
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float tm;
                    CK(hipEventElapsedTime(&tm, a, b));
                    if (it > 0) ms[p][mi].push_back(tm);
                }
            }
        }
    for (int p = 0; p < K; ++p) {
        printf("{\"pool\": %d", p);
        for (size_t mi = 0; mi < modes.size(); ++mi) {
            auto v = ms[p][mi];
            std::sort(v.begin(), v.end());
            printf(", \"%s\": %.4f", modes[mi].c_str(), v[v.size() / 2]);
        }
        printf("}\n");
    }
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
