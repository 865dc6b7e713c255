// exp_phase.hip -- experiment (GPU box): separate the output stream from the input streams in TIME.
//
// Slow pools lose their time only when the output stream runs beside the 32 input streams
// (tools/exp_slow.hip): the inputs alone read at 7.1 TB/s in every pool (1.21 ms), a 256 MiB
// write-only stream takes 0.043 ms, but together they take 1.30 (fast pools) to 1.41 ms (slow).
// Variants of the same f32 chain (32 clients, 16 loads in flight), results staged in LDS:
//   product   fa_reduce_device (reference point)
//   wgburst   one-shot grid, each workgroup reduces 16 vectors per lane into 64 KiB of LDS, then
//             writes them as one burst (bursty per workgroup, no global order)
//   phase     persistent grid (CUs x 2 workgroups, checked against the occupancy API): each phase
//             every workgroup reduces 16 vectors per lane into LDS, arrives on a device counter,
//             waits for all (bounded spin: an exit every wave reaches, error flag if it ran out),
//             then all write -- reads and writes alternate chip-wide
//   phase32   the same with 32 vectors per lane (128 KiB LDS, one workgroup per CU)
// Each variant's output is checked bit-for-bit against the product's.
//
//   ./exp_phase [n_log2] [K] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__device__ __forceinline__ u32x4 chain(const Tab& t, int64_t v) {
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
    return u32x4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
}

__device__ __forceinline__ void st_sc1(void* p, u32x4 r) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(r) : "memory");
}

// one-shot: workgroup b owns vectors [b*256*R, (b+1)*256*R), lane-interleaved
template <int R>
__global__ __launch_bounds__(256) void wgburst_kernel(Tab t, float* out, int64_t nvec) {
    __shared__ u32x4 buf[R * 256];
    const int64_t base = (int64_t)blockIdx.x * 256 * R;
#pragma unroll 1
    for (int i = 0; i < R; ++i) {
        const int64_t v = base + i * 256 + threadIdx.x;
        if (v < nvec) buf[i * 256 + threadIdx.x] = chain(t, v);
    }
#pragma unroll 1
    for (int i = 0; i < R; ++i) {
        const int64_t v = base + i * 256 + threadIdx.x;
        if (v < nvec) st_sc1(reinterpret_cast<u32x4*>(out) + v, buf[i * 256 + threadIdx.x]);
    }
}

// persistent phases: phase p covers vectors [p*G*256*R, (p+1)*G*256*R); inside it, vector
// p*G*256*R + i*G*256 + b*256 + lane (the linear walk over the phase window)
template <int R>
__global__ __launch_bounds__(256) void phase_kernel(Tab t, float* out, int64_t nvec, int* ctr, int* err) {
    __shared__ u32x4 buf[R * 256];
    const int64_t G = gridDim.x;
    const int64_t per_phase = G * 256 * R;
    const int phases = (int)((nvec + per_phase - 1) / per_phase);
    for (int p = 0; p < phases; ++p) {
        const int64_t base = (int64_t)p * per_phase + (int64_t)blockIdx.x * 256 + threadIdx.x;
#pragma unroll 1
        for (int i = 0; i < R; ++i) {
            const int64_t v = base + (int64_t)i * G * 256;
            if (v < nvec) buf[i * 256 + threadIdx.x] = chain(t, v);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int target = (int)G * (p + 1);
            int spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 16)) {  // every wave leaves: a grid that is not co-resident cannot hang
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
#pragma unroll 1
        for (int i = 0; i < R; ++i) {
            const int64_t v = base + (int64_t)i * G * 256;
            if (v < nvec) st_sc1(reinterpret_cast<u32x4*>(out) + v, buf[i * 256 + threadIdx.x]);
        }
    }
}

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int K = argc > 2 ? atoi(argv[2]) : 4;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 2048;
    const int64_t nvec = (int64_t)(n / 4);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    int occ16 = 0, occ32 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ16, phase_kernel<16>, 256, 0));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ32, phase_kernel<32>, 256, 0));
    const int G16 = cus * std::min(occ16, 2), G32 = cus * std::min(occ32, 1);
    fprintf(stderr, "CUs %d, occupancy phase16 %d phase32 %d -> grids %d %d\n", cus, occ16, occ32, G16, G32);
    if (occ16 < 1 || occ32 < 1) return 1;
    std::vector<char*> pools(K);
    for (int p = 0; p < K; ++p) {
        CK(hipMalloc((void**)&pools[p], stride * (D + 2)));
        for (int k = 0; k < D; ++k)
            if (fa_fill_uniform(pools[p] + k * stride, n, FA_F32, 0x5EED, k, 0, nullptr) != FA_OK) return 1;
    }
    int *ctr, *err;
    CK(hipMalloc((void**)&ctr, 4));
    CK(hipMalloc((void**)&err, 4));
    CK(hipMemset(err, 0, 4));
    CK(hipDeviceSynchronize());
    std::vector<float> w(D);
    for (int k = 0; k < D; ++k) w[k] = (float)(k + 1) / (D * (D + 1) / 2);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const std::vector<std::string> modes = {"product", "wgburst", "phase", "phase32"};
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(modes.size()));
    std::vector<int> mismatches(modes.size(), 0);
    std::vector<uint32_t> ref(n), got(n);
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
            float* out_ref = (float*)(pools[p] + (D + 1) * stride);
            for (size_t mi = 0; mi < modes.size(); ++mi) {
                const std::string& m = modes[mi];
                for (int it = 0; it < 4; ++it) {
                    if (m == "phase" || m == "phase32") CK(hipMemsetAsync(ctr, 0, 4, st));
                    CK(hipEventRecord(a, st));
                    if (m == "product") {
                        if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out_ref, FA_F32, FA_FEDAVG,
                                             nullptr, st) != FA_OK)
                            return 1;
                    } else if (m == "wgburst") {
                        hipLaunchKernelGGL(wgburst_kernel<16>, dim3((unsigned)((nvec + 4095) / 4096)), dim3(256), 0, st,
                                           t, out, nvec);
                    } else if (m == "phase") {
                        hipLaunchKernelGGL(phase_kernel<16>, dim3(G16), dim3(256), 0, st, t, out, nvec, ctr, err);
                    } else {
                        hipLaunchKernelGGL(phase_kernel<32>, dim3(G32), dim3(256), 0, st, t, out, nvec, ctr, err);
                    }
                    CK(hipGetLastError());
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float tm;
                    CK(hipEventElapsedTime(&tm, a, b));
                    if (it > 0) ms[p][mi].push_back(tm);
                }
                if (r == 0 && p == 0 && m != "product") {
                    CK(hipMemcpy(ref.data(), out_ref, n * 4, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < n; ++i) mismatches[mi] += ref[i] != got[i];
                }
            }
        }
    int h_err = 0;
    CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
    for (int p = 0; p < K; ++p) {
        printf("{\"pool\": %d", p);
        for (size_t mi = 0; mi < modes.size(); ++mi) {
            auto v = ms[p][mi];
            std::sort(v.begin(), v.end());
            printf(", \"%s\": %.4f", modes[mi].c_str(), v[v.size() / 2]);
        }
        printf("}\n");
    }
    printf("{\"mismatches\": {\"wgburst\": %d, \"phase\": %d, \"phase32\": %d}, \"spin_timeout\": %d, \"grids\": [%d, %d]}\n",
           mismatches[1], mismatches[2], mismatches[3], h_err, G16, G32);
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
