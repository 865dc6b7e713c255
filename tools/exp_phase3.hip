// exp_phase3.hip -- experiment (GPU box): bigger phases (results staged in registers beside LDS) and
// soft barriers for the phased kernel of tools/exp_phase2.hip.
//   r40            256 threads, 40 vectors per lane in LDS (160 KiB), full chip-wide barrier
//   r40_regN       + N more vectors per lane held in VGPRs (1 wave per SIMD: up to 512 VGPRs), so
//                  a phase covers (40+N)/40 times more of the bucket and fewer barriers are paid
//   ..._slackS     the write part starts once all but S workgroups have arrived
//
// exp_phase2.hip's header follows.
//
// exp_phase2.hip -- experiment (GPU box): where the phased kernel of tools/exp_phase.hip loses its time.
//
// exp_phase.hip (r01s14): with reads and writes separated chip-wide in time, a persistent grid of one
// 256-thread workgroup per CU, 32 vectors per lane staged in 128 KiB of LDS, ran 1.32 ms in EVERY
// pool (the product: 1.28 fast, 1.42 slow).  Variants of that kernel:
//   phase(T,R,L,B)  T threads per workgroup, R vectors per lane per phase (T*R*16 B of LDS),
//                   L client loads in flight per lane (16, or all 32), B = with / without the
//                   chip-wide barrier between the read and the write part of a phase.
// The original exp_phase.hip header follows.
//
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

template <int L>
__device__ __forceinline__ u32x4 chain(const Tab& t, int64_t v) {
    float acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < D; g += L) {
        u32x4 raw[L];
#pragma unroll
        for (int u = 0; u < L; ++u)
            raw[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t.p[g + u]) + v);
#pragma unroll
        for (int u = 0; u < L; ++u) {
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

template <int R, int RR, int SLACK>
__global__ __launch_bounds__(256) void phase_kernel(Tab t, float* out, int64_t nvec, int* ctr, int* err) {
    constexpr int T = 256;
    __shared__ u32x4 buf[R * T];
    const int64_t G = gridDim.x;
    const int64_t per_phase = G * T * (R + RR);
    const int phases = (int)((nvec + per_phase - 1) / per_phase);
    for (int p = 0; p < phases; ++p) {
        const int64_t base = (int64_t)p * per_phase + (int64_t)blockIdx.x * T + threadIdx.x;
#pragma unroll 1
        for (int i = 0; i < R; ++i) {
            const int64_t v = base + (int64_t)i * G * T;
            if (v < nvec) buf[i * T + threadIdx.x] = chain<16>(t, v);
        }
        u32x4 keep[RR > 0 ? RR : 1];
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const int64_t v = base + (int64_t)(R + j) * G * T;
            keep[j] = v < nvec ? chain<16>(t, v) : u32x4{0, 0, 0, 0};
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int target = (int)G * (p + 1) - SLACK;
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
            const int64_t v = base + (int64_t)i * G * T;
            if (v < nvec) st_sc1(reinterpret_cast<u32x4*>(out) + v, buf[i * T + threadIdx.x]);
        }
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const int64_t v = base + (int64_t)(R + j) * G * T;
            if (v < nvec) st_sc1(reinterpret_cast<u32x4*>(out) + v, keep[j]);
        }
    }
}

struct Variant {
    const char* name;
    void (*kern)(Tab, float*, int64_t, int*, int*);
    int threads;
};

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int K = argc > 2 ? atoi(argv[2]) : 4;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + 2048;
    const int64_t nvec = (int64_t)(n / 4);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const std::vector<Variant> vars = {
        {"r40", phase_kernel<40, 0, 0>, 256},
        {"r40_slack8", phase_kernel<40, 0, 8>, 256},
        {"r40_slack32", phase_kernel<40, 0, 32>, 256},
        {"r40_reg16", phase_kernel<40, 16, 0>, 256},
        {"r40_reg32", phase_kernel<40, 32, 0>, 256},
        {"r40_reg48", phase_kernel<40, 48, 0>, 256},
        {"r40_reg32_slack8", phase_kernel<40, 32, 8>, 256},
    };
    std::vector<int> grid(vars.size());
    for (size_t i = 0; i < vars.size(); ++i) {
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vars[i].kern, vars[i].threads, 0));
        if (occ < 1) {
            fprintf(stderr, "%s: occupancy %d\n", vars[i].name, occ);
            return 1;
        }
        grid[i] = cus;  // one workgroup per CU
    }
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
    const size_t nm = vars.size() + 1;  // + product
    std::vector<std::vector<std::vector<float>>> ms(K, std::vector<std::vector<float>>(nm));
    std::vector<int> mismatches(nm, 0);
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
            for (size_t mi = 0; mi < nm; ++mi) {
                for (int it = 0; it < 4; ++it) {
                    if (mi > 0) CK(hipMemsetAsync(ctr, 0, 4, st));
                    CK(hipEventRecord(a, st));
                    if (mi == 0) {
                        if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out_ref, FA_F32, FA_FEDAVG,
                                             nullptr, st) != FA_OK)
                            return 1;
                    } else {
                        const Variant& v = vars[mi - 1];
                        hipLaunchKernelGGL(v.kern, dim3(grid[mi - 1]), dim3(v.threads), 0, st, t, out, nvec, ctr, err);
                    }
                    CK(hipGetLastError());
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    float tm;
                    CK(hipEventElapsedTime(&tm, a, b));
                    if (it > 0) ms[p][mi].push_back(tm);
                }
                if (r == 0 && p == 0 && mi > 0) {
                    CK(hipMemcpy(ref.data(), out_ref, n * 4, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < n; ++i) mismatches[mi] += ref[i] != got[i];
                }
            }
        }
    int h_err = 0;
    CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
    for (int p = 0; p < K; ++p) {
        printf("{\"pool\": %d, \"product\": ", p);
        for (size_t mi = 0; mi < nm; ++mi) {
            auto v = ms[p][mi];
            std::sort(v.begin(), v.end());
            if (mi) printf(", \"%s\": ", vars[mi - 1].name);
            printf("%.4f", v[v.size() / 2]);
        }
        printf("}\n");
    }
    int bad = 0;
    for (size_t mi = 1; mi < nm; ++mi) bad += mismatches[mi];
    printf("{\"mismatches_total\": %d, \"spin_timeout\": %d}\n", bad, h_err);
    for (auto p : pools) CK(hipFree(p));
    return 0;
}
