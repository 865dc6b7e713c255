// exp_sync.hip -- experiment (not product): ceilings of the compute-node state sync (SURVEY 8f row 4,
// fedavg_sync_kernel: every one of D slots := the ordered chain over them, in place; per element D reads
// + D writes).  D = 8 fp32 at C2's size (12.56 M) and VGG-19's FC part (119.6 M).  Variants: the sync with
// each store policy, R vectors per lane (all R*D reads before the R*D writes), and the D-stream read-only
// and write-only ceilings.  Prints one JSON line per (variant, size): median / min us, algorithmic rate.
//   hipcc --offload-arch=gfx950 -O3 tools/exp_sync.hip -o tools/exp_sync && tools/exp_sync [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int D = 8;

struct Tab {
    u32x4* src[D];
    float w[D];
};

enum { kPlain = 0, kNt = 1, kSc1 = 2, kSc01 = 3 };
template <int SP>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    if constexpr (SP == kNt) __builtin_nontemporal_store(v, p);
    else if constexpr (SP == kSc1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == kSc01) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else *p = v;
}

__device__ __forceinline__ u32x4 chain(const u32x4* raw, const float* w) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        a0 = __builtin_fmaf(__uint_as_float(raw[k].x), w[k], a0);
        a1 = __builtin_fmaf(__uint_as_float(raw[k].y), w[k], a1);
        a2 = __builtin_fmaf(__uint_as_float(raw[k].z), w[k], a2);
        a3 = __builtin_fmaf(__uint_as_float(raw[k].w), w[k], a3);
    }
    return u32x4{__float_as_uint(a0), __float_as_uint(a1), __float_as_uint(a2), __float_as_uint(a3)};
}

// MODE 0: sync (read D, write D); 1: read-only; 2: write-only.  Workgroup b covers 256*R vectors, lane l
// takes b*256*R + j*256 + l.
template <int R, int SP, int MODE>
__global__ __launch_bounds__(256) void sync_k(const Tab t, int64_t nvec, float* sink) {
    const int64_t v0 = (int64_t)blockIdx.x * 256 * R + threadIdx.x;
    u32x4 res[R];
    if constexpr (MODE != 2) {
        u32x4 raw[R][D];
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (v0 + j * 256 < nvec) {
#pragma unroll
                for (int k = 0; k < D; ++k) raw[j][k] = __builtin_nontemporal_load(t.src[k] + v0 + j * 256);
            }
#pragma unroll
        for (int j = 0; j < R; ++j) res[j] = chain(raw[j], t.w);
    } else {
#pragma unroll
        for (int j = 0; j < R; ++j) res[j] = u32x4{0x3f800000u, 0x3f800000u, 0x3f800000u, (uint32_t)(v0 + j)};
    }
    if constexpr (MODE == 1) {
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (res[j].x == 0x7fc01234u) sink[threadIdx.x] = 1.f;
    } else {
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (v0 + j * 256 < nvec) {
#pragma unroll
                for (int k = 0; k < D; ++k) st16<SP>(t.src[k] + v0 + j * 256, res[j]);
            }
    }
}

__global__ void fill(uint32_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = 0x3f800000u | ((uint32_t)z >> 9);  // [1, 2)
    }
}

struct Variant {
    const char* name;
    int mode;
    void (*launch)(const Tab&, int64_t, float*, hipStream_t);
};
template <int R, int SP, int MODE>
void run(const Tab& t, int64_t nvec, float* sink, hipStream_t s) {
    const int64_t blocks = (nvec + 256 * R - 1) / (256 * R);
    sync_k<R, SP, MODE><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(t, nvec, sink);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const int64_t sizes[] = {12557960, 119586824};
    std::vector<Variant> vs = {
        {"sync_r1_sc1 (product store)", 0, run<1, kSc1, 0>},
        {"sync_r1_nt", 0, run<1, kNt, 0>},
        {"sync_r1_plain", 0, run<1, kPlain, 0>},
        {"sync_r1_sc01", 0, run<1, kSc01, 0>},
        {"sync_r2_sc1", 0, run<2, kSc1, 0>},
        {"sync_r4_sc1", 0, run<4, kSc1, 0>},
        {"sync_r2_nt", 0, run<2, kNt, 0>},
        {"read8_r1", 1, run<1, kSc1, 1>},
        {"write8_r1_sc1", 2, run<1, kSc1, 2>},
        {"write8_r1_nt", 2, run<1, kNt, 2>},
        {"write8_r1_plain", 2, run<1, kPlain, 2>},
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    float* sink;
    CHECK(hipMalloc(&sink, 4096 * sizeof(float)));
    for (int64_t n : sizes) {
        const int64_t nvec = n / 4;
        const int sets = n < (1 << 26) ? 3 : 1;
        std::vector<Tab> tabs(sets);
        for (int st = 0; st < sets; ++st)
            for (int k = 0; k < D; ++k) {
                CHECK(hipMalloc(&tabs[st].src[k], n * 4));
                tabs[st].w[k] = 0.1f + 0.01f * k;
            }
        auto refill = [&](int st) {
            for (int k = 0; k < D; ++k) fill<<<4096, 256, 0, s>>>((uint32_t*)tabs[st].src[k], n, 977u * st + k);
        };
        for (int st = 0; st < sets; ++st) refill(st);
        std::vector<uint32_t> ref(n), got(n);
        std::vector<std::vector<float>> ms(vs.size());
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int pass = 0; pass < 3; ++pass) {
            for (size_t iv = 0; iv < vs.size(); ++iv) {
                const size_t vi = pass & 1 ? vs.size() - 1 - iv : iv;
                for (int r = 0; r < 3; ++r) vs[vi].launch(tabs[r % sets], nvec, sink, s);
                for (int r = 0; r < reps; ++r) {
                    CHECK(hipEventRecord(a, s));
                    vs[vi].launch(tabs[r % sets], nvec, sink, s);
                    CHECK(hipEventRecord(b, s));
                    CHECK(hipEventSynchronize(b));
                    float t;
                    CHECK(hipEventElapsedTime(&t, a, b));
                    ms[vi].push_back(t);
                }
                CHECK(hipGetLastError());
                if (pass == 0 && vs[vi].mode == 0) {  // bits of slot 5 after one sync of fresh inputs vs variant 0
                    refill(0);
                    vs[vi].launch(tabs[0], nvec, sink, s);
                    CHECK(hipMemcpyAsync(vi == 0 ? ref.data() : got.data(), tabs[0].src[5], nvec * 16,
                                         hipMemcpyDeviceToHost, s));
                    CHECK(hipStreamSynchronize(s));
                    if (vi != 0 && memcmp(ref.data(), got.data(), nvec * 16) != 0) {
                        fprintf(stderr, "MISMATCH %s n=%ld\n", vs[vi].name, (long)n);
                        return 3;
                    }
                }
                refill(0);  // values stay in range for the timing (repeated syncs shrink them)
            }
        }
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            std::vector<float> v = ms[vi];
            std::sort(v.begin(), v.end());
            const double bytes = (double)nvec * 16 * D * (vs[vi].mode == 0 ? 2 : 1);
            const double med = v[v.size() / 2];
            printf("{\"variant\": \"%s\", \"n\": %ld, \"median_us\": %.2f, \"min_us\": %.2f, \"GBs\": %.0f, \"frac\": %.4f}\n",
                   vs[vi].name, (long)n, med * 1e3, v[0] * 1e3, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 1e9 / 8000.0);
        }
        fflush(stdout);
        for (auto& t : tabs)
            for (int k = 0; k < D; ++k) CHECK(hipFree(t.src[k]));
    }
    return 0;
}
