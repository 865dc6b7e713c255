// exp_small_d.hip -- experiment (not product): launch shapes for the few-client buckets (C2: D = 8 fp32,
// 12.56 M elements full model, 9.44 M the round's phase-2 bucket), where the product's one-shot kernel
// runs at 0.75 of spec (VERDICT r01 "kernel furthest below its roofline").  Every variant computes the
// product's ordered chain acc = fma(x_k, w_k, acc), k = 0..7 from +0, so the outputs are checked equal
// to variant 0's bit for bit.  Prints one JSON line per (variant, size): median / min us over the timed
// launches and the algorithmic rate ((D+1) n 4 bytes / t).
//   hipcc --offload-arch=gfx950 -O3 tools/exp_small_d.hip -o exp_small_d && ./exp_small_d [reps]
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
    const u32x4* src[D];
    float w[D];
};

enum { kPlain = 0, kNt = 1, kSc1 = 2 };
template <int SP>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    if constexpr (SP == kNt) __builtin_nontemporal_store(v, p);
    else if constexpr (SP == kSc1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
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

// One-shot: workgroup slot s covers TH*VPL consecutive vectors; lane l takes s*TH*VPL + j*TH + l, j < VPL.
// All VPL*D loads are issued before the first FMA.  WALK: slot = (b % 8) * nb8 + b / 8 (XCD eighths).
template <int VPL, int TH, int SP, bool WALK, bool READONLY>
__global__ __launch_bounds__(TH) void oneshot(const Tab t, u32x4* out, int64_t nvec, float* sink) {
    int64_t slot = blockIdx.x;
    if (WALK) {
        const int64_t nb8 = gridDim.x >> 3;
        if ((int64_t)blockIdx.x < nb8 * 8) slot = (blockIdx.x & 7) * nb8 + (blockIdx.x >> 3);
    }
    const int64_t v0 = slot * TH * VPL + threadIdx.x;
    u32x4 raw[VPL][D];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int64_t v = v0 + (int64_t)j * TH;
        if (v < nvec) {
#pragma unroll
            for (int k = 0; k < D; ++k) raw[j][k] = __builtin_nontemporal_load(t.src[k] + v);
        }
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int64_t v = v0 + (int64_t)j * TH;
        if (v < nvec) {
            u32x4 r = chain(raw[j], t.w);
            if (READONLY) {
                if (r.x == 0x7fc01234u) sink[threadIdx.x] = 1.f;
            } else {
                st16<SP>(out + v, r);
            }
        }
    }
}

// Grid-stride, software-pipelined: a grid of WPC workgroups per CU; each lane loads the next vector's D
// inputs before it reduces and stores the current one, so D loads stay in flight across iterations.
template <int TH, int SP>
__global__ __launch_bounds__(TH) void pipelined(const Tab t, u32x4* out, int64_t nvec, float* sink) {
    const int64_t stride = (int64_t)gridDim.x * TH;
    int64_t v = (int64_t)blockIdx.x * TH + threadIdx.x;
    if (v >= nvec) return;
    u32x4 cur[D], nxt[D];
#pragma unroll
    for (int k = 0; k < D; ++k) cur[k] = __builtin_nontemporal_load(t.src[k] + v);
    for (; v < nvec; v += stride) {
        const int64_t vn = v + stride;
        if (vn < nvec) {
#pragma unroll
            for (int k = 0; k < D; ++k) nxt[k] = __builtin_nontemporal_load(t.src[k] + vn);
        }
        st16<SP>(out + v, chain(cur, t.w));
#pragma unroll
        for (int k = 0; k < D; ++k) cur[k] = nxt[k];
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
    void (*launch)(const Tab&, u32x4*, int64_t, float*, hipStream_t);
};

template <int VPL, int TH, int SP, bool WALK, bool RO>
void run_oneshot(const Tab& t, u32x4* out, int64_t nvec, float* sink, hipStream_t s) {
    int64_t blocks = (nvec + (int64_t)TH * VPL - 1) / ((int64_t)TH * VPL);
    if (WALK) blocks = (blocks + 7) / 8 * 8;
    oneshot<VPL, TH, SP, WALK, RO><<<dim3((unsigned)blocks), dim3(TH), 0, s>>>(t, out, nvec, sink);
}
template <int TH, int SP, int WPC>
void run_pipe(const Tab& t, u32x4* out, int64_t nvec, float* sink, hipStream_t s) {
    pipelined<TH, SP><<<dim3(256 * WPC), dim3(TH), 0, s>>>(t, out, nvec, sink);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 40;
    const int64_t sizes[] = {12557960, 9442304};  // C2 full model (4-aligned), C2 round phase 2
    const int sets = 3;                             // rotated input sets (> 256 MiB MALL per step)
    std::vector<Variant> vs = {
        {"v1_t256_sc1_walk (product shape)", run_oneshot<1, 256, kSc1, true, false>},
        {"v1_t256_sc1", run_oneshot<1, 256, kSc1, false, false>},
        {"v1_t256_nt_walk", run_oneshot<1, 256, kNt, true, false>},
        {"v1_t256_plain_walk", run_oneshot<1, 256, kPlain, true, false>},
        {"v1_t512_sc1_walk", run_oneshot<1, 512, kSc1, true, false>},
        {"v1_t1024_sc1_walk", run_oneshot<1, 1024, kSc1, true, false>},
        {"v2_t256_sc1_walk", run_oneshot<2, 256, kSc1, true, false>},
        {"v4_t256_sc1_walk", run_oneshot<4, 256, kSc1, true, false>},
        {"v2_t512_sc1_walk", run_oneshot<2, 512, kSc1, true, false>},
        {"pipe_t256_sc1_x8", run_pipe<256, kSc1, 8>},
        {"pipe_t256_sc1_x4", run_pipe<256, kSc1, 4>},
        {"pipe_t512_sc1_x4", run_pipe<512, kSc1, 4>},
        {"pipe_t256_sc1_x16", run_pipe<256, kSc1, 16>},
        {"readonly_v1_t256_walk", run_oneshot<1, 256, kSc1, true, true>},
        {"readonly_v2_t256_walk", run_oneshot<2, 256, kSc1, true, true>},
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    float* sink;
    CHECK(hipMalloc(&sink, 4096 * sizeof(float)));
    for (int64_t n : sizes) {
        const int64_t nvec = n / 4;
        std::vector<void*> in(sets * D), outs(sets);
        std::vector<Tab> tabs(sets);
        for (int st = 0; st < sets; ++st) {
            for (int k = 0; k < D; ++k) {
                CHECK(hipMalloc(&in[st * D + k], n * 4));
                fill<<<4096, 256, 0, s>>>((uint32_t*)in[st * D + k], n, 977u * st + k);
                tabs[st].src[k] = (const u32x4*)in[st * D + k];
                tabs[st].w[k] = 0.05f + 0.01f * k;
            }
            CHECK(hipMalloc(&outs[st], n * 4));
        }
        std::vector<uint32_t> ref(n), got(n);
        std::vector<std::vector<float>> ms(vs.size());
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int pass = 0; pass < 3; ++pass) {
            for (size_t iv = 0; iv < vs.size(); ++iv) {
                const size_t vi = pass & 1 ? vs.size() - 1 - iv : iv;
                for (int r = 0; r < 5; ++r) vs[vi].launch(tabs[r % sets], (u32x4*)outs[r % sets], nvec, sink, s);
                for (int r = 0; r < reps; ++r) {
                    CHECK(hipEventRecord(a, s));
                    vs[vi].launch(tabs[r % sets], (u32x4*)outs[r % sets], nvec, sink, s);
                    CHECK(hipEventRecord(b, s));
                    CHECK(hipEventSynchronize(b));
                    float t;
                    CHECK(hipEventElapsedTime(&t, a, b));
                    ms[vi].push_back(t);
                }
                CHECK(hipGetLastError());
                if (pass == 0 && strncmp(vs[vi].name, "readonly", 8) != 0) {  // bits vs variant 0
                    CHECK(hipMemsetAsync(outs[0], 0xff, n * 4, s));
                    vs[vi].launch(tabs[0], (u32x4*)outs[0], nvec, sink, s);
                    CHECK(hipMemcpyAsync(vi == 0 ? ref.data() : got.data(), outs[0], nvec * 16, hipMemcpyDeviceToHost, s));
                    CHECK(hipStreamSynchronize(s));
                    if (vi != 0 && memcmp(ref.data(), got.data(), nvec * 16) != 0) {
                        fprintf(stderr, "MISMATCH %s n=%ld\n", vs[vi].name, (long)n);
                        return 3;
                    }
                }
            }
        }
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            std::vector<float> v = ms[vi];
            std::sort(v.begin(), v.end());
            const bool ro = strncmp(vs[vi].name, "readonly", 8) == 0;
            const double bytes = (double)nvec * 16 * (ro ? D : D + 1);
            printf("{\"variant\": \"%s\", \"n\": %ld, \"median_us\": %.2f, \"min_us\": %.2f, \"GBs\": %.0f, \"frac\": %.4f}\n",
                   vs[vi].name, (long)n, v[v.size() / 2] * 1e3, v[0] * 1e3, bytes / (v[v.size() / 2] * 1e-3) / 1e9,
                   bytes / (v[v.size() / 2] * 1e-3) / 1e9 / 8000.0);
        }
        fflush(stdout);
        for (void* p : in) CHECK(hipFree(p));
        for (void* p : outs) CHECK(hipFree(p));
    }
    return 0;
}
