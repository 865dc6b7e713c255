// exp_streams.hip -- experiment (not product): read rate of the phased kernel's two access patterns as the
// client count grows (the timeline shows phase-0 reads at 7.2 TB/s with 32 clients, 6.9 with 64 and 6.8
// with 128, r02s67).  Read-only, persistent grid (one 256-thread workgroup per CU), fixed 8.6 GB per launch:
//   rows:  the LDS stage -- workgroup b, row i = block (i*G + b) of 256 vectors; per vector all D clients
//          in groups of 16 loads (chain order), the next row after;
//   chunk: the register stage -- each wave owns R*64 contiguous vectors; clients outer, R loads of one
//          client (1 KiB apart, contiguous) in groups of 16, R accumulators.
// Prints one JSON line per (pattern, D): median / min us, TB/s of reads.
//   hipcc --offload-arch=gfx950 -O3 tools/exp_streams.hip -o tools/exp_streams && tools/exp_streams
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxD = 128;
struct Tab {
    const f32x4* src[kMaxD];
};

template <int D>
__global__ __launch_bounds__(256) void rows_k(const Tab t, int64_t nvec, float* sink) {
    const int64_t G = gridDim.x;
    f32x4 tot = {0, 0, 0, 0};
    for (int64_t i = 0;; ++i) {
        const int64_t v = (i * G + blockIdx.x) * 256 + threadIdx.x;
        if ((i * G) * 256 >= nvec) break;
        if (v < nvec) {
            f32x4 acc = {0, 0, 0, 0};
#pragma unroll
            for (int k0 = 0; k0 < D; k0 += 16) {
                f32x4 x[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) x[u] = __builtin_nontemporal_load(t.src[k0 + u] + v);
#pragma unroll
                for (int u = 0; u < 16; ++u) acc += x[u] * (float)(k0 + u + 1);
            }
            tot += acc;
        }
    }
    if (tot.x == 1.0e30f) sink[threadIdx.x] = tot.y;
}

template <int D, int R>
__global__ __launch_bounds__(256) void chunk_k(const Tab t, int64_t nvec, float* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4, wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    f32x4 tot = {0, 0, 0, 0};
    for (int64_t c0 = wave * R * 64; c0 + R * 64 <= nvec; c0 += waves * R * 64) {
        f32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = f32x4{0, 0, 0, 0};
        for (int k = 0; k < D; ++k) {
            const f32x4* p = t.src[k] + c0 + lane;
#pragma unroll
            for (int r0 = 0; r0 < R; r0 += 16) {
                f32x4 x[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) x[u] = __builtin_nontemporal_load(p + (r0 + u) * 64);
#pragma unroll
                for (int u = 0; u < 16; ++u) acc[r0 + u] += x[u] * (float)(k + 1);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) tot += acc[r];
    }
    if (tot.x == 1.0e30f) sink[threadIdx.x] = tot.y;
}

__global__ void fill(float* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)(i & 1023) * 1e-3f;
}

template <int D>
void run(int reps, float* sink, int cus) {
    const int64_t total = 8LL << 30;            // 8 GiB of reads per launch
    const int64_t n = total / 4 / D;            // elements per client
    const int64_t nvec = n / 4;
    std::vector<float*> bufs(D);
    Tab t{};
    for (int k = 0; k < D; ++k) {
        CHECK(hipMalloc(&bufs[k], n * 4 + 2048 * (k % 16)));  // a little skew, as the product's slots
        fill<<<2048, 256>>>(bufs[k], n);
        t.src[k] = (const f32x4*)bufs[k];
    }
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const char* names[3] = {"rows", "chunk_r16", "chunk_r32"};
    std::vector<float> ms[3];
    for (int pass = 0; pass < 3; ++pass)
        for (int v = 0; v < 3; ++v)
            for (int r = 0; r < reps + 2; ++r) {
                CHECK(hipEventRecord(a));
                if (v == 0) rows_k<D><<<cus, 256>>>(t, nvec, sink);
                else if (v == 1) chunk_k<D, 16><<<cus, 256>>>(t, nvec, sink);
                else chunk_k<D, 32><<<cus, 256>>>(t, nvec, sink);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float x;
                CHECK(hipEventElapsedTime(&x, a, b));
                if (r >= 2) ms[v].push_back(x);
            }
    for (int v = 0; v < 3; ++v) {
        std::sort(ms[v].begin(), ms[v].end());
        const double med = ms[v][ms[v].size() / 2];
        printf("{\"pattern\": \"%s\", \"D\": %d, \"elems_per_client\": %ld, \"median_us\": %.1f, \"min_us\": %.1f, \"TBs\": %.3f}\n",
               names[v], D, (long)n, med * 1e3, ms[v][0] * 1e3, (double)nvec * 16 * D / (med * 1e-3) / 1e12);
    }
    fflush(stdout);
    for (float* p : bufs) CHECK(hipFree(p));
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float* sink;
    CHECK(hipMalloc(&sink, 4096 * sizeof(float)));
    run<32>(reps, sink, cus);
    run<64>(reps, sink, cus);
    run<128>(reps, sink, cus);
    return 0;
}
