// hbm_probe.hip -- measured HBM ceilings on this MI355X for the roofline report.
// Not part of the product: a standalone tool that times a read-only stream, a
// copy and a write stream over 8 GiB buffers (far beyond the 256 MiB
// Infinity Cache) with hipEvents and prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                          \
        }                                                                      \
    } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const f32x4* __restrict__ p, int64_t nvec, float* sink) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
        f32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = NT ? __builtin_nontemporal_load(p + v + u * stride) : p[v + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += x[u];
    }
    for (; v < nvec; v += stride) acc += p[v];
    float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.678f) sink[threadIdx.x] = s;  // keeps the loads live, never true for the fill below
}

__global__ __launch_bounds__(256) void copy_kernel(const f32x4* __restrict__ a, f32x4* __restrict__ b, int64_t nvec) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(a + v), b + v);
}

__global__ __launch_bounds__(256) void write_kernel(f32x4* __restrict__ b, int64_t nvec) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride)
        __builtin_nontemporal_store(f32x4{1.f, 2.f, 3.f, 4.f}, b + v);
}

struct Table {
    const f32x4* p[32];
};

// 32-stream read with the FedAvg kernel's structure (8 clients per load group, one float4 per lane) but no
// store: the read-only ceiling of the aggregation access pattern.
__global__ __launch_bounds__(256) void mstream_read_kernel(Table t, int64_t nvec, float* sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        f32x4 acc = {0, 0, 0, 0};
        for (int k = 0; k < 32; k += 8) {
            f32x4 x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(t.p[k + u] + v);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += x[u];
        }
        float s = acc.x + acc.y + acc.z + acc.w;
        if (s == 12345.678f) sink[threadIdx.x] = s;
    }
}

// The same 32-stream pattern WITH the per-lane result store (STORE: 0 none, 1 nt store, 2 plain store,
// 3 store into a 1 MiB L2-resident window): isolates what the output stream costs.
template <int STORE, int U>
__global__ __launch_bounds__(128) void mstream_store_kernel(Table t, int64_t nvec, f32x4* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        f32x4 acc = {0, 0, 0, 0};
        for (int k = 0; k < 32; k += U) {
            f32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(t.p[k + u] + v);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = acc * 0.5f + x[u];
        }
        if constexpr (STORE == 0) {
            float s = acc.x + acc.y + acc.z + acc.w;
            if (s == 12345.678f) out[threadIdx.x] = acc;
        } else if constexpr (STORE == 1) {
            __builtin_nontemporal_store(acc, out + v);
        } else if constexpr (STORE == 2) {
            out[v] = acc;
        } else {
            out[v & 65535] = acc;
        }
    }
}

// Store policy variants through buffer stores (aux: 1 = sc0, 2 = nt, 16 = sc1).
template <int AUX>
__global__ __launch_bounds__(128) void mstream_bstore_kernel(Table t, int64_t nvec, f32x4* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        f32x4 acc = {0, 0, 0, 0};
        for (int k = 0; k < 32; k += 8) {
            f32x4 x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(t.p[k + u] + v);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = acc * 0.5f + x[u];
        }
        // 32-bit byte offset within a 2 GiB window of the output
        __builtin_amdgcn_raw_buffer_store_b128(acc, r, (int)((v & ((1 << 27) - 1)) * 16), 0, AUX);
    }
}

// Write-combining: a workgroup computes TILES consecutive 256-vector tiles, keeps the results in LDS and
// writes them out as one contiguous TILES * 4 KiB burst.
template <int TILES>
__global__ __launch_bounds__(256) void mstream_lds_burst_kernel(Table t, int64_t nvec, f32x4* out) {
    __shared__ f32x4 buf[TILES * 256];
    const int64_t base = (int64_t)blockIdx.x * TILES * 256;
    for (int tile = 0; tile < TILES; ++tile) {
        const int64_t v = base + tile * 256 + threadIdx.x;
        f32x4 acc = {0, 0, 0, 0};
        if (v < nvec) {
            for (int k = 0; k < 32; k += 8) {
                f32x4 x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(t.p[k + u] + v);
#pragma unroll
                for (int u = 0; u < 8; ++u) acc = acc * 0.5f + x[u];
            }
        }
        buf[tile * 256 + threadIdx.x] = acc;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TILES * 256; i += 256)
        if (base + i < nvec) __builtin_nontemporal_store(buf[i], out + base + i);
}

template <typename F>
double time_ms(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a, 0);
        f();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float t;
        (void)hipEventElapsedTime(&t, a, b);
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const size_t bytes = 8ull << 30;
    const int64_t nvec = (int64_t)(bytes / 16);
    f32x4 *a, *b;
    float* sink;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes / 2));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes / 2));
    printf("{");
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    bool first = true;
    for (int g : grids) {
        double r8 = time_ms([&] { read_kernel<8, false><<<g, 256>>>(a, nvec, sink); }, 10);
        double r8n = time_ms([&] { read_kernel<8, true><<<g, 256>>>(a, nvec, sink); }, 10);
        double r16 = time_ms([&] { read_kernel<16, true><<<g, 256>>>(a, nvec, sink); }, 10);
        printf("%s\"read_grid%d\":{\"u8\":%.1f,\"u8_nt\":%.1f,\"u16_nt\":%.1f}", first ? "" : ",", g,
               bytes / r8 / 1e6, bytes / r8n / 1e6, bytes / r16 / 1e6);
        first = false;
    }
    const int64_t nh = nvec / 2;
    double c = time_ms([&] { copy_kernel<<<4096, 256>>>(a, b, nh); }, 10);
    double w = time_ms([&] { write_kernel<<<4096, 256>>>(b, nh); }, 10);
    // 32 streams of 256 MiB inside the 8 GiB buffer, one-shot grid like the FedAvg kernel
    Table t;
    const int64_t per = nvec / 32;
    for (int k = 0; k < 32; ++k) t.p[k] = a + k * per;
    double m = time_ms([&] { mstream_read_kernel<<<(unsigned)(per / 256), 256>>>(t, per, sink); }, 10);
    printf(",\"mstream32_read_GBs\":%.1f", bytes / m / 1e6);
    // output stream ablation: 32 x 128 MiB clients + 128 MiB output (in b)
    {
        Table t2;
        const int64_t per2 = nvec / 64;  // 128 MiB per client
        for (int k = 0; k < 32; ++k) t2.p[k] = a + k * per2;
        const unsigned g = (unsigned)(per2 / 128);
        const double rd = 32.0 * per2 * 16, wr = per2 * 16.0;
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s16 = 0;
        for (int rep = 0; rep < 3; ++rep) {  // interleaved
            s0 += time_ms([&] { mstream_store_kernel<0, 8><<<g, 128>>>(t2, per2, b); }, 5);
            s1 += time_ms([&] { mstream_store_kernel<1, 8><<<g, 128>>>(t2, per2, b); }, 5);
            s2 += time_ms([&] { mstream_store_kernel<2, 8><<<g, 128>>>(t2, per2, b); }, 5);
            s3 += time_ms([&] { mstream_store_kernel<3, 8><<<g, 128>>>(t2, per2, b); }, 5);
            s16 += time_ms([&] { mstream_store_kernel<1, 16><<<g, 128>>>(t2, per2, b); }, 5);
        }
        double pol[8] = {0};
        const int auxs[8] = {0, 1, 2, 3, 16, 17, 18, 19};
        double lb8 = 0, lb16 = 0;
        for (int rep = 0; rep < 3; ++rep) {
            pol[0] += time_ms([&] { mstream_bstore_kernel<0><<<g, 128>>>(t2, per2, b); }, 5);
            pol[1] += time_ms([&] { mstream_bstore_kernel<1><<<g, 128>>>(t2, per2, b); }, 5);
            pol[2] += time_ms([&] { mstream_bstore_kernel<2><<<g, 128>>>(t2, per2, b); }, 5);
            pol[3] += time_ms([&] { mstream_bstore_kernel<3><<<g, 128>>>(t2, per2, b); }, 5);
            pol[4] += time_ms([&] { mstream_bstore_kernel<16><<<g, 128>>>(t2, per2, b); }, 5);
            pol[5] += time_ms([&] { mstream_bstore_kernel<17><<<g, 128>>>(t2, per2, b); }, 5);
            pol[6] += time_ms([&] { mstream_bstore_kernel<18><<<g, 128>>>(t2, per2, b); }, 5);
            pol[7] += time_ms([&] { mstream_bstore_kernel<19><<<g, 128>>>(t2, per2, b); }, 5);
            lb8 += time_ms([&] { mstream_lds_burst_kernel<8><<<(unsigned)((per2 + 2047) / 2048), 256>>>(t2, per2, b); }, 5);
            lb16 += time_ms([&] { mstream_lds_burst_kernel<16><<<(unsigned)((per2 + 4095) / 4096), 256>>>(t2, per2, b); }, 5);
        }
        printf(",\"store_policy_ms\":{");
        for (int i = 0; i < 8; ++i) printf("%s\"aux%d\":%.4f", i ? "," : "", auxs[i], pol[i] / 3);
        printf(",\"lds_burst8\":%.4f,\"lds_burst16\":%.4f}", lb8 / 3, lb16 / 3);
        printf(",\"store_ablation_ms\":{\"no_store\":%.4f,\"nt_store\":%.4f,\"plain_store\":%.4f,"
               "\"l2_window_store\":%.4f,\"nt_store_u16\":%.4f,\"algo_GBs_nt_store\":%.1f,\"read_GBs_no_store\":%.1f}",
               s0 / 3, s1 / 3, s2 / 3, s3 / 3, s16 / 3, (rd + wr) / (s1 / 3) / 1e6, rd / (s0 / 3) / 1e6);
    }
    printf(",\"copy_GBs\":%.1f,\"write_GBs\":%.1f,\"unit\":\"GB/s (1e9 B/s), median of 10, 8 GiB read / 4 GiB copy+write\"}\n",
           2.0 * (bytes / 2) / c / 1e6, (bytes / 2) / w / 1e6);
    return 0;
}
