// exp_vmm.hip -- experiment (GPU box): north-star reduce time vs the PHYSICAL placement of the
// client pool, controlled with HIP's virtual memory API.
//
// The same virtual layout (33 buffers of n fp32, slot stride = align(4 KiB) + skew) is backed by
// 2 MiB physical granules mapped in different orders:
//   malloc      one hipMalloc (what the ctx does)
//   contiguous  hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   vmm_ident   granules created in virtual order (physically linear if the allocator is)
//   vmm_perm    granules mapped in a random permutation
//   vmm_ileave  granules created granule-major across buffers (phys order g0b0 g0b1 ... g1b0 ...)
//   vmm_rot     buffer k's granules rotated by k * (granules / D)
// Prints one JSON line per pool: median kernel ms over rounds interleaved across pools.
//
//   hipcc --offload-arch=gfx950 -O2 tools/exp_vmm.hip -Iinclude -Lmultihop-federeated-split-learning_amd/lib -lfa \
//         -Wl,-rpath,$PWD/multihop-federeated-split-learning_amd/lib -o exp_vmm && ./exp_vmm [n_log2] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "fedavg/fa.h"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static const int D = 32;

struct Pool {
    std::string name;
    char* base = nullptr;
    size_t bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles;
    bool vmm = false;
};

static size_t g_gran = 0;

static void vmm_pool(Pool& p, size_t bytes, const std::string& order) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    if (!g_gran) {
        CK(hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityRecommended));
        g_gran = std::max<size_t>(g_gran, 2u << 20);
    }
    const size_t G = (bytes + g_gran - 1) / g_gran;
    p.bytes = G * g_gran;
    p.vmm = true;
    void* va = nullptr;
    CK(hipMemAddressReserve(&va, p.bytes, g_gran, nullptr, 0));
    p.base = (char*)va;
    // creation order defines (likely) physical order; map[v] = handle index for virtual granule v
    std::vector<size_t> create_order(G);  // create_order[i] = virtual granule created i-th
    std::iota(create_order.begin(), create_order.end(), 0);
    const size_t per_buf = G / (D + 1) ? G / (D + 1) : 1;
    if (order == "perm") {
        std::mt19937_64 rng(12345);
        std::shuffle(create_order.begin(), create_order.end(), rng);
    } else if (order == "ileave") {
        std::vector<size_t> o;
        for (size_t g = 0; g < per_buf + 1; ++g)
            for (size_t b = 0; b <= (size_t)D; ++b) {
                const size_t v = b * per_buf + g;
                if (v < G && g < per_buf) o.push_back(v);
            }
        for (size_t v = (D + 1) * per_buf; v < G; ++v) o.push_back(v);
        create_order = o;
    } else if (order == "rot") {
        std::vector<size_t> o;
        for (size_t b = 0; b <= (size_t)D; ++b)
            for (size_t g = 0; g < per_buf; ++g) o.push_back(b * per_buf + (g + b * (per_buf / D)) % per_buf);
        for (size_t v = (D + 1) * per_buf; v < G; ++v) o.push_back(v);
        create_order = o;
    }
    p.handles.resize(G);
    for (size_t i = 0; i < G; ++i) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, g_gran, &prop, 0));
        const size_t v = create_order[i];
        p.handles[v] = h;
        CK(hipMemMap(p.base + v * g_gran, g_gran, 0, h, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = 0;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(p.base, p.bytes, &acc, 1));
}

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 26);
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    const size_t skew = 512;
    const size_t stride = (n * 4 + 4095) / 4096 * 4096 + skew;
    const size_t bytes = stride * (D + 1);
    std::vector<Pool> pools;
    const char* names[] = {"malloc", "contiguous", "vmm_ident", "vmm_perm", "vmm_ileave", "vmm_rot", "malloc2"};
    for (const char* nm : names) {
        Pool p;
        p.name = nm;
        std::string s = nm;
        if (s == "malloc" || s == "malloc2") {
            CK(hipMalloc((void**)&p.base, bytes));
            p.bytes = bytes;
        } else if (s == "contiguous") {
            CK(hipExtMallocWithFlags((void**)&p.base, bytes, hipDeviceMallocContiguous));
            p.bytes = bytes;
        } else {
            vmm_pool(p, bytes, s.substr(4));
        }
        for (int k = 0; k < D; ++k)
            if (fa_fill_uniform(p.base + k * stride, n, FA_F32, 0x5EED, k, 0, nullptr) != FA_OK) {
                fprintf(stderr, "fill: %s\n", fa_last_error());
                return 1;
            }
        pools.push_back(std::move(p));
    }
    CK(hipDeviceSynchronize());
    std::vector<float> w(D, 1.0f / D);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> ms(pools.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < pools.size(); ++i) {
            const void* cl[D];
            for (int k = 0; k < D; ++k) cl[k] = pools[i].base + k * stride;
            void* out = pools[i].base + D * stride;
            for (int it = 0; it < 6; ++it) {
                CK(hipEventRecord(a, st));
                if (fa_reduce_device(nullptr, 0, cl, w.data(), D, n, FA_F32, out, FA_F32, FA_FEDAVG, nullptr, st) !=
                    FA_OK) {
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
    for (size_t i = 0; i < pools.size(); ++i) {
        auto v = ms[i];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("{\"pool\": \"%s\", \"n\": %zu, \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBs\": %.0f, \"base_mod_2M\": %zu}\n",
               pools[i].name.c_str(), n, med, v[0], algo / (med * 1e-3) / 1e9, (size_t)pools[i].base % (2u << 20));
    }
    for (auto& p : pools) {
        if (p.vmm) {
            CK(hipMemUnmap(p.base, p.bytes));
            for (auto h : p.handles) CK(hipMemRelease(h));
            CK(hipMemAddressFree(p.base, p.bytes));
        } else {
            CK(hipFree(p.base));
        }
    }
    return 0;
}
