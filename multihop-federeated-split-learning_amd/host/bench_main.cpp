// bench_main.cpp -- fa_bench: the device-resident round timed from C++ through the C ABI alone (no
// Python, no torch), as the reference's aggregator process would drive it (aggregator.cpp:55-167 on
// libfa): fa_create -> fa_bucket_define -> the client slots filled in place (fa_fill_uniform on
// fa_bucket_slot) -> fa_reduce_part per round.  One GPU, range layout: HIP events on the launch stream;
// the rs layout (its exchange and bf16 rounding run on the context's own exchange stream) and several GPUs
// (FA_SHARD_RANGE or FA_SHARD_CLIENT_RS over the first G devices): host wall clock around the rounds,
// fa_sync at both ends.  Prints one JSON line with bench.py's metric (GiB/s of client input).
//
//   fa_bench [--workload northstar|c2|c3|c4|c5r] [--steps K] [--warmup W] [--gpus G] [--layout range|rs]
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fedavg/fa.h"

namespace {

struct Workload {
    const char* name;
    int clients;
    size_t elems;
    fa_dtype in, out;
};

// the bench.py workloads (BASELINE.json configs) that fit one GPU
const Workload kWorkloads[] = {
    {"northstar", 32, (size_t)64 << 20, FA_F32, FA_F32},  // 256 MiB fp32 x 32 clients
    {"c2", 8, 12557962, FA_F32, FA_F32},                   // ResNet-18 full model, 8 owners
    {"c3", 32, 42737546, FA_BF16, FA_BF16},                // ResNet-101 (basic blocks), 32 owners, bf16
    {"c4", 64, 139611210, FA_F32, FA_F32},                 // VGG-19, 64 owners
    {"c5r", 128, (size_t)1 << 25, FA_F32, FA_F32},         // C5's per-GPU share at 8 GPUs
};

void check(int rc, const char* what) {
    if (rc != FA_OK) {
        std::fprintf(stderr, "fa_bench: %s: %s\n", what, fa_last_error());
        std::exit(1);
    }
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "fa_bench: %s: %s\n", what, hipGetErrorString(e));
        std::exit(1);
    }
}

}  // namespace

int main(int argc, char** argv) {
    std::string name = "northstar", layout = "range";
    int steps = 20, warmup = 5, gpus = 1;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : "";
        if (a == "--workload") name = v, ++i;
        else if (a == "--steps") steps = std::atoi(v), ++i;
        else if (a == "--warmup") warmup = std::atoi(v), ++i;
        else if (a == "--gpus") gpus = std::atoi(v), ++i;
        else if (a == "--layout") layout = v, ++i;
        else {
            std::fprintf(stderr, "usage: fa_bench [--workload W] [--steps K] [--warmup W] [--gpus G] [--layout range|rs]\n");
            return 2;
        }
    }
    const Workload* wl = nullptr;
    for (auto& w : kWorkloads)
        if (name == w.name) wl = &w;
    if (!wl || steps < 1 || warmup < 0 || gpus < 1 || (layout != "range" && layout != "rs")) {
        std::fprintf(stderr, "fa_bench: bad arguments\n");
        return 2;
    }
    const bool rs = layout == "rs";
    const int flags = rs ? FA_SHARD_CLIENT_RS : gpus > 1 ? FA_SHARD_RANGE : 0;
    fa_ctx* ctx = nullptr;
    check(fa_create(&ctx, gpus, flags), "fa_create");
    const int part = 1, D = wl->clients;
    const fa_dtype out = wl->out;  // the rs layout sums fp32 partials, rounded once for a bf16 output
    const size_t n = wl->elems, s_in = wl->in == FA_F32 ? 4 : 2, s_out = out == FA_F32 ? 4 : 2;
    check(fa_bucket_define(ctx, part, n, wl->in, out, D, FA_FEDAVG), "fa_bucket_define");
    // synthetic client buckets generated in HBM (bench.py's inputs: seed 0x5EED, client k, global index)
    for (int g = 0; g < gpus; ++g) {
        hip_check(hipSetDevice(g), "hipSetDevice");
        int npc = 1;
        check(fa_bucket_pieces(ctx, part, g, &npc), "fa_bucket_pieces");
        for (int k = 0; k < D; ++k)
            for (int j = 0; j < npc; ++j) {
                void* p = nullptr;
                size_t cnt = 0, off = 0;
                if (fa_bucket_piece(ctx, part, g, j, k, &p, &cnt, &off) != FA_OK) break;  // rs: another GPU's client
                check(fa_fill_uniform(p, cnt, wl->in, 0x5EED, (uint32_t)k, off, nullptr), "fa_fill_uniform");
            }
    }
    for (int g = 0; g < gpus; ++g) {
        hip_check(hipSetDevice(g), "hipSetDevice");
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    }
    hip_check(hipSetDevice(0), "hipSetDevice");
    std::vector<float> w((size_t)D, 1.0f / (float)D);
    double ms = 0;
    if (gpus == 1 && !rs) {
        hipStream_t s;
        hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
        hipEvent_t a, b;
        hip_check(hipEventCreate(&a), "hipEventCreate");
        hip_check(hipEventCreate(&b), "hipEventCreate");
        for (int i = 0; i < warmup; ++i) check(fa_reduce_part(ctx, part, w.data(), s), "fa_reduce_part");
        hip_check(hipEventRecord(a, s), "hipEventRecord");
        for (int i = 0; i < steps; ++i) check(fa_reduce_part(ctx, part, w.data(), s), "fa_reduce_part");
        hip_check(hipEventRecord(b, s), "hipEventRecord");
        hip_check(hipEventSynchronize(b), "hipEventSynchronize");
        float t = 0;
        hip_check(hipEventElapsedTime(&t, a, b), "hipEventElapsedTime");
        ms = t / steps;
        hip_check(hipStreamDestroy(s), "hipStreamDestroy");
    } else {
        for (int i = 0; i < warmup; ++i) check(fa_reduce_part(ctx, part, w.data(), nullptr), "fa_reduce_part");
        check(fa_sync(ctx), "fa_sync");
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < steps; ++i) check(fa_reduce_part(ctx, part, w.data(), nullptr), "fa_reduce_part");
        check(fa_sync(ctx), "fa_sync");
        ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / steps;
    }
    const double in_bytes = (double)D * (double)n * (double)s_in;
    const double algo = in_bytes + (double)n * (double)s_out;  // + the output
    std::printf("{\"tool\": \"fa_bench\", \"workload\": \"%s\", \"gpus\": %d, \"layout\": \"%s\", \"clients\": %d, "
                "\"elems_per_client\": %zu, \"steps\": %d, \"ms_per_round\": %.4f, \"gib_s\": %.1f, "
                "\"algorithmic_GBs\": %.1f, \"frac_of_8TBs_per_gpu\": %.4f}\n",
                wl->name, gpus, layout.c_str(), D, n, steps, ms, in_bytes / (ms * 1e-3) / (1024.0 * 1024 * 1024),
                algo / (ms * 1e-3) / 1e9, algo / (ms * 1e-3) / 1e9 / 8000.0 / gpus);
    fa_destroy(ctx);
    return 0;
}
