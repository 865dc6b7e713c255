// fa_api.hip -- the C ABI (include/fedavg/fa.h): aggregation context, device
// slots, pinned staging, multi-GPU range sharding, and the raw device entry.
//
// What it replaces in the reference (paths relative to the reference root):
//   fa_create / fa_bucket_define  <- systemAPI(true,-1,..) + refactor() ->
//       init_model_sate (aggregator.cpp:47,53; systemAPI.cpp:17-38): the global
//       model parts the aggregator owns.
//   fa_submit                     <- one receipt: torch::load of Task.model_parts
//       into parts_[..] and the per-parameter update (aggregator.cpp:60-92,
//       :113-149).  Here the bytes are staged to HBM; the arithmetic is deferred
//       to finalize so that it runs as one ordered chain over all clients.
//   fa_finalize                   <- the reduced module handed to new_message()
//       (aggregator.cpp:96-106, :153-166).
// No CPU fallback exists: without a gfx950 device every entry that needs one
// returns FA_ERR_NODEV.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "fa_internal.h"

namespace {

thread_local std::string g_err;
// block 128, one-shot grid, 16 clients per load group, nt loads, write-through (sc1) stores:
// tools/sweep.py over 3 pools (profiles/r01_summary.json): sc1 stores 2.7% faster than nt,
// unroll 16 ~1% faster than 8, block 128 2-3% faster than 256; XCD-eighths walk 0.5-1.5% faster than
// linear in 7 of 9 pools over the north star, C3 and C4 (gpurun_out r01s11, profiles/r01_summary.json).
// Default walk: phased with the larger register stage (fa_kernels.hip, fedavg_phased_kernel) wherever
// a bucket holds a full phase, the XCD-eighths one-shot grid below that: in one process over 3 pools
// each (gpurun_out r01s18) 1.269 ms north star in every pool (XCD walk 1.42 there: all slow pools),
// and ahead of the XCD walk on C3, C4 and C5's per-rank share too.
fa::Tuning g_tuning{128, 0, 16, 1, 2, 4};
// Byte skew between consecutive client slots of one bucket (see slot_stride).
size_t g_slot_skew = 2048;
// Placement probing of large FedAvg bucket pools (see alloc_placed): at most this many candidates.
int g_placement_probes = 8;
constexpr size_t kProbeMinBytes = 1ull << 30;  // smaller pools: one allocation, no probe
constexpr double kFastGBs = 0.83 * 8000.0;     // a candidate at >= 83% of the 8 TB/s spec is kept at once
constexpr int kMaxProbeRecord = 8;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define FA_HIP(call)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) return fail(FA_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                     \
    } while (0)

inline size_t dsize(fa_dtype t) { return t == FA_F32 ? 4 : 2; }
inline bool dvalid(int t) { return t == FA_F32 || t == FA_BF16; }

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

constexpr size_t kStageBytes = 32u << 20;  // pinned staging chunk per buffer

struct GpuRes {
    int dev = 0;
    hipStream_t compute = nullptr, copy = nullptr;
    char* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int stage_i = 0;
    void* scratch = nullptr;  // fp32 chain accumulator for bf16-out, D > kMaxClients
    size_t scratch_bytes = 0;
};

struct Part {
    size_t n = 0;
    fa_dtype in = FA_F32, out = FA_F32;
    int D = 0;
    fa_mode mode = FA_FEDAVG;
    float divisor = FA_DEFAULT_DIVISOR;
    std::vector<size_t> off, cnt;  // per-GPU element range
    std::vector<char*> pool;       // per GPU: D client slots + the output, one allocation
    std::vector<size_t> stride;    // per GPU: bytes between consecutive slots
    std::vector<char*> slots;      // per GPU: == pool (slot k at pool + k * stride)
    std::vector<void*> dout;       // per GPU: pool + D * stride
    std::vector<float> w;
    std::vector<std::vector<float>> probe_ms;  // per GPU: probe time of each placement candidate
    std::vector<int> chosen;                   // per GPU: the candidate kept
    std::vector<char> submitted;
    int n_submitted = 0;
    int last_slot = -1;
};

}  // namespace

namespace {
// Host memcpy into / out of the pinned staging chunks, split over worker threads:
// one thread copies ~8-10 GB/s, a PCIe Gen5 x16 link takes ~50 GB/s.
class CopyPool {
public:
    explicit CopyPool(int n) : n_(std::max(1, n)) {
        for (int i = 1; i < n_; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // dst[0, len) = src(0, len), split over the workers (the caller copies part 0).
    void copy(char* dst, size_t len, const std::function<void(size_t, size_t, char*)>& src) {
        if (n_ == 1 || len < (4u << 20)) {
            src(0, len, dst);
            return;
        }
        const size_t per = (len / n_ + 4095) / 4096 * 4096;
        std::function<void(int)> part = [&](int p) {
            const size_t lo = std::min(len, (size_t)p * per), hi = std::min(len, lo + per);
            if (hi > lo) src(lo, hi - lo, dst + lo);
        };
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &part;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        part(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
    }

private:
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                job = job_;
            }
            (*job)(id);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
    const std::function<void(int)>* job_ = nullptr;
};

int default_copy_threads() {
    if (const char* e = std::getenv("FA_COPY_THREADS")) return std::max(1, std::atoi(e));
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hw / 2));
}
}  // namespace

struct fa_ctx {
    int G = 1;
    int flags = 0;
    float divisor = FA_DEFAULT_DIVISOR;
    std::vector<GpuRes> gpu;
    std::map<int, Part> parts;
    std::unique_ptr<CopyPool> pool{new CopyPool(default_copy_threads())};
};

namespace {

// Scratch of at least `bytes` on GPU g (only used by bf16 output with D > kMaxClients).
int ensure_scratch(fa_ctx* ctx, int g, size_t bytes) {
    GpuRes& r = ctx->gpu[g];
    if (r.scratch_bytes >= bytes) return FA_OK;
    DeviceGuard dg(r.dev);
    if (r.scratch) FA_HIP(hipFree(r.scratch));
    r.scratch = nullptr;
    r.scratch_bytes = 0;
    if (hipMalloc(&r.scratch, bytes) != hipSuccess) return fail(FA_ERR_NOMEM, "scratch alloc of %zu B failed", bytes);
    r.scratch_bytes = bytes;
    return FA_OK;
}

bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

// The device reduction for one GPU, shared by fa_reduce_device and fa_finalize.
int reduce_on(fa_ctx* ctx, int g, const void* const* clients, const float* w, int D, size_t n, fa_dtype in,
              void* dst, fa_dtype out, fa_mode mode, float divisor, const float* init, hipStream_t s) {
    if (n == 0) return FA_OK;
    const size_t si = dsize(in), so = dsize(out);
    const int V = (int)(16 / si);
    for (int k = 0; k < D; ++k)
        if (!clients[k]) return fail(FA_ERR_ARG, "client pointer %d is null", k);
    if (!dst) return fail(FA_ERR_ARG, "output pointer is null");
    for (int k = 0; k < D; ++k)
        if (!aligned(clients[k], si)) return fail(FA_ERR_ALIGN, "client %d not %zu-byte aligned", k, si);
    if (!aligned(dst, so)) return fail(FA_ERR_ALIGN, "output not %zu-byte aligned", so);
    if (init && !aligned(init, 4)) return fail(FA_ERR_ALIGN, "init not 4-byte aligned");

    // Vector path: every input shares one 16-byte phase; head elements bring it to 0.
    const size_t phase = ((uintptr_t)clients[mode == FA_LITERAL ? D - 1 : 0] % 16) / si;
    int64_t head = (int64_t)((V - phase) % V);
    if ((size_t)head > n) head = (int64_t)n;
    const int64_t nvec = (int64_t)(n - (size_t)head) / V;
    bool vec = true;
    if (mode == FA_FEDAVG)
        for (int k = 0; k < D; ++k) vec = vec && (((uintptr_t)clients[k] % 16) / si == phase);
    const size_t out_vec_bytes = (size_t)V * so;  // 16 or 32 (f32 out of bf16) or 8 (bf16 out of f32)
    vec = vec && ((uintptr_t)dst + (size_t)head * so) % std::min<size_t>(16, out_vec_bytes) == 0;
    if (init) vec = vec && ((uintptr_t)init + (size_t)head * 4) % 16 == 0;

    if (mode == FA_LITERAL) {
        FA_HIP(fa::launch_literal(clients[D - 1], in, dst, out, divisor, head, nvec, (int64_t)n, vec, g_tuning, s));
        return FA_OK;
    }

    const int passes = (D + fa::kMaxClients - 1) / fa::kMaxClients;
    float* acc = nullptr;  // fp32 accumulator between passes
    if (passes > 1) {
        if (out == FA_F32) {
            acc = static_cast<float*>(dst);
        } else {
            if (!ctx) return fail(FA_ERR_ARG, "bf16 output with D > %d needs a ctx for scratch", fa::kMaxClients);
            int rc = ensure_scratch(ctx, g, n * 4);
            if (rc) return rc;
            acc = static_cast<float*>(ctx->gpu[g].scratch);
            vec = vec && ((uintptr_t)acc + (size_t)head * 4) % 16 == 0;
        }
    }
    for (int p = 0; p < passes; ++p) {
        fa::ClientTable t;
        const int k0 = p * fa::kMaxClients, nc = std::min(fa::kMaxClients, D - k0);
        for (int k = 0; k < nc; ++k) {
            t.src[k] = clients[k0 + k];
            t.w[k] = w[k0 + k];
        }
        const float* pin = p == 0 ? init : acc;
        const bool last = p == passes - 1;
        void* pdst = last ? dst : acc;
        FA_HIP(fa::launch_chain(t, nc, in, last ? out : FA_F32, pin, pdst, head, nvec, (int64_t)n, vec, g_tuning, s));
    }
    return FA_OK;
}

// In-place state sync on GPU g: every slot := sum_k w_k slot_k (rounded to dt).  D <= kMaxClients:
// one fused launch; more: the chain into fp32 scratch, then broadcast launches of kMaxClients slots.
int sync_on(fa_ctx* ctx, int g, void* const* slots, const float* w, int D, size_t n, fa_dtype dt, hipStream_t s) {
    if (n == 0) return FA_OK;
    const size_t si = dsize(dt);
    const int V = (int)(16 / si);
    for (int k = 0; k < D; ++k) {
        if (!slots[k]) return fail(FA_ERR_ARG, "client slot pointer %d is null", k);
        if (!aligned(slots[k], si)) return fail(FA_ERR_ALIGN, "client slot %d not %zu-byte aligned", k, si);
    }
    if (D > fa::kMaxClients) {
        if (!ctx) return fail(FA_ERR_ARG, "state sync of more than %d slots needs a ctx for scratch", fa::kMaxClients);
        int rc = ensure_scratch(ctx, g, n * 4);
        if (rc) return rc;
        float* acc = static_cast<float*>(ctx->gpu[g].scratch);
        rc = reduce_on(ctx, g, (const void* const*)slots, w, D, n, dt, acc, FA_F32, FA_FEDAVG, 0.0f, nullptr, s);
        if (rc) return rc;
        for (int k0 = 0; k0 < D; k0 += fa::kMaxClients) {
            fa::ClientTable t;
            const int nc = std::min(fa::kMaxClients, D - k0);
            for (int k = 0; k < nc; ++k) {
                t.src[k] = slots[k0 + k];
                t.w[k] = 0.0f;
            }
            FA_HIP(fa::launch_broadcast(t, nc, dt, acc, (int64_t)n, g_tuning, s));
        }
        return FA_OK;
    }
    const size_t phase = ((uintptr_t)slots[0] % 16) / si;
    int64_t head = (int64_t)((V - phase) % V);
    if ((size_t)head > n) head = (int64_t)n;
    const int64_t nvec = (int64_t)(n - (size_t)head) / V;
    bool vec = true;
    for (int k = 0; k < D; ++k) vec = vec && (((uintptr_t)slots[k] % 16) / si == phase);
    fa::ClientTable t;
    for (int k = 0; k < D; ++k) {
        t.src[k] = slots[k];
        t.w[k] = w[k];
    }
    FA_HIP(fa::launch_sync(t, D, dt, nullptr, head, nvec, (int64_t)n, vec, g_tuning, s));
    return FA_OK;
}

// Placement of a bucket pool.  The same reduction over the same layout runs at two speeds depending
// on which physical HBM a large allocation receives: 1.29-1.30 ms vs 1.41-1.42 ms for 32 x 256 MiB
// (tools/exp_pick.hip: of 8 pools allocated in sequence, 6 fast and 2 slow, each stable over
// interleaved rounds; physically contiguous pools and 2 MiB-granule VMM pools in any mapping order
// were slow, tools/exp_vmm.hip; the output's placement does not matter, tools/exp_out.hip).  So a
// large FedAvg pool is chosen by measurement: allocate a candidate, time the part's own reduction
// over it (uninitialized contents: the timing does not depend on the values), keep it if it reaches
// kFastGBs, else keep it allocated (so the next candidate lands elsewhere) and try another, up to
// g_placement_probes candidates; the fastest is kept and the others are freed.
int probe_pool(fa_ctx* ctx, int g, const Part& p, size_t stride, char* pool, float* ms_out) {
    GpuRes& r = ctx->gpu[(size_t)g];
    const size_t n = p.cnt[(size_t)g];
    std::vector<const void*> cl((size_t)p.D);
    for (int k = 0; k < p.D; ++k) cl[(size_t)k] = pool + (size_t)k * stride;
    std::vector<float> w((size_t)p.D, 1.0f / (float)p.D);
    void* out = pool + (size_t)p.D * stride;
    struct Ev {  // destroyed on every return path
        hipEvent_t e = nullptr;
        ~Ev() { if (e) (void)hipEventDestroy(e); }
    } a, b;
    FA_HIP(hipEventCreate(&a.e));
    FA_HIP(hipEventCreate(&b.e));
    float best = 1e30f;
    int rc = FA_OK;
    for (int it = 0; it < 4 && rc == FA_OK; ++it) {
        FA_HIP(hipEventRecord(a.e, r.compute));
        rc = reduce_on(ctx, g, cl.data(), w.data(), p.D, n, p.in, out, p.out, FA_FEDAVG, 1.0f, nullptr, r.compute);
        FA_HIP(hipEventRecord(b.e, r.compute));
        FA_HIP(hipEventSynchronize(b.e));
        float t = 0;
        FA_HIP(hipEventElapsedTime(&t, a.e, b.e));
        if (it > 0) best = std::min(best, t);  // first launch warms up
    }
    *ms_out = best;
    return rc;
}

int alloc_placed(fa_ctx* ctx, int g, Part& p, size_t stride, size_t bytes, char** out) {
    const size_t algo = (size_t)p.D * p.cnt[(size_t)g] * dsize(p.in) + p.cnt[(size_t)g] * dsize(p.out);
    // The phased walk runs at the same speed in every pool: a part it covers needs no probe.
    const int64_t phased_from = fa::phased_min_elems(p.in, g_tuning);
    const bool phased = phased_from > 0 && (int64_t)p.cnt[(size_t)g] >= phased_from;
    const int probes = (p.mode == FA_FEDAVG && !phased && bytes >= kProbeMinBytes && p.cnt[(size_t)g] > 0)
                           ? std::max(1, g_placement_probes) : 1;
    std::vector<char*> cand;
    std::vector<float>& ms = p.probe_ms[(size_t)g];
    int best = -1, rc = FA_OK;
    for (int i = 0; i < probes; ++i) {
        char* c = nullptr;
        if (hipMalloc((void**)&c, bytes) != hipSuccess) {  // out of memory for another candidate: stop
            (void)hipGetLastError();
            break;
        }
        cand.push_back(c);
        if (probes == 1) {
            best = 0;
            break;
        }
        float t = 0;
        if ((rc = probe_pool(ctx, g, p, stride, c, &t))) break;
        if (ms.size() < (size_t)kMaxProbeRecord) ms.push_back(t);
        if (best < 0 || t < ms[(size_t)best]) best = i;
        if ((double)algo / (t * 1e-3) / 1e9 >= kFastGBs) break;
    }
    if (cand.empty()) return fail(FA_ERR_NOMEM, "device alloc of %zu B failed on GPU %d", bytes, g);
    if (best < 0) best = 0;
    for (size_t i = 0; i < cand.size(); ++i)
        if ((int)i != best) (void)hipFree(cand[i]);
    if (rc) {
        (void)hipFree(cand[(size_t)best]);
        return rc;
    }
    p.chosen[(size_t)g] = best;
    *out = cand[(size_t)best];
    return FA_OK;
}

int check_part(fa_ctx* ctx, int part_id, Part** out) {
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    auto it = ctx->parts.find(part_id);
    if (it == ctx->parts.end()) return fail(FA_ERR_ARG, "part %d not defined", part_id);
    *out = &it->second;
    return FA_OK;
}

void free_part(fa_ctx* ctx, Part& p) {
    for (size_t g = 0; g < p.pool.size(); ++g) {
        DeviceGuard dg(ctx->gpu[g].dev);
        if (p.pool[g]) (void)hipFree(p.pool[g]);
    }
    p.pool.clear();
    p.slots.clear();
    p.dout.clear();
}

// HBM placement of a bucket's slots.  Client buckets that start at the same
// address modulo a large power of two put the U simultaneous loads of a wave
// (and its store) on the same HBM channels; a small per-slot skew spreads them.
// Measured on MI355X (profiles/r01_summary.json, tools/exp_layout.py): 256-512 B
// skew -> 1.30-1.32 ms for 32 x 256 MiB vs 1.47-1.51 ms unskewed.  Re-laid out
// inside the same six pools (tools/exp_skew.hip), 2048 B beat 512 B in every one
// (by 0.6-2.9%); 8 KiB + 512 and 2 MiB + 512 are 7-12% slower.  Slots stay
// 16-byte aligned.
size_t slot_stride(size_t bytes) { return (bytes + 4095) / 4096 * 4096 + g_slot_skew; }

inline char* slot_ptr(const Part& p, int g, int k) { return p.slots[g] + (size_t)k * p.stride[g]; }

// Enqueue the reduction of part p on every GPU's compute stream (or `s` for a single GPU).
int reduce_part(fa_ctx* ctx, Part& p, const float* w, hipStream_t s) {
    std::vector<const void*> ptrs(p.D);
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[g];
        DeviceGuard dg(r.dev);
        hipStream_t st = s ? s : r.compute;
        for (int k = 0; k < p.D; ++k) ptrs[k] = slot_ptr(p, g, k);
        int rc;
        if (p.mode == FA_LITERAL) {
            const void* last = ptrs[p.last_slot >= 0 ? p.last_slot : p.D - 1];
            rc = reduce_on(ctx, g, &last, w, 1, p.cnt[g], p.in, p.dout[g], p.out, p.mode, p.divisor, nullptr, st);
        } else {
            rc = reduce_on(ctx, g, ptrs.data(), w, p.D, p.cnt[g], p.in, p.dout[g], p.out, p.mode, p.divisor, nullptr,
                           st);
        }
        if (rc) return rc;
    }
    return FA_OK;
}

// A host buffer given as the concatenation of `n` segments (one segment for a flat buffer, one per
// parameter record for an archive mapped in place): the source of a receipt or the destination of a
// reduced bucket.
struct Gather {
    int n;
    const void* const* seg;
    const size_t* bytes;
    // fn(piece, rel, take) for each piece of bytes [a, a + len) of the concatenation; rel = offset of
    // the piece from a.
    template <class F>
    void pieces(size_t a, size_t len, F&& fn) const {
        size_t seg_lo = 0, rel = 0;
        for (int k = 0; k < n && len > 0; ++k) {
            const size_t seg_hi = seg_lo + bytes[k];
            if (a < seg_hi) {
                const size_t off = a - seg_lo, take = std::min(len, seg_hi - a);
                fn(const_cast<char*>(static_cast<const char*>(seg[k])) + off, rel, take);
                a += take;
                rel += take;
                len -= take;
            }
            seg_lo = seg_hi;
        }
    }
    void copy_out(size_t a, size_t len, char* dst) const {  // concatenation[a, a+len) -> dst
        pieces(a, len, [&](char* p, size_t rel, size_t take) { std::memcpy(dst + rel, p, take); });
    }
    void copy_in(size_t a, size_t len, const char* src) const {  // src -> concatenation[a, a+len)
        pieces(a, len, [&](char* p, size_t rel, size_t take) { std::memcpy(p, src + rel, take); });
    }
    size_t total() const {
        size_t t = 0;
        for (int k = 0; k < n; ++k) t += bytes[k];
        return t;
    }
    int check(const char* what) const {
        if (n < 0 || (n > 0 && (!seg || !bytes))) return fail(FA_ERR_ARG, "bad %s segment list", what);
        for (int k = 0; k < n; ++k)
            if (!seg[k] && bytes[k]) return fail(FA_ERR_ARG, "%s segment %d is null", what, k);
        return FA_OK;
    }
};

int submit_impl(fa_ctx* ctx, int part_id, int slot, const Gather& src, float weight, bool pinned) {
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (slot < 0 || slot >= p->D) return fail(FA_ERR_ARG, "client slot %d out of range [0,%d)", slot, p->D);
    if ((rc = src.check("host source"))) return rc;
    const size_t si = dsize(p->in), total = src.total();
    if (total != p->n * si)
        return fail(FA_ERR_ARG, "part %d expects %zu bytes per receipt, got %zu", part_id, p->n * si, total);
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[g];
        DeviceGuard dg(r.dev);
        const size_t base = p->off[g] * si;
        char* ds = slot_ptr(*p, g, slot);
        const size_t bytes = p->cnt[g] * si;
        if (pinned) {  // pinned segments: DMA straight from them, one copy per piece of this GPU's range
            hipError_t e = hipSuccess;
            src.pieces(base, bytes, [&](char* piece, size_t rel, size_t take) {
                if (e == hipSuccess) e = hipMemcpyAsync(ds + rel, piece, take, hipMemcpyHostToDevice, r.copy);
            });
            FA_HIP(e);
            continue;
        }
        // Double-buffered staging: fill one pinned chunk while the other is in flight.
        for (size_t o = 0; o < bytes; o += kStageBytes) {
            const size_t b = std::min(kStageBytes, bytes - o);
            const int i = r.stage_i;
            r.stage_i ^= 1;
            FA_HIP(hipEventSynchronize(r.stage_ev[i]));
            ctx->pool->copy(r.stage[i], b, [&](size_t lo, size_t len, char* d) { src.copy_out(base + o + lo, len, d); });
            FA_HIP(hipMemcpyAsync(ds + o, r.stage[i], b, hipMemcpyHostToDevice, r.copy));
            FA_HIP(hipEventRecord(r.stage_ev[i], r.copy));
        }
    }
    if (!p->submitted[slot]) {
        p->submitted[slot] = 1;
        ++p->n_submitted;
    }
    p->w[slot] = weight;
    p->last_slot = slot;
    return FA_OK;
}

// D2H of the part's device output (the result leaves for new_message()) into `dst`: straight into
// pinned segments, else through the pinned chunks, double-buffered.  Waits for all work on the
// device first (the reduction may have run on a caller's stream).
int copy_output(fa_ctx* ctx, Part& p, const Gather& dst, bool pinned) {
    const size_t so = dsize(p.out);
    if (dst.total() != p.n * so)
        return fail(FA_ERR_ARG, "output of %zu bytes expected, destination holds %zu", p.n * so, dst.total());
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[g];
        DeviceGuard dg(r.dev);
        FA_HIP(hipDeviceSynchronize());
        const char* src = static_cast<const char*>(p.dout[g]);
        const size_t base = p.off[g] * so;
        const size_t bytes = p.cnt[g] * so;
        if (pinned) {
            hipError_t e = hipSuccess;
            dst.pieces(base, bytes, [&](char* piece, size_t rel, size_t take) {
                if (e == hipSuccess) e = hipMemcpyAsync(piece, src + rel, take, hipMemcpyDeviceToHost, r.compute);
            });
            FA_HIP(e);
            FA_HIP(hipStreamSynchronize(r.compute));
            continue;
        }
        const size_t chunks = (bytes + kStageBytes - 1) / kStageBytes;
        // double-buffered: the D2H of chunk c+1 overlaps the host copy-out of chunk c
        auto issue = [&](size_t c) -> int {
            const size_t o = c * kStageBytes, b = std::min(kStageBytes, bytes - o);
            FA_HIP(hipMemcpyAsync(r.stage[c & 1], src + o, b, hipMemcpyDeviceToHost, r.compute));
            FA_HIP(hipEventRecord(r.stage_ev[c & 1], r.compute));
            return FA_OK;
        };
        if (chunks > 0) {
            int rc = issue(0);
            if (rc) return rc;
        }
        for (size_t c = 0; c < chunks; ++c) {
            FA_HIP(hipEventSynchronize(r.stage_ev[c & 1]));
            if (c + 1 < chunks) {
                int rc = issue(c + 1);
                if (rc) return rc;
            }
            const size_t o = c * kStageBytes, b = std::min(kStageBytes, bytes - o);
            char* st = r.stage[c & 1];
            // the pool partitions [0, b); each worker scatters its share of the chunk
            ctx->pool->copy(st, b, [&](size_t lo, size_t len, char*) { dst.copy_in(base + o + lo, len, st + lo); });
        }
        FA_HIP(hipStreamSynchronize(r.compute));
    }
    return FA_OK;
}

int copy_output_flat(fa_ctx* ctx, Part& p, void* host_dst) {
    const size_t bytes = p.n * dsize(p.out);
    const void* segs[1] = {host_dst};
    return copy_output(ctx, p, Gather{1, segs, &bytes}, false);
}

// The end of a phase: wait for the submits, reduce on every GPU, copy the result out, reset the round.
int finalize_impl(fa_ctx* ctx, int part_id, const Gather& dst, bool pinned) {
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (p->mode == FA_FEDAVG && p->n_submitted != p->D)
        return fail(FA_ERR_STATE, "part %d: %d of %d clients submitted", part_id, p->n_submitted, p->D);
    if (p->n_submitted == 0) return fail(FA_ERR_STATE, "part %d: nothing submitted", part_id);
    if ((rc = dst.check("host destination"))) return rc;
    for (int g = 0; g < ctx->G; ++g) {  // the reduction waits for this round's H2D copies
        GpuRes& r = ctx->gpu[g];
        DeviceGuard dg(r.dev);
        hipEvent_t ev;
        FA_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        FA_HIP(hipEventRecord(ev, r.copy));
        FA_HIP(hipStreamWaitEvent(r.compute, ev, 0));
        FA_HIP(hipEventDestroy(ev));
    }
    rc = reduce_part(ctx, *p, p->w.data(), nullptr);
    if (rc) return rc;
    rc = copy_output(ctx, *p, dst, pinned);
    if (rc) return rc;
    std::fill(p->submitted.begin(), p->submitted.end(), 0);
    p->n_submitted = 0;
    p->last_slot = -1;
    return FA_OK;
}

}  // namespace

extern "C" {

int fa_version(void) { return FA_ABI_VERSION; }

const char* fa_last_error(void) { return g_err.c_str(); }

int fa_device_count(int* out) {
    g_err.clear();
    if (!out) return fail(FA_ERR_ARG, "out is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return FA_OK;
}

int fa_set_tuning(const fa_tuning* t) {
    g_err.clear();
    if (!t) return fail(FA_ERR_ARG, "tuning is null");
    fa::Tuning nt = g_tuning;
    size_t skew = g_slot_skew;
    if (t->block) {
        if (t->block != 64 && t->block != 128 && t->block != 256) return fail(FA_ERR_ARG, "block must be 64/128/256");
        nt.block = t->block;
    }
    if (t->max_blocks) nt.max_blocks = t->max_blocks < 0 ? 0 : t->max_blocks;
    if (t->unroll) {
        if (t->unroll != 4 && t->unroll != 8 && t->unroll != 16) return fail(FA_ERR_ARG, "unroll must be 4/8/16");
        nt.unroll = t->unroll;
    }
    if (t->load_policy) {
        if (t->load_policy < 1 || t->load_policy > 2) return fail(FA_ERR_ARG, "load_policy must be 1 or 2");
        nt.load_nt = t->load_policy == 2;
    }
    if (t->store_policy) {
        if (t->store_policy < 1 || t->store_policy > 4) return fail(FA_ERR_ARG, "store_policy must be 1..4");
        nt.store_policy = t->store_policy - 1;
    }
    if (t->slot_skew) {
        if (t->slot_skew > 0 && t->slot_skew % 16) return fail(FA_ERR_ARG, "slot_skew must be a multiple of 16");
        skew = t->slot_skew < 0 ? 0 : (size_t)t->slot_skew;
    }
    if (t->walk) {
        if (t->walk < 1 || t->walk > 6) return fail(FA_ERR_ARG, "walk must be 1..6");
        nt.walk = t->walk - 1;
    }
    int probes = g_placement_probes;
    if (t->placement_probes) {
        if (t->placement_probes > 16) return fail(FA_ERR_ARG, "placement_probes must be <= 16");
        probes = t->placement_probes < 0 ? 1 : t->placement_probes;
    }
    g_tuning = nt;
    g_slot_skew = skew;
    g_placement_probes = probes;
    return FA_OK;
}

int fa_get_tuning(fa_tuning* t) {
    g_err.clear();
    if (!t) return fail(FA_ERR_ARG, "tuning is null");
    t->block = g_tuning.block;
    t->max_blocks = g_tuning.max_blocks;
    t->unroll = g_tuning.unroll;
    t->load_policy = g_tuning.load_nt ? 2 : 1;
    t->store_policy = g_tuning.store_policy + 1;
    t->slot_skew = (int)g_slot_skew;
    t->placement_probes = g_placement_probes;
    t->walk = g_tuning.walk + 1;
    return FA_OK;
}

int fa_create(fa_ctx** out, int n_gpus, int flags) {
    std::vector<int> ids;
    for (int g = 0; g < n_gpus; ++g) ids.push_back(g);
    return fa_create_ex(out, ids.data(), n_gpus, flags);
}

int fa_create_ex(fa_ctx** out, const int* device_ids, int n_gpus, int flags) {
    g_err.clear();
    if (!out) return fail(FA_ERR_ARG, "out is null");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(FA_ERR_NODEV, "no HIP device visible");
    if (n_gpus < 1 || n_gpus > count || (!device_ids && n_gpus > 0))
        return fail(FA_ERR_ARG, "n_gpus=%d but %d device(s) visible", n_gpus, count);
    if (n_gpus > 1 && !(flags & FA_SHARD_RANGE)) return fail(FA_ERR_ARG, "n_gpus > 1 needs FA_SHARD_RANGE");
    for (int g = 0; g < n_gpus; ++g) {
        const int d = device_ids[g];
        if (d < 0 || d >= count) return fail(FA_ERR_ARG, "device id %d out of range [0,%d)", d, count);
        for (int h = 0; h < g; ++h)
            if (device_ids[h] == d) return fail(FA_ERR_ARG, "device id %d listed twice", d);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) return fail(FA_ERR_NODEV, "device %d unreadable", d);
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(FA_ERR_NODEV, "device %d is %s; libfa.so is built for gfx950 only", d, prop.gcnArchName);
    }
    fa_ctx* ctx = new fa_ctx();
    ctx->G = n_gpus;
    ctx->flags = flags;
    ctx->gpu.resize(n_gpus);
    for (int g = 0; g < n_gpus; ++g) {
        GpuRes& r = ctx->gpu[g];
        r.dev = device_ids[g];
        DeviceGuard dg(r.dev);
        bool ok = hipStreamCreateWithFlags(&r.compute, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&r.copy, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; ok && i < 2; ++i)
            ok = hipHostMalloc((void**)&r.stage[i], kStageBytes, hipHostMallocDefault) == hipSuccess &&
                 hipEventCreateWithFlags(&r.stage_ev[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            fa_destroy(ctx);
            return fail(FA_ERR_NOMEM, "stream/staging setup failed on device %d", device_ids[g]);
        }
    }
    *out = ctx;
    return FA_OK;
}

void fa_destroy(fa_ctx* ctx) {
    if (!ctx) return;
    for (auto& kv : ctx->parts) free_part(ctx, kv.second);
    for (auto& r : ctx->gpu) {
        DeviceGuard dg(r.dev);
        if (r.compute) (void)hipStreamSynchronize(r.compute);
        if (r.copy) (void)hipStreamSynchronize(r.copy);
        for (int i = 0; i < 2; ++i) {
            if (r.stage[i]) (void)hipHostFree(r.stage[i]);
            if (r.stage_ev[i]) (void)hipEventDestroy(r.stage_ev[i]);
        }
        if (r.scratch) (void)hipFree(r.scratch);
        if (r.compute) (void)hipStreamDestroy(r.compute);
        if (r.copy) (void)hipStreamDestroy(r.copy);
    }
    delete ctx;
}

int fa_bucket_define(fa_ctx* ctx, int part_id, size_t n_elems, fa_dtype in, fa_dtype out, int n_clients,
                     fa_mode mode) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    if (!dvalid(in) || !dvalid(out)) return fail(FA_ERR_ARG, "bad dtype");
    if (mode != FA_FEDAVG && mode != FA_LITERAL) return fail(FA_ERR_ARG, "bad mode");
    if (n_clients < 1) return fail(FA_ERR_ARG, "n_clients must be >= 1");
    auto it = ctx->parts.find(part_id);
    if (it != ctx->parts.end()) {
        free_part(ctx, it->second);
        ctx->parts.erase(it);
    }
    Part p;
    p.n = n_elems;
    p.in = in;
    p.out = out;
    p.D = n_clients;
    p.mode = mode;
    p.divisor = ctx->divisor;
    p.w.assign(n_clients, 0.0f);
    p.submitted.assign(n_clients, 0);
    // Range shards: multiples of 64 elements so every shard keeps 16-B phase 0.
    const size_t G = (size_t)ctx->G, unit = 64;
    size_t per = ((n_elems + G - 1) / G + unit - 1) / unit * unit;
    for (size_t g = 0; g < G; ++g) {
        size_t lo = std::min(n_elems, g * per), hi = std::min(n_elems, lo + per);
        p.off.push_back(lo);
        p.cnt.push_back(hi - lo);
    }
    p.pool.assign(G, nullptr);
    p.slots.assign(G, nullptr);
    p.dout.assign(G, nullptr);
    p.stride.assign(G, 0);
    p.probe_ms.assign(G, {});
    p.chosen.assign(G, 0);
    for (size_t g = 0; g < G; ++g) {
        DeviceGuard dg(ctx->gpu[g].dev);
        p.stride[g] = slot_stride(p.cnt[g] * dsize(in));
        const size_t bytes = (size_t)n_clients * p.stride[g] + std::max<size_t>(1, p.cnt[g] * dsize(out));
        int rc = alloc_placed(ctx, (int)g, p, p.stride[g], bytes, &p.pool[g]);
        if (rc) {
            free_part(ctx, p);
            return rc;
        }
        p.slots[g] = p.pool[g];
        p.dout[g] = p.pool[g] + (size_t)n_clients * p.stride[g];
    }
    ctx->parts.emplace(part_id, std::move(p));
    return FA_OK;
}

int fa_set_literal_divisor(fa_ctx* ctx, int part_id, float divisor) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    if (!(divisor != 0.0f)) return fail(FA_ERR_ARG, "divisor must be non-zero");
    if (part_id < 0) {
        ctx->divisor = divisor;
        return FA_OK;
    }
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    p->divisor = divisor;
    return FA_OK;
}

static int submit_flat(fa_ctx* ctx, int part_id, int client_slot, const void* host_src, float weight, bool pinned) {
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (!host_src && p->n) return fail(FA_ERR_ARG, "host_src is null");
    const size_t bytes = p->n * dsize(p->in);
    const void* srcs[1] = {host_src};
    return submit_impl(ctx, part_id, client_slot, Gather{1, srcs, &bytes}, weight, pinned);
}

int fa_submit(fa_ctx* ctx, int part_id, int client_slot, const void* host_src, float weight) {
    g_err.clear();
    return submit_flat(ctx, part_id, client_slot, host_src, weight, false);
}

int fa_submit_pinned(fa_ctx* ctx, int part_id, int client_slot, const void* host_src, float weight) {
    g_err.clear();
    return submit_flat(ctx, part_id, client_slot, host_src, weight, true);
}

int fa_submit_gather(fa_ctx* ctx, int part_id, int client_slot, int n_segments, const void* const* srcs,
                     const size_t* bytes, float weight) {
    g_err.clear();
    return submit_impl(ctx, part_id, client_slot, Gather{n_segments, srcs, bytes}, weight, false);
}

int fa_submit_gather_pinned(fa_ctx* ctx, int part_id, int client_slot, int n_segments, const void* const* srcs,
                            const size_t* bytes, float weight) {
    g_err.clear();
    return submit_impl(ctx, part_id, client_slot, Gather{n_segments, srcs, bytes}, weight, true);
}

int fa_finalize(fa_ctx* ctx, int part_id, void* host_dst) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (!host_dst && p->n) return fail(FA_ERR_ARG, "host_dst is null");
    const size_t bytes = p->n * dsize(p->out);
    const void* segs[1] = {host_dst};
    return finalize_impl(ctx, part_id, Gather{1, segs, &bytes}, false);
}

int fa_finalize_gather(fa_ctx* ctx, int part_id, int n_segments, void* const* dsts, const size_t* bytes,
                       int flags) {
    g_err.clear();
    if (flags & ~FA_HOST_PINNED) return fail(FA_ERR_ARG, "unknown flags 0x%x", flags);
    return finalize_impl(ctx, part_id, Gather{n_segments, (const void* const*)dsts, bytes}, (flags & FA_HOST_PINNED) != 0);
}

int fa_host_alloc(size_t bytes, void** out) {
    g_err.clear();
    if (!out) return fail(FA_ERR_ARG, "out is null");
    *out = nullptr;
    if (bytes == 0) return FA_OK;
    if (hipHostMalloc(out, bytes, hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return fail(FA_ERR_NOMEM, "pinned host alloc of %zu B failed", bytes);
    }
    return FA_OK;
}

int fa_host_free(void* p) {
    g_err.clear();
    if (p) FA_HIP(hipHostFree(p));
    return FA_OK;
}

int fa_bucket_slot(fa_ctx* ctx, int part_id, int gpu, int client_slot, void** d_ptr, size_t* n_elems,
                   size_t* elem_offset) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    if (client_slot < 0 || client_slot >= p->D) return fail(FA_ERR_ARG, "client slot %d out of range", client_slot);
    if (d_ptr) *d_ptr = slot_ptr(*p, gpu, client_slot);
    if (n_elems) *n_elems = p->cnt[gpu];
    if (elem_offset) *elem_offset = p->off[gpu];
    return FA_OK;
}

int fa_bucket_placement(fa_ctx* ctx, int part_id, int gpu, int* n_probes, float* probe_ms, int* chosen) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    const auto& ms = p->probe_ms[(size_t)gpu];
    if (n_probes) *n_probes = (int)ms.size();
    if (probe_ms)
        for (size_t i = 0; i < ms.size(); ++i) probe_ms[i] = ms[i];
    if (chosen) *chosen = p->chosen[(size_t)gpu];
    return FA_OK;
}

int fa_bucket_output(fa_ctx* ctx, int part_id, int gpu, void** d_ptr) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    if (d_ptr) *d_ptr = p->dout[gpu];
    return FA_OK;
}

int fa_reduce_part(fa_ctx* ctx, int part_id, const float* h_weights, void* hip_stream) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (hip_stream && ctx->G != 1) return fail(FA_ERR_ARG, "an explicit stream needs a single-GPU ctx");
    return reduce_part(ctx, *p, h_weights ? h_weights : p->w.data(), static_cast<hipStream_t>(hip_stream));
}

int fa_copy_output(fa_ctx* ctx, int part_id, void* host_dst) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (!host_dst && p->n) return fail(FA_ERR_ARG, "host_dst is null");
    return copy_output_flat(ctx, *p, host_dst);
}

int fa_sync(fa_ctx* ctx) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    for (auto& r : ctx->gpu) {
        DeviceGuard dg(r.dev);
        FA_HIP(hipStreamSynchronize(r.copy));
        FA_HIP(hipStreamSynchronize(r.compute));
    }
    return FA_OK;
}

int fa_reduce_device(fa_ctx* ctx, int gpu, const void* const* d_clients, const float* h_weights, int D, size_t n,
                     fa_dtype in, void* d_out, fa_dtype out, fa_mode mode, const float* d_init, void* hip_stream) {
    g_err.clear();
    if (!d_clients || !h_weights) return fail(FA_ERR_ARG, "client or weight array is null");
    if (D < 1) return fail(FA_ERR_ARG, "D must be >= 1");
    if (!dvalid(in) || !dvalid(out)) return fail(FA_ERR_ARG, "bad dtype");
    if (mode != FA_FEDAVG && mode != FA_LITERAL) return fail(FA_ERR_ARG, "bad mode");
    if (ctx && (gpu < 0 || gpu >= ctx->G)) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    int dev = ctx ? ctx->gpu[gpu].dev : gpu;
    if (!s && ctx) s = ctx->gpu[gpu].compute;
    DeviceGuard dg(dev);
    return reduce_on(ctx, ctx ? gpu : 0, d_clients, h_weights, D, n, in, d_out, out, mode,
                     ctx ? ctx->divisor : FA_DEFAULT_DIVISOR, d_init, s);
}

int fa_sync_device(fa_ctx* ctx, int gpu, void* const* d_clients, const float* h_weights, int D, size_t n, fa_dtype dt,
                   void* hip_stream) {
    g_err.clear();
    if (!d_clients || !h_weights) return fail(FA_ERR_ARG, "client or weight array is null");
    if (D < 1) return fail(FA_ERR_ARG, "D must be >= 1");
    if (!dvalid(dt)) return fail(FA_ERR_ARG, "bad dtype");
    if (ctx && (gpu < 0 || gpu >= ctx->G)) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (!s && ctx) s = ctx->gpu[gpu].compute;
    if (ctx) {
        DeviceGuard dg(ctx->gpu[gpu].dev);
        return sync_on(ctx, gpu, d_clients, h_weights, D, n, dt, s);
    }
    return sync_on(nullptr, gpu, d_clients, h_weights, D, n, dt, s);
}

int fa_sync_part(fa_ctx* ctx, int part_id, const float* h_weights, void* hip_stream) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (p->mode != FA_FEDAVG) return fail(FA_ERR_ARG, "part %d is not a FedAvg part", part_id);
    if (hip_stream && ctx->G != 1) return fail(FA_ERR_ARG, "an explicit stream needs a single-GPU ctx");
    const float* w = h_weights ? h_weights : p->w.data();
    std::vector<void*> ptrs(p->D);
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[g];
        DeviceGuard dg(r.dev);
        for (int k = 0; k < p->D; ++k) ptrs[k] = slot_ptr(*p, g, k);
        hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : r.compute;
        if ((rc = sync_on(ctx, g, ptrs.data(), w, p->D, p->cnt[g], p->in, st))) return rc;
    }
    return FA_OK;
}

int fa_fill_uniform(void* d_dst, size_t n, fa_dtype dt, uint64_t seed, uint32_t client, uint64_t idx0,
                    void* hip_stream) {
    g_err.clear();
    if (!dvalid(dt)) return fail(FA_ERR_ARG, "bad dtype");
    if (n == 0) return FA_OK;
    if (!d_dst) return fail(FA_ERR_ARG, "dst is null");
    FA_HIP(fa::launch_fill(d_dst, (int64_t)n, dt, seed, client, idx0, static_cast<hipStream_t>(hip_stream)));
    return FA_OK;
}

}  // extern "C"
