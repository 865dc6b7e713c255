// fa_api.hip -- the C ABI (include/fedavg/fa.h): aggregation context, device
// slots, pinned staging, multi-GPU layouts (range shards; client shards + an
// RCCL reduce-scatter), batched and accumulate-on-arrival reductions, and the
// raw device entry.
//
// What it replaces in the reference (paths relative to the reference root):
//   fa_create / fa_bucket_define  <- systemAPI(true,-1,..) + refactor() ->
//       init_model_sate (aggregator.cpp:47,53; systemAPI.cpp:17-38): the global
//       model parts the aggregator owns.
//   fa_submit                     <- one receipt: torch::load of Task.model_parts
//       into parts_[..] and the per-parameter update (aggregator.cpp:60-92,
//       :113-149).  Here the bytes are staged to HBM; the arithmetic runs as one
//       ordered chain over all clients, at the phase end or (FA_ACCUMULATE_ON_ARRIVAL)
//       continued as the in-order prefix of receipts grows.
//   fa_finalize                   <- the reduced module handed to new_message()
//       (aggregator.cpp:96-106, :153-166).
// No CPU fallback exists: without a gfx950 device every entry that needs one
// returns FA_ERR_NODEV.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fa_internal.h"

namespace {

thread_local std::string g_err;

constexpr size_t kSkewAuto = SIZE_MAX;  // fa_tuning.slot_skew -2: chosen per bucket by slot_skew_for

// Per-context tuning (fa_ctx_set_tuning); fa_set_tuning sets the process defaults that new contexts and
// context-less fa_reduce_device calls start from.
struct CtxTuning {
    // block 128, one-shot grid, 16 clients per load group, nt loads, write-through (sc1) stores, phased
    // walk with the larger register stage where a bucket holds a phase (tools/sweep.py over 3
    // pools, profiles/r01_summary.json: sc1 stores 2.7% faster than nt, unroll 16 ~1% faster than 8,
    // block 128 2-3% faster than 256; the phased walk 1.269 ms on the north star in every pool).
    fa::Tuning tu{128, 0, 16, 1, 2, 4};
    // Byte skew between consecutive client slots of one bucket (see slot_stride); kSkewAuto = by slot size.
    size_t slot_skew = kSkewAuto;
    // FA_SHARD_CLIENT_RS: pieces per round (the reduce-scatter of piece c overlaps the reduce of c+1).
    int rs_chunks = 8;
    // Range pieces (piece_len_for): bytes of slots per piece (0 = never cut) and the span of a GPU's slots
    // above which they are cut.
    size_t piece_span = size_t(16) << 30;
    size_t piece_split = size_t(48) << 30;
};
std::mutex g_defaults_mu;
CtxTuning g_defaults;

CtxTuning defaults() {
    std::lock_guard<std::mutex> g(g_defaults_mu);
    return g_defaults;
}

// A roctx range around a host-side entry (submit, finalize, batched reduce, ...), so that
// `rocprofv3 --marker-trace` shows the aggregation round's host phases beside its kernels and copies.
struct Trace {
    explicit Trace(const char* fmt, int a = -1, int b = -1) {
        char buf[96];
        snprintf(buf, sizeof buf, fmt, a, b);
        roctxRangePushA(buf);
    }
    ~Trace() { roctxRangePop(); }
};

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

#define FA_NCCL(call)                                                                                   \
    do {                                                                                                \
        ncclResult_t r_ = (call);                                                                       \
        if (r_ != ncclSuccess) return fail(FA_ERR_NCCL, "%s: %s (%s:%d)", #call, ncclGetErrorString(r_), \
                                           __FILE__, __LINE__);                                         \
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
constexpr size_t kShardUnit = 64;          // range shards / rs pieces: multiples of 64 elements (16-B phase kept)
constexpr int kMaxSegments = 256;          // buckets per batched launch
constexpr int kSegRing = 4;                // device segment tables per GPU (GpuRes::seg)
// Small receipts read in place (host_keep / host_reduce): a one-GPU range part whose D receipts total at most
// kHostReadMax bytes, in pinned memory, is reduced by kernels that read the receipts' segments over PCIe,
// in at most kHostReadPieces launches (the pieces on which every receipt and the destination are contiguous)
constexpr size_t kHostReadMax = FA_HOST_READ_MAX_BYTES;
constexpr size_t kHostReadPieces = 16;
constexpr int kNotHostReadable = 1;  // host_reduce: the path does not apply (nothing was launched)

// Host memcpy into / out of the pinned staging chunks, split over worker threads:
// one thread copies ~8-10 GB/s, a PCIe Gen5 x16 link takes ~50 GB/s.  One pool per GPU, so the GPUs of a
// range-sharded context stage their pieces concurrently.
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
    int size() const { return n_; }
    // fn(i) for every i in [0, size()): i = 0 on the calling thread, the others on the workers; returns when
    // all have.  One caller at a time.
    void run(const std::function<void(int)>& fn) {
        if (n_ == 1) {
            fn(0);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
    }
    // dst[0, len) = src(0, len), split over the workers (the caller copies part 0).
    void copy(char* dst, size_t len, const std::function<void(size_t, size_t, char*)>& src) {
        if (n_ == 1 || len < (4u << 20)) {
            src(0, len, dst);
            return;
        }
        const size_t per = (len / n_ + 4095) / 4096 * 4096;
        run([&](int p) {
            const size_t lo = std::min(len, (size_t)p * per), hi = std::min(len, lo + per);
            if (hi > lo) src(lo, hi - lo, dst + lo);
        });
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
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hw / 2));
}

// Runs fn(g) for g in [0, G): G > 1 on the context's persistent per-GPU workers (the host-side staging of
// each GPU is independent; no thread is created per call), returning the first non-zero status.
int for_each_gpu(CopyPool* workers, int G, const std::function<int(int)>& fn) {
    if (G == 1 || !workers) return fn(0);
    std::vector<int> rc((size_t)G, FA_OK);
    std::vector<std::string> err((size_t)G);
    workers->run([&](int g) {
        rc[(size_t)g] = fn(g);
        if (rc[(size_t)g]) err[(size_t)g] = g_err;  // g_err is thread-local
    });
    for (int g = 0; g < G; ++g)
        if (rc[(size_t)g]) {
            g_err = err[(size_t)g];
            return rc[(size_t)g];
        }
    return FA_OK;
}

struct GpuRes {
    int dev = 0;
    hipStream_t compute = nullptr, copy = nullptr, comm = nullptr;
    char* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int stage_i = 0;
    hipEvent_t copy_ev = nullptr;  // orders a reduction after the H2D copies queued on `copy`
    uint64_t copy_gen = 0;         // H2D batches queued on `copy` so far (a submit adds one)
    uint64_t copy_ev_gen = 0;      // the batch copy_ev was last recorded after
    std::map<hipStream_t, uint64_t> waited;  // per stream: the copy batch it last waited for
    hipEvent_t step_ev = nullptr;  // orders the rs exchange of a piece after its reduction
    void* scratch = nullptr;       // fp32 chain accumulator for bf16-out, D > kMaxClients
    // fa_output_crc32: the piece table (pinned staging + device copy) and the per-piece results, grown on use
    char* crc_host = nullptr;
    char* crc_dev = nullptr;
    size_t crc_bytes = 0;
    size_t scratch_bytes = 0;
    // Device segment tables of batched launches (fa_reduce_parts beyond the kernel-argument table): a ring,
    // so a changed table is uploaded into a slot whose last launch is long done; each slot remembers the
    // stream and event of its last launch, which orders a reuse or an overwrite after it (allocated on
    // first use).
    struct SegTable {
        fa::SegDesc* host = nullptr;  // pinned staging of the upload
        fa::SegDesc* dev = nullptr;
        hipEvent_t ev = nullptr;      // recorded after the slot's last launch (its upload precedes it)
        hipStream_t stream = nullptr; // the stream of that launch
        size_t bytes = 0;             // bytes of the table the slot holds
    };
    SegTable seg[kSegRing];
    int seg_last = -1;                // the slot of the last batched launch
    std::unique_ptr<CopyPool> pool;
    ncclComm_t nccl = nullptr;
};

// One copy-out run: elements [src, src + cnt) of a GPU's output buffer are bucket elements [dst, dst + cnt).
struct Run {
    size_t src, dst, cnt;
};

struct Part {
    size_t n = 0;
    fa_dtype in = FA_F32, out = FA_F32;
    int D = 0;
    fa_mode mode = FA_FEDAVG;
    float divisor = FA_DEFAULT_DIVISOR;
    bool rs = false;               // FA_SHARD_CLIENT_RS layout
    size_t npad = 0;               // rs: slot length (n padded to a multiple of G * 64)
    std::vector<size_t> off, cnt;  // per GPU: bucket elements held by its slots (range: its shard; rs: [0, n))
    std::vector<int> c0, c1;       // per GPU: the client slots it holds, [c0, c1)
    std::vector<char*> pool;       // per GPU: its client slots + the output (+ rs partial, eager acc)
    std::vector<size_t> stride;    // per GPU: bytes between consecutive slots of one piece
    // Pieces (range layout): a GPU whose slots would span more than 48 GiB (piece_len_for) holds its range as
    // npiece[g] pieces of piece_len[g] elements (the last one shorter): piece j of every slot lies in the
    // j-th region of the pool (slots of one piece stride[g] apart), so one launch reads clients that lie
    // close together (the address span).  One piece = the plain layout.
    std::vector<int> npiece;
    std::vector<size_t> piece_len;
    std::vector<void*> dout;       // per GPU: the output (range: cnt elements of `out`; rs: its fp32 shard)
    std::vector<void*> dout16;     // rs with a bf16 output: per GPU, its shard rounded to bf16 (the copy-out's source)
    std::vector<float*> partial;   // rs: per GPU, fp32 partial over its clients, npad elements
    std::vector<float*> acc;       // FA_ACCUMULATE_ON_ARRIVAL: per GPU, fp32 chain of the reduced prefix
    std::vector<hipEvent_t> done;  // per GPU: orders the copy-out after the reduction (see mark_done)
    std::vector<hipStream_t> done_stream;  // per GPU: the stream the last reduction ran on
    std::vector<float> w;
    std::vector<char> submitted;
    int n_submitted = 0;
    int last_slot = -1;
    int reduced = 0;    // accumulate on arrival: slots [0, reduced) are chained into acc (or dout)
    bool ready = false; // this round's output is reduced already (eager prefix reached D, fa_reduce_parts)
    std::vector<std::vector<Run>> runs;  // per GPU: where its output goes (set by the last reduction)
    std::vector<void*> run_src;          // per GPU: the buffer the runs read
    // Small receipts kept where they arrived (host_keep): per slot the receipt's pinned segments -- the host
    // address (for a later DMA, host_flush) and the address a kernel reads it at -- empty = in the slot.
    struct HostSeg {
        const char* host;
        const char* dev;
        size_t bytes;
    };
    std::vector<std::vector<HostSeg>> host_src;
    int n_host = 0;  // slots whose receipt is kept host-side this round
};

}  // namespace

struct fa_ctx {
    int G = 1;
    int flags = 0;
    float divisor = FA_DEFAULT_DIVISOR;
    CtxTuning tuning;
    std::vector<GpuRes> gpu;
    std::map<int, Part> parts;
    std::unique_ptr<CopyPool> workers;  // G > 1: one persistent host thread per GPU (for_each_gpu)
    unsigned long long host_reads = 0;  // reductions that read their receipts in place (fa_diag_host_reads)
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

// The device reduction for one GPU, shared by every entry: D clients (any D >= 1; more than kMaxClients
// continue the chain from an fp32 accumulator in further passes) -> dst.
int reduce_on(fa_ctx* ctx, int g, const fa::Tuning& tu, const void* const* clients, const float* w, int D, size_t n,
              fa_dtype in, void* dst, fa_dtype out, fa_mode mode, float divisor, const float* init, hipStream_t s) {
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
        FA_HIP(fa::launch_literal(clients[D - 1], in, dst, out, divisor, head, nvec, (int64_t)n, vec, tu, s));
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
        FA_HIP(fa::launch_chain(t, nc, in, last ? out : FA_F32, pin, pdst, head, nvec, (int64_t)n, vec, tu, s));
    }
    return FA_OK;
}

// In-place state sync on GPU g: every slot := sum_k w_k slot_k (rounded to dt).  D <= kMaxClients:
// one fused launch; more: the chain into fp32 scratch, then broadcast launches of kMaxClients slots.
int sync_on(fa_ctx* ctx, int g, const fa::Tuning& tu, void* const* slots, const float* w, int D, size_t n,
            fa_dtype dt, hipStream_t s) {
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
        rc = reduce_on(ctx, g, tu, (const void* const*)slots, w, D, n, dt, acc, FA_F32, FA_FEDAVG, 0.0f, nullptr, s);
        if (rc) return rc;
        for (int k0 = 0; k0 < D; k0 += fa::kMaxClients) {
            fa::ClientTable t;
            const int nc = std::min(fa::kMaxClients, D - k0);
            for (int k = 0; k < nc; ++k) {
                t.src[k] = slots[k0 + k];
                t.w[k] = 0.0f;
            }
            FA_HIP(fa::launch_broadcast(t, nc, dt, acc, (int64_t)n, tu, s));
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
    FA_HIP(fa::launch_sync(t, D, dt, nullptr, head, nvec, (int64_t)n, vec, tu, s));
    return FA_OK;
}

// ------------------------------------------------------------------ layouts

// [c0, c1) of the D client slots held by GPU g of G under the rs layout (contiguous, balanced; chain
// order kept within a GPU).  Same rule as shard.client_bounds.
void client_bounds(int D, int G, int g, int* c0, int* c1) {
    const int base = D / G, extra = D % G;
    *c0 = g * base + std::min(g, extra);
    *c1 = *c0 + base + (g < extra ? 1 : 0);
}

// The rs pieces of a bucket padded to npad (a multiple of G * 64): `chunks` contiguous pieces, each a
// multiple of G * 64 elements, so each splits into G equal blocks; GPU g owns block g of every piece
// (block-cyclic, the same rule as shard.cyclic_pieces / cyclic_bounds).
std::vector<std::pair<size_t, size_t>> rs_pieces(size_t npad, int G, int chunks) {
    const size_t unit = (size_t)G * kShardUnit, m = npad / unit;
    chunks = std::max(1, chunks);
    std::vector<size_t> edges;
    for (int c = 0; c < chunks; ++c) edges.push_back(m * (size_t)c / (size_t)chunks * unit);
    edges.push_back(npad);
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
    std::vector<std::pair<size_t, size_t>> out;
    for (size_t i = 0; i + 1 < edges.size(); ++i) out.emplace_back(edges[i], edges[i + 1]);
    return out;
}

// HBM placement of a bucket's slots.  Client buckets that start at the same address modulo a large
// power of two put the U simultaneous loads of a wave (and its store) on the same HBM channels; a small
// per-slot skew spreads them.  Measured on MI355X (round 1, profiles/r01_summary.json):
// 256-512 B skew -> 1.30-1.32 ms for 32 x 256 MiB vs 1.47-1.51 ms unskewed; re-laid out inside the
// same six pools (round 1), 2048 B beat 512 B in every one (by 0.6-2.9%); 8 KiB + 512 and
// 2 MiB + 512 are 7-12% slower.  Slots stay 16-byte aligned.
// Re-measured on the phased kernel (tools/ab_lib.py AB_TUNE, fresh processes on several boxes, gpurun_out
// r02s79-s92): slots of >= 56 MiB read faster at 512 B (one rank's share at 4 GPUs, 32 x 64 MiB: 0.320
// vs 0.330-0.334 ms; C4 0.7%, north star 0.4%, 2 ranks' share 0.6%, the C3 round's 56 MiB bf16 slots
// 0.8%), while 32 MiB slots (8 ranks' share) are 3-4% slower at 512 and 9% slower at 1024 than at 2048,
// and C2's 47.9 MiB slots are equal.  The default (kSkewAuto) therefore takes 512 B from 48 MiB up and
// 2048 B below.
size_t slot_skew_for(size_t bytes, size_t skew) {
    if (skew != kSkewAuto) return skew;
    return bytes >= (size_t(48) << 20) ? 512 : 2048;
}
// A slot's length rounded up to 4 KiB, then the skew.
size_t slot_stride(size_t bytes, size_t skew) {
    constexpr size_t a = 4096;
    return (bytes + a - 1) / a * a + slot_skew_for(bytes, skew);
}

// Range pieces ("the address span").  A GPU whose held slots span more than 48 GiB reads
// them much slower than their bytes say (C5, 128 x 1 GiB: 0.76-0.80 of HBM; the same bytes as 8 pools of
// 16 GiB: +6-13%, gpurun_out r03s19): the range layout then cuts its elements into pieces of <= 16 GiB of
// slots each (a multiple of 64 elements) and reduces them one launch after another.  Below the threshold
// (C4's 34 GiB included: no gain measured) a part is one piece.  The two sizes are the context's tuning
// (fa_tuning.piece_span_kib / piece_split_kib, taken at each fa_bucket_define): `piece` bytes of slots per
// piece (0: never cut), `split` the span above which a GPU's slots are cut.
size_t piece_len_for(size_t held, size_t cnt, size_t si, size_t piece, size_t split) {
    const size_t span = held * cnt * si;
    if (piece == 0 || held == 0 || cnt == 0 || span <= split) return std::max<size_t>(cnt, 1);
    const size_t n = (span + piece - 1) / piece;
    const size_t len = ((cnt + n - 1) / n + 63) / 64 * 64;
    return std::max<size_t>(64, std::min(len, cnt));
}
size_t piece_len_for(size_t held, size_t cnt, size_t si, const CtxTuning& t) {
    return piece_len_for(held, cnt, si, t.piece_span, t.piece_split);
}

inline bool holds(const Part& p, int g, int k) { return k >= p.c0[(size_t)g] && k < p.c1[(size_t)g]; }
// Piece j of GPU g: GPU-local elements [piece_lo, piece_lo + piece_cnt), the slot of client k at piece_ptr.
inline size_t piece_lo(const Part& p, int g, int j) { return (size_t)j * p.piece_len[(size_t)g]; }
inline size_t piece_cnt(const Part& p, int g, int j) {
    const size_t lo = piece_lo(p, g, j), n = p.cnt[(size_t)g];
    return lo >= n ? 0 : std::min(p.piece_len[(size_t)g], n - lo);
}
inline char* piece_ptr(const Part& p, int g, int k, int j) {
    const size_t held = (size_t)(p.c1[(size_t)g] - p.c0[(size_t)g]);
    return p.pool[(size_t)g] + ((size_t)j * held + (size_t)(k - p.c0[(size_t)g])) * p.stride[(size_t)g];
}
inline char* slot_ptr(const Part& p, int g, int k) { return piece_ptr(p, g, k, 0); }  // one-piece parts

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
        if (g < p.done.size() && p.done[g]) (void)hipEventDestroy(p.done[g]);
    }
    p.pool.clear();
    p.dout.clear();
    p.dout16.clear();
    p.done.clear();
}

// Makes stream s of GPU g wait for the H2D copies queued so far on its copy stream (the submits) -- only
// if copies were queued since s last waited: a cross-stream wait costs the launch ~7-10 us on the device
// (fa_reduce_part rounds, gpurun_out r02s05), which a device-resident round (slots written in place, no
// submits) must not pay.
int wait_copies(fa_ctx* ctx, int g, hipStream_t s) {
    GpuRes& r = ctx->gpu[g];
    auto it = r.waited.find(s);
    if (it != r.waited.end() ? it->second == r.copy_gen : r.copy_gen == 0) return FA_OK;
    if (r.copy_ev_gen != r.copy_gen) {
        FA_HIP(hipEventRecord(r.copy_ev, r.copy));
        r.copy_ev_gen = r.copy_gen;
    }
    FA_HIP(hipStreamWaitEvent(s, r.copy_ev, 0));
    r.waited[s] = r.copy_gen;
    return FA_OK;
}

// Copy-out runs of a range part: GPU g's output holds its shard.
void set_range_runs(Part& p, int G) {
    for (int g = 0; g < G; ++g) {
        p.runs[(size_t)g] = {Run{0, p.off[(size_t)g], p.cnt[(size_t)g]}};
        p.run_src[(size_t)g] = p.dout[(size_t)g];
    }
}

// The rs exchange state of a part: GPU g's shard holds block g of every piece, clipped to n.
void set_rs_runs(Part& p, int G, int chunks) {
    const auto pieces = rs_pieces(p.npad, G, chunks);
    for (int g = 0; g < G; ++g) {
        auto& rr = p.runs[(size_t)g];
        rr.clear();
        size_t off = 0;
        for (auto& pc : pieces) {
            const size_t q = (pc.second - pc.first) / (size_t)G;
            const size_t lo = pc.first + (size_t)g * q, hi = std::min(p.n, lo + q);
            if (hi > lo) rr.push_back(Run{off, lo, hi - lo});
            off += q;
        }
        p.run_src[(size_t)g] = p.out == FA_BF16 ? p.dout16[(size_t)g] : p.dout[(size_t)g];
    }
}

// Notes the stream the part's reduction on GPU g ran on; the copy-out orders itself after it
// (copy_output records p.done there at copy time, which covers everything enqueued so far, and waits
// only when that stream is not its own).  Nothing is recorded in the reduction's path.
int mark_done(fa_ctx*, Part& p, int g, hipStream_t s) {
    p.done_stream[(size_t)g] = s;
    return FA_OK;
}

// Range layout: enqueue the ordered chain over clients [k0, k1) of part p on GPU g, continuing the
// fp32 accumulator when k0 > 0 (accumulate on arrival) and writing the output dtype when k1 == D.
int chain_range(fa_ctx* ctx, Part& p, int g, int k0, int k1, const float* w, hipStream_t st) {
    const bool last = k1 == p.D;
    for (int j = 0; j < p.npiece[(size_t)g]; ++j) {
        const size_t lo = piece_lo(p, g, j);
        std::vector<const void*> ptrs;
        for (int k = k0; k < k1; ++k) ptrs.push_back(piece_ptr(p, g, k, j));
        const float* init = k0 > 0 ? p.acc[(size_t)g] + lo : nullptr;
        void* dst = last ? static_cast<char*>(p.dout[(size_t)g]) + lo * dsize(p.out) : (void*)(p.acc[(size_t)g] + lo);
        int rc = reduce_on(ctx, g, ctx->tuning.tu, ptrs.data(), w + k0, k1 - k0, piece_cnt(p, g, j), p.in, dst,
                           last ? p.out : FA_F32, FA_FEDAVG, p.divisor, init, st);
        if (rc) return rc;
    }
    return FA_OK;
}

// Every launch of the rs layout (the piece reductions, the bf16 rounding, the test-only emulated exchange) may
// run beside an RCCL exchange -- of the previous piece, or of the previous round.  RCCL's blocks need CU slots
// and LDS, which a persistent phased grid holds on every CU (all 160 KiB of it) for its whole launch: the
// exchange would wait for the reduction it is meant to overlap, and a phased grid that RCCL's blocks keep from
// being co-resident would spin at its meetings (769 bounded waits ran out, 24 ms per launch
// instead of 1.4).  So the rs layout never takes the phased kernel: its launches use the one-shot grid
// (walk 2, each XCD's workgroups on one contiguous eighth), which retires workgroup by workgroup and leaves
// room for RCCL's blocks as it goes.  fa_diag_rs_plan shows the resulting plan to the CPU suite.
fa::Tuning rs_launch_tuning(const fa::Tuning& tu) {
    fa::Tuning r = tu;
    if (r.walk >= 3) r.walk = 1;
    return r;
}

// FA_TEST_SHARED_DEVICE with FA_SHARD_CLIENT_RS: RCCL refuses two ranks on one device, so the
// reduce-scatter of piece [a, a + G q) is replaced by its definition -- shard g block [off, off + q) :=
// sum over h of partial_h[a + g q, a + (g + 1) q), one launch per shard on its exchange stream after every
// shard's piece reduction -- so that the rest of the layout (client dealing, pieces, padding, shard
// offsets, copy-out runs) runs on a one-GPU box.  The sum runs in ring order, as a ring reduce-scatter
// accumulates block g (it starts at rank g + 1 and ends at rank g), not rank order; RCCL's channels may
// still order it otherwise, which is why the layout's parity is a tolerance.  Never used with distinct
// devices.
int emulated_reduce_scatter(fa_ctx* ctx, Part& p, size_t a, size_t q, size_t off) {
    const int G = ctx->G;
    for (int g = 0; g < G; ++g)
        for (int h = 0; h < G; ++h) FA_HIP(hipStreamWaitEvent(ctx->gpu[(size_t)g].comm, ctx->gpu[(size_t)h].step_ev, 0));
    std::vector<const void*> ptrs((size_t)G);
    const std::vector<float> ones((size_t)G, 1.0f);
    for (int g = 0; g < G; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        for (int i = 0; i < G; ++i) ptrs[(size_t)i] = p.partial[(size_t)((g + 1 + i) % G)] + a + (size_t)g * q;
        int rc = reduce_on(ctx, g, rs_launch_tuning(ctx->tuning.tu), ptrs.data(), ones.data(), G, q, FA_F32,
                           static_cast<float*>(p.dout[(size_t)g]) + off, FA_F32, FA_FEDAVG, 1.0f, nullptr, r.comm);
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

// ------------------------------------------------------------------ small receipts read in place
//
// A small model's round is bound by stream round trips, not bytes: BASELINE C1 (LeNet-5, two owners) spent
// ~0.23 ms per round inside this library for 31 us of kernels (profiles/r05_c1_trace.json) -- an H2D copy per
// receipt segment, the reduction, a D2H copy, each a queue hop.  So a pinned receipt of a one-GPU range part
// whose D receipts total at most kHostReadMax bytes stays where it arrived (host_keep): its segments'
// device-visible addresses are noted and the finalize that ends the round has the reduction's kernels read
// them over PCIe -- straight into the reply's pinned records at fa_finalize_gather(FA_HOST_PINNED), else
// into the output before the copy-out (host_reduce) -- one launch per piece and one synchronization.  Same
// kernels, same chain, same bits.  The caller keeps pinned receipts until that finalize returns (fa.h), and
// anything before it that needs the slots -- a reduction, a state sync, a slot address, a pageable submit --
// first copies the kept receipts in (host_flush), so every other path sees exactly what the plain submit gives.
// FA_HOST_READ=0 in the environment turns it off (fa.h).

bool host_read_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("FA_HOST_READ");
        return !e || std::atoi(e) != 0;
    }();
    return on;
}

// The address a kernel on the current device reads pinned host memory at, or null.
const char* device_visible(const void* ptr) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return static_cast<const char*>(a.devicePointer) + (static_cast<const char*>(ptr) - static_cast<const char*>(a.hostPointer));
}

bool host_read_part(const fa_ctx* ctx, const Part& p) {
    return host_read_enabled() && ctx->G == 1 && !p.rs && !(ctx->flags & FA_ACCUMULATE_ON_ARRIVAL) &&
           p.npiece[0] == 1 && p.n > 0 && (size_t)p.D * p.n * dsize(p.in) <= kHostReadMax;
}

// Keeps a pinned receipt of slot `slot` where it is, if the part and every segment allow it (element-aligned,
// device-visible); false = submit it the plain way.
bool host_keep(fa_ctx* ctx, Part& p, int slot, const Gather& src) {
    if (!host_read_part(ctx, p) || (size_t)src.n > 4 * kHostReadPieces) return false;
    const size_t si = dsize(p.in);
    std::vector<Part::HostSeg> segs;
    DeviceGuard dg(ctx->gpu[0].dev);
    for (int k = 0; k < src.n; ++k) {
        if (!src.bytes[k]) continue;
        const char* h = static_cast<const char*>(src.seg[k]);
        if ((uintptr_t)h % si || src.bytes[k] % si) return false;
        const char* d = device_visible(h);
        if (!d || (uintptr_t)d % si) return false;
        segs.push_back({h, d, src.bytes[k]});
    }
    auto& slot_src = p.host_src[(size_t)slot];
    if (slot_src.empty()) ++p.n_host;
    slot_src = std::move(segs);
    return true;
}

// Copies every kept receipt into its slot (what the plain pinned submit would have done) and forgets them.
int host_flush(fa_ctx* ctx, Part& p) {
    if (p.n_host == 0) return FA_OK;
    GpuRes& r = ctx->gpu[0];
    DeviceGuard dg(r.dev);
    for (int k = 0; k < p.D; ++k) {
        auto& segs = p.host_src[(size_t)k];
        size_t o = 0;
        for (auto& sg : segs) {
            FA_HIP(hipMemcpyAsync(slot_ptr(p, 0, k) + o, sg.host, sg.bytes, hipMemcpyHostToDevice, r.copy));
            o += sg.bytes;
        }
        segs.clear();
    }
    ++r.copy_gen;
    p.n_host = 0;
    return FA_OK;
}

// Every receipt the reduction reads is kept host-side (FedAvg: all D; literal: the last one).
bool host_read_all(const Part& p) {
    if (p.n_host == 0) return false;
    if (p.mode == FA_LITERAL) {
        const int k = p.last_slot >= 0 ? p.last_slot : p.D - 1;
        return !p.host_src[(size_t)k].empty();
    }
    return p.n_host == p.D;
}

// The reduction over the kept receipts: into the part's output (dst null; the copy-out follows as usual) or
// straight into the pinned destination segments, synchronized.  kNotHostReadable (nothing launched) when the
// destination is not device-visible or element-aligned, or the pieces would be more than kHostReadPieces.
int host_reduce(fa_ctx* ctx, Part& p, const float* w, hipStream_t s, const Gather* dst) {
    const size_t si = dsize(p.in), so = dsize(p.out);
    std::vector<int> ks;  // the slots the chain reads, in order
    if (p.mode == FA_LITERAL) ks.push_back(p.last_slot >= 0 ? p.last_slot : p.D - 1);
    else for (int k = 0; k < p.D; ++k) ks.push_back(k);
    GpuRes& r = ctx->gpu[0];
    DeviceGuard dg(r.dev);
    std::vector<size_t> cuts{0, p.n};
    for (int k : ks) {
        size_t e = 0;
        for (auto& sg : p.host_src[(size_t)k]) cuts.push_back(e += sg.bytes / si);
    }
    std::vector<Part::HostSeg> out;
    if (dst) {
        size_t e = 0;
        for (int j = 0; j < dst->n; ++j) {
            if (!dst->bytes[j]) continue;
            const char* h = static_cast<const char*>(dst->seg[j]);
            const char* d = device_visible(h);
            if (!d || (uintptr_t)h % so || (uintptr_t)d % so || dst->bytes[j] % so) return kNotHostReadable;
            out.push_back({h, d, dst->bytes[j]});
            cuts.push_back(e += dst->bytes[j] / so);
        }
    }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    while (!cuts.empty() && cuts.back() > p.n) cuts.pop_back();
    if (cuts.size() - 1 > kHostReadPieces) return kNotHostReadable;
    // element e of a segment list (si bytes per element) -> its device-visible address
    auto at = [](const std::vector<Part::HostSeg>& segs, size_t e, size_t es) -> const char* {
        size_t b = e * es;
        for (auto& sg : segs) {
            if (b < sg.bytes) return sg.dev + b;
            b -= sg.bytes;
        }
        return nullptr;
    };
    hipStream_t st = s ? s : r.compute;
    const size_t npc = cuts.size() - 1, nk = ks.size();
    std::vector<const void*> ptrs(npc * nk);
    std::vector<void*> outs(npc);
    bool aligned16 = true;  // every piece 16-byte aligned at both ends of the chain: one batched launch
    for (size_t c = 0; c < npc; ++c) {
        for (size_t i = 0; i < nk; ++i) {
            ptrs[c * nk + i] = at(p.host_src[(size_t)ks[i]], cuts[c], si);
            aligned16 = aligned16 && (uintptr_t)ptrs[c * nk + i] % 16 == 0;
        }
        outs[c] = dst ? const_cast<char*>(at(out, cuts[c], so)) : static_cast<char*>(p.dout[0]) + cuts[c] * so;
        aligned16 = aligned16 && (uintptr_t)outs[c] % 16 == 0;
    }
    const fa::Tuning& tu = ctx->tuning.tu;
    if (p.mode == FA_FEDAVG && aligned16 && nk <= (size_t)fa::kMaxClients && npc <= (size_t)fa::kSegArgMax &&
        npc * nk <= (size_t)fa::kSegArgClients) {
        // the archive records are 64-byte aligned in the frames (host/wire.cpp), so the pieces of a receipt
        // and of its reply usually are: every piece in one segment launch (the same chain, the same bits)
        fa::SegArgs a{};
        const size_t V = 16 / si;
        int64_t blocks = 0;
        for (size_t c = 0; c < npc; ++c) {
            const size_t len = cuts[c + 1] - cuts[c];
            a.nc[c] = (int)nk;
            a.src0[c] = (int)(c * nk);
            a.blk0[c] = blocks;
            a.nvec[c] = (int64_t)(len / V);
            a.n[c] = (int64_t)len;
            a.out[c] = outs[c];
            blocks += std::max<int64_t>(1, (a.nvec[c] + tu.block - 1) / tu.block);
            for (size_t i = 0; i < nk; ++i) {
                a.src[c * nk + i] = ptrs[c * nk + i];
                a.w[c * nk + i] = w[ks[i]];
            }
        }
        a.nseg = (int)npc;
        a.blk0[npc] = blocks;
        FA_HIP(fa::launch_segargs(a, p.in, p.out, (int)nk, tu, st));
    } else {
        for (size_t c = 0; c < npc; ++c) {
            int rc = reduce_on(ctx, 0, tu, &ptrs[c * nk], w, (int)nk, cuts[c + 1] - cuts[c], p.in, outs[c], p.out,
                               p.mode, p.divisor, nullptr, st);
            if (rc) return rc;
        }
    }
    ++ctx->host_reads;
    if (dst) {
        FA_HIP(hipStreamSynchronize(st));
        return FA_OK;
    }
    int rc = mark_done(ctx, p, 0, st);
    if (rc) return rc;
    set_range_runs(p, 1);
    return FA_OK;
}

// Enqueue the full reduction of part p on every GPU (the ctx's streams, or `s` for a one-GPU ctx):
// range -> each GPU's shard; rs -> the clients' fp32 partials, piece by piece, each piece's RCCL
// reduce-scatter (ring over xGMI) overlapping the reduction of the next.
int reduce_part(fa_ctx* ctx, Part& p, const float* w, hipStream_t s) {
    Trace tr(p.rs ? "fa_reduce rs D %d" : "fa_reduce D %d", p.D);
    const int G = ctx->G;
    // small receipts kept where they arrived are read there only by the finalize that ends their round (the
    // caller keeps them until then); a reduction before it takes them into the slots first
    if (int rc = host_flush(ctx, p)) return rc;
    if (!p.rs) {
        for (int g = 0; g < G; ++g) {
            GpuRes& r = ctx->gpu[(size_t)g];
            DeviceGuard dg(r.dev);
            hipStream_t st = s ? s : r.compute;
            int rc = wait_copies(ctx, g, st);
            if (rc) return rc;
            for (int j = 0; j < p.npiece[(size_t)g] && !rc; ++j) {  // one launch per piece, in order
                void* dst = static_cast<char*>(p.dout[(size_t)g]) + piece_lo(p, g, j) * dsize(p.out);
                if (p.mode == FA_LITERAL) {
                    const void* last = piece_ptr(p, g, p.last_slot >= 0 ? p.last_slot : p.D - 1, j);
                    rc = reduce_on(ctx, g, ctx->tuning.tu, &last, w, 1, piece_cnt(p, g, j), p.in, dst, p.out,
                                   FA_LITERAL, p.divisor, nullptr, st);
                } else {
                    std::vector<const void*> ptrs;
                    for (int k = 0; k < p.D; ++k) ptrs.push_back(piece_ptr(p, g, k, j));
                    rc = reduce_on(ctx, g, ctx->tuning.tu, ptrs.data(), w, p.D, piece_cnt(p, g, j), p.in, dst, p.out,
                                   FA_FEDAVG, p.divisor, nullptr, st);
                }
            }
            if (rc || (rc = mark_done(ctx, p, g, st))) return rc;
        }
        set_range_runs(p, G);
        return FA_OK;
    }
    if (p.mode == FA_LITERAL) {  // the last client's GPU computes the whole bucket; nothing to exchange
        const int k = p.last_slot >= 0 ? p.last_slot : p.D - 1;
        int o = 0;
        while (!holds(p, o, k)) ++o;
        GpuRes& r = ctx->gpu[(size_t)o];
        DeviceGuard dg(r.dev);
        hipStream_t st = s ? s : r.compute;
        int rc = wait_copies(ctx, o, st);
        const void* last = slot_ptr(p, o, k);
        if (rc || (rc = reduce_on(ctx, o, ctx->tuning.tu, &last, w, 1, p.n, p.in, p.partial[(size_t)o], p.out,
                                  FA_LITERAL, p.divisor, nullptr, st)))
            return rc;
        if ((rc = mark_done(ctx, p, o, st))) return rc;
        for (int g = 0; g < G; ++g) p.runs[(size_t)g].clear();
        p.runs[(size_t)o] = {Run{0, 0, p.n}};
        p.run_src[(size_t)o] = p.partial[(size_t)o];
        return FA_OK;
    }
    const auto pieces = rs_pieces(p.npad, G, ctx->tuning.rs_chunks);
    const fa::Tuning rtu = rs_launch_tuning(ctx->tuning.tu);
    for (int g = 0; g < G; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        hipStream_t st = s ? s : r.compute;
        int rc = wait_copies(ctx, g, st);
        if (rc) return rc;
        // the previous round's exchange still reads the partials (back-to-back device-resident rounds)
        FA_HIP(hipEventRecord(r.step_ev, r.comm));
        FA_HIP(hipStreamWaitEvent(st, r.step_ev, 0));
        if (p.c1[(size_t)g] == p.c0[(size_t)g])  // a GPU without clients contributes zeros
            FA_HIP(hipMemsetAsync(p.partial[(size_t)g], 0, p.npad * 4, st));
    }
    size_t off = 0;
    for (auto& pc : pieces) {
        const size_t a = pc.first, len = pc.second - pc.first, q = len / (size_t)G;
        for (int g = 0; g < G; ++g) {
            GpuRes& r = ctx->gpu[(size_t)g];
            DeviceGuard dg(r.dev);
            hipStream_t st = s ? s : r.compute;
            const int k0 = p.c0[(size_t)g], k1 = p.c1[(size_t)g];
            if (k1 > k0) {
                std::vector<const void*> ptrs;
                for (int k = k0; k < k1; ++k) ptrs.push_back(slot_ptr(p, g, k) + a * dsize(p.in));
                int rc = reduce_on(ctx, g, rtu, ptrs.data(), w + k0, k1 - k0, len, p.in, p.partial[(size_t)g] + a,
                                   FA_F32, FA_FEDAVG, p.divisor, nullptr, st);
                if (rc) return rc;
            }
            FA_HIP(hipEventRecord(r.step_ev, st));
            FA_HIP(hipStreamWaitEvent(r.comm, r.step_ev, 0));
        }
        if (ctx->flags & FA_TEST_SHARED_DEVICE) {  // test only: every shard on one GPU, no RCCL (below)
            int rc = emulated_reduce_scatter(ctx, p, a, q, off);
            if (rc) return rc;
            off += q;
            continue;
        }
        FA_NCCL(ncclGroupStart());
        for (int g = 0; g < G; ++g) {
            GpuRes& r = ctx->gpu[(size_t)g];
            ncclResult_t e = ncclReduceScatter(p.partial[(size_t)g] + a, static_cast<float*>(p.dout[(size_t)g]) + off,
                                               q, ncclFloat32, ncclSum, r.nccl, r.comm);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail(FA_ERR_NCCL, "ncclReduceScatter: %s", ncclGetErrorString(e));
            }
        }
        FA_NCCL(ncclGroupEnd());
        off += q;
    }
    if (p.out == FA_BF16) {  // the fp32 shard rounded once to bf16 (fma(x, 1, +0) = x: the sums are never -0)
        const float one = 1.0f;
        for (int g = 0; g < G; ++g) {
            GpuRes& r = ctx->gpu[(size_t)g];
            DeviceGuard dg(r.dev);
            const void* shard = p.dout[(size_t)g];
            int rc = reduce_on(ctx, g, rtu, &shard, &one, 1, p.npad / (size_t)G, FA_F32, p.dout16[(size_t)g], FA_BF16,
                               FA_FEDAVG, 1.0f, nullptr, r.comm);
            if (rc) return rc;
        }
    }
    for (int g = 0; g < G; ++g) {
        int rc = mark_done(ctx, p, g, ctx->gpu[(size_t)g].comm);
        if (rc) return rc;
    }
    set_rs_runs(p, G, ctx->tuning.rs_chunks);
    return FA_OK;
}


// Accumulate on arrival: extend the chain over the in-order prefix of submitted slots.  Slots
// [p.reduced, j) are all submitted: one launch continues the fp32 accumulator over them (or, when j == D,
// finishes the chain into the output), after their H2D copies.  Same bits as one chain over all D.
int advance_prefix(fa_ctx* ctx, Part& p) {
    if (!(ctx->flags & FA_ACCUMULATE_ON_ARRIVAL) || p.rs || p.mode != FA_FEDAVG || p.ready) return FA_OK;
    int j = p.reduced;
    while (j < p.D && p.submitted[(size_t)j]) ++j;
    if (j == p.reduced) return FA_OK;
    Trace tr("fa_accumulate slots %d..%d", p.reduced, j);
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        int rc = wait_copies(ctx, g, r.compute);
        if (rc || (rc = chain_range(ctx, p, g, p.reduced, j, p.w.data(), r.compute))) return rc;
        if (j == p.D && (rc = mark_done(ctx, p, g, r.compute))) return rc;
    }
    p.reduced = j;
    if (j == p.D) {
        p.ready = true;
        set_range_runs(p, ctx->G);
    }
    return FA_OK;
}

// The bookkeeping of one receipt in slot `slot`: it counts for the round (a second one replaces it), with its
// weight; on arrival the chain advances over the in-order prefix.
int mark_submitted(fa_ctx* ctx, Part& p, int slot, float weight) {
    p.ready = false;  // a new receipt invalidates a finished reduction (fa_reduce_parts, a full prefix)
    if (!p.submitted[(size_t)slot]) {
        p.submitted[(size_t)slot] = 1;
        ++p.n_submitted;
    } else if (slot < p.reduced) {  // a receipt already chained was replaced: restart the chain
        p.reduced = 0;
        p.ready = false;
    }
    p.w[(size_t)slot] = weight;
    p.last_slot = slot;
    return advance_prefix(ctx, p);
}

int submit_impl(fa_ctx* ctx, int part_id, int slot, const Gather& src, float weight, bool pinned) {
    Trace tr("fa_submit part %d slot %d", part_id, slot);
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (slot < 0 || slot >= p->D) return fail(FA_ERR_ARG, "client slot %d out of range [0,%d)", slot, p->D);
    if ((rc = src.check("host source"))) return rc;
    const size_t si = dsize(p->in), total = src.total();
    if (total != p->n * si)
        return fail(FA_ERR_ARG, "part %d expects %zu bytes per receipt, got %zu", part_id, p->n * si, total);
    const bool kept = pinned && host_keep(ctx, *p, slot, src);  // a small receipt stays where it arrived
    if (!kept && (rc = host_flush(ctx, *p))) return rc;         // else the kept ones go to their slots first
    if (!kept) rc = for_each_gpu(ctx->workers.get(), ctx->G, [&](int g) -> int {
        if (!holds(*p, g, slot)) return FA_OK;  // rs: only the slot's GPU receives it
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        const size_t base = p->off[(size_t)g] * si;
        const size_t bytes = p->cnt[(size_t)g] * si;
        // bytes [x, x + len) of this GPU's range -> fn(device address, x', take) per stretch within one piece
        const size_t piece_bytes = p->piece_len[(size_t)g] * si;
        auto to_device = [&](size_t x, size_t len, const std::function<void(char*, size_t, size_t)>& fn) {
            while (len > 0) {
                const int j = (int)(x / piece_bytes);
                const size_t in = x - (size_t)j * piece_bytes, take = std::min(len, piece_bytes - in);
                fn(piece_ptr(*p, g, slot, j) + in, x, take);
                x += take;
                len -= take;
            }
        };
        if (pinned) {  // pinned segments: DMA straight from them, one copy per piece of this GPU's range
            hipError_t e = hipSuccess;
            src.pieces(base, bytes, [&](char* piece, size_t rel, size_t take) {
                to_device(rel, take, [&](char* dev, size_t x, size_t t) {
                    if (e == hipSuccess) e = hipMemcpyAsync(dev, piece + (x - rel), t, hipMemcpyHostToDevice, r.copy);
                });
            });
            ++r.copy_gen;
            FA_HIP(e);
            return FA_OK;
        }
        ++r.copy_gen;
        // Double-buffered staging: fill one pinned chunk while the other is in flight.
        for (size_t o = 0; o < bytes; o += kStageBytes) {
            const size_t b = std::min(kStageBytes, bytes - o);
            const int i = r.stage_i;
            r.stage_i ^= 1;
            FA_HIP(hipEventSynchronize(r.stage_ev[i]));
            r.pool->copy(r.stage[i], b, [&](size_t lo, size_t len, char* d) { src.copy_out(base + o + lo, len, d); });
            hipError_t e = hipSuccess;
            to_device(o, b, [&](char* dev, size_t x, size_t t) {
                if (e == hipSuccess) e = hipMemcpyAsync(dev, r.stage[i] + (x - o), t, hipMemcpyHostToDevice, r.copy);
            });
            FA_HIP(e);
            FA_HIP(hipEventRecord(r.stage_ev[i], r.copy));
        }
        return FA_OK;
    });
    if (rc) return rc;
    return mark_submitted(ctx, *p, slot, weight);
}

// Streaming ingest (fa_submit_piece_pinned): bytes [at, at + len) of a receipt -- one parameter record of an
// archive that is still arriving -- DMA'd from pinned memory into the slot's bytes on every GPU that holds
// them.  Only the copies: the slot counts as a receipt once fa_submit_commit names it.
int piece_impl(fa_ctx* ctx, int part_id, int slot, size_t at, const void* src, size_t len) {
    Trace tr("fa_submit_piece part %d slot %d", part_id, slot);
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (slot < 0 || slot >= p->D) return fail(FA_ERR_ARG, "client slot %d out of range [0,%d)", slot, p->D);
    const size_t si = dsize(p->in);
    if (at > p->n * si || len > p->n * si - at)
        return fail(FA_ERR_ARG, "piece [%zu, %zu) outside part %d's %zu bytes", at, at + len, part_id, p->n * si);
    if (len && !src) return fail(FA_ERR_ARG, "piece source is null");
    if (len == 0) return FA_OK;
    if ((rc = host_flush(ctx, *p))) return rc;  // kept receipts first: the plain path from here on
    for (int g = 0; g < ctx->G; ++g) {
        if (!holds(*p, g, slot)) continue;
        const size_t base = p->off[(size_t)g] * si, end = base + p->cnt[(size_t)g] * si;
        const size_t a = std::max(at, base), b = std::min(at + len, end);
        if (a >= b) continue;
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        const size_t piece_bytes = p->piece_len[(size_t)g] * si;
        for (size_t x = a - base; x < b - base;) {  // GPU-local bytes, one copy per range piece
            const int j = (int)(x / piece_bytes);
            const size_t in = x - (size_t)j * piece_bytes, take = std::min(b - base - x, piece_bytes - in);
            FA_HIP(hipMemcpyAsync(piece_ptr(*p, g, slot, j) + in, static_cast<const char*>(src) + (base + x - at), take,
                                  hipMemcpyHostToDevice, r.copy));
            x += take;
        }
        ++r.copy_gen;
    }
    return FA_OK;
}

// D2H of the part's output (the result leaves for new_message()) into `dst`, following the runs of its
// last reduction: straight into pinned segments, else through the pinned chunks, double-buffered.  Every
// GPU's copies wait on that GPU's done event (no device-wide synchronization); pinned copies of all GPUs
// are issued before any is waited for, staged ones run on one host thread per GPU.
int copy_output(fa_ctx* ctx, Part& p, const Gather& dst, bool pinned) {
    Trace tr("fa_copy_output n %d", (int)std::min<size_t>(p.n, 0x7fffffff));
    const size_t so = dsize(p.out);
    if (dst.total() != p.n * dsize(p.out))
        return fail(FA_ERR_ARG, "output of %zu bytes expected, destination holds %zu", p.n * dsize(p.out),
                    dst.total());
    const int G = ctx->G;
    for (int g = 0; g < G; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        hipStream_t ds = p.done_stream[(size_t)g];
        if (p.runs[(size_t)g].empty() || !ds || ds == r.compute) continue;
        DeviceGuard dg(r.dev);
        FA_HIP(hipEventRecord(p.done[(size_t)g], ds));
        FA_HIP(hipStreamWaitEvent(r.compute, p.done[(size_t)g], 0));
    }
    if (pinned) {
        for (int g = 0; g < G; ++g) {
            GpuRes& r = ctx->gpu[(size_t)g];
            DeviceGuard dg(r.dev);
            const char* src = static_cast<const char*>(p.run_src[(size_t)g]);
            hipError_t e = hipSuccess;
            for (const Run& run : p.runs[(size_t)g])
                dst.pieces(run.dst * so, run.cnt * so, [&](char* piece, size_t rel, size_t take) {
                    if (e == hipSuccess)
                        e = hipMemcpyAsync(piece, src + run.src * so + rel, take, hipMemcpyDeviceToHost, r.compute);
                });
            FA_HIP(e);
        }
        for (int g = 0; g < G; ++g) {
            DeviceGuard dg(ctx->gpu[(size_t)g].dev);
            FA_HIP(hipStreamSynchronize(ctx->gpu[(size_t)g].compute));
        }
        return FA_OK;
    }
    return for_each_gpu(ctx->workers.get(), G, [&](int g) -> int {
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        const char* src = static_cast<const char*>(p.run_src[(size_t)g]);
        for (const Run& run : p.runs[(size_t)g]) {
            const size_t bytes = run.cnt * so, base = run.dst * so;
            const char* rsrc = src + run.src * so;
            const size_t chunks = (bytes + kStageBytes - 1) / kStageBytes;
            // double-buffered: the D2H of chunk c+1 overlaps the host copy-out of chunk c
            auto issue = [&](size_t c) -> int {
                const size_t o = c * kStageBytes, b = std::min(kStageBytes, bytes - o);
                FA_HIP(hipMemcpyAsync(r.stage[c & 1], rsrc + o, b, hipMemcpyDeviceToHost, r.compute));
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
                r.pool->copy(st, b, [&](size_t lo, size_t len, char*) { dst.copy_in(base + o + lo, len, st + lo); });
            }
        }
        FA_HIP(hipStreamSynchronize(r.compute));
        return FA_OK;
    });
}

void reset_round(Part& p) {
    for (auto& h : p.host_src) h.clear();
    p.n_host = 0;
    std::fill(p.submitted.begin(), p.submitted.end(), 0);
    p.n_submitted = 0;
    p.last_slot = -1;
    p.reduced = 0;
    p.ready = false;
}

// The end of a phase: wait for the submits, reduce on every GPU (unless the round's reduction is done
// already: accumulate on arrival reached D, or fa_reduce_parts), copy the result out, reset the round.
int finalize_impl(fa_ctx* ctx, int part_id, const Gather& dst, bool pinned) {
    Trace tr("fa_finalize part %d", part_id);
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (p->mode == FA_FEDAVG && p->n_submitted != p->D)
        return fail(FA_ERR_STATE, "part %d: %d of %d clients submitted", part_id, p->n_submitted, p->D);
    if (p->n_submitted == 0) return fail(FA_ERR_STATE, "part %d: nothing submitted", part_id);
    if ((rc = dst.check("host destination"))) return rc;
    if (dst.total() != p->n * dsize(p->out))
        return fail(FA_ERR_ARG, "output of %zu bytes expected, destination holds %zu", p->n * dsize(p->out),
                    dst.total());
    if (!p->ready && p->reduced == 0 && host_read_all(*p)) {  // the kept receipts, read where they are:
        rc = pinned ? host_reduce(ctx, *p, p->w.data(), nullptr, &dst) : kNotHostReadable;  // into the reply,
        const bool into_reply = rc == FA_OK;
        if (rc == kNotHostReadable) {                                                      // or the output
            if ((rc = host_reduce(ctx, *p, p->w.data(), nullptr, nullptr)) == FA_OK) rc = copy_output(ctx, *p, dst, pinned);
        }
        if (rc == kNotHostReadable) {
            rc = FA_OK;  // more pieces than kHostReadPieces: the plain path below
        } else {
            if (rc) return rc;
            // the device output was not written this round: fa_copy_output must not hand out the last one
            if (into_reply)
                for (auto& rr : p->runs) rr.clear();
            reset_round(*p);
            return FA_OK;
        }
    }
    if (!p->ready) {
        if (p->reduced > 0) {  // accumulate on arrival: finish the chain after the reduced prefix
            for (int g = 0; g < ctx->G; ++g) {
                GpuRes& r = ctx->gpu[(size_t)g];
                DeviceGuard dg(r.dev);
                if ((rc = wait_copies(ctx, g, r.compute))) return rc;
                if ((rc = chain_range(ctx, *p, g, p->reduced, p->D, p->w.data(), r.compute))) return rc;
                if ((rc = mark_done(ctx, *p, g, r.compute))) return rc;
            }
            set_range_runs(*p, ctx->G);
        } else if ((rc = reduce_part(ctx, *p, p->w.data(), nullptr))) {
            return rc;
        }
    }
    rc = copy_output(ctx, *p, dst, pinned);
    if (rc) return rc;
    reset_round(*p);
    return FA_OK;
}

// One launch per GPU for every batchable part (FedAvg, range layout, <= kMaxClients clients, same dtypes,
// not taken by the phased kernel); the others launch one by one.  Marks the parts ready for finalize.
int reduce_parts_impl(fa_ctx* ctx, int n_parts, const int* ids, const float* const* weights, hipStream_t s) {
    Trace tr("fa_reduce_parts n %d", n_parts);
    std::vector<Part*> ps;
    for (int i = 0; i < n_parts; ++i) {
        Part* p;
        int rc = check_part(ctx, ids[i], &p);
        if (rc) return rc;
        for (Part* q : ps)
            if (q == p) return fail(FA_ERR_ARG, "part %d listed twice", ids[i]);
        ps.push_back(p);
    }
    const fa::Tuning& tu = ctx->tuning.tu;
    // group the batchable parts by dtype pair
    std::map<std::pair<int, int>, std::vector<int>> groups;
    std::vector<int> single;
    for (int i = 0; i < n_parts; ++i) {
        Part& p = *ps[(size_t)i];
        bool batch = !p.rs && p.mode == FA_FEDAVG && p.D <= fa::kMaxClients && p.n_host == 0;
        for (int g = 0; batch && g < ctx->G; ++g) {
            DeviceGuard dg(ctx->gpu[(size_t)g].dev);
            batch = p.npiece[(size_t)g] == 1 &&
                    !fa::phased_takes(p.in, p.out, (int64_t)(p.cnt[(size_t)g] * dsize(p.in) / 16), p.D, tu);
        }
        if (batch) groups[{(int)p.in, (int)p.out}].push_back(i);
        else single.push_back(i);
    }
    for (int i : single) {
        Part& p = *ps[(size_t)i];
        const float* w = weights && weights[i] ? weights[i] : p.w.data();
        int rc = reduce_part(ctx, p, w, s);
        if (rc) return rc;
        p.ready = true;
    }
    for (auto& kv : groups) {
        const fa_dtype in = (fa_dtype)kv.first.first, out = (fa_dtype)kv.first.second;
        const auto& members = kv.second;
        const size_t V = 16 / dsize(in);
        for (size_t m0 = 0; m0 < members.size(); m0 += kMaxSegments) {
            const size_t m1 = std::min(members.size(), m0 + kMaxSegments);
            for (int g = 0; g < ctx->G; ++g) {
                GpuRes& r = ctx->gpu[(size_t)g];
                DeviceGuard dg(r.dev);
                hipStream_t st = s ? s : r.compute;
                int rc = wait_copies(ctx, g, st);
                if (rc) return rc;
                // the buckets of this GPU: their ranges, clients and weights
                int nseg = 0, max_nc = 0, clients = 0;
                for (size_t m = m0; m < m1; ++m) {
                    Part& p = *ps[(size_t)members[m]];
                    if (p.cnt[(size_t)g] == 0) continue;
                    ++nseg;
                    clients += p.D;
                    max_nc = std::max(max_nc, p.D);
                }
                auto each = [&](const std::function<void(Part&, const float*, size_t)>& fn) {
                    for (size_t m = m0; m < m1; ++m) {
                        Part& p = *ps[(size_t)members[m]];
                        if (p.cnt[(size_t)g] == 0) continue;
                        fn(p, weights && weights[members[m]] ? weights[members[m]] : p.w.data(), p.cnt[(size_t)g]);
                    }
                };
                if (nseg > 0 && nseg <= fa::kSegArgMax && clients <= fa::kSegArgClients) {
                    fa::SegArgs a{};  // the whole table in the kernel arguments
                    int i = 0, c = 0;
                    int64_t blocks = 0;
                    each([&](Part& p, const float* w, size_t n) {
                        a.nc[i] = p.D;
                        a.src0[i] = c;
                        a.blk0[i] = blocks;
                        a.nvec[i] = (int64_t)(n / V);
                        a.n[i] = (int64_t)n;
                        a.out[i] = p.dout[(size_t)g];
                        blocks += std::max<int64_t>(1, (a.nvec[i] + tu.block - 1) / tu.block);
                        for (int k = 0; k < p.D; ++k, ++c) {
                            a.src[c] = slot_ptr(p, g, k);
                            a.w[c] = w[k];
                        }
                        ++i;
                    });
                    a.nseg = i;
                    a.blk0[i] = blocks;
                    FA_HIP(fa::launch_segargs(a, in, out, max_nc, tu, st));
                } else if (nseg > 0) {  // a device table, uploaded only when it changed since the last batch
                    std::vector<fa::SegDesc> tab((size_t)nseg);
                    int i = 0;
                    int64_t blocks = 0;
                    each([&](Part& p, const float* w, size_t n) {
                        fa::SegDesc& sd = tab[(size_t)i++];
                        std::memset(&sd, 0, sizeof sd);
                        sd.nvec = (int64_t)(n / V);
                        sd.n = (int64_t)n;
                        sd.nblk = std::max<int64_t>(1, (sd.nvec + tu.block - 1) / tu.block);
                        sd.blk0 = blocks;
                        blocks += sd.nblk;
                        sd.out = p.dout[(size_t)g];
                        sd.nc = p.D;
                        for (int k = 0; k < p.D; ++k) {
                            sd.src[k] = slot_ptr(p, g, k);
                            sd.w[k] = w[k];
                        }
                    });
                    const size_t bytes = sizeof(fa::SegDesc) * (size_t)nseg;
                    int ti = r.seg_last;
                    if (ti >= 0 && r.seg[ti].bytes == bytes && std::memcmp(r.seg[ti].host, tab.data(), bytes) == 0) {
                        // the same table again: its upload (and last launch) may have run on another stream
                        if (r.seg[ti].stream != st) FA_HIP(hipStreamWaitEvent(st, r.seg[ti].ev, 0));
                    } else {
                        ti = (r.seg_last + 1) % kSegRing;
                        GpuRes::SegTable& t = r.seg[ti];
                        if (!t.host) {
                            // all three or none: a ring entry is either fully usable or allocated afresh next time
                            fa::SegDesc *h = nullptr, *d = nullptr;
                            hipEvent_t ev = nullptr;
                            if (hipHostMalloc((void**)&h, sizeof(fa::SegDesc) * kMaxSegments, hipHostMallocDefault) !=
                                    hipSuccess ||
                                hipMalloc((void**)&d, sizeof(fa::SegDesc) * kMaxSegments) != hipSuccess ||
                                hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
                                if (h) (void)hipHostFree(h);
                                if (d) (void)hipFree(d);
                                (void)hipGetLastError();
                                return fail(FA_ERR_NOMEM, "segment table allocation failed");
                            }
                            t.host = h;
                            t.dev = d;
                            t.ev = ev;
                        } else {
                            // the slot's last launch (on any stream) has read the device table, and its upload
                            // the pinned one, before either is rewritten
                            FA_HIP(hipEventSynchronize(t.ev));
                        }
                        std::memcpy(t.host, tab.data(), bytes);
                        FA_HIP(hipMemcpyAsync(t.dev, t.host, bytes, hipMemcpyHostToDevice, st));
                        t.bytes = bytes;
                    }
                    FA_HIP(fa::launch_segments(r.seg[ti].dev, nseg, blocks, in, out, max_nc, tu, st));
                    FA_HIP(hipEventRecord(r.seg[ti].ev, st));
                    r.seg[ti].stream = st;
                    r.seg_last = ti;
                }
                for (size_t m = m0; m < m1; ++m)
                    if ((rc = mark_done(ctx, *ps[(size_t)members[m]], g, st))) return rc;
            }
            for (size_t m = m0; m < m1; ++m) {
                Part& p = *ps[(size_t)members[m]];
                set_range_runs(p, ctx->G);
                p.ready = true;
            }
        }
    }
    return FA_OK;
}

int tuning_from(const fa_tuning* t, CtxTuning* io) {
    if (!t) return fail(FA_ERR_ARG, "tuning is null");
    CtxTuning nt = *io;
    if (t->block) {
        if (t->block != 64 && t->block != 128 && t->block != 256) return fail(FA_ERR_ARG, "block must be 64/128/256");
        nt.tu.block = t->block;
    }
    if (t->max_blocks) nt.tu.max_blocks = t->max_blocks < 0 ? 0 : t->max_blocks;
    if (t->unroll) {
        if (t->unroll != 4 && t->unroll != 8 && t->unroll != 16) return fail(FA_ERR_ARG, "unroll must be 4/8/16");
        nt.tu.unroll = t->unroll;
    }
    if (t->load_policy) {
        if (t->load_policy < 1 || t->load_policy > 2) return fail(FA_ERR_ARG, "load_policy must be 1 or 2");
        nt.tu.load_nt = t->load_policy == 2;
    }
    if (t->store_policy) {
        if (t->store_policy < 1 || t->store_policy > 4) return fail(FA_ERR_ARG, "store_policy must be 1..4");
        nt.tu.store_policy = t->store_policy - 1;
    }
    if (t->slot_skew) {
        if (t->slot_skew < -2 || (t->slot_skew > 0 && t->slot_skew % 16))
            return fail(FA_ERR_ARG, "slot_skew must be -2 (by slot size), -1 (none) or a multiple of 16");
        nt.slot_skew = t->slot_skew == -2 ? kSkewAuto : t->slot_skew < 0 ? 0 : (size_t)t->slot_skew;
    }
    if (t->walk) {
        if (t->walk < 1 || t->walk > 6) return fail(FA_ERR_ARG, "walk must be 1..6");
        nt.tu.walk = t->walk - 1;
    }
    if (t->rs_chunks) {
        if (t->rs_chunks < 1 || t->rs_chunks > 1024) return fail(FA_ERR_ARG, "rs_chunks must be 1..1024");
        nt.rs_chunks = t->rs_chunks;
    }
    if (t->piece_span_kib) {
        if (t->piece_span_kib < -1) return fail(FA_ERR_ARG, "piece_span_kib must be -1 (never cut) or > 0");
        nt.piece_span = t->piece_span_kib < 0 ? 0 : (size_t)t->piece_span_kib << 10;
    }
    if (t->piece_split_kib) {
        if (t->piece_split_kib < -1) return fail(FA_ERR_ARG, "piece_split_kib must be -1 (always cut) or > 0");
        nt.piece_split = t->piece_split_kib < 0 ? 0 : (size_t)t->piece_split_kib << 10;
    }
    *io = nt;
    return FA_OK;
}

void tuning_to(const CtxTuning& c, fa_tuning* t) {
    t->block = c.tu.block;
    t->max_blocks = c.tu.max_blocks;
    t->unroll = c.tu.unroll;
    t->load_policy = c.tu.load_nt ? 2 : 1;
    t->store_policy = c.tu.store_policy + 1;
    t->slot_skew = c.slot_skew == kSkewAuto ? -2 : (int)c.slot_skew;
    t->walk = c.tu.walk + 1;
    t->rs_chunks = c.rs_chunks;
    t->piece_span_kib = c.piece_span ? (int)(c.piece_span >> 10) : -1;
    t->piece_split_kib = c.piece_split ? (int)(c.piece_split >> 10) : -1;
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
    std::lock_guard<std::mutex> g(g_defaults_mu);
    return tuning_from(t, &g_defaults);
}

int fa_get_tuning(fa_tuning* t) {
    g_err.clear();
    if (!t) return fail(FA_ERR_ARG, "tuning is null");
    tuning_to(defaults(), t);
    return FA_OK;
}

int fa_ctx_set_tuning(fa_ctx* ctx, const fa_tuning* t) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    return tuning_from(t, &ctx->tuning);
}

int fa_ctx_get_tuning(fa_ctx* ctx, fa_tuning* t) {
    g_err.clear();
    if (!ctx || !t) return fail(FA_ERR_ARG, "ctx or tuning is null");
    tuning_to(ctx->tuning, t);
    return FA_OK;
}

int fa_rs_segments(size_t n, int n_gpus, int chunks, int gpu, size_t* lo_hi, int cap) {
    g_err.clear();
    if (n_gpus < 1 || gpu < 0 || gpu >= n_gpus || chunks < 1) return fail(FA_ERR_ARG, "bad n_gpus/gpu/chunks");
    const size_t unit = (size_t)n_gpus * kShardUnit, npad = (n + unit - 1) / unit * unit;
    int k = 0;
    for (auto& pc : rs_pieces(npad, n_gpus, chunks)) {
        const size_t q = (pc.second - pc.first) / (size_t)n_gpus, lo = pc.first + (size_t)gpu * q;
        if (lo_hi && k < cap) {
            lo_hi[2 * k] = lo;
            lo_hi[2 * k + 1] = lo + q;
        }
        ++k;
    }
    return k;
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
    if (flags & ~(FA_SHARD_RANGE | FA_SHARD_CLIENT_RS | FA_ACCUMULATE_ON_ARRIVAL | FA_TEST_SHARED_DEVICE))
        return fail(FA_ERR_ARG, "unknown flags 0x%x", flags);
    if ((flags & FA_SHARD_RANGE) && (flags & FA_SHARD_CLIENT_RS))
        return fail(FA_ERR_ARG, "FA_SHARD_RANGE and FA_SHARD_CLIENT_RS exclude each other");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(FA_ERR_NODEV, "no HIP device visible");
    if (n_gpus < 1 || !device_ids) return fail(FA_ERR_ARG, "n_gpus=%d with %d device(s) visible", n_gpus, count);
    if (n_gpus > 1 && !(flags & (FA_SHARD_RANGE | FA_SHARD_CLIENT_RS)))
        return fail(FA_ERR_ARG, "n_gpus > 1 needs FA_SHARD_RANGE or FA_SHARD_CLIENT_RS");
    for (int g = 0; g < n_gpus; ++g) {
        const int d = device_ids[g];
        if (d < 0 || d >= count) return fail(FA_ERR_ARG, "device id %d out of range [0,%d)", d, count);
        for (int h = 0; h < g && !(flags & FA_TEST_SHARED_DEVICE); ++h)
            if (device_ids[h] == d) return fail(FA_ERR_ARG, "device id %d listed twice", d);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) return fail(FA_ERR_NODEV, "device %d unreadable", d);
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(FA_ERR_NODEV, "device %d is %s; libfa.so is built for gfx950 only", d, prop.gcnArchName);
    }
    fa_ctx* ctx = new fa_ctx();
    ctx->G = n_gpus;
    ctx->flags = flags;
    ctx->tuning = defaults();
    ctx->gpu.resize((size_t)n_gpus);
    const int threads = std::max(1, default_copy_threads() / n_gpus);
    // The exchange stream exists only where there is an exchange (the rs layout).  A high-priority stream
    // costs every launch on the device ~2% while its queue lives, even idle (the c4 workload 0.875 -> 0.858
    // of spec once one more high-priority stream had been created, and it stays so after the stream is
    // destroyed -- the runtime keeps the queue; tools/order_effect.py, gpurun_out r05s27-s29).
    const bool need_comm = (flags & FA_SHARD_CLIENT_RS) != 0;
    for (int g = 0; g < n_gpus; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        r.dev = device_ids[g];
        DeviceGuard dg(r.dev);
        int prio_lo = 0, prio_hi = 0;
        if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = 0;
        bool ok = hipStreamCreateWithFlags(&r.compute, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&r.copy, hipStreamNonBlocking) == hipSuccess &&
                  // the rs exchange's stream at the highest priority: its RCCL blocks are dispatched ahead of
                  // the next piece's reduction waiting on the compute stream
                  (!need_comm || hipStreamCreateWithPriority(&r.comm, hipStreamNonBlocking, prio_hi) == hipSuccess) &&
                  hipEventCreateWithFlags(&r.copy_ev, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&r.step_ev, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < 2; ++i)
            ok = hipHostMalloc((void**)&r.stage[i], kStageBytes, hipHostMallocDefault) == hipSuccess &&
                 hipEventCreateWithFlags(&r.stage_ev[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            fa_destroy(ctx);
            return fail(FA_ERR_NOMEM, "stream/staging setup failed on device %d", device_ids[g]);
        }
        r.pool.reset(new CopyPool(threads));
    }
    if (n_gpus > 1) ctx->workers.reset(new CopyPool(n_gpus));
    if ((flags & FA_SHARD_CLIENT_RS) && !(flags & FA_TEST_SHARED_DEVICE)) {  // one RCCL communicator per GPU
        std::vector<ncclComm_t> comms((size_t)n_gpus, nullptr);
        const ncclResult_t e = ncclCommInitAll(comms.data(), n_gpus, device_ids);
        if (e != ncclSuccess) {
            fa_destroy(ctx);
            return fail(FA_ERR_NCCL, "ncclCommInitAll over %d GPU(s): %s", n_gpus, ncclGetErrorString(e));
        }
        for (int g = 0; g < n_gpus; ++g) ctx->gpu[(size_t)g].nccl = comms[(size_t)g];
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
        if (r.comm) (void)hipStreamSynchronize(r.comm);
        if (r.nccl) (void)ncclCommDestroy(r.nccl);
        for (int i = 0; i < 2; ++i) {
            if (r.stage[i]) (void)hipHostFree(r.stage[i]);
            if (r.stage_ev[i]) (void)hipEventDestroy(r.stage_ev[i]);
        }
        for (auto& t : r.seg) {
            if (t.host) (void)hipHostFree(t.host);
            if (t.dev) (void)hipFree(t.dev);
            if (t.ev) (void)hipEventDestroy(t.ev);
        }
        for (hipEvent_t e : {r.copy_ev, r.step_ev})
            if (e) (void)hipEventDestroy(e);
        if (r.scratch) (void)hipFree(r.scratch);
        if (r.crc_host) (void)hipHostFree(r.crc_host);
        if (r.crc_dev) (void)hipFree(r.crc_dev);
        for (hipStream_t s : {r.compute, r.copy, r.comm})
            if (s) {
                fa::phased_release_stream(r.dev, s);  // its phased counter slot goes to the next new stream
                (void)hipStreamDestroy(s);
            }
        r.pool.reset();
    }
    ctx->workers.reset();
    delete ctx;
}

int fa_bucket_define(fa_ctx* ctx, int part_id, size_t n_elems, fa_dtype in, fa_dtype out, int n_clients,
                     fa_mode mode) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    if (!dvalid(in) || !dvalid(out)) return fail(FA_ERR_ARG, "bad dtype");
    if (mode != FA_FEDAVG && mode != FA_LITERAL) return fail(FA_ERR_ARG, "bad mode");
    if (n_clients < 1) return fail(FA_ERR_ARG, "n_clients must be >= 1");
    const bool rs = (ctx->flags & FA_SHARD_CLIENT_RS) != 0;
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
    p.rs = rs;
    p.w.assign((size_t)n_clients, 0.0f);
    p.submitted.assign((size_t)n_clients, 0);
    p.host_src.assign((size_t)n_clients, {});
    const size_t G = (size_t)ctx->G;
    const bool eager = (ctx->flags & FA_ACCUMULATE_ON_ARRIVAL) && !rs && mode == FA_FEDAVG;
    if (rs) {
        const size_t unit = G * kShardUnit;
        p.npad = (n_elems + unit - 1) / unit * unit;
        for (size_t g = 0; g < G; ++g) {
            int c0, c1;
            client_bounds(n_clients, (int)G, (int)g, &c0, &c1);
            p.c0.push_back(c0);
            p.c1.push_back(c1);
            p.off.push_back(0);
            p.cnt.push_back(n_elems);
        }
    } else {
        // Range shards: multiples of 64 elements so every shard keeps 16-B phase 0.
        size_t per = ((n_elems + G - 1) / G + kShardUnit - 1) / kShardUnit * kShardUnit;
        for (size_t g = 0; g < G; ++g) {
            size_t lo = std::min(n_elems, g * per), hi = std::min(n_elems, lo + per);
            p.off.push_back(lo);
            p.cnt.push_back(hi - lo);
            p.c0.push_back(0);
            p.c1.push_back(n_clients);
        }
    }
    p.pool.assign(G, nullptr);
    p.dout.assign(G, nullptr);
    p.dout16.assign(G, nullptr);
    p.stride.assign(G, 0);
    p.npiece.assign(G, 1);
    p.piece_len.assign(G, 0);
    p.partial.assign(G, nullptr);
    p.acc.assign(G, nullptr);
    p.done.assign(G, nullptr);
    p.runs.assign(G, {});
    p.done_stream.assign(G, nullptr);
    p.run_src.assign(G, nullptr);
    for (size_t g = 0; g < G; ++g) {
        DeviceGuard dg(ctx->gpu[g].dev);
        if (hipEventCreateWithFlags(&p.done[g], hipEventDisableTiming) != hipSuccess) {
            free_part(ctx, p);
            return fail(FA_ERR_HIP, "event creation failed");
        }
        const size_t held = (size_t)(p.c1[g] - p.c0[g]);
        if (rs) {
            p.npiece[g] = 1;
            p.piece_len[g] = p.npad;
        } else {
            p.piece_len[g] = piece_len_for(held, p.cnt[g], dsize(in), ctx->tuning);
            p.npiece[g] = p.cnt[g] ? (int)((p.cnt[g] + p.piece_len[g] - 1) / p.piece_len[g]) : 1;
        }
        p.stride[g] = slot_stride(p.piece_len[g] * dsize(in), ctx->tuning.slot_skew);
        // one allocation: the slots (piece-major: piece j of every held slot, then piece j+1), then the
        // output (range: cnt of `out`; rs: the fp32 shard, + its bf16 rounding for a bf16 output), then the
        // rs partial or the eager accumulator, each 4 KiB aligned
        const size_t shard16_bytes = rs && out == FA_BF16 ? (p.npad / G * 2 + 4095) / 4096 * 4096 : 0;
        const size_t out_bytes = rs ? p.npad / G * 4 : p.cnt[g] * dsize(out);
        const size_t out_off = (size_t)p.npiece[g] * held * p.stride[g];
        const size_t extra_off = out_off + (out_bytes + 4095) / 4096 * 4096 + shard16_bytes;
        const size_t extra_bytes = rs ? p.npad * 4 : eager ? p.cnt[g] * 4 : 0;
        const size_t bytes = std::max<size_t>(1, extra_off + extra_bytes);
        if (hipMalloc((void**)&p.pool[g], bytes) != hipSuccess) {
            (void)hipGetLastError();
            free_part(ctx, p);
            return fail(FA_ERR_NOMEM, "device alloc of %zu B failed on GPU %zu", bytes, g);
        }
        p.dout[g] = p.pool[g] + out_off;
        if (shard16_bytes) p.dout16[g] = p.pool[g] + out_off + (out_bytes + 4095) / 4096 * 4096;
        if (rs) {
            p.partial[g] = reinterpret_cast<float*>(p.pool[g] + extra_off);
            // the padding of every slot stays zero: the pieces past n reduce to 0
            for (size_t k = 0; k < held && p.npad > n_elems; ++k)
                if (hipMemset(p.pool[g] + k * p.stride[g] + n_elems * dsize(in), 0, (p.npad - n_elems) * dsize(in)) !=
                    hipSuccess) {
                    free_part(ctx, p);
                    return fail(FA_ERR_HIP, "slot padding memset failed");
                }
        } else if (eager) {
            p.acc[g] = reinterpret_cast<float*>(p.pool[g] + extra_off);
        }
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

int fa_submit_piece_pinned(fa_ctx* ctx, int part_id, int client_slot, size_t byte_offset, const void* host_src,
                           size_t bytes) {
    g_err.clear();
    return piece_impl(ctx, part_id, client_slot, byte_offset, host_src, bytes);
}

int fa_submit_commit(fa_ctx* ctx, int part_id, int client_slot, float weight) {
    g_err.clear();
    Trace tr("fa_submit_commit part %d slot %d", part_id, client_slot);
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (client_slot < 0 || client_slot >= p->D)
        return fail(FA_ERR_ARG, "client slot %d out of range [0,%d)", client_slot, p->D);
    if (p->host_src[(size_t)client_slot].size()) {  // an earlier receipt kept in place would shadow the pieces
        p->host_src[(size_t)client_slot].clear();
        --p->n_host;
    }
    return mark_submitted(ctx, *p, client_slot, weight);
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

int fa_reduce_parts(fa_ctx* ctx, int n_parts, const int* part_ids, const float* const* h_weights, void* hip_stream) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    if (n_parts < 0 || (n_parts > 0 && !part_ids)) return fail(FA_ERR_ARG, "bad part list");
    if (hip_stream && ctx->G != 1) return fail(FA_ERR_ARG, "an explicit stream needs a single-GPU ctx");
    for (int i = 0; i < n_parts; ++i) {
        Part* p;
        int rc = check_part(ctx, part_ids[i], &p);
        if (rc) return rc;
        if (p->mode == FA_FEDAVG && p->n_submitted != p->D && !(h_weights && h_weights[i]))
            return fail(FA_ERR_STATE, "part %d: %d of %d clients submitted", part_ids[i], p->n_submitted, p->D);
    }
    return reduce_parts_impl(ctx, n_parts, part_ids, h_weights, static_cast<hipStream_t>(hip_stream));
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
    if (!holds(*p, gpu, client_slot))
        return fail(FA_ERR_ARG, "client slot %d is not held by GPU %d (rs layout: slots [%d,%d))", client_slot, gpu,
                    p->c0[(size_t)gpu], p->c1[(size_t)gpu]);
    if (p->npiece[(size_t)gpu] > 1)
        return fail(FA_ERR_STATE, "part %d is held as %d pieces on GPU %d: use fa_bucket_piece", part_id,
                    p->npiece[(size_t)gpu], gpu);
    if ((rc = host_flush(ctx, *p))) return rc;  // the caller may read the slot: the kept receipts land first
    if (d_ptr) *d_ptr = slot_ptr(*p, gpu, client_slot);
    if (n_elems) *n_elems = p->cnt[(size_t)gpu];
    if (elem_offset) *elem_offset = p->off[(size_t)gpu];
    return FA_OK;
}

int fa_bucket_pieces(fa_ctx* ctx, int part_id, int gpu, int* n_pieces) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    if (!n_pieces) return fail(FA_ERR_ARG, "n_pieces is null");
    *n_pieces = p->npiece[(size_t)gpu];
    return FA_OK;
}

int fa_bucket_piece(fa_ctx* ctx, int part_id, int gpu, int piece, int client_slot, void** d_ptr, size_t* n_elems,
                    size_t* elem_offset) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    if (piece < 0 || piece >= p->npiece[(size_t)gpu]) return fail(FA_ERR_ARG, "piece %d out of range", piece);
    if (client_slot < 0 || client_slot >= p->D) return fail(FA_ERR_ARG, "client slot %d out of range", client_slot);
    if (!holds(*p, gpu, client_slot))
        return fail(FA_ERR_ARG, "client slot %d is not held by GPU %d (rs layout: slots [%d,%d))", client_slot, gpu,
                    p->c0[(size_t)gpu], p->c1[(size_t)gpu]);
    if ((rc = host_flush(ctx, *p))) return rc;
    if (d_ptr) *d_ptr = piece_ptr(*p, gpu, client_slot, piece);
    if (n_elems) *n_elems = piece_cnt(*p, gpu, piece);
    if (elem_offset) *elem_offset = p->off[(size_t)gpu] + piece_lo(*p, gpu, piece);
    return FA_OK;
}

int fa_bucket_output(fa_ctx* ctx, int part_id, int gpu, void** d_ptr) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (gpu < 0 || gpu >= ctx->G) return fail(FA_ERR_ARG, "gpu %d out of range", gpu);
    if (d_ptr) *d_ptr = p->dout[(size_t)gpu];
    return FA_OK;
}

int fa_bucket_progress(fa_ctx* ctx, int part_id, int* n_submitted, int* n_reduced) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (n_submitted) *n_submitted = p->n_submitted;
    if (n_reduced) *n_reduced = p->ready ? p->D : p->reduced;
    return FA_OK;
}

int fa_bucket_host_read(fa_ctx* ctx, int part_id, int* kept) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (!kept) return fail(FA_ERR_ARG, "kept is null");
    *kept = !p->ready && p->reduced == 0 && host_read_all(*p) ? 1 : 0;
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

int fa_output_crc32(fa_ctx* ctx, int part_id, int n_segments, const size_t* bytes, uint32_t* crcs) {
    g_err.clear();
    Trace tr("fa_output_crc32 part %d n %d", part_id, n_segments);
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (n_segments < 0 || (n_segments > 0 && (!bytes || !crcs))) return fail(FA_ERR_ARG, "bad segment list");
    const size_t so = dsize(p->out);
    size_t total = 0;
    for (int k = 0; k < n_segments; ++k) total += bytes[k];
    if (total != p->n * so)
        return fail(FA_ERR_ARG, "segments hold %zu bytes, part %d's output %zu", total, part_id, p->n * so);
    bool any = false;
    for (auto& rr : p->runs) any = any || !rr.empty();
    if (!any && p->n) return fail(FA_ERR_STATE, "part %d has no device output", part_id);
    // segment k = output bytes [seg_lo[k], seg_lo[k] + bytes[k]); each GPU's runs map bucket bytes to its
    // output buffer: the pieces are their intersections, in segment order on every GPU
    std::vector<size_t> seg_lo((size_t)n_segments + 1, 0);
    for (int k = 0; k < n_segments; ++k) seg_lo[(size_t)k + 1] = seg_lo[(size_t)k] + bytes[k];
    struct Piece {
        size_t dev_off, len;  // bytes of the GPU's output buffer
        int seg;
        size_t end;           // the piece's end, relative to its segment's start
    };
    std::vector<std::vector<Piece>> pieces((size_t)ctx->G);
    for (int g = 0; g < ctx->G; ++g)
        for (const Run& run : p->runs[(size_t)g]) {
            const size_t a = run.dst * so, b = (run.dst + run.cnt) * so;  // bucket bytes of this run
            int k = (int)(std::upper_bound(seg_lo.begin(), seg_lo.end(), a) - seg_lo.begin()) - 1;
            for (size_t x = a; x < b && k < n_segments; ++k) {
                const size_t e = std::min(b, seg_lo[(size_t)k + 1]);
                if (e > x) pieces[(size_t)g].push_back(Piece{run.src * so + (x - a), e - x, k, e - seg_lo[(size_t)k]});
                x = std::max(x, e);
            }
        }
    std::vector<uint32_t> raw;  // R(piece, 0) per piece, all GPUs in order
    for (int g = 0; g < ctx->G; ++g) {
        auto& pc = pieces[(size_t)g];
        if (pc.empty()) continue;
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        const size_t np = pc.size();
        const size_t need = np * 16 + (np + 1) * 8 + np * 4 + 64;
        if (r.crc_bytes < need) {
            if (r.crc_host) (void)hipHostFree(r.crc_host);
            if (r.crc_dev) (void)hipFree(r.crc_dev);
            r.crc_host = r.crc_dev = nullptr;
            r.crc_bytes = 0;
            const size_t cap = std::max<size_t>(need, 64u << 10);
            if (hipHostMalloc((void**)&r.crc_host, cap, hipHostMallocDefault) != hipSuccess ||
                hipMalloc((void**)&r.crc_dev, cap) != hipSuccess) {
                (void)hipGetLastError();
                if (r.crc_host) (void)hipHostFree(r.crc_host);
                r.crc_host = nullptr;
                return fail(FA_ERR_NOMEM, "crc table allocation failed");
            }
            r.crc_bytes = cap;
        }
        uint64_t* h_off = reinterpret_cast<uint64_t*>(r.crc_host);
        uint64_t* h_len = h_off + np;
        uint64_t* h_chunk0 = h_len + np;
        uint32_t* h_out = reinterpret_cast<uint32_t*>(h_chunk0 + np + 1);
        uint64_t chunks = 0;
        for (size_t i = 0; i < np; ++i) {
            h_off[i] = pc[i].dev_off;
            h_len[i] = pc[i].len;
            h_chunk0[i] = chunks;
            chunks += (pc[i].len + fa::kCrcChunkBytes - 1) / fa::kCrcChunkBytes;
        }
        h_chunk0[np] = chunks;
        const size_t table = (np * 2 + np + 1) * 8;
        uint64_t* d_off = reinterpret_cast<uint64_t*>(r.crc_dev);
        uint32_t* d_out = reinterpret_cast<uint32_t*>(d_off + np * 3 + 1);
        // after the reduction that wrote the output (on whatever stream it ran)
        hipStream_t ds = p->done_stream[(size_t)g];
        if (ds && ds != r.compute) {
            FA_HIP(hipEventRecord(p->done[(size_t)g], ds));
            FA_HIP(hipStreamWaitEvent(r.compute, p->done[(size_t)g], 0));
        }
        FA_HIP(hipMemcpyAsync(d_off, h_off, table, hipMemcpyHostToDevice, r.compute));
        FA_HIP(hipMemsetAsync(d_out, 0, np * 4, r.compute));
        FA_HIP(fa::launch_crc32_pieces(p->run_src[(size_t)g], d_off, d_off + np, d_off + 2 * np, (int)np, chunks, d_out,
                                       r.compute));
        FA_HIP(hipMemcpyAsync(h_out, d_out, np * 4, hipMemcpyDeviceToHost, r.compute));
        FA_HIP(hipStreamSynchronize(r.compute));
        raw.insert(raw.end(), h_out, h_out + np);
    }
    // join a segment's pieces: R(seg, ~0) = shift(~0, L) ^ XOR_i shift(R(piece_i, 0), L - end_i); CRC = ~R
    for (int k = 0; k < n_segments; ++k) crcs[k] = fa::crc32_mulmod(fa::crc32_x8n(bytes[k]), 0xFFFFFFFFu);
    size_t i = 0;
    for (int g = 0; g < ctx->G; ++g)
        for (const Piece& pc : pieces[(size_t)g]) {
            const size_t L = bytes[pc.seg];
            crcs[pc.seg] ^= fa::crc32_mulmod(fa::crc32_x8n(L - pc.end), raw[i++]);
        }
    for (int k = 0; k < n_segments; ++k) crcs[k] = ~crcs[k];
    return FA_OK;
}

int fa_copy_output(fa_ctx* ctx, int part_id, void* host_dst) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (!host_dst && p->n) return fail(FA_ERR_ARG, "host_dst is null");
    bool any = false;
    for (auto& rr : p->runs) any = any || !rr.empty();
    if (!any && p->n) return fail(FA_ERR_STATE, "part %d has not been reduced", part_id);
    const size_t bytes = p->n * dsize(p->out);
    const void* segs[1] = {host_dst};
    return copy_output(ctx, *p, Gather{1, segs, &bytes}, false);
}

int fa_sync(fa_ctx* ctx) {
    g_err.clear();
    if (!ctx) return fail(FA_ERR_ARG, "ctx is null");
    for (auto& r : ctx->gpu) {
        DeviceGuard dg(r.dev);
        FA_HIP(hipStreamSynchronize(r.copy));
        FA_HIP(hipStreamSynchronize(r.compute));
        if (r.comm) FA_HIP(hipStreamSynchronize(r.comm));
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
    const int dev = ctx ? ctx->gpu[(size_t)gpu].dev : gpu;
    if (!s && ctx) s = ctx->gpu[(size_t)gpu].compute;
    DeviceGuard dg(dev);
    const CtxTuning tu = ctx ? ctx->tuning : defaults();
    return reduce_on(ctx, ctx ? gpu : 0, tu.tu, d_clients, h_weights, D, n, in, d_out, out, mode,
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
    if (!s && ctx) s = ctx->gpu[(size_t)gpu].compute;
    if (ctx) {
        DeviceGuard dg(ctx->gpu[(size_t)gpu].dev);
        return sync_on(ctx, gpu, ctx->tuning.tu, d_clients, h_weights, D, n, dt, s);
    }
    const CtxTuning tu = defaults();
    return sync_on(nullptr, gpu, tu.tu, d_clients, h_weights, D, n, dt, s);
}

int fa_sync_part(fa_ctx* ctx, int part_id, const float* h_weights, void* hip_stream) {
    g_err.clear();
    Part* p;
    int rc = check_part(ctx, part_id, &p);
    if (rc) return rc;
    if (p->mode != FA_FEDAVG) return fail(FA_ERR_ARG, "part %d is not a FedAvg part", part_id);
    if (p->rs) return fail(FA_ERR_ARG, "part %d: state sync needs every client on every GPU (range layout)", part_id);
    if (hip_stream && ctx->G != 1) return fail(FA_ERR_ARG, "an explicit stream needs a single-GPU ctx");
    const float* w = h_weights ? h_weights : p->w.data();
    if ((rc = host_flush(ctx, *p))) return rc;  // the sync works on the slots
    std::vector<void*> ptrs((size_t)p->D);
    for (int g = 0; g < ctx->G; ++g) {
        GpuRes& r = ctx->gpu[(size_t)g];
        DeviceGuard dg(r.dev);
        hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : r.compute;
        if ((rc = wait_copies(ctx, g, st))) return rc;  // the slots' submits land first
        for (int j = 0; j < p->npiece[(size_t)g]; ++j) {
            for (int k = 0; k < p->D; ++k) ptrs[(size_t)k] = piece_ptr(*p, g, k, j);
            if ((rc = sync_on(ctx, g, ctx->tuning.tu, ptrs.data(), w, p->D, piece_cnt(*p, g, j), p->in, st))) return rc;
        }
    }
    return FA_OK;
}

int fa_release_stream(int device, void* hip_stream) {
    g_err.clear();
    int n = 0;
    FA_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(FA_ERR_ARG, "device %d", device);
    fa::phased_release_stream(device, static_cast<hipStream_t>(hip_stream));
    return FA_OK;
}

int fa_phased_timeouts(int device, uint64_t* count) {
    g_err.clear();
    if (!count) return fail(FA_ERR_ARG, "count is null");
    if (device < 0) return fail(FA_ERR_ARG, "device %d", device);
    FA_HIP(fa::phased_timeouts(device, count));
    return FA_OK;
}

namespace {
// a 256-byte device word per device for the read diagnostics' never-taken store
int read_sink(float** out) {
    static float* sinks[64] = {};
    static std::mutex mu;
    int dev = 0;
    FA_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(FA_ERR_ARG, "device %d", dev);
    std::lock_guard<std::mutex> lk(mu);
    if (!sinks[dev]) FA_HIP(hipMalloc((void**)&sinks[dev], 256));
    *out = sinks[dev];
    return FA_OK;
}

int read_table(const void* const* d_bufs, int nc, size_t n, fa::ClientTable* t) {
    if (!d_bufs || nc < 1 || nc > fa::kMaxClients || n % 4) return fail(FA_ERR_ARG, "bad read-stream arguments");
    for (int k = 0; k < nc; ++k) {
        if (!d_bufs[k] || (uintptr_t)d_bufs[k] % 16) return fail(FA_ERR_ARG, "buffer %d null or misaligned", k);
        t->src[k] = d_bufs[k];
    }
    return FA_OK;
}
}  // namespace

// Diagnostic, not part of the ABI in fa.h: one read-stream probe launch over nc device buffers of n fp32
// elements each (16-byte aligned, n a multiple of 4, nc <= 128) on `hip_stream`, enqueued; bench.py times
// it with events on that stream (roofline.read_stream_peak).
extern "C" int fa_diag_read_stream(const void* const* d_bufs, int nc, size_t n, void* hip_stream) {
    g_err.clear();
    fa::ClientTable t{};
    float* sink = nullptr;
    int rc;
    if ((rc = read_table(d_bufs, nc, n, &t)) || (rc = read_sink(&sink))) return rc;
    FA_HIP(fa::launch_read_probe(t, nc, (int64_t)(n / 4), sink, static_cast<hipStream_t>(hip_stream)));
    return FA_OK;
}

// Diagnostic, not part of the ABI in fa.h: the independent read ceiling -- a plain grid-stride read of the
// same buffers (grid workgroups of 256 lanes, `unroll` 8 or 16 non-temporal 16-byte loads in flight per
// lane, buffer after buffer), none of the product kernels' structure; bench.py times it on the launch stream
// (roofline.read_stream_peak_independent).
extern "C" int fa_diag_read_plain(const void* const* d_bufs, int nc, size_t n, int grid, int unroll,
                                  void* hip_stream) {
    g_err.clear();
    if (grid < 1 || grid > (1 << 20) || (unroll != 8 && unroll != 16)) return fail(FA_ERR_ARG, "bad grid or unroll");
    fa::ClientTable t{};
    float* sink = nullptr;
    int rc;
    if ((rc = read_table(d_bufs, nc, n, &t)) || (rc = read_sink(&sink))) return rc;
    FA_HIP(fa::launch_read_plain(t, nc, (int64_t)(n / 4), grid, unroll, sink, static_cast<hipStream_t>(hip_stream)));
    return FA_OK;
}

// Diagnostic, not part of the ABI in fa.h: the independent in-place read+write ceiling -- every buffer read
// and written back where it lies (x * 1), a plain grid-stride walk buffer after buffer (grid workgroups of 256
// lanes, `unroll` 8 or 16 non-temporal 16-byte loads in flight per lane, plain or non-temporal stores); bench.py
// times it on the sync legs' own slots (copy_ceiling_independent).  The values are left as they were.
extern "C" int fa_diag_rw_plain(const void* const* d_bufs, int nc, size_t n, int grid, int unroll, int nt,
                                void* hip_stream) {
    g_err.clear();
    if (grid < 1 || grid > (1 << 20) || (unroll != 8 && unroll != 16)) return fail(FA_ERR_ARG, "bad grid or unroll");
    fa::ClientTable t{};
    int rc;
    if ((rc = read_table(d_bufs, nc, n, &t))) return rc;
    FA_HIP(fa::launch_rw_plain(t, nc, (int64_t)(n / 4), grid, unroll, nt != 0, static_cast<hipStream_t>(hip_stream)));
    return FA_OK;
}

// Diagnostic, not part of the ABI in fa.h: how many reductions of this context read their receipts in place
// (small pinned receipts, host_reduce); -1 for a null context.
extern "C" long long fa_diag_host_reads(fa_ctx* ctx) { return ctx ? (long long)ctx->host_reads : -1; }

// GPUs of the context that hold an exchange stream: the rs layout's high-priority stream, none otherwise
// (fa_create: a second high-priority stream on a device slows every later launch there).
extern "C" int fa_diag_exchange_streams(fa_ctx* ctx) {
    if (!ctx) return -1;
    int n = 0;
    for (auto& r : ctx->gpu) n += r.comm ? 1 : 0;
    return n;
}

// Diagnostic, not part of the ABI in fa.h: the per-workgroup timeline of the last phased launch on `device`
// when the process runs with FA_TIMELINE=1 (tools/timeline.py).
extern "C" int fa_diag_phased_timeline(int device, unsigned long long* out, int cap) {
    return out && cap > 0 ? fa::phased_timeline(device, out, cap) : -1;
}

// Diagnostic, not part of the ABI in fa.h: the phased kernel's counter slot of `hip_stream` on `device`
// (assigned now if the stream has none, exactly as its first phased launch would); *own = 1 when the slot is
// the stream's alone, 0 for a hashed slot shared with other streams (tests/test_gpu_parity.py).
extern "C" int fa_diag_phased_slot(int device, void* hip_stream, int* own) {
    g_err.clear();
    bool o = false;
    const int slot = fa::phased_slot(device, static_cast<hipStream_t>(hip_stream), &o);
    if (slot < 0) return fail(FA_ERR_ARG, "device %d", device);
    if (own) *own = o ? 1 : 0;
    return slot;
}

// Diagnostic, not part of the ABI in fa.h: how many of the owned counter slots are taken on `device` (a
// destroyed context gives its streams' slots back).
extern "C" int fa_diag_phased_owned(int device) {
    g_err.clear();
    const int n = fa::phased_owned_slots(device);
    return n < 0 ? fail(FA_ERR_ARG, "device %d", device) : n;
}

// Diagnostic, not part of the ABI in fa.h: the kernel plan (fa::plan_chain) of one FedAvg chain launch of n
// elements (16-byte aligned) and nc clients under fa_tuning.walk `walk` (0 = the process default) on a chip of
// `cus` CUs: *kind 0 one-shot grid, 1 one element per lane, 2 phased persistent grid of *phases phases (more
// than one: chip-wide meetings).  Pure host arithmetic.
extern "C" int fa_diag_plan_chain(int in, int out, size_t n, int nc, int walk, int cus, int* kind, long long* phases) {
    g_err.clear();
    if (!dvalid(in) || !dvalid(out) || walk < 0 || walk > 6 || cus < 0 || nc < 0)
        return fail(FA_ERR_ARG, "bad plan arguments");
    fa::Tuning tu = defaults().tu;
    if (walk) tu.walk = walk - 1;
    const fa::ChainPlan pl =
        fa::plan_chain((fa_dtype)in, (fa_dtype)out, (int64_t)(n / (16 / dsize((fa_dtype)in))), nc, true, tu, cus);
    if (kind) *kind = pl.kind;
    if (phases) *phases = pl.phases;
    return FA_OK;
}

// Diagnostic, not part of the ABI in fa.h: the plan of every launch one FA_SHARD_CLIENT_RS round enqueues for a
// FedAvg bucket of n elements over n_clients clients on n_gpus GPUs of `cus` CUs (as reduce_part does: each
// GPU's piece reductions into its fp32 partial, then, for a bf16 output, the rounding of its shard), under the
// process-default tuning with `chunks` pieces (0 = the default).  *launches counts them, *phased_launches
// those that take the phased kernel, *max_phases the most phases of one launch.  Pure host arithmetic.
extern "C" int fa_diag_rs_plan(size_t n, int n_gpus, int n_clients, int chunks, int in, int out, int cus,
                               int* launches, int* phased_launches, long long* max_phases) {
    g_err.clear();
    if (n_gpus < 1 || n_clients < 1 || chunks < 0 || !dvalid(in) || !dvalid(out) || cus < 0)
        return fail(FA_ERR_ARG, "bad rs plan arguments");
    const CtxTuning ct = defaults();
    const fa::Tuning rtu = rs_launch_tuning(ct.tu);
    const size_t unit = (size_t)n_gpus * kShardUnit, npad = (n + unit - 1) / unit * unit;
    const int V = (int)(16 / dsize((fa_dtype)in));
    int nl = 0, np = 0;
    long long mp = 0;
    auto note = [&](const fa::ChainPlan& pl) {
        ++nl;
        if (pl.kind == fa::kPlanPhased) ++np;
        mp = std::max<long long>(mp, pl.phases);
    };
    const auto pieces = rs_pieces(npad, n_gpus, chunks ? chunks : ct.rs_chunks);
    for (int g = 0; g < n_gpus; ++g) {
        int c0, c1;
        client_bounds(n_clients, n_gpus, g, &c0, &c1);
        if (c1 > c0)
            for (auto& pc : pieces)
                note(fa::plan_chain((fa_dtype)in, FA_F32, (int64_t)((pc.second - pc.first) / V), c1 - c0, true, rtu, cus));
        if (out == FA_BF16) note(fa::plan_chain(FA_F32, FA_BF16, (int64_t)(npad / n_gpus / 4), 1, true, rtu, cus));
    }
    if (launches) *launches = nl;
    if (phased_launches) *phased_launches = np;
    if (max_phases) *max_phases = mp;
    return FA_OK;
}

// Diagnostic, not part of the ABI in fa.h: how a range-layout GPU holding `held` slots of n elements of
// `in` cuts them (piece_len_for under the process default tuning, fa_set_tuning): *n_pieces pieces of
// *piece_elems elements (the last one shorter).  Pure host arithmetic.
extern "C" int fa_diag_pieces(size_t n, int held, int in, int* n_pieces, size_t* piece_elems) {
    g_err.clear();
    if (held < 0 || !dvalid(in)) return fail(FA_ERR_ARG, "bad piece arguments");
    const size_t len = piece_len_for((size_t)held, n, dsize((fa_dtype)in), defaults());
    if (n_pieces) *n_pieces = n ? (int)((n + len - 1) / len) : 1;
    if (piece_elems) *piece_elems = len;
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
