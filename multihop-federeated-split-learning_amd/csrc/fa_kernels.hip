// fa_kernels.hip -- CDNA4 (gfx950) kernels of the FedAvg aggregation path.
//
// The reduction replaces the per-parameter loop of the reference aggregator
// (pipeline_simulation/aggregator.cpp:72-88 and :126-142).  It is pure
// element-wise, HBM-bound work: per element, D client reads and one write, two
// flops per client.  No MFMA, no LDS reuse to exploit -- what matters is the
// number of 16-byte loads in flight per CU.
//
// Layout: each client bucket is one contiguous array in HBM (the flattened
// named_parameters() of a model part).  A wave reads 1 KiB contiguous from U
// client buckets (16 B per lane, one global_load_dwordx4 each), then runs the
// ordered FMA chain acc = fma(x_k, w_k, acc) in client order for the 4 (f32)
// or 8 (bf16) elements it owns, and writes the result once.  Client pointers
// and weights sit in the kernel-argument segment (scalar loads, uniform per
// wave); more than kMaxClients clients are handled by further passes that
// continue the chain from the fp32 accumulator (bit-identical to one chain).
//
// Numerics follow oracle/fa_oracle.c exactly: fmaf chain from +0, exact bf16
// widening, one round-to-nearest-even at the end; literal mode uses IEEE
// division (hipcc's default correctly rounded f32 divide).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <vector>

#include "fa_internal.h"

namespace fa {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------- helpers

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}
// Store cache policies (fa_tuning.store_policy - 1): plain, nt, sc1 (write-through, the
// line is dropped from the XCD L2), sc0 sc1.  The asm stores need no waitcnt (nothing in
// the kernel reads the output back) but end with s_nop 1: hipcc does not pad hazards
// inside an asm statement and would otherwise overwrite the data VGPRs before the store
// has read them (cdna_hip_programming.md 5.7 item 1).
enum { kStPlain = 0, kStNt = 1, kStSc1 = 2, kStSc01 = 3 };
template <int SP>
__device__ __forceinline__ void st16(void* p, u32x4 v) {
    if constexpr (SP == kStNt) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else if constexpr (SP == kStSc1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == kStSc01)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else *reinterpret_cast<u32x4*>(p) = v;
}
template <int SP>
__device__ __forceinline__ void st8(void* p, u32x2 v) {
    if constexpr (SP == kStNt) __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(p));
    else if constexpr (SP == kStSc1) asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == kStSc01)
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else *reinterpret_cast<u32x2*>(p) = v;
}

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

// Same integer rounding as oracle fa_oracle_f32_to_bf16 (NaN kept a quiet NaN).
__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// Element-type traits: a lane owns 16 bytes of every input bucket.
template <typename T> struct In;
template <> struct In<float> {
    static constexpr int kVec = 4;
    __device__ static __forceinline__ void widen(u32x4 r, float* x) {
        x[0] = __uint_as_float(r.x); x[1] = __uint_as_float(r.y);
        x[2] = __uint_as_float(r.z); x[3] = __uint_as_float(r.w);
    }
    __device__ static __forceinline__ float scalar(const void* p, int64_t i) {
        return reinterpret_cast<const float*>(p)[i];
    }
};
template <> struct In<uint16_t> {
    static constexpr int kVec = 8;
    __device__ static __forceinline__ void widen(u32x4 r, float* x) {
        x[0] = __uint_as_float(r.x << 16); x[1] = __uint_as_float(r.x & 0xffff0000u);
        x[2] = __uint_as_float(r.y << 16); x[3] = __uint_as_float(r.y & 0xffff0000u);
        x[4] = __uint_as_float(r.z << 16); x[5] = __uint_as_float(r.z & 0xffff0000u);
        x[6] = __uint_as_float(r.w << 16); x[7] = __uint_as_float(r.w & 0xffff0000u);
    }
    __device__ static __forceinline__ float scalar(const void* p, int64_t i) {
        return bf16_to_f32(reinterpret_cast<const uint16_t*>(p)[i]);
    }
};

template <typename T> struct Out;
template <> struct Out<float> {
    template <int V, int SP>
    __device__ static __forceinline__ void store(void* base, int64_t e, const float* a) {
        float* p = reinterpret_cast<float*>(base) + e;
#pragma unroll
        for (int j = 0; j < V; j += 4)
            st16<SP>(p + j, u32x4{__float_as_uint(a[j]), __float_as_uint(a[j + 1]), __float_as_uint(a[j + 2]),
                                  __float_as_uint(a[j + 3])});
    }
    __device__ static __forceinline__ void scalar(void* base, int64_t i, float a) {
        reinterpret_cast<float*>(base)[i] = a;
    }
};
template <> struct Out<uint16_t> {
    template <int V, int SP>
    __device__ static __forceinline__ void store(void* base, int64_t e, const float* a) {
        uint16_t* p = reinterpret_cast<uint16_t*>(base) + e;
        if constexpr (V == 8) {
            st16<SP>(p, u32x4{f32_to_bf16(a[0]) | (f32_to_bf16(a[1]) << 16), f32_to_bf16(a[2]) | (f32_to_bf16(a[3]) << 16),
                              f32_to_bf16(a[4]) | (f32_to_bf16(a[5]) << 16), f32_to_bf16(a[6]) | (f32_to_bf16(a[7]) << 16)});
        } else {
            st8<SP>(p, u32x2{f32_to_bf16(a[0]) | (f32_to_bf16(a[1]) << 16), f32_to_bf16(a[2]) | (f32_to_bf16(a[3]) << 16)});
        }
    }
    __device__ static __forceinline__ void scalar(void* base, int64_t i, float a) {
        reinterpret_cast<uint16_t*>(base)[i] = (uint16_t)f32_to_bf16(a);
    }
};

// ---------------------------------------------------------------- FedAvg chain

// Scalar elements [0, head) and [tail0, n): handled by the first workgroup.
template <typename IN, typename OUT, bool INIT>
__device__ __forceinline__ void chain_scalar_edges(const ClientTable& t, int nc, const float* init, void* out,
                                                   int64_t head, int64_t tail0, int64_t n) {
    if (blockIdx.x != 0) return;
    const int64_t n_tail = n - tail0;
    for (int64_t s = threadIdx.x; s < head + n_tail; s += blockDim.x) {
        const int64_t i = s < head ? s : tail0 + (s - head);
        float acc = INIT ? init[i] : 0.0f;
        for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<IN>::scalar(t.src[k], i), t.w[k], acc);
        Out<OUT>::scalar(out, i, acc);
    }
}

// The last r < U clients of the chain (k .. k+r-1) in groups of up to G: a group's loads are all
// issued before its first FMA (r is uniform, so the guards are scalar branches), instead of a runtime
// loop that the compiler emits as load / wait / fma per client -- one HBM round trip per client, which
// a bucket with D < U (e.g. C2, D = 8 under U = 16) would otherwise pay for every vector.  G = 8 keeps
// the f32 kernel at 64 VGPRs (8 waves per SIMD); a 15-wide group would take 72.
template <typename IN, int U, bool LNT, int V, class Tab = ClientTable>
__device__ __forceinline__ void chain_tail(const Tab& t, int k, int r, int64_t e, float* acc) {
    constexpr int G = U < 8 ? U : 8;
    for (; r > 0; k += G, r -= G) {
        u32x4 raw[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
            if (u < r) raw[u] = ld16<LNT>(reinterpret_cast<const IN*>(t.src[k + u]) + e);
#pragma unroll
        for (int u = 0; u < G; ++u) {
            if (u < r) {
                float x[V];
                In<IN>::widen(raw[u], x);
                const float w = t.w[k + u];
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] = __builtin_fmaf(x[j], w, acc[j]);
            }
        }
    }
}

// Clients [k, k1) of the ordered chain for the V elements starting at element e, continuing acc: groups of
// U loads in flight before their FMAs, then the grouped tail.
template <typename IN, int U, bool LNT, class Tab = ClientTable>
__device__ __forceinline__ void chain_from(const Tab& t, int k, int k1, int64_t e, float* acc) {
    constexpr int V = In<IN>::kVec;
    for (; k + U <= k1; k += U) {
        u32x4 raw[U];  // U loads in flight before the first FMA of the group
#pragma unroll
        for (int u = 0; u < U; ++u) raw[u] = ld16<LNT>(reinterpret_cast<const IN*>(t.src[k + u]) + e);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float x[V];
            In<IN>::widen(raw[u], x);
            const float w = t.w[k + u];
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] = __builtin_fmaf(x[j], w, acc[j]);
        }
    }
    chain_tail<IN, U, LNT, V, Tab>(t, k, k1 - k, e, acc);
}

// The ordered chain for the V elements of every client bucket starting at element e: groups of U
// loads in flight before their FMAs, then the grouped tail.  acc starts at +0 or at init[e..].
// Tab: anything with t.src[k] / t.w[k] (the kernarg ClientTable, or a SegView into a batched launch's
// kernel arguments).
template <typename IN, int U, bool LNT, bool INIT, class Tab = ClientTable>
__device__ __forceinline__ void chain_vec(const Tab& t, int nc, const float* init, int64_t e, float* acc) {
    constexpr int V = In<IN>::kVec;
    if constexpr (INIT) {
#pragma unroll
        for (int j = 0; j < V; j += 4) {
            u32x4 r = ld16<LNT>(init + e + j);
            acc[j] = __uint_as_float(r.x); acc[j + 1] = __uint_as_float(r.y);
            acc[j + 2] = __uint_as_float(r.z); acc[j + 3] = __uint_as_float(r.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.0f;
    }
    chain_from<IN, U, LNT, Tab>(t, 0, nc, e, acc);
}

// Vector body over nvec lane-vectors starting at element `head`; lane-vector v
// covers elements head + v*V .. head + v*V + V-1 of every bucket.  LNT: nt
// loads; SP: store policy (st16).
// walk (fa_tuning.walk - 1): 0 = linear grid-stride; 1 = XCD eighths: on a one-shot grid of 8*nb8
// workgroups, workgroup b takes block slot (b % 8) * nb8 + b / 8, so the workgroups of one XCD (blocks
// are dealt round-robin over the 8 XCDs; speed only, never correctness) walk one contiguous eighth of
// the bucket; 2 = the same with the odd eighths walked backwards.
template <typename IN, typename OUT, int U, bool LNT, int SP, bool INIT>
__global__ __launch_bounds__(256) void fedavg_chain_kernel(const ClientTable t, int nc, const float* init, void* out,
                                                           int64_t head, int64_t nvec, int64_t n, int walk) {
    constexpr int V = In<IN>::kVec;
    chain_scalar_edges<IN, OUT, INIT>(t, nc, init, out, head, head + nvec * V, n);
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (walk) {
        const int64_t nb8 = gridDim.x >> 3;
        const int x = blockIdx.x & 7;
        int64_t j = blockIdx.x >> 3;
        if (walk == 2 && (x & 1)) j = nb8 - 1 - j;
        v0 = (x * nb8 + j) * blockDim.x + threadIdx.x;
        stride = nvec;  // one vector per lane
    }
    for (int64_t v = v0; v < nvec; v += stride) {
        const int64_t e = head + v * V;  // first element owned by this lane
        float acc[V];
        chain_vec<IN, U, LNT, INIT>(t, nc, init, e, acc);
        Out<OUT>::template store<V, SP>(out, e, acc);
    }
}

// ---------------------------------------------------------------- phased FedAvg chain
//
// The same chain, with the output stream separated from the input streams in TIME.  On MI355X the
// 32 input streams of the north star read at 7.1 TB/s in every HBM pool, and a write-only stream
// runs at 6.2 TB/s, but interleaved they lose 0.07 ms (fast pools) to 0.2 ms (slow pools) to
// read/write turnaround -- which of the two a pool gets depends only on where the allocation of the
// INPUTS lands physically (round-1 experiments, profiles/r01_summary.json).  Here a persistent grid
// (one 256-thread workgroup per CU) works in phases: every lane reduces RL vectors into LDS (160 KiB
// per CU) and RR more into registers, the workgroups meet at a chip-wide counter, then all of them
// write the phase's results.  With the larger register stage (REGS 192, walk 5) three phases cover
// the north star, and it runs at 1.268-1.270 ms in every pool (gpurun_out r01s18: the one-shot XCD
// walk took 1.42 ms in the same, slow, pools; 1.27-1.30 in fast ones).  Results are bit-identical:
// the phases only reorder stores in time.
//
// The meeting point is a counter slot picked per stream: a 64-bit ticket word, then a ring of
// kSyncRing arrival and kSyncRing departure counters.  Every workgroup takes a ticket when it starts;
// tickets [jG, (j+1)G) form epoch j, which counts on ring entry j % kSyncRing.  Launches on one stream
// (or replays of a captured graph) are serialized, so each launch is exactly one epoch; the last
// workgroup of an epoch to leave zeroes its entry.  Launches on two streams that share a slot may
// mix their workgroups within an epoch, but every epoch still holds G workgroups, so its entry is
// zeroed all the same: they lose speed (the wait is bounded), never results or the counters.  The
// bound also lets every wave reach the exit if the grid were not co-resident.  The write part starts
// once all but `slack` workgroups have arrived.
constexpr int kPhasedThreads = 256;
constexpr int kSyncRing = 8;

// An LDS row holds a lane's finished vector (the whole chain is done before it is stored), so it is kept in
// the OUTPUT dtype: rounded once to bf16 there exactly as the global store would, same bits, and a bf16
// output fits twice the rows (the 512-thread bf16 form: 20 instead of 10, a phase of 33.5 M elements
// instead of 23.1 M).
template <typename OUT> using LdsT = typename std::conditional<std::is_same<OUT, uint16_t>::value, uint16_t, float>::type;

template <typename IN, int REGS, int TH = kPhasedThreads, typename OUT = float>
struct Phased {  // vectors per lane per phase: LDS (160 KiB per workgroup) + registers
    static constexpr int V = In<IN>::kVec;
    // 256 threads: f32 -> f32 40; 512 threads: bf16 -> bf16 20, bf16 -> f32 10
    static constexpr int RL = 160 * 1024 / (TH * V * (int)sizeof(LdsT<OUT>));
    static constexpr int RR = REGS / V;  // REGS 128: 32 / 16 vectors (arch VGPRs); 192: 48 / 24 (+ AGPRs)
};

// The register-staged part of a phase: wave w of workgroup b owns a contiguous chunk of RR*64
// vectors (RR KiB of every bucket for f32), lane l holds vectors c0 + r*64 + l for r < RR in keep[].
// The loops are swapped -- clients outside (a runtime loop), the RR vectors inside (unrolled, so
// every index into keep[] is a constant and it stays in VGPRs); each element still sees its clients
// in order, so the chain is unchanged.  The wave's base address is uniform (SGPRs) and r*1 KiB a
// constant, so a load needs no per-vector address registers: keep[] (128 VGPRs) and 16 loads in
// flight fit the 256 architectural VGPRs.  Returns false (nothing staged) for a wave whose chunk
// runs past the end of the bucket; the caller reduces and stores those vectors directly.
template <typename IN, bool INIT, int RR, int G16>
__device__ __forceinline__ bool stage_regs(const ClientTable& t, int nc, const float* init, int64_t head, int64_t c0,
                                           int64_t nvec, float (&keep)[RR][In<IN>::kVec]) {
    constexpr int V = In<IN>::kVec;
    if (c0 + (int64_t)RR * 64 > nvec) return false;
    const int lane = threadIdx.x & 63;
    const int64_t ubase = (head + c0 * V) * (int64_t)sizeof(IN);      // wave-uniform
    const uint32_t loff = (uint32_t)(lane * V * (int)sizeof(IN));     // this lane's 16 B
    constexpr int64_t kRowBytes = 64 * V * (int64_t)sizeof(IN);        // one vector per lane: 1 KiB
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        if constexpr (INIT) {
            const float* ip = init + head + (c0 + r * 64 + lane) * V;
#pragma unroll
            for (int j = 0; j < V; j += 4) {
                u32x4 q = ld16<true>(ip + j);
                keep[r][j] = __uint_as_float(q.x); keep[r][j + 1] = __uint_as_float(q.y);
                keep[r][j + 2] = __uint_as_float(q.z); keep[r][j + 3] = __uint_as_float(q.w);
            }
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) keep[r][j] = 0.0f;
        }
    }
    for (int k = 0; k < nc; ++k) {
        const char* src = reinterpret_cast<const char*>(t.src[k]) + ubase;
        const float w = t.w[k];
#pragma unroll
        for (int r0 = 0; r0 < RR; r0 += G16) {
            u32x4 raw[G16];
#pragma unroll
            for (int u = 0; u < G16; ++u)
                if (r0 + u < RR) raw[u] = ld16<true>(src + (r0 + u) * kRowBytes + loff);
#pragma unroll
            for (int u = 0; u < G16; ++u) {
                if (r0 + u < RR) {
                    float x[V];
                    In<IN>::widen(raw[u], x);
#pragma unroll
                    for (int j = 0; j < V; ++j) keep[r0 + u][j] = __builtin_fmaf(x[j], w, keep[r0 + u][j]);
                }
            }
        }
    }
    return true;
}

template <typename T, bool INIT>
__device__ __forceinline__ void sync_scalar_edges(const ClientTable& t, int nc, const float* init, int64_t head,
                                                  int64_t tail0, int64_t n) {
    if (blockIdx.x != 0) return;
    const int64_t n_tail = n - tail0;
    for (int64_t s = threadIdx.x; s < head + n_tail; s += blockDim.x) {
        const int64_t i = s < head ? s : tail0 + (s - head);
        float acc = INIT ? init[i] : 0.0f;
        for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<T>::scalar(t.src[k], i), t.w[k], acc);
        for (int k = 0; k < nc; ++k) Out<T>::scalar(const_cast<void*>(t.src[k]), i, acc);
    }
}

// A reduced vector leaves the phased kernel: to the output, or (SYNC, compute-node state sync) back to
// every client slot in place.
template <typename OUT, int V, bool SYNC>
__device__ __forceinline__ void put(const ClientTable& t, int nc, void* out, int64_t e, const float* acc) {
    if (!SYNC && !out) return;  // the read-stream probe (launch_read_probe): the same reads, no output stream
    if constexpr (SYNC) {
        for (int k = 0; k < nc; ++k) Out<OUT>::template store<V, kStSc1>(const_cast<void*>(t.src[k]), e, acc);
    } else {
        Out<OUT>::template store<V, kStSc1>(out, e, acc);
    }
}

// LDS rows of a bf16 output: the finished vector as bf16 bits (pack_bf16), stored as they are.
template <int V>
__device__ __forceinline__ void pack_bf16(uint16_t* row, const float* acc) {
    if constexpr (V == 8) {
        *reinterpret_cast<u32x4*>(row) =
            u32x4{f32_to_bf16(acc[0]) | (f32_to_bf16(acc[1]) << 16), f32_to_bf16(acc[2]) | (f32_to_bf16(acc[3]) << 16),
                  f32_to_bf16(acc[4]) | (f32_to_bf16(acc[5]) << 16), f32_to_bf16(acc[6]) | (f32_to_bf16(acc[7]) << 16)};
    } else {
        *reinterpret_cast<u32x2*>(row) =
            u32x2{f32_to_bf16(acc[0]) | (f32_to_bf16(acc[1]) << 16), f32_to_bf16(acc[2]) | (f32_to_bf16(acc[3]) << 16)};
    }
}
template <int V, bool SYNC>
__device__ __forceinline__ void put_bf16_bits(const ClientTable& t, int nc, void* out, int64_t e, const uint16_t* row) {
    auto one = [&](void* base) {
        uint16_t* p = reinterpret_cast<uint16_t*>(base) + e;
        if constexpr (V == 8) st16<kStSc1>(p, *reinterpret_cast<const u32x4*>(row));
        else st8<kStSc1>(p, *reinterpret_cast<const u32x2*>(row));
    };
    if constexpr (SYNC) {
        for (int k = 0; k < nc; ++k) one(const_cast<void*>(t.src[k]));
    } else {
        one(out);
    }
}

template <typename IN, typename OUT, bool INIT, int REGS, bool SYNC, int TH>
__global__ __launch_bounds__(TH) void fedavg_phased_kernel(const ClientTable t, int nc, const float* init,
                                                                       void* out, int64_t head, int64_t nvec, int64_t n,
                                                                       unsigned* sync, int slack, int rl_last,
                                                                       int skew, int skew_last, int last_meet,
                                                                       unsigned long long* tl) {
    constexpr int V = In<IN>::kVec, T = TH, RL = Phased<IN, REGS, TH, OUT>::RL, RR = Phased<IN, REGS, TH, OUT>::RR;
    constexpr int U = TH > 256 ? 8 : 16;  // loads in flight per wave (2 waves per SIMD at 512 threads)
    constexpr bool kPacked = std::is_same<LdsT<OUT>, uint16_t>::value;  // LDS rows hold bf16 output bits
    __shared__ LdsT<OUT> buf[RL * T * V];
    // thread 0 takes the ticket; its value is first needed at the phase-0 meeting, so the atomic's
    // latency hides under the phase's loads
    unsigned long long ticket = 0;
    int wait_budget = 1 << 16;  // thread 0: spins per meeting; 0 after one ran out (the grid is not co-resident)
    // diagnostic timeline (FA_TIMELINE, fa_diag_phased_timeline): per workgroup, 8 slots of the 100 MHz
    // wall clock -- start, phase-0 arrival / departure at the meeting, last arrival / departure, end
    unsigned long long* my_tl = tl ? tl + (size_t)blockIdx.x * 8 : nullptr;
    if (my_tl && threadIdx.x == 0) my_tl[0] = (unsigned long long)wall_clock64();
    if (threadIdx.x == 0)
        ticket = __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(sync), 1ull, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (SYNC) sync_scalar_edges<IN, INIT>(t, nc, init, head, head + nvec * V, n);
    else chain_scalar_edges<IN, OUT, INIT>(t, nc, init, out, head, head + nvec * V, n);
    const int64_t G = gridDim.x;
    // skew: the workgroups of the odd XCDs (blockIdx odd; blocks are dealt round-robin over the 8 XCDs)
    // take `skew` fewer LDS rows than the even ones in every full phase, and 2 skew_last fewer in the last
    // (rl_last - skew_last against rl_last + skew_last) -- those XCDs read 5-10% slower (tools/timeline.py)
    const int64_t per_phase = G * T * (RL + RR) - (G / 2) * T * skew;
    const int phases = (int)((nvec + per_phase - 1) / per_phase);
    const bool odd = blockIdx.x & 1;
    // the meeting before phase p's writes: every workgroup's reads of the phase are done (all but `slack`)
    auto meet = [&](int p) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long t_arrive = my_tl ? (unsigned long long)wall_clock64() : 0;
            unsigned* arrive = sync + 4 + (unsigned)((ticket / (unsigned long long)G) % kSyncRing);
            __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)(G * (p + 1) - slack);
            int spins = 0;
            for (; __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && spins < wait_budget;
                 ++spins)
                __builtin_amdgcn_s_sleep(1);
            if (wait_budget && spins == wait_budget) {
                // the grid was not co-resident (GPU shared with other kernels): counted (fa_phased_timeouts),
                // and this workgroup stops waiting at the launch's later meetings, which would run out too
                __hip_atomic_fetch_add(sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wait_budget = 0;
            }
            if (my_tl) {
                const unsigned long long t_leave = (unsigned long long)wall_clock64();
                if (p == 0) my_tl[1] = t_arrive, my_tl[2] = t_leave;
                my_tl[3] = t_arrive, my_tl[4] = t_leave, my_tl[6] = (unsigned long long)(p + 1);
            }
        }
        __syncthreads();
    };
    for (int p = 0; p < phases; ++p) {
        const bool last = p == phases - 1;
        // LDS vectors per lane in this phase: r_all rows every workgroup takes, then r_even more that only
        // the even XCDs' take.  Full phases: RL - skew and skew; the last phase is balanced by the host
        // (rl_last per lane on average, registers first: phased_rl_last)
        const int r_all = last ? rl_last - skew_last : RL - skew;
        const int r_even = last ? 2 * skew_last : skew;
        const int rl = r_all + (odd ? 0 : r_even);
        // LDS row i: block (i G + b) of T vectors for i < r_all, block (r_all G + (i - r_all) G/2 + b/2) after
        const int64_t p0 = (int64_t)p * per_phase + threadIdx.x;
        const int64_t lds_rows = (int64_t)r_all * G + (int64_t)r_even * (G / 2);
        auto row_vec = [&](int i) {
            return i < r_all ? p0 + ((int64_t)i * G + blockIdx.x) * T
                             : p0 + ((int64_t)r_all * G + (int64_t)(i - r_all) * (G / 2) + blockIdx.x / 2) * T;
        };
#pragma unroll 1
        for (int i = 0; i < rl; ++i) {
            const int64_t v = row_vec(i);
            if (v < nvec) {
                float acc[V];
                chain_vec<IN, U, true, INIT>(t, nc, init, head + v * V, acc);
                if constexpr (kPacked) {
                    pack_bf16<V>(reinterpret_cast<uint16_t*>(&buf[(i * T + threadIdx.x) * V]), acc);
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) buf[(i * T + threadIdx.x) * V + j] = acc[j];
                }
            }
        }
        if (my_tl && p == 0) {
            __syncthreads();
            if (threadIdx.x == 0) my_tl[7] = (unsigned long long)wall_clock64();
        }
        // register part: this wave's contiguous chunk after the phase's LDS part
        const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int64_t c0 = (int64_t)p * per_phase + lds_rows * T + ((int64_t)blockIdx.x * (T / 64) + wave) * RR * 64;
        float keep[RR][V];
        const bool staged = stage_regs<IN, INIT, RR, U>(t, nc, init, head, c0, nvec, keep);
        if (!staged) {  // the chunk that holds the end of the bucket (or lies past it): no staging
            for (int r = 0; r < RR; ++r) {
                const int64_t v = c0 + r * 64 + (threadIdx.x & 63);
                if (v < nvec) {
                    float acc[V];
                    chain_vec<IN, U, true, INIT>(t, nc, init, head + v * V, acc);
                    put<OUT, V, SYNC>(t, nc, out, head + v * V, acc);
                }
            }
        }
        if (!last || last_meet) meet(p);
        else __syncthreads();
#pragma unroll 1
        for (int i = 0; i < rl; ++i) {
            const int64_t v = row_vec(i);
            if (v < nvec) {
                if constexpr (kPacked)
                    put_bf16_bits<V, SYNC>(t, nc, out, head + v * V,
                                           reinterpret_cast<const uint16_t*>(&buf[(i * T + threadIdx.x) * V]));
                else
                    put<OUT, V, SYNC>(t, nc, out, head + v * V, reinterpret_cast<const float*>(&buf[(i * T + threadIdx.x) * V]));
            }
        }
        if (staged) {
            const int64_t c = c0 + (threadIdx.x & 63);
#pragma unroll
            for (int r = 0; r < RR; ++r) put<OUT, V, SYNC>(t, nc, out, head + (c + r * 64) * V, keep[r]);
        }
    }
    if (my_tl) {  // end: this workgroup's stores have completed
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) my_tl[5] = (unsigned long long)wall_clock64();
    }
    if (threadIdx.x == 0) {
        const unsigned e = (unsigned)((ticket / (unsigned long long)G) % kSyncRing);
        if (__hip_atomic_fetch_add(sync + 4 + kSyncRing + e, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)G - 1) {
            __hip_atomic_store(sync + 4 + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(sync + 4 + kSyncRing + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Fully general path (pointers whose 16-byte phases differ): one element per lane.
template <typename IN, typename OUT, bool INIT>
__global__ __launch_bounds__(256) void fedavg_chain_scalar_kernel(const ClientTable t, int nc, const float* init,
                                                                  void* out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float acc = INIT ? init[i] : 0.0f;
        for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<IN>::scalar(t.src[k], i), t.w[k], acc);
        Out<OUT>::scalar(out, i, acc);
    }
}

// ---------------------------------------------------------------- state sync (compute nodes)
//
// Compute-node aggregation of an intermediate model part: a compute node keeps
// one State per client (systemAPI::init_state_vector, systemAPI.cpp:3-15); after a round every
// client's copy becomes the FedAvg of all copies.  In place: a lane reads its 16-byte vector of all
// nc client slots, runs the same ordered FMA chain, and writes the rounded result back to every
// slot (all reads of a vector precede its writes, so aliasing input and output is safe).
// Per element: nc*s reads + nc*s writes.

template <typename T, int U, int SP, bool INIT>
__global__ __launch_bounds__(256) void fedavg_sync_kernel(const ClientTable t, int nc, const float* init,
                                                          int64_t head, int64_t nvec, int64_t n) {
    constexpr int V = In<T>::kVec;
    sync_scalar_edges<T, INIT>(t, nc, init, head, head + nvec * V, n);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const int64_t e = head + v * V;
        float acc[V];
        if constexpr (INIT) {
#pragma unroll
            for (int j = 0; j < V; j += 4) {
                u32x4 r = ld16<true>(init + e + j);
                acc[j] = __uint_as_float(r.x); acc[j + 1] = __uint_as_float(r.y);
                acc[j + 2] = __uint_as_float(r.z); acc[j + 3] = __uint_as_float(r.w);
            }
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] = 0.0f;
        }
        int k = 0;
        for (; k + U <= nc; k += U) {
            u32x4 raw[U];
#pragma unroll
            for (int u = 0; u < U; ++u) raw[u] = ld16<true>(reinterpret_cast<const T*>(t.src[k + u]) + e);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float x[V];
                In<T>::widen(raw[u], x);
                const float w = t.w[k + u];
#pragma unroll
                for (int j = 0; j < V; ++j) acc[j] = __builtin_fmaf(x[j], w, acc[j]);
            }
        }
        chain_tail<T, U, true, V>(t, k, nc - k, e, acc);
        for (int k2 = 0; k2 < nc; ++k2) Out<T>::template store<V, SP>(const_cast<void*>(t.src[k2]), e, acc);
    }
}

template <typename T, bool INIT>
__global__ __launch_bounds__(256) void fedavg_sync_scalar_kernel(const ClientTable t, int nc, const float* init,
                                                                 int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float acc = INIT ? init[i] : 0.0f;
        for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<T>::scalar(t.src[k], i), t.w[k], acc);
        for (int k = 0; k < nc; ++k) Out<T>::scalar(const_cast<void*>(t.src[k]), i, acc);
    }
}

// More than kMaxClients slots: the chain ran into an fp32 accumulator; write it (rounded) to nc slots.
template <typename T>
__global__ __launch_bounds__(256) void broadcast_kernel(const ClientTable t, int nc, const float* acc, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float a = acc[i];
        for (int k = 0; k < nc; ++k) Out<T>::scalar(const_cast<void*>(t.src[k]), i, a);
    }
}

// ---------------------------------------------------------------- literal mode

template <typename IN, typename OUT, bool LNT, int SP>
__global__ __launch_bounds__(256) void literal_kernel(const void* x, void* out, float divisor, int64_t head,
                                                      int64_t nvec, int64_t n) {
    constexpr int V = In<IN>::kVec;
    if (blockIdx.x == 0) {
        const int64_t tail0 = head + nvec * V, n_tail = n - tail0;
        for (int64_t s = threadIdx.x; s < head + n_tail; s += blockDim.x) {
            const int64_t i = s < head ? s : tail0 + (s - head);
            const float xi = In<IN>::scalar(x, i);
            Out<OUT>::scalar(out, i, (xi + xi) / divisor);
        }
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const int64_t e = head + v * V;
        float xv[V], r[V];
        In<IN>::widen(ld16<LNT>(reinterpret_cast<const IN*>(x) + e), xv);
#pragma unroll
        for (int j = 0; j < V; ++j) r[j] = (xv[j] + xv[j]) / divisor;
        Out<OUT>::template store<V, SP>(out, e, r);
    }
}

template <typename IN, typename OUT>
__global__ __launch_bounds__(256) void literal_scalar_kernel(const void* x, void* out, float divisor, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float xi = In<IN>::scalar(x, i);
        Out<OUT>::scalar(out, i, (xi + xi) / divisor);
    }
}

// ---------------------------------------------------------------- batched buckets (segment table)
//
// All model-part buckets of one aggregator phase (aggregator.cpp:108-150: model_part 2..L+1, e.g.
// ResNet-18's 9,442,304 + 5,130 elements) reduced by ONE launch: segment s owns workgroups
// [blk0, blk0 + nblk) of a one-shot grid; a workgroup finds its segment by binary search, copies the
// segment's client table into LDS and runs the same ordered chain as fedavg_chain_kernel (so the bits
// equal one launch per bucket).  Its last workgroup also takes the segment's scalar tail.  Tiny
// buckets then cost a few workgroups instead of a launch each.

template <typename IN, typename OUT, int U>
__global__ __launch_bounds__(256) void fedavg_segments_kernel(const SegDesc* __restrict__ segs, int nseg) {
    constexpr int V = In<IN>::kVec;
    __shared__ ClientTable t;
    __shared__ int s_seg;
    if (threadIdx.x == 0) {
        int lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (segs[mid].blk0 <= (int64_t)blockIdx.x) lo = mid;
            else hi = mid - 1;
        }
        s_seg = lo;
    }
    __syncthreads();
    const SegDesc* sd = segs + __builtin_amdgcn_readfirstlane(s_seg);
    const int nc = sd->nc;
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        t.src[i] = sd->src[i];
        t.w[i] = sd->w[i];
    }
    __syncthreads();
    const int64_t b = (int64_t)blockIdx.x - sd->blk0;
    const int64_t nvec = sd->nvec;
    const int64_t v = b * blockDim.x + threadIdx.x;
    if (v < nvec) {
        float acc[V];
        chain_vec<IN, U, true, false>(t, nc, nullptr, v * V, acc);
        Out<OUT>::template store<V, kStSc1>(sd->out, v * V, acc);
    }
    if (b == sd->nblk - 1) {
        for (int64_t i = nvec * V + threadIdx.x; i < sd->n; i += blockDim.x) {
            float acc = 0.0f;
            for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<IN>::scalar(t.src[k], i), t.w[k], acc);
            Out<OUT>::scalar(sd->out, i, acc);
        }
    }
}

// The same over a small batch whose whole table travels in the kernel arguments (SegArgs: up to
// kSegArgMax buckets and kSegArgClients client pointers): no table upload before the launch (a 4 us
// blit on the stream, gpurun_out r02s07) and no dependent load of the table inside the kernel.
struct SegView {
    const void* const* src;
    const float* w;
};

template <typename IN, typename OUT, int U>
__global__ __launch_bounds__(256) void fedavg_segargs_kernel(const SegArgs a) {
    constexpr int V = In<IN>::kVec;
    int s = 0;
    while (s + 1 < a.nseg && a.blk0[s + 1] <= (int64_t)blockIdx.x) ++s;
    const SegView t{&a.src[a.src0[s]], &a.w[a.src0[s]]};
    const int nc = a.nc[s];
    const int64_t b = (int64_t)blockIdx.x - a.blk0[s], nvec = a.nvec[s];
    const int64_t v = b * blockDim.x + threadIdx.x;
    if (v < nvec) {
        float acc[V];
        chain_vec<IN, U, true, false, SegView>(t, nc, nullptr, v * V, acc);
        Out<OUT>::template store<V, kStSc1>(a.out[s], v * V, acc);
    }
    if (b == a.blk0[s + 1] - a.blk0[s] - 1) {
        for (int64_t i = nvec * V + threadIdx.x; i < a.n[s]; i += blockDim.x) {
            float acc = 0.0f;
            for (int k = 0; k < nc; ++k) acc = __builtin_fmaf(In<IN>::scalar(t.src[k], i), t.w[k], acc);
            Out<OUT>::scalar(a.out[s], i, acc);
        }
    }
}

// ---------------------------------------------------------------- generator

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ float gen_value(uint64_t seed, uint32_t client, uint64_t idx) {
    const uint64_t h = splitmix64(seed ^ ((uint64_t)client << 40) ^ idx);
    return (float)(uint32_t)(h >> 40) * 0x1p-23f - 1.0f;
}

template <typename OUT>
__global__ __launch_bounds__(256) void fill_kernel(void* dst, int64_t n, uint64_t seed, uint32_t client,
                                                   uint64_t idx0) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        Out<OUT>::scalar(dst, i, gen_value(seed, client, idx0 + (uint64_t)i));
}

// ---------------------------------------------------------------- launchers

namespace {

inline int64_t grid_for(int64_t work, const Tuning& tu) {
    int64_t g = (work + tu.block - 1) / tu.block;
    if (g < 1) g = 1;
    if (tu.max_blocks > 0 && g > tu.max_blocks) g = tu.max_blocks;
    return g;
}

// Grid of the one-element-per-lane kernels (scalar chain, literal, sync, broadcast): grid-stride loops,
// so the grid is capped -- a bucket of 2^32 elements would otherwise ask for more than 2^32 threads.
constexpr int64_t kScalarMaxBlocks = 1 << 16;
inline int64_t grid_scalar(int64_t n, const Tuning& tu) { return std::min(grid_for(n, tu), kScalarMaxBlocks); }

template <typename IN, typename OUT, int U, bool LNT, int SP>
hipError_t launch_chain_u(const ClientTable& t, int nc, const float* init, void* out, int64_t head, int64_t nvec,
                          int64_t n, const Tuning& tu, hipStream_t s) {
    int64_t g = grid_for(nvec > 0 ? nvec : 1, tu);
    // the XCD walks need the one-shot grid (one vector per lane), rounded up to whole eighths
    const int walk = (tu.walk && tu.max_blocks <= 0 && nvec >= 8 * (int64_t)tu.block) ? tu.walk : 0;
    if (walk) g = (g + 7) / 8 * 8;
    if (init)
        hipLaunchKernelGGL((fedavg_chain_kernel<IN, OUT, U, LNT, SP, true>), dim3((unsigned)g), dim3(tu.block), 0, s,
                           t, nc, init, out, head, nvec, n, walk);
    else
        hipLaunchKernelGGL((fedavg_chain_kernel<IN, OUT, U, LNT, SP, false>), dim3((unsigned)g), dim3(tu.block), 0,
                           s, t, nc, init, out, head, nvec, n, walk);
    return hipGetLastError();
}

template <typename IN, typename OUT, bool LNT, int SP>
hipError_t launch_chain_sp(const ClientTable& t, int nc, const float* init, void* out, int64_t head, int64_t nvec,
                           int64_t n, const Tuning& tu, hipStream_t s) {
    // D <= 8 never fills a 16-wide group: the 8-wide body (loads and FMAs interleaved by the
    // compiler) is ~2% faster there than the guarded tail group (tools/sweep.py c2, profiles/).
    const int unroll = (nc <= 8 && tu.unroll == 16) ? 8 : tu.unroll;
    switch (unroll) {
        case 4: return launch_chain_u<IN, OUT, 4, LNT, SP>(t, nc, init, out, head, nvec, n, tu, s);
        case 16: return launch_chain_u<IN, OUT, 16, LNT, SP>(t, nc, init, out, head, nvec, n, tu, s);
        default: return launch_chain_u<IN, OUT, 8, LNT, SP>(t, nc, init, out, head, nvec, n, tu, s);
    }
}

template <typename IN, typename OUT, bool LNT>
hipError_t launch_chain_lnt(const ClientTable& t, int nc, const float* init, void* out, int64_t head, int64_t nvec,
                            int64_t n, const Tuning& tu, hipStream_t s) {
    switch (tu.store_policy) {
        case kStNt: return launch_chain_sp<IN, OUT, LNT, kStNt>(t, nc, init, out, head, nvec, n, tu, s);
        case kStSc1: return launch_chain_sp<IN, OUT, LNT, kStSc1>(t, nc, init, out, head, nvec, n, tu, s);
        case kStSc01: return launch_chain_sp<IN, OUT, LNT, kStSc01>(t, nc, init, out, head, nvec, n, tu, s);
        default: return launch_chain_sp<IN, OUT, LNT, kStPlain>(t, nc, init, out, head, nvec, n, tu, s);
    }
}

// Per-device state of the phased kernel: the CU count (= its grid) and a table of zeroed counter
// slots (ticket + ring, fedavg_phased_kernel), one picked per stream, 256 B apart.
constexpr int kMaxDevices = 64, kSyncSlots = 64, kSyncStride = 64;
static_assert(4 + 2 * kSyncRing <= kSyncStride, "a counter slot holds the ticket and both rings");
// Counter slots [0, kOwnedSlots) belong to one stream each (first come, until the stream is released:
// fa_destroy releases its context's streams), so launches on two streams never mix their workgroups in one
// epoch; further streams share the hashed slots [kOwnedSlots, kSyncSlots) (speed only, never results: see
// the ring above).  A released slot is handed to the next new stream; it needs no reset, since a slot's
// ticket and ring already serve any sequence of launches from any streams (the hashed slots rely on it).
constexpr int kOwnedSlots = 48;
struct PhasedDevice {
    std::once_flag once;
    int cus = 0;
    unsigned* sync = nullptr;  // kSyncSlots slots, kSyncStride words apart
    unsigned long long* tl = nullptr;  // FA_TIMELINE=1: the last phased launch's per-workgroup timeline
    std::mutex mu;
    hipStream_t owner[kOwnedSlots] = {};
    bool taken[kOwnedSlots] = {};  // owner[i] is valid (the null stream may own a slot too)
    // this stream's counter slot; *own: the slot is the stream's alone
    int slot_of(hipStream_t s, bool* own) {
        std::lock_guard<std::mutex> g(mu);
        int free_slot = -1;
        for (int i = 0; i < kOwnedSlots; ++i) {
            if (taken[i] && owner[i] == s) return *own = true, i;
            if (!taken[i] && free_slot < 0) free_slot = i;
        }
        if (free_slot >= 0) {
            owner[free_slot] = s;
            taken[free_slot] = true;
            return *own = true, free_slot;
        }
        *own = false;
        return kOwnedSlots + (int)(((uintptr_t)s >> 4) % (kSyncSlots - kOwnedSlots));
    }
    int taken_count() {
        std::lock_guard<std::mutex> g(mu);
        int c = 0;
        for (int i = 0; i < kOwnedSlots; ++i) c += taken[i] ? 1 : 0;
        return c;
    }
    void release(hipStream_t s) {
        std::lock_guard<std::mutex> g(mu);
        for (int i = 0; i < kOwnedSlots; ++i)
            if (taken[i] && owner[i] == s) taken[i] = false;
    }
};
PhasedDevice g_phased[kMaxDevices];

PhasedDevice* phased_device() {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
    PhasedDevice& d = g_phased[dev];
    std::call_once(d.once, [&] {
        int cus = 0;
        unsigned* p = nullptr;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return;
        const size_t words = (size_t)kSyncStride * kSyncSlots;
        if (hipMalloc((void**)&p, sizeof(unsigned) * words) != hipSuccess) return;
        if (hipMemset(p, 0, sizeof(unsigned) * words) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipFree(p);
            return;
        }
        d.cus = cus;
        d.sync = p;
        const char* e = std::getenv("FA_TIMELINE");
        if (e && std::atoi(e) > 0 && hipMalloc((void**)&d.tl, sizeof(unsigned long long) * 8 * cus) == hipSuccess)
            (void)hipMemset(d.tl, 0, sizeof(unsigned long long) * 8 * cus);
    });
    (void)hipGetLastError();
    return d.sync ? &d : nullptr;
}

// LDS vectors per lane in the last phase (fedavg_phased_kernel's rl_last), whose `rem` vectors are spread
// evenly over all `lanes` of the grid.  Up to RL vectors per lane go to LDS alone; more fill every wave's
// register chunk (RR) and LDS takes the rest, so no lane holds more than one vector above the average
// (filling LDS first and then whole register chunks left half the waves of a partial phase idle while the
// others did RL + RR).
inline int phased_rl_last(int64_t rem, int64_t lanes, int RL, int RR) {
    if (rem >= lanes * (RL + RR)) return RL;
    const int64_t q = (rem + lanes - 1) / lanes;
    if (q <= RL) return (int)q;
    return (int)std::max<int64_t>(0, q - RR);
}

// LDS rows the odd XCDs' workgroups leave to the even ones in every full phase (fedavg_phased_kernel's
// skew): RL / 10 in the f32 form -- 4 of its 40 (north star 1.259-1.261 against 1.271 ms, C4 5.25 against
// 5.30, one rank's share at 2 GPUs 0.668-0.673 against 0.677-0.684; gpurun_out r02s25-s26); more loses
// again.  None in the 512-thread bf16 form: with fp32 rows (10) no step was small enough (C3: 1 row
// 0.425-0.427 ms against 0.424, 4 rows 0.444-0.449; r02s26-s27), and its bf16 rows (20) keep none either.
int phased_skew(int RL) { return RL >= 40 ? std::min(RL / 10, RL / 2 - 1) : 0; }

// Enqueue one phased launch on stream s, on the stream's counter slot.
template <typename Kern>
hipError_t phased_enqueue(PhasedDevice* d, Kern kern, int th, int RL, int RR, hipStream_t s, const ClientTable& t,
                          int nc, const float* init, void* out, int64_t head, int64_t nvec, int64_t n) {
    bool own = false;
    const int slot = d->slot_of(s, &own);
    const int slack = d->cus / 32;  // the write part starts once all but ~3% of the workgroups have arrived
    const int64_t lanes = (int64_t)d->cus * th;
    // the skew follows the whole chip's round-robin of workgroups over its 8 XCDs (blockIdx parity = XCD
    // parity); a partition of the chip (fewer CUs per device) keeps the plain layout
    const int skew = d->cus >= 256 && d->cus % 16 == 0 ? phased_skew(RL) : 0;
    const int64_t per_phase = lanes * (RL + RR) - (int64_t)(d->cus / 2) * th * skew;
    const int64_t phases = (nvec + per_phase - 1) / per_phase;
    const int rl_last = phased_rl_last(nvec - (phases - 1) * per_phase, lanes, RL, RR);
    const int skew_last = std::min({(skew + 1) / 2, rl_last, RL - rl_last});
    // The last phase writes without the meeting: each workgroup as soon as it has read its share, beside
    // the slower workgroups' last reads (one rank's share at 2 / 4 / 8 GPUs 0.664 / 0.344 / 0.173 ms
    // against 0.670 / 0.346 / 0.176 with the meeting, north star, C3 and C4 unchanged; gpurun_out r02s36).
    constexpr int last_meet = 0;
    // FA_TIMELINE: a launch without meetings leaves their stamps alone, so clear the previous launch's
    if (d->tl) (void)hipMemsetAsync(d->tl, 0, sizeof(unsigned long long) * 8 * d->cus, s);
    hipLaunchKernelGGL(kern, dim3((unsigned)d->cus), dim3(th), 0, s, t, nc, init, out, head, nvec, n,
                       d->sync + slot * kSyncStride, slack, rl_last, skew, skew_last, last_meet, d->tl);
    return hipGetLastError();
}

// One occupancy query per kernel instantiation (same on every gfx950 device).
template <typename Kern>
bool phased_fits(std::atomic<int>& occ, Kern kern, int th) {
    int o = occ.load(std::memory_order_relaxed);
    if (o < 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, th, 0) != hipSuccess) o = 0;
        occ.store(o, std::memory_order_relaxed);
    }
    return o >= 1;
}

// The phased kernel launch of one instantiation (the plan, below, chose it and the bucket's size): one
// workgroup per CU, all co-resident -- hipErrorNotSupported if not even one fits (the caller then takes the
// one-shot grid).
template <typename IN, typename OUT, int REGS, int TH>
hipError_t launch_phased_r(PhasedDevice* d, const ClientTable& t, int nc, const float* init, void* out, int64_t head,
                           int64_t nvec, int64_t n, hipStream_t s) {
    constexpr int RL = Phased<IN, REGS, TH, OUT>::RL, RR = Phased<IN, REGS, TH, OUT>::RR;
    static std::atomic<int> occ[2] = {-1, -1};  // per INIT variant
    auto kern = init ? fedavg_phased_kernel<IN, OUT, true, REGS, false, TH> : fedavg_phased_kernel<IN, OUT, false, REGS, false, TH>;
    if (!phased_fits(occ[init ? 1 : 0], kern, TH)) return hipErrorNotSupported;
    return phased_enqueue(d, kern, TH, RL, RR, s, t, nc, init, out, head, nvec, n);
}

// Clients from which a bucket smaller than one phase takes a phase sized to it (plan_chain); fewer
// clients make the output a larger share of the traffic, and its write burst after the meeting costs
// more than the one-shot grid's interleaving (C2, D = 8: 0.085 vs 0.075 ms).
constexpr int kSizedMinClients = 16;

template <typename T> constexpr fa_dtype dtype_of() { return std::is_same<T, float>::value ? FA_F32 : FA_BF16; }

// The instantiations a plan may name (threads, register-stage bytes per lane): 256-thread f32 forms with
// the register stages of the sized phases (192, 128, 32), the 512-thread form of walk 6 and of bf16 inputs
// (96, and 64 / 32 for sized bf16 phases), and walk 4's 128-register form.
template <typename IN, typename OUT>
hipError_t launch_phased_plan(PhasedDevice* d, const ChainPlan& pl, const ClientTable& t, int nc, const float* init,
                              void* out, int64_t head, int64_t nvec, int64_t n, hipStream_t s) {
    constexpr bool bf = std::is_same<IN, uint16_t>::value;
    switch (pl.threads * 1000 + pl.regs) {
        case 256128: return launch_phased_r<IN, OUT, 128, 256>(d, t, nc, init, out, head, nvec, n, s);
        case 512096: return launch_phased_r<IN, OUT, 96, 512>(d, t, nc, init, out, head, nvec, n, s);
        default: break;
    }
    if constexpr (!bf) {
        switch (pl.threads * 1000 + pl.regs) {
            case 256192: return launch_phased_r<IN, OUT, 192, 256>(d, t, nc, init, out, head, nvec, n, s);
            case 256032: return launch_phased_r<IN, OUT, 32, 256>(d, t, nc, init, out, head, nvec, n, s);
            default: break;
        }
    } else {
        switch (pl.threads * 1000 + pl.regs) {
            case 512064: return launch_phased_r<IN, OUT, 64, 512>(d, t, nc, init, out, head, nvec, n, s);
            case 512032: return launch_phased_r<IN, OUT, 32, 512>(d, t, nc, init, out, head, nvec, n, s);
            default: break;
        }
    }
    return hipErrorNotSupported;
}

template <typename IN, typename OUT>
hipError_t launch_chain_t(const ClientTable& t, int nc, const float* init, void* out, int64_t head, int64_t nvec,
                          int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s) {
    PhasedDevice* d = vector_ok && tu.walk >= 3 && tu.walk <= 5 ? phased_device() : nullptr;
    const ChainPlan pl = plan_chain(dtype_of<IN>(), dtype_of<OUT>(), nvec, nc, vector_ok, tu, d ? d->cus : 0);
    if (pl.kind == kPlanPhased) {
        const hipError_t e = launch_phased_plan<IN, OUT>(d, pl, t, nc, init, out, head, nvec, n, s);
        if (e != hipErrorNotSupported) return e;
    }
    if (pl.kind == kPlanScalar) {
        const int64_t g = grid_scalar(n, tu);
        if (init)
            hipLaunchKernelGGL((fedavg_chain_scalar_kernel<IN, OUT, true>), dim3((unsigned)g), dim3(tu.block), 0, s,
                               t, nc, init, out, n);
        else
            hipLaunchKernelGGL((fedavg_chain_scalar_kernel<IN, OUT, false>), dim3((unsigned)g), dim3(tu.block), 0,
                               s, t, nc, init, out, n);
        return hipGetLastError();
    }
    if (tu.load_nt) return launch_chain_lnt<IN, OUT, true>(t, nc, init, out, head, nvec, n, tu, s);
    return launch_chain_lnt<IN, OUT, false>(t, nc, init, out, head, nvec, n, tu, s);
}

}  // namespace

// ---------------------------------------------------------------- launch planning
//
// Which kernel one FedAvg chain launch takes, decided on the host from the bucket's shape, the tuning and
// the device's CU count alone (no device call), so that fa_diag_plan_chain can show the selection to the
// CPU suite.  The phased kernel takes buckets of at least one full phase (walks 4-6), and with walk 5 (the
// default) also buckets below one phase with >= kSizedMinClients clients, in one phase sized to them,
// q vectors per lane spread evenly (phased_rl_last): up to RL of them go to LDS alone and the register stage
// stays empty, so the smallest instantiation serves every q <= RL; above RL the register stage takes the
// largest RR <= q of the instantiated set and LDS the rest (q - RR <= RL).  E.g. the strong-scaled north
// star at 4 ranks (16.8 M f32 elements per rank): q = 64 -> 48 in registers + 16 in LDS, where the
// full-phase layout gave half the waves 88 and half 40; at 8 ranks q = 32 -> all 32 in LDS.
ChainPlan plan_chain(fa_dtype in, fa_dtype out, int64_t nvec, int nc, bool vector_ok, const Tuning& tu, int cus) {
    ChainPlan p{vector_ok ? kPlanOneShot : kPlanScalar, 0, 0, 0};
    if (!vector_ok || cus <= 0 || tu.walk < 3 || tu.walk > 5) return p;
    const bool bf = in == FA_BF16;
    const int V = bf ? 8 : 4;
    // walk 4 (fa_tuning.walk 5, the default): bf16 inputs take the 512-thread form (2 waves per SIMD hide
    // the widening VALU work of 8 elements per load: C3 0.430 vs 0.439 ms), f32 the 256-thread one (C4 5.43
    // vs 5.49 ms, C5's share 2.55 vs 2.56), gpurun_out r01s25
    const int th = tu.walk == 3 ? 256 : (tu.walk == 5 || bf) ? 512 : 256;
    int regs = tu.walk == 3 ? 128 : (tu.walk == 5 || bf) ? 96 : 192;
    const int rl = 160 * 1024 / (th * V * (out == FA_BF16 ? 2 : 4));  // Phased<>::RL
    const int64_t lanes = (int64_t)cus * th;
    if (nvec < lanes * (rl + regs / V)) {  // below one full phase
        if (tu.walk != 4 || nc < kSizedMinClients) return p;
        const int64_t q = (nvec + lanes - 1) / lanes;
        if (q < (bf ? 4 : 8)) return p;  // too few vectors per lane: the one-shot grid
        // register stages (bytes per lane) instantiated for the sized phase, largest first
        static const int kF32[] = {192, 128, 32}, kBf16[] = {96, 64, 32};
        const int* tiers = bf ? kBf16 : kF32;
        regs = tiers[2];  // q <= RL: LDS only, the register stage unused
        if (q > rl)
            for (int i = 0; i < 3; ++i)
                if (q >= tiers[i] / V) {
                    regs = tiers[i];
                    break;
                }
    }
    const int skew = cus >= 256 && cus % 16 == 0 ? phased_skew(rl) : 0;  // as phased_enqueue
    const int64_t per_phase = lanes * (rl + regs / V) - (int64_t)(cus / 2) * th * skew;
    return ChainPlan{kPlanPhased, regs, th, (nvec + per_phase - 1) / per_phase};
}

hipError_t phased_timeouts(int dev, uint64_t* count) {
    *count = 0;
    if (dev < 0 || dev >= kMaxDevices || !g_phased[dev].sync) return hipSuccess;  // no phased launch yet
    // on that device (the caller's current one may differ), after the launches still in flight there: they
    // run on non-blocking streams, which a plain hipMemcpy would not wait for
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    std::vector<unsigned> tab((size_t)kSyncStride * kSyncSlots);
    if (e == hipSuccess)
        e = hipMemcpy(tab.data(), g_phased[dev].sync, tab.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    if (e != hipSuccess) return e;
    for (int slot = 0; slot < kSyncSlots; ++slot) *count += tab[(size_t)slot * kSyncStride + 2];
    return hipSuccess;
}

int phased_timeline(int dev, unsigned long long* out, int cap) {
    if (dev < 0 || dev >= kMaxDevices || !g_phased[dev].tl) return 0;
    const int n = std::min(cap, g_phased[dev].cus * 8);
    // on that device, after its launches in flight (as phased_timeouts): the caller's current one may differ
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess)
        e = hipMemcpy(out, g_phased[dev].tl, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost);
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    return e == hipSuccess ? n : -1;
}

void phased_release_stream(int dev, hipStream_t s) {
    if (dev >= 0 && dev < kMaxDevices) g_phased[dev].release(s);
}

int phased_slot(int dev, hipStream_t s, bool* own) {
    if (dev < 0 || dev >= kMaxDevices) return -1;
    return g_phased[dev].slot_of(s, own);
}

int phased_owned_slots(int dev) { return dev >= 0 && dev < kMaxDevices ? g_phased[dev].taken_count() : -1; }

hipError_t launch_chain(const ClientTable& t, int nc, fa_dtype in, fa_dtype outdt, const float* init, void* out,
                        int64_t head, int64_t nvec, int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s) {
    if (in == FA_F32 && outdt == FA_F32)
        return launch_chain_t<float, float>(t, nc, init, out, head, nvec, n, vector_ok, tu, s);
    if (in == FA_F32 && outdt == FA_BF16)
        return launch_chain_t<float, uint16_t>(t, nc, init, out, head, nvec, n, vector_ok, tu, s);
    if (in == FA_BF16 && outdt == FA_F32)
        return launch_chain_t<uint16_t, float>(t, nc, init, out, head, nvec, n, vector_ok, tu, s);
    return launch_chain_t<uint16_t, uint16_t>(t, nc, init, out, head, nvec, n, vector_ok, tu, s);
}

namespace {
template <typename IN, typename OUT>
hipError_t launch_literal_t(const void* x, void* out, float divisor, int64_t head, int64_t nvec, int64_t n,
                            bool vector_ok, const Tuning& tu, hipStream_t s) {
    if (!vector_ok) {
        hipLaunchKernelGGL((literal_scalar_kernel<IN, OUT>), dim3((unsigned)grid_scalar(n, tu)), dim3(tu.block), 0, s,
                           x, out, divisor, n);
    } else {  // two streams only: nt loads, write-through stores
        hipLaunchKernelGGL((literal_kernel<IN, OUT, true, kStSc1>), dim3((unsigned)grid_for(nvec > 0 ? nvec : 1, tu)),
                           dim3(tu.block), 0, s, x, out, divisor, head, nvec, n);
    }
    return hipGetLastError();
}
}  // namespace

hipError_t launch_literal(const void* x, fa_dtype in, void* out, fa_dtype outdt, float divisor, int64_t head,
                          int64_t nvec, int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s) {
    if (in == FA_F32 && outdt == FA_F32)
        return launch_literal_t<float, float>(x, out, divisor, head, nvec, n, vector_ok, tu, s);
    if (in == FA_F32 && outdt == FA_BF16)
        return launch_literal_t<float, uint16_t>(x, out, divisor, head, nvec, n, vector_ok, tu, s);
    if (in == FA_BF16 && outdt == FA_F32)
        return launch_literal_t<uint16_t, float>(x, out, divisor, head, nvec, n, vector_ok, tu, s);
    return launch_literal_t<uint16_t, uint16_t>(x, out, divisor, head, nvec, n, vector_ok, tu, s);
}

namespace {
template <typename T, int SP>
hipError_t launch_sync_sp(const ClientTable& t, int nc, const float* init, int64_t head, int64_t nvec, int64_t n,
                          const Tuning& tu, hipStream_t s) {
    const int64_t g = grid_for(nvec > 0 ? nvec : 1, tu);
    if (init)
        hipLaunchKernelGGL((fedavg_sync_kernel<T, 8, SP, true>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc, init,
                           head, nvec, n);
    else
        hipLaunchKernelGGL((fedavg_sync_kernel<T, 8, SP, false>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc,
                           init, head, nvec, n);
    return hipGetLastError();
}

// The phased kernel in state-sync form (no init: sync_on chains more than kMaxClients slots into
// scratch and broadcasts instead).
template <typename T, int REGS, int TH>
hipError_t launch_sync_phased_r(const ClientTable& t, int nc, int64_t head, int64_t nvec, int64_t n, hipStream_t s) {
    PhasedDevice* d = phased_device();
    if (!d) return hipErrorNotSupported;
    constexpr int RL = Phased<T, REGS, TH, T>::RL, RR = Phased<T, REGS, TH, T>::RR;
    const int64_t per_phase = (int64_t)d->cus * TH * (RL + RR);
    if (nvec < per_phase) return hipErrorNotSupported;
    static std::atomic<int> occ{-1};
    auto kern = fedavg_phased_kernel<T, T, false, REGS, true, TH>;
    if (!phased_fits(occ, kern, TH)) return hipErrorNotSupported;
    return phased_enqueue(d, kern, TH, RL, RR, s, t, nc,
                          (const float*)nullptr, (void*)nullptr, head, nvec, n);
}

template <typename T>
hipError_t launch_sync_t(const ClientTable& t, int nc, const float* init, int64_t head, int64_t nvec, int64_t n,
                         bool vector_ok, const Tuning& tu, hipStream_t s) {
    if (vector_ok && !init && tu.walk >= 3 && tu.walk <= 5) {
        const hipError_t e = tu.walk == 3   ? launch_sync_phased_r<T, 128, 256>(t, nc, head, nvec, n, s)
                             : tu.walk == 4 ? launch_sync_phased_r<T, 192, 256>(t, nc, head, nvec, n, s)
                                            : launch_sync_phased_r<T, 96, 512>(t, nc, head, nvec, n, s);
        if (e != hipErrorNotSupported) return e;
    }
    if (!vector_ok) {
        const int64_t g = grid_scalar(n, tu);
        if (init)
            hipLaunchKernelGGL((fedavg_sync_scalar_kernel<T, true>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc,
                               init, n);
        else
            hipLaunchKernelGGL((fedavg_sync_scalar_kernel<T, false>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc,
                               init, n);
        return hipGetLastError();
    }
    switch (tu.store_policy) {
        case kStNt: return launch_sync_sp<T, kStNt>(t, nc, init, head, nvec, n, tu, s);
        case kStSc1: return launch_sync_sp<T, kStSc1>(t, nc, init, head, nvec, n, tu, s);
        case kStSc01: return launch_sync_sp<T, kStSc01>(t, nc, init, head, nvec, n, tu, s);
        default: return launch_sync_sp<T, kStPlain>(t, nc, init, head, nvec, n, tu, s);
    }
}
}  // namespace

hipError_t launch_sync(const ClientTable& t, int nc, fa_dtype dt, const float* init, int64_t head, int64_t nvec,
                       int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s) {
    if (dt == FA_F32) return launch_sync_t<float>(t, nc, init, head, nvec, n, vector_ok, tu, s);
    return launch_sync_t<uint16_t>(t, nc, init, head, nvec, n, vector_ok, tu, s);
}

hipError_t launch_broadcast(const ClientTable& t, int nc, fa_dtype dt, const float* acc, int64_t n,
                            const Tuning& tu, hipStream_t s) {
    const int64_t g = grid_scalar(n, tu);
    if (dt == FA_F32)
        hipLaunchKernelGGL((broadcast_kernel<float>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc, acc, n);
    else
        hipLaunchKernelGGL((broadcast_kernel<uint16_t>), dim3((unsigned)g), dim3(tu.block), 0, s, t, nc, acc, n);
    return hipGetLastError();
}

namespace {
template <typename IN, typename OUT>
hipError_t launch_segments_t(const SegDesc* d_segs, int nseg, int64_t blocks, int max_nc, int block,
                             hipStream_t s) {
    if (max_nc <= 8)
        hipLaunchKernelGGL((fedavg_segments_kernel<IN, OUT, 8>), dim3((unsigned)blocks), dim3(block), 0, s, d_segs,
                           nseg);
    else
        hipLaunchKernelGGL((fedavg_segments_kernel<IN, OUT, 16>), dim3((unsigned)blocks), dim3(block), 0, s,
                           d_segs, nseg);
    return hipGetLastError();
}
}  // namespace

namespace {
template <typename IN, typename OUT>
hipError_t launch_segargs_t(const SegArgs& a, int max_nc, int block, hipStream_t s) {
    const unsigned blocks = (unsigned)a.blk0[a.nseg];
    if (max_nc <= 8) hipLaunchKernelGGL((fedavg_segargs_kernel<IN, OUT, 8>), dim3(blocks), dim3(block), 0, s, a);
    else hipLaunchKernelGGL((fedavg_segargs_kernel<IN, OUT, 16>), dim3(blocks), dim3(block), 0, s, a);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_segargs(const SegArgs& a, fa_dtype in, fa_dtype outdt, int max_nc, const Tuning& tu, hipStream_t s) {
    if (a.nseg <= 0) return hipSuccess;
    if (in == FA_F32 && outdt == FA_F32) return launch_segargs_t<float, float>(a, max_nc, tu.block, s);
    if (in == FA_F32 && outdt == FA_BF16) return launch_segargs_t<float, uint16_t>(a, max_nc, tu.block, s);
    if (in == FA_BF16 && outdt == FA_F32) return launch_segargs_t<uint16_t, float>(a, max_nc, tu.block, s);
    return launch_segargs_t<uint16_t, uint16_t>(a, max_nc, tu.block, s);
}

hipError_t launch_segments(const SegDesc* d_segs, int nseg, int64_t blocks, fa_dtype in, fa_dtype outdt, int max_nc,
                           const Tuning& tu, hipStream_t s) {
    if (nseg <= 0) return hipSuccess;
    if (in == FA_F32 && outdt == FA_F32) return launch_segments_t<float, float>(d_segs, nseg, blocks, max_nc, tu.block, s);
    if (in == FA_F32 && outdt == FA_BF16)
        return launch_segments_t<float, uint16_t>(d_segs, nseg, blocks, max_nc, tu.block, s);
    if (in == FA_BF16 && outdt == FA_F32)
        return launch_segments_t<uint16_t, float>(d_segs, nseg, blocks, max_nc, tu.block, s);
    return launch_segments_t<uint16_t, uint16_t>(d_segs, nseg, blocks, max_nc, tu.block, s);
}

bool phased_takes(fa_dtype in, fa_dtype out, int64_t nvec, int nc, const Tuning& tu) {
    if (tu.walk < 3 || tu.walk > 5) return false;
    PhasedDevice* d = phased_device();
    return d && plan_chain(in, out, nvec, nc, true, tu, d->cus).kind == kPlanPhased;
}

// Read-stream probe (SURVEY.md 8d "also report a measured read-STREAM peak").  From one phase up it is the
// phased kernel itself with no output (launch_read_probe): the same reads, LDS staging and meetings,
// no writes -- the best read rate measured on this chip for these buffers (simple grid-stride read
// kernels reach ~6.95 TB/s, this ~7.2).  Below one phase, this kernel: every lane reads one 16-byte
// vector of each of nc buffers per step with U loads in flight, over a grid of 8 workgroups per CU
// walking the XCD eighths; the sum is stored only if it equals a value uniform[-1,1) inputs never
// produce, so nothing is written and nothing is elided.
__global__ __launch_bounds__(256) void read_probe_kernel(const ClientTable t, int nc, int64_t nvec, float* sink) {
    const int64_t nb8 = gridDim.x >> 3;
    const int64_t per = (nvec + nb8 * 8 * 256 - 1) / (nb8 * 8 * 256);  // vectors per lane
    const int64_t slot = (int64_t)(blockIdx.x & 7) * nb8 + (blockIdx.x >> 3);
    float acc = 0.0f;
    for (int64_t i = 0; i < per; ++i) {
        const int64_t v = (slot * per + i) * 256 + threadIdx.x;
        if (v >= nvec) break;
        float a[4];
        chain_vec<float, 16, true, false>(t, nc, nullptr, v * 4, a);
        acc += a[0] + a[1] + a[2] + a[3];
    }
    if (acc == 1.0e30f) sink[0] = acc;
}

hipError_t launch_read_probe(const ClientTable& t, int nc, int64_t nvec, float* sink, hipStream_t s) {
    // the phased kernel itself with no output (its reads, LDS and meetings, no writes) wherever an f32 chain of
    // this shape takes it: from one phase up, and below one phase with >= kSizedMinClients clients in one
    // phase sized to the buffers (the product's launch for such buckets; the simple probe below reads those
    // up to 14% slower than the product reduces them, r04s16)
    PhasedDevice* d = phased_device();
    Tuning tu{256, 0, 16, 1, 2, 4};  // walk 5's f32 form
    if (d) {
        const ChainPlan pl = plan_chain(FA_F32, FA_F32, nvec, nc, true, tu, d->cus);
        if (pl.kind == kPlanPhased) {
            const hipError_t e = launch_phased_plan<float, float>(d, pl, t, nc, nullptr, nullptr, 0, nvec, nvec * 4, s);
            if (e != hipErrorNotSupported) return e;
        }
    }
    const int g = (d ? d->cus : 256) * 8;
    hipLaunchKernelGGL(read_probe_kernel, dim3((unsigned)g), dim3(256), 0, s, t, nc, nvec, sink);
    return hipGetLastError();
}

// Independent read ceiling (roofline.read_stream_peak_independent): nothing of the product's access pattern --
// a plain grid-stride walk with U non-temporal 16-byte loads in flight per lane, buffer after buffer within one
// launch (tools/hbm_probe.hip's read kernel over the same slots).  The sum is stored only if it equals a value
// uniform[-1,1) inputs never produce, so nothing is written and nothing is elided.
template <int U>
__global__ __launch_bounds__(256) void read_plain_kernel(const ClientTable t, int nc, int64_t nvec, float* sink) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nc; ++k) {
        const f32x4* p = static_cast<const f32x4*>(t.src[k]);
        int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
        for (; v + (U - 1) * stride < nvec; v += U * stride) {
            f32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(p + v + u * stride);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += x[u];
        }
        for (; v < nvec; v += stride) acc += __builtin_nontemporal_load(p + v);
    }
    const float sum = acc.x + acc.y + acc.z + acc.w;
    if (sum == 1.0e30f) sink[0] = sum;
}

hipError_t launch_read_plain(const ClientTable& t, int nc, int64_t nvec, int grid, int unroll, float* sink,
                             hipStream_t s) {
    if (unroll == 8)
        hipLaunchKernelGGL(read_plain_kernel<8>, dim3((unsigned)grid), dim3(256), 0, s, t, nc, nvec, sink);
    else
        hipLaunchKernelGGL(read_plain_kernel<16>, dim3((unsigned)grid), dim3(256), 0, s, t, nc, nvec, sink);
    return hipGetLastError();
}

// Independent in-place read+write ceiling (the compute-node sync legs' copy_ceiling_independent): every
// slot read and written back where it lies, a plain grid-stride walk slot after slot with U non-temporal
// 16-byte loads in flight per lane, stored plain or non-temporal -- the sync's traffic (D reads + D writes of
// the same addresses) with none of its element-major structure.  x * scale with scale = 1 leaves every
// finite value as it was and keeps the store from being folded away.
template <int U, bool NT>
__global__ __launch_bounds__(256) void rw_plain_kernel(const ClientTable t, int nc, int64_t nvec, float scale) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int k = 0; k < nc; ++k) {
        f32x4* p = static_cast<f32x4*>(const_cast<void*>(t.src[k]));
        int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
        for (; v + (U - 1) * stride < nvec; v += U * stride) {
            f32x4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(p + v + u * stride);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (NT) __builtin_nontemporal_store(x[u] * scale, p + v + u * stride);
                else p[v + u * stride] = x[u] * scale;
            }
        }
        for (; v < nvec; v += stride) {
            const f32x4 x = __builtin_nontemporal_load(p + v) * scale;
            if constexpr (NT) __builtin_nontemporal_store(x, p + v);
            else p[v] = x;
        }
    }
}

hipError_t launch_rw_plain(const ClientTable& t, int nc, int64_t nvec, int grid, int unroll, bool nt, hipStream_t s) {
    const dim3 g((unsigned)grid), b(256);
    if (unroll == 8 && nt) hipLaunchKernelGGL((rw_plain_kernel<8, true>), g, b, 0, s, t, nc, nvec, 1.0f);
    else if (unroll == 8) hipLaunchKernelGGL((rw_plain_kernel<8, false>), g, b, 0, s, t, nc, nvec, 1.0f);
    else if (nt) hipLaunchKernelGGL((rw_plain_kernel<16, true>), g, b, 0, s, t, nc, nvec, 1.0f);
    else hipLaunchKernelGGL((rw_plain_kernel<16, false>), g, b, 0, s, t, nc, nvec, 1.0f);
    return hipGetLastError();
}

hipError_t launch_fill(void* dst, int64_t n, fa_dtype dt, uint64_t seed, uint32_t client, uint64_t idx0,
                       hipStream_t s) {
    Tuning tu{256, 8192, 8, 0, 0};
    const int64_t g = grid_for(n, tu);
    if (dt == FA_F32)
        hipLaunchKernelGGL((fill_kernel<float>), dim3((unsigned)g), dim3(256), 0, s, dst, n, seed, client, idx0);
    else
        hipLaunchKernelGGL((fill_kernel<uint16_t>), dim3((unsigned)g), dim3(256), 0, s, dst, n, seed, client, idx0);
    return hipGetLastError();
}

// ------------------------------------------------------------------ CRC-32 of output byte ranges
//
// The reply of a phase is the last receipt's zip archive around the reduced parameters, and every parameter
// record carries the CRC-32 of its bytes (torch::save's zip, which torch::load on the data owner checks,
// data_owner.cpp:232-253).  Those bytes are the part's device output, so their CRCs are computed here, from
// HBM, instead of by the host reading the reply back after its D2H (C2: 37.7 MB, ~0.7 ms of host time per
// phase; C4's FC reply 478 MB).  zlib's CRC-32 (reflected IEEE 802.3 polynomial) is linear: with R(M, r) the
// register after message M from register r, R(A || B, r) = R(B, 0) ^ shift(R(A, r), |B|), where shift(c, n)
// = c * x^(8n) mod P.  So every lane takes one 256-byte chunk of a piece, computes R(chunk, 0) with a byte
// table in LDS and shifts it by the bytes after the chunk in its piece; the XOR of a piece's lanes is
// R(piece, 0) (one wave reduction and one atomic XOR per wave when its lanes share a piece, which they do
// but at piece edges).  The host joins the pieces of a segment and applies the initial and final inversion.
namespace {

constexpr uint32_t kCrcPoly = 0xEDB88320u;
constexpr int kCrcChunk = 256;

// a(x) * b(x) mod P in the reflected representation (bit 31 = x^0), 32 fixed steps
__host__ __device__ constexpr uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; ++i) {
        if (a & (0x80000000u >> i)) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}

struct CrcX2n {  // t[k] = x^(2^k) mod P
    uint32_t t[64];
    constexpr CrcX2n() : t() {
        uint32_t p = 1u << 30;  // x^1
        t[0] = p;
        for (int k = 1; k < 64; ++k) t[k] = p = crc_mulmod(p, p);
    }
};
__constant__ CrcX2n kCrcX2n;

// x^(8 n) mod P: the multiplier that moves a CRC register over n zero bytes
__device__ inline uint32_t crc_x8n(uint64_t n) {
    uint32_t p = 0x80000000u;  // x^0
    for (int k = 3; n; n >>= 1, ++k)
        if (n & 1) p = crc_mulmod(kCrcX2n.t[k], p);
    return p;
}

__global__ __launch_bounds__(256) void crc32_pieces_kernel(const uint8_t* __restrict__ base,
                                                           const uint64_t* __restrict__ off,
                                                           const uint64_t* __restrict__ len,
                                                           const uint64_t* __restrict__ chunk0, int np,
                                                           uint32_t* __restrict__ out) {
    __shared__ uint32_t tab[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        uint32_t c = (uint32_t)i;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kCrcPoly : c >> 1;
        tab[i] = c;
    }
    __syncthreads();
    const uint64_t total = chunk0[np];
    const int lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // wave-uniform trip count: every lane of a wave runs every iteration (the shuffles need all 64)
    for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < total; g0 += stride) {
        const uint64_t g = g0 + lane;
        int p = -1;
        uint32_t r = 0;
        if (g < total) {
            int lo = 0, hi = np - 1;  // the piece whose chunks hold chunk g
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (chunk0[mid] <= g) lo = mid;
                else hi = mid - 1;
            }
            p = lo;
            const uint64_t a = (g - chunk0[p]) * kCrcChunk, L = len[p];
            const uint64_t e = a + kCrcChunk < L ? a + kCrcChunk : L;
            const uint8_t* q = base + off[p] + a;
            for (uint64_t i = 0; i < e - a; ++i) r = tab[(r ^ q[i]) & 0xFFu] ^ (r >> 8);
            r = crc_mulmod(crc_x8n(L - e), r);
        }
        const int p0 = __shfl(p, 0);
        if (__all(p == p0)) {
            for (int o = 32; o > 0; o >>= 1) r ^= __shfl_xor(r, o);
            if (lane == 0 && p0 >= 0) atomicXor(out + p0, r);
        } else if (p >= 0) {
            atomicXor(out + p, r);
        }
    }
}

}  // namespace

uint32_t crc32_mulmod(uint32_t a, uint32_t b) { return crc_mulmod(a, b); }

uint32_t crc32_x8n(uint64_t n) {
    static constexpr CrcX2n x2n;
    uint32_t p = 0x80000000u;
    for (int k = 3; n; n >>= 1, ++k)
        if (n & 1) p = crc_mulmod(x2n.t[k], p);
    return p;
}

hipError_t launch_crc32_pieces(const void* base, const uint64_t* d_off, const uint64_t* d_len, const uint64_t* d_chunk0,
                               int np, uint64_t chunks, uint32_t* d_out, hipStream_t s) {
    if (np <= 0 || chunks == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((chunks + 255) / 256, 4096);
    hipLaunchKernelGGL(crc32_pieces_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const uint8_t*>(base), d_off, d_len, d_chunk0, np, d_out);
    return hipGetLastError();
}

}  // namespace fa
