// fa_internal.h -- shared declarations between the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fedavg/fa.h"

namespace fa {

// Clients per launch.  Pointers + weights travel in the kernel-argument segment
// (1.5 KiB of the 4 KiB kernarg segment), read with scalar loads; more clients continue the chain in
// another pass.  128 covers C5 (D = 128) in one pass.
constexpr int kMaxClients = 128;

struct ClientTable {
    const void* src[kMaxClients];
    float w[kMaxClients];
};

// One bucket of a batched launch (fedavg_segments_kernel): workgroups [blk0, blk0 + nblk) of the grid
// reduce its nvec 16-byte vectors, the last of them also the scalar tail [nvec * V, n).  Device memory.
struct SegDesc {
    int64_t blk0, nblk, nvec, n;
    void* out;
    int nc, pad;
    const void* src[kMaxClients];
    float w[kMaxClients];
};

// A small batch in the kernel arguments: segment s = workgroups [blk0[s], blk0[s+1]), its clients are
// src/w[src0[s], src0[s] + nc[s]).
constexpr int kSegArgMax = 8, kSegArgClients = 192;
struct SegArgs {
    int nseg;
    int nc[kSegArgMax], src0[kSegArgMax];
    int64_t blk0[kSegArgMax + 1], nvec[kSegArgMax], n[kSegArgMax];
    void* out[kSegArgMax];
    const void* src[kSegArgClients];
    float w[kSegArgClients];
};

struct Tuning {
    int block;       // threads per workgroup: 64, 128 or 256
    int max_blocks;  // grid cap (grid-stride beyond it), <= 0: uncapped
    int unroll;      // clients per load group: 4, 8, 16
    int load_nt;      // non-temporal client loads
    int store_policy; // 0 plain, 1 nt, 2 sc1 (write-through), 3 sc0 sc1
    int walk;         // FedAvg grid walk: 0 linear, 1 XCD eighths, 2 XCD eighths, odd ones reversed,
                      // 3 phased (persistent grid, reads and writes separated in time; XCD eighths
                      // for buckets smaller than one phase), 4 phased with the larger register stage
};

// CRC-32 of byte ranges of device memory (the reply's zip records): piece i = [base + off[i], + len[i]),
// chunk0 the prefix count of its 256-byte chunks (np + 1 entries, chunks = chunk0[np]); out[i] (zeroed by the
// caller) gets R(piece i, 0), the CRC register over the piece from 0, without the inversions.  Device arrays.
hipError_t launch_crc32_pieces(const void* base, const uint64_t* d_off, const uint64_t* d_len, const uint64_t* d_chunk0,
                               int np, uint64_t chunks, uint32_t* d_out, hipStream_t s);
constexpr uint64_t kCrcChunkBytes = 256;
// Host side of the same algebra: a * b mod P (reflected) and x^(8 n) mod P.
uint32_t crc32_mulmod(uint32_t a, uint32_t b);
uint32_t crc32_x8n(uint64_t n);

hipError_t launch_chain(const ClientTable& t, int nc, fa_dtype in, fa_dtype out, const float* init, void* dst,
                        int64_t head, int64_t nvec, int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s);
// Meetings of the phased kernel on device `dev` that gave up waiting (the grid was not co-resident).
hipError_t phased_timeouts(int dev, uint64_t* count);
// FA_TIMELINE=1 diagnostic: copies the last phased launch's per-workgroup timeline (8 words each) on device
// dev into out; returns the words copied (0: no timeline, -1: HIP error).
int phased_timeline(int dev, unsigned long long* out, int cap);
// The phased kernel's counter slot of stream s on device dev (assigned on first use, as a launch would;
// *own: the slot is the stream's alone), and the release of a stream's owned slot (fa_destroy).
int phased_slot(int dev, hipStream_t s, bool* own);
void phased_release_stream(int dev, hipStream_t s);
int phased_owned_slots(int dev);  // owned slots currently taken on dev
// What one FedAvg chain launch runs (plan_chain, host-only): the one-shot vector grid, the one-element-per-
// lane kernel (mixed 16-byte phases), or the phased persistent grid (`threads` per workgroup, `regs` bytes of
// register stage per lane, `phases` phases; phases > 1 means chip-wide meetings).
enum { kPlanOneShot = 0, kPlanScalar = 1, kPlanPhased = 2 };
struct ChainPlan {
    int kind, regs, threads;
    int64_t phases;
};
// cus: the device's CU count (0 = no phased kernel).
ChainPlan plan_chain(fa_dtype in, fa_dtype out, int64_t nvec, int nc, bool vector_ok, const Tuning& tu, int cus);
hipError_t launch_literal(const void* x, fa_dtype in, void* dst, fa_dtype out, float divisor, int64_t head,
                          int64_t nvec, int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s);
// In-place state sync: every slot t.src[0..nc) := the chain over them (continuing `init` if given).
hipError_t launch_sync(const ClientTable& t, int nc, fa_dtype dt, const float* init, int64_t head, int64_t nvec,
                       int64_t n, bool vector_ok, const Tuning& tu, hipStream_t s);
// slots t.src[0..nc) := acc (rounded to dt).
hipError_t launch_broadcast(const ClientTable& t, int nc, fa_dtype dt, const float* acc, int64_t n,
                            const Tuning& tu, hipStream_t s);
// One launch over nseg buckets (FedAvg, no init, every pointer 16-byte aligned); blocks = sum of nblk.
hipError_t launch_segments(const SegDesc* d_segs, int nseg, int64_t blocks, fa_dtype in, fa_dtype out, int max_nc,
                           const Tuning& tu, hipStream_t s);
// The same with the table in the kernel arguments (a.nseg <= kSegArgMax, sum of nc <= kSegArgClients).
hipError_t launch_segargs(const SegArgs& a, fa_dtype in, fa_dtype out, int max_nc, const Tuning& tu, hipStream_t s);
// Whether launch_chain takes the phased kernel for a bucket of nvec vectors and nc clients.
bool phased_takes(fa_dtype in, fa_dtype out, int64_t nvec, int nc, const Tuning& tu);
hipError_t launch_fill(void* dst, int64_t n, fa_dtype dt, uint64_t seed, uint32_t client, uint64_t idx0,
                       hipStream_t s);
// Read-stream probe over nc f32 buffers of nvec 16-byte vectors (16-byte aligned); nothing is written.
hipError_t launch_read_probe(const ClientTable& t, int nc, int64_t nvec, float* sink, hipStream_t s);
hipError_t launch_read_plain(const ClientTable& t, int nc, int64_t nvec, int grid, int unroll, float* sink,
                             hipStream_t s);
hipError_t launch_rw_plain(const ClientTable& t, int nc, int64_t nvec, int grid, int unroll, bool nt, hipStream_t s);

}  // namespace fa
