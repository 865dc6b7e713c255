/*
 * fa.h -- C ABI of the MI355X FedAvg aggregation path (libfa.so).
 *
 * The reference has no plugin/FFI seam: the reduction is inline in the
 * aggregator's main() (pipeline_simulation/aggregator.cpp:55-167).  These
 * entry points replace that inline code; each declaration names the reference
 * lines it stands in for.  Plain pointers and sizes only, no torch types, no
 * C++ exceptions across the boundary.  Every call returns FA_OK (0) or a
 * negative fa_status; fa_last_error() gives a thread-local message.
 *
 * Threading: one fa_ctx per aggregator; calls on one ctx are serialized by the
 * caller (the reference's single consumer main thread, aggregator.cpp:60/:113).
 * Device work runs on ctx-owned HIP streams (one compute + one copy stream per
 * GPU, plus a high-priority exchange stream per GPU for FA_SHARD_CLIENT_RS only)
 * or on the caller's stream for fa_reduce_device.
 *
 * Numerics (tests/, DESIGN.md "Parity"):
 *   FA_FEDAVG  out_i = sum_k w_k x_{k,i} as an ordered fp32 FMA chain in client
 *              order starting from +0 (== libtorch acc.add_(x_k, w_k)),
 *              bf16 inputs widened exactly, bf16 output rounded to nearest-even
 *              once at the end.  Bit-exact vs oracle/ on every GPU layout
 *              except FA_SHARD_CLIENT_RS (summation order changes, <=1e-6
 *              relative to sum_k |w_k x_k|).
 *   FA_LITERAL out_i = fl(fl(x_i + x_i) / divisor), x = the LAST client
 *              submitted (aggregator.cpp:63-88 with parts/parts_ aliased,
 *              systemAPI.cpp:34-37); divisor defaults to kTrainSize_10 = 1000
 *              (aggregator.cpp:48).  Correctly rounded division.
 */
#ifndef FEDAVG_FA_H_
#define FEDAVG_FA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_ABI_VERSION 7

typedef struct fa_ctx fa_ctx; /* opaque: device slots, streams, pinned staging */

typedef enum { FA_F32 = 0, FA_BF16 = 1 } fa_dtype;
typedef enum { FA_FEDAVG = 0, FA_LITERAL = 1 } fa_mode;

typedef enum {
    FA_OK = 0,
    FA_ERR_ARG = -1,     /* bad argument (null pointer, size, dtype, slot) */
    FA_ERR_HIP = -2,     /* a HIP runtime call failed */
    FA_ERR_NOMEM = -3,   /* device or pinned allocation failed */
    FA_ERR_STATE = -4,   /* call out of order (e.g. finalize before any submit) */
    FA_ERR_NODEV = -5,   /* no usable gfx950 device */
    FA_ERR_ALIGN = -6,   /* pointer not 4-byte (f32) / 2-byte (bf16) aligned */
    FA_ERR_NCCL = -7     /* an RCCL call failed (FA_SHARD_CLIENT_RS) */
} fa_status;

/* fa_create flags */
/* n_gpus > 1: GPU g owns elements [g*n/G, (g+1)*n/G) of every client bucket; bit-exact, no collective. */
#define FA_SHARD_RANGE 0x1
/* Client-sharded: GPU g holds whole buckets of clients [c_g, c_{g+1}) (contiguous, balanced), reduces them
 * into an fp32 partial, and an RCCL reduce-scatter over xGMI (one communicator per GPU, ncclCommInitAll in
 * this process) sums the partials piece by piece, overlapped with the reduction of the next piece
 * (fa_tuning.rs_chunks pieces; GPU g ends with block g of every piece, fa_rs_segments).  The summation
 * order changes: within 1e-6 of sum_k |w_k x_k| (bit-exact at n_gpus = 1).  A bf16 output is the fp32
 * result rounded once to bf16 on each GPU after the exchange (so within one bf16 rounding of that). */
#define FA_SHARD_CLIENT_RS 0x2
/* Accumulate on arrival (range layout, FedAvg): as soon as receipts 0..k-1 of a round are all in, their
 * ordered chain is enqueued (continued in an fp32 accumulator), so the phase end only reduces the
 * clients that came late or out of order.  Same bits as one chain. */
#define FA_ACCUMULATE_ON_ARRIVAL 0x4
/* Test only: accept a device id more than once (several shards of one context on one GPU), so the
 * multi-GPU host logic runs on a one-GPU box.  RCCL refuses two ranks on one device, so with
 * FA_SHARD_CLIENT_RS the reduce-scatter is replaced by its definition (shard g's block := the sum of the
 * GPUs' partials in ring order, starting at rank g + 1 and ending at rank g as a ring reduce-scatter
 * accumulates it; one device launch); everything else of the layout is unchanged. */
#define FA_TEST_SHARED_DEVICE 0x100

int fa_version(void);
const char* fa_last_error(void); /* thread-local; "" when the last call succeeded */
int fa_device_count(int* out);   /* visible HIP devices */

/* Replaces the aggregator's state construction: systemAPI sys_(true, -1, ...)
 * + refactor() -> init_model_sate (aggregator.cpp:47,53; systemAPI.cpp:17-38).
 * Uses devices 0..n_gpus-1. */
int fa_create(fa_ctx** out, int n_gpus, int flags);
/* Same on an explicit device list (e.g. {LOCAL_RANK} for one process per GPU).  Every id once
 * (FA_SHARD_CLIENT_RS needs distinct devices for its RCCL communicators). */
int fa_create_ex(fa_ctx** out, const int* device_ids, int n_gpus, int flags);
void fa_destroy(fa_ctx* ctx);

/* One reduced bucket = the flattened named_parameters() of one model part
 * (model_part 1 -> parts[0].layers[0], aggregator.cpp:64; model_part m >= 2 ->
 * parts[1].layers[m-2], :118).  Allocates n_clients device slots per GPU. */
int fa_bucket_define(fa_ctx* ctx, int part_id, size_t n_elems, fa_dtype in, fa_dtype out, int n_clients,
                     fa_mode mode);
/* kTrainSize_10 of aggregator.cpp:48 for FA_LITERAL buckets (default 1000). */
int fa_set_literal_divisor(fa_ctx* ctx, int part_id, float divisor);

/* Replaces one receipt: torch::load into the global module + the per-parameter
 * update (aggregator.cpp:63-88 / :117-142).  Copies host_src (n_elems of the
 * bucket dtype, caller-owned, reusable on return) through ctx pinned staging
 * to the device slot asynchronously.  weight = w_k for FA_FEDAVG (ignored for
 * FA_LITERAL).  Submitting a slot twice in one round overwrites it. */
int fa_submit(fa_ctx* ctx, int part_id, int client_slot, const void* host_src, float weight);
/* Same, but host_src is pinned (hipHostMalloc'd / registered) memory that the
 * caller keeps unchanged until fa_finalize returns: no staging copy.
 * Small receipts are read where they are: on a one-GPU range context without
 * FA_ACCUMULATE_ON_ARRIVAL, a part whose D receipts total at most
 * FA_HOST_READ_MAX_BYTES keeps element-aligned pinned receipts in place, and the
 * fa_finalize* that ends the round has its kernels read them over PCIe -- with
 * FA_HOST_PINNED straight into the pinned destination: one stream round trip for
 * the phase (a small model's round is bound by round trips, not bytes).  Same
 * bits.  Calls before it that need the device slots (fa_reduce_part(s),
 * fa_sync_part, fa_bucket_slot/_piece, a pageable submit to the part) copy the
 * kept receipts in first.  A finalize that wrote a pinned destination this way
 * leaves the part's device output (fa_bucket_output) as it was, and
 * fa_copy_output of the part then fails with FA_ERR_STATE until its next
 * reduction.  fa_bucket_host_read tells whether a part's round is being kept
 * this way.  FA_HOST_READ=0 in the environment turns this off. */
#define FA_HOST_READ_MAX_BYTES (1u << 20)
int fa_submit_pinned(fa_ctx* ctx, int part_id, int client_slot, const void* host_src, float weight);

/* Same as fa_submit for a receipt scattered over n_segments host pieces whose
 * concatenation is the bucket (e.g. the parameter records of a torch::save
 * archive mapped in place, in named_parameters() order): gathered straight into
 * the pinned staging chunks, no intermediate flat copy. */
int fa_submit_gather(fa_ctx* ctx, int part_id, int client_slot, int n_segments, const void* const* srcs,
                     const size_t* bytes, float weight);
/* Zero-copy ingest: the segments lie in pinned memory (fa_host_alloc), e.g. the
 * parameter records of an archive inside a frame the network layer received
 * into a pinned buffer, and stay unchanged until fa_finalize* returns.  The
 * H2D DMA runs from them directly, no staging copy. */
int fa_submit_gather_pinned(fa_ctx* ctx, int part_id, int client_slot, int n_segments, const void* const* srcs,
                            const size_t* bytes, float weight);

/* Streaming ingest: a receipt handed over while its frame is still arriving (network_layer.cpp:48-65 reads
 * the whole frame first; aggregator.cpp:63-64 then decodes it).  fa_submit_piece_pinned enqueues the H2D
 * DMA of bytes [byte_offset, byte_offset + bytes) of the bucket (e.g. one parameter record, as soon as its
 * bytes are in) from pinned memory the caller keeps unchanged until fa_finalize* returns.  The slot counts
 * as the client's receipt only after fa_submit_commit (weight as for fa_submit); pieces never committed are
 * overwritten by the slot's next submit.  A piece overlapping one already sent replaces those bytes. */
int fa_submit_piece_pinned(fa_ctx* ctx, int part_id, int client_slot, size_t byte_offset, const void* host_src,
                           size_t bytes);
int fa_submit_commit(fa_ctx* ctx, int part_id, int client_slot, float weight);

/* Replaces the end of a phase: the reduced module handed to new_message()
 * (aggregator.cpp:96-106 / :153-166).  Waits for the submits, reduces on every
 * GPU, copies the result (out dtype) to host_dst and resets the round. */
int fa_finalize(fa_ctx* ctx, int part_id, void* host_dst);
/* Same, scattering the result over n_segments host pieces (e.g. the parameter
 * records of the reply archive inside the outgoing frame, aggregator.cpp:96-101
 * + network_layer.cpp:305-313).  flags: FA_HOST_PINNED = every segment is pinned
 * memory, DMA'd into directly; 0 = pageable, copied through the pinned chunks. */
#define FA_HOST_PINNED 0x1
int fa_finalize_gather(fa_ctx* ctx, int part_id, int n_segments, void* const* dsts, const size_t* bytes,
                       int flags);

/* Pinned (page-locked, every device can DMA it) host memory, for frame buffers
 * that feed fa_submit_gather_pinned / fa_finalize_gather(FA_HOST_PINNED). */
int fa_host_alloc(size_t bytes, void** out);
int fa_host_free(void* p);

/* Device-resident round (the data path with buckets already in HBM, e.g. a
 * zero-copy ingest that lands receipts straight in the slots): reduce the
 * part's slots into its device output on every GPU, no host copies.
 * h_weights: D floats, NULL = the weights given to fa_submit.  hip_stream:
 * NULL = ctx compute streams; non-NULL only for a single-GPU ctx.  Async. */
int fa_reduce_part(fa_ctx* ctx, int part_id, const float* h_weights, void* hip_stream);
/* Device pointer of client slot `client_slot` on GPU `gpu` (n_elems elements of
 * the input dtype, covering bucket elements [elem_offset, elem_offset+n_elems);
 * FA_SHARD_CLIENT_RS: only the GPU holding the client, whole bucket).  Slots of one bucket share one allocation
 * with a small per-slot byte skew (fa_tuning.slot_skew) so that the wave's
 * simultaneous loads spread over HBM channels. */
int fa_bucket_slot(fa_ctx* ctx, int part_id, int gpu, int client_slot, void** d_ptr, size_t* n_elems,
                   size_t* elem_offset);
/* Range layout: a GPU whose client slots would span more than 48 GiB holds them as pieces of <= 16 GiB of
 * slots each (fa_tuning.piece_span_kib / piece_split_kib, taken at fa_bucket_define), reduced
 * one launch per piece.  fa_bucket_slot then fails (FA_ERR_STATE); a slot is written piece by piece instead.
 * n_pieces: 1 for every other part. */
int fa_bucket_pieces(fa_ctx* ctx, int part_id, int gpu, int* n_pieces);
/* Piece `piece` of client slot `client_slot` on GPU `gpu`: n_elems elements of the input dtype covering
 * bucket elements [elem_offset, elem_offset+n_elems). */
int fa_bucket_piece(fa_ctx* ctx, int part_id, int gpu, int piece, int client_slot, void** d_ptr, size_t* n_elems,
                    size_t* elem_offset);
/* The part's device output on GPU `gpu` (range: its shard, `out` dtype; rs: its fp32 shard, the blocks
 * fa_rs_segments lists, concatenated). */
int fa_bucket_output(fa_ctx* ctx, int part_id, int gpu, void** d_ptr);
/* This round's receipts so far and how many leading client slots are already reduced
 * (FA_ACCUMULATE_ON_ARRIVAL; n_reduced == D once the round's result is ready). */
int fa_bucket_progress(fa_ctx* ctx, int part_id, int* n_submitted, int* n_reduced);
/* Whether the part's round so far is kept host-side to be read in place (fa_submit_pinned, small receipts):
 * *kept = 1 when every receipt its reduction reads is held that way, so the fa_finalize* ending the round
 * reduces them itself (a caller then skips fa_reduce_parts for it, which would copy them in first); else 0. */
int fa_bucket_host_read(fa_ctx* ctx, int part_id, int* kept);
/* Batched device-resident reduction of several parts (e.g. all last-part layers of a phase,
 * aggregator.cpp:108-150): one launch per GPU covers every part that is FedAvg, range-laid-out, has at
 * most 128 clients and is below the phased kernel's size (a segment table: one bucket per segment,
 * the same ordered chain, the same bits); larger parts get their own launch.  h_weights: NULL or one
 * entry per part (NULL entry = the weights given to fa_submit).  A following fa_finalize* of these
 * parts only copies the result out.  Async on hip_stream (NULL = ctx compute streams). */
int fa_reduce_parts(fa_ctx* ctx, int n_parts, const int* part_ids, const float* const* h_weights, void* hip_stream);
/* D2H of the part's current device output (after fa_reduce_part), waiting for it.  FA_ERR_STATE when the
 * part has no device output: never reduced, or its last round was read in place straight into a pinned
 * reply (fa_submit_pinned). */
int fa_copy_output(fa_ctx* ctx, int part_id, void* host_dst);
/* CRC-32 (zlib's: IEEE 802.3, reflected, initial and final inversion) of consecutive byte segments of the
 * part's current device output: segment k = bytes [sum_{j<k} bytes[j], + bytes[k]) of the reduced bucket in
 * its out dtype; the segments cover it exactly.  Computed on the GPU(s) holding the output, from HBM: for the
 * zip records of a reply built around the reduced parameters (aggregator.cpp:96-101 hands the module to
 * torch::save, which writes a CRC-32 per record), so the host need not read the reply back.  Waits for the
 * reduction and returns with the CRCs.  FA_ERR_STATE when the part has no device output (never reduced, or
 * its last round was read in place straight into a pinned reply). */
int fa_output_crc32(fa_ctx* ctx, int part_id, int n_segments, const size_t* bytes, uint32_t* crcs);
/* Wait for all copy and compute work of the ctx. */
int fa_sync(fa_ctx* ctx);

/* Raw device entry for benches and device-resident callers: reduce D client
 * buckets already resident on device `gpu` into d_out.  d_clients[k] are device
 * pointers, h_weights a host array of D floats (copied into kernel arguments,
 * any D >= 1).  d_init (nullable, fp32, n) continues an earlier chain: acc
 * starts at d_init[i] instead of +0 (used to split clients across launches or
 * GPUs bit-exactly).  Enqueued on hip_stream (a hipStream_t; NULL = the
 * ctx's compute stream of `gpu`); returns without synchronizing.  ctx may be
 * NULL except for bf16 output with D > 128 (needs ctx scratch). */
int fa_reduce_device(fa_ctx* ctx, int gpu, const void* const* d_clients, const float* h_weights, int D, size_t n,
                     fa_dtype in, void* d_out, fa_dtype out, fa_mode mode, const float* d_init, void* hip_stream);

/* Compute-node aggregation of an intermediate model part.
 * A compute node keeps one State per client (systemAPI::init_state_vector,
 * systemAPI.cpp:3-15; compute_node.cpp), and the paper (EdgeSys 3) aggregates
 * them, which the reference code never does.  Here every client copy becomes
 * sum_k w_k x_k, in place: the same ordered fp32 FMA chain as FA_FEDAVG,
 * rounded once to the slot dtype and written back to all D slots, so each
 * client continues training from the FedAvg model.  HBM traffic is D*s read +
 * D*s written per element.
 * fa_sync_device: raw device pointers, any D >= 1 (ctx needed only for D > 128).
 * fa_sync_part: the part's own slots on every GPU of the ctx (range shards sync
 * their ranges); h_weights NULL = the weights given to fa_submit.  Both are
 * async on hip_stream (NULL = ctx compute stream). */
int fa_sync_device(fa_ctx* ctx, int gpu, void* const* d_clients, const float* h_weights, int D, size_t n, fa_dtype dt,
                   void* hip_stream);
int fa_sync_part(fa_ctx* ctx, int part_id, const float* h_weights, void* hip_stream);

/* Phased-kernel meetings on HIP device `device` that stopped waiting for the rest of the grid since the
 * process started (each counts one workgroup's bounded wait running out).  Non-zero means the persistent
 * grid was not co-resident -- the GPU was shared with other kernels -- and those launches ran slower;
 * results are unaffected.  Synchronizes with the device. */
int fa_phased_timeouts(int device, uint64_t* count);

/* The phased kernel gives each HIP stream it runs on a counter slot of its own on that device (the first
 * 48 streams; later ones share hashed slots, which costs speed, never results).  A context returns its own
 * streams' slots in fa_destroy; a caller that passed its own stream (fa_reduce_device, fa_sync_device,
 * fa_reduce_part / fa_reduce_parts / fa_sync_part with hip_stream) returns that stream's slot here before it
 * destroys or stops using the stream, so a long-lived process cycling through many streams keeps owned
 * slots.  Launches still in flight on the stream stay correct.  A stream without a slot: FA_OK, no-op. */
int fa_release_stream(int device, void* hip_stream);

/* Literal mode divisor used by fa_reduce_device when ctx == NULL. */
#define FA_DEFAULT_DIVISOR 1000.0f

/* Synthetic input generator on device, identical to oracle/fa_oracle.c:
 * element i = uniform[-1,1) from splitmix64(seed ^ client<<40 ^ (idx0+i)),
 * bf16 = round-to-nearest-even of that value. */
int fa_fill_uniform(void* d_dst, size_t n, fa_dtype dt, uint64_t seed, uint32_t client, uint64_t idx0,
                    void* hip_stream);

/* Kernel and layout tuning knobs for benches (every field: 0 = keep the current value). */
typedef struct {
    int block;        /* threads per workgroup: 64, 128 or 256 */
    int max_blocks;   /* grid cap, grid-stride beyond it; -1 = uncapped (one-shot grid) */
    int unroll;       /* clients loaded per FMA group: 4, 8 or 16 */
    int load_policy;  /* client loads: 1 default cache policy, 2 non-temporal */
    int store_policy; /* output stores: 1 plain, 2 nt, 3 sc1 (write-through), 4 sc0 sc1 */
    int slot_skew;    /* bytes between consecutive client slots beyond 4 KiB alignment (multiple of 16);
                         -1 = none, -2 (default) = by slot size: 512 for slots of >= 48 MiB, else 2048;
                         applies to buckets defined afterwards */
    int walk;         /* FedAvg grid walk over a bucket: 1 linear, 2 each XCD's workgroups own one contiguous
                         eighth, 3 the same with the odd eighths walked backwards (one-shot grid only),
                         4 phased: a persistent grid (one workgroup per CU) reduces a phase into LDS and
                         registers, then writes it, so the output never streams beside the inputs,
                         5 (default) phased with a larger register stage (fewer phases; bf16 inputs
                         take the form of walk 6), 6 phased with 512-thread workgroups (2 waves per
                         SIMD).  Buckets smaller than one phase (walk 4: 18.9 M, walks 5 and 6:
                         23.1 M elements per GPU on 256 CUs, f32 or bf16) take walk 2.  The phased
                         kernels always use nt loads and sc1 stores.  With walk 5, a bucket below one
                         phase with >= 16 clients takes one phase sized to it */
    int rs_chunks;    /* FA_SHARD_CLIENT_RS: pieces per round (default 8) */
    int piece_span_kib;  /* range pieces: KiB of a GPU's slots per piece (default 16 GiB); -1 = never cut */
    int piece_split_kib; /* range pieces: a GPU's slots are cut above this many KiB (default 48 GiB); -1 = always */
} fa_tuning;
/* Process defaults: every fa_ctx created afterwards starts from them, and fa_reduce_device /
 * fa_sync_device without a ctx use them. */
int fa_set_tuning(const fa_tuning* t);
int fa_get_tuning(fa_tuning* t);
/* One context's own tuning (buckets defined afterwards take its slot_skew). */
int fa_ctx_set_tuning(fa_ctx* ctx, const fa_tuning* t);
int fa_ctx_get_tuning(fa_ctx* ctx, fa_tuning* t);

/* The rs layout's block-cyclic ownership (FA_SHARD_CLIENT_RS): bucket elements [lo, hi) that GPU `gpu`
 * of n_gpus holds after the reduce-scatter of a bucket of n elements in `chunks` pieces, in the order of
 * its shard (lo_hi: room for 2 * cap values; elements >= n are padding).  Returns the segment count.
 * Pure host arithmetic (no device needed). */
int fa_rs_segments(size_t n, int n_gpus, int chunks, int gpu, size_t* lo_hi, int cap);

#ifdef __cplusplus
}
#endif
#endif /* FEDAVG_FA_H_ */
