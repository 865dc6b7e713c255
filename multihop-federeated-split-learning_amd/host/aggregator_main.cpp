// aggregator_main.cpp -- drop-in replacement for pipeline_simulation/aggregator.cpp.
//
// Same process role (node id -1), same CLI (-i/-d/-c, aggregator.cpp:13-32),
// same wire protocol and the same round structure (aggregator.cpp:55-167):
//   refactor  <- the init node's REFACTOR_DATA_OWNER message (:52-53)
//   phase 1   <- D receipts of model_part 1, reduced, reply to 0 and i+c+1 (:59-106)
//   phase 2   <- D*L receipts of model_parts 2..L+1, reduced, reply per layer (:108-166)
// What changes is only how a receipt is consumed: frames are received into
// pooled pinned buffers (one reader thread per connection), the archive is
// mapped in place (host/archive.h) and its parameter records are DMA'd straight
// from the frame to the client's device slot (fa_submit_gather_pinned); at the
// end of a phase one ordered FMA chain per bucket runs on the MI355X and the
// result is DMA'd straight into the parameter records of the reply frame
// (fa_finalize_gather).  The reply archive is the last receipt's with the
// reduced parameters (buffers stay the last receipt's, as in the reference),
// built once and sent to every data owner.
//
// Client slots (the FMA chain order) are fixed, not arrival-ordered: the
// refactor message's data-owner list when it has D entries, else the reply
// convention of aggregator.cpp:102-106 (owner ids 0, C+1, ..., C+D-1).
//
// --mode literal reproduces the reference's arithmetic bit-for-bit
// (fl(fl(x_last + x_last) / 1000)); --mode fedavg (default) is
// the north star's weighted mean (weights n_k/N from --samples, else 1/D).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <set>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "archive.h"
#include "fedavg/fa.h"
#include "net.h"
#include "receipts.h"

using namespace fahost;

namespace {

struct Options {
    int id = -1, data_owners = 1, compute_nodes = 1;
    int gpus = 1, rounds = -1, port_base = 8079, last_layers = -1;
    fa_mode mode = FA_FEDAVG;
    float divisor = 1000.0f;  // kTrainSize_10, aggregator.cpp:48
    bool discover = false, pinned = true;
    bool rs = false;     // --layout rs: clients dealt to the GPUs, RCCL reduce-scatter of fp32 partials
    bool eager = false;  // --eager: accumulate on arrival (the chain advances with the in-order receipts)
    // --test-shared-device: the --gpus G shards all on GPU 0 (FA_TEST_SHARED_DEVICE; the rs exchange replaced
    // by its definition), so the multi-GPU layouts run end to end on a one-GPU box (tests only)
    bool shared_device = false;
    int rs_chunks = 0;
    double link_mbps = 0;
    // failure detection: after stall_report_s without a receipt, name the data owners still missing;
    // after receipt_timeout_s (0 = wait forever, the reference's behaviour), give up with exit code 3
    double stall_report_s = 60, receipt_timeout_s = 0;
    // large receipts received at once (NetLayer::set_rx_concurrency; 0 = no limit).  C4 at D = 64 over
    // loopback (gpurun_out r02s40), owner-view round: unlimited 3.15-3.32 s, 4 at a time 2.05-2.48 s,
    // 16 at a time 2.15-2.31 s -- the phase end drops from 0.48-0.51 s to 0.04-0.17 s
    int rx_concurrency = 8;
    int senders = 8;  // fan-out sender threads (each destination keeps to one, in order)
    // streaming ingest: receipt frames of at least this many bytes go to their slot record by record while
    // they arrive (NetLayer::set_streaming; pinned frames only); 0 = off
    size_t stream_min = 1u << 20;
    bool gpu_crc = true;  // --crc gpu|host: the reply records' CRC-32s from the GPU (fa_output_crc32) or the host
    std::map<int, double> samples;  // client id -> n_k
};

void usage() {
    std::cerr << "usage: fa_aggregator -i ID -d DATA_OWNERS -c COMPUTE_NODES [--mode fedavg|literal] [--gpus G]\n"
                 "       [--rounds R] [--port-base P] [--discover] [--link-mbps M] [--samples id:n,...]\n"
                 "       [--divisor K] [--last-layers L] [--no-pinned] [--layout range|rs] [--rs-chunks C]\n"
                 "       [--eager] [--stall-report S] [--receipt-timeout S] [--rx-concurrency K]\n"
                 "       [--senders S] [--stream-min-bytes N] [--crc gpu|host] [--test-shared-device]\n";
}

bool parse_args(int argc, char** argv, Options* o) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&](const char* what) -> const char* {
            if (i + 1 >= argc) {
                std::cerr << "missing value for " << what << "\n";
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "-i" || a == "--id") o->id = std::atoi(val("-i"));
        else if (a == "-d" || a == "--data_owners") o->data_owners = std::atoi(val("-d"));
        else if (a == "-c" || a == "--compute_nodes") o->compute_nodes = std::atoi(val("-c"));
        else if (a == "--gpus") o->gpus = std::atoi(val("--gpus"));
        else if (a == "--rounds") o->rounds = std::atoi(val("--rounds"));
        else if (a == "--port-base") o->port_base = std::atoi(val("--port-base"));
        else if (a == "--last-layers") o->last_layers = std::atoi(val("--last-layers"));
        else if (a == "--divisor") o->divisor = (float)std::atof(val("--divisor"));
        else if (a == "--discover") o->discover = true;
        else if (a == "--no-pinned") o->pinned = false;
        else if (a == "--eager") o->eager = true;
        else if (a == "--test-shared-device") o->shared_device = true;
        else if (a == "--rs-chunks") o->rs_chunks = std::atoi(val("--rs-chunks"));
        else if (a == "--stall-report") o->stall_report_s = std::atof(val("--stall-report"));
        else if (a == "--receipt-timeout") o->receipt_timeout_s = std::atof(val("--receipt-timeout"));
        else if (a == "--rx-concurrency") o->rx_concurrency = std::atoi(val("--rx-concurrency"));
        else if (a == "--senders") o->senders = std::atoi(val("--senders"));
        else if (a == "--stream-min-bytes") o->stream_min = (size_t)std::strtoull(val("--stream-min-bytes"), nullptr, 0);
        else if (a == "--crc") {
            std::string c = val("--crc");
            if (c == "host") o->gpu_crc = false;
            else if (c != "gpu") return false;
        }
        else if (a == "--layout") {
            std::string l = val("--layout");
            if (l == "rs") o->rs = true;
            else if (l != "range") return false;
        }
        else if (a == "--link-mbps") o->link_mbps = std::atof(val("--link-mbps"));
        else if (a == "--mode") {
            std::string m = val("--mode");
            if (m == "literal") o->mode = FA_LITERAL;
            else if (m == "fedavg") o->mode = FA_FEDAVG;
            else return false;
        } else if (a == "--samples") {
            std::stringstream ss(val("--samples"));
            std::string tok;
            while (std::getline(ss, tok, ',')) {
                const size_t c = tok.find(':');
                if (c == std::string::npos) return false;
                o->samples[std::atoi(tok.substr(0, c).c_str())] = std::atof(tok.substr(c + 1).c_str());
            }
        } else if (a == "-h" || a == "--help") {
            return false;
        } else {
            std::cerr << "unknown argument " << a << "\n";
            return false;
        }
    }
    return o->data_owners >= 1 && o->stall_report_s > 0 && o->receipt_timeout_s >= 0;
}

// parts[1].layers.size() for the aggregator's ModelPart(start, -1) (systemAPI.cpp:19):
// resnet_part / lenet_part always return two Sequentials for end == -1
// (resnet_split.cpp:176-188, lenet_help.cpp:170-183); vgg_part returns two iff
// start - 1 <= 20 (vgg_help.cpp:250-256, ModelPart passes start - 1, models.h:25).
int last_part_layers(int model_name, int start) {
    if (model_name == 0) return (start - 1) <= 20 ? 2 : 1;
    return 2;
}

long now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

double secs_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
}

#define FA_CHECK(call)                                                                       \
    do {                                                                                     \
        int rc_ = (call);                                                                    \
        if (rc_ != FA_OK) {                                                                  \
            std::cerr << "[aggregator] " #call " failed: " << fa_last_error() << "\n";       \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

// Replies of at least this many parameter bytes get their records' CRC-32s from the GPU (fa_output_crc32);
// smaller ones are sealed on the host, which takes less than the call's round trip.
constexpr size_t kGpuCrcMinBytes = 1u << 20;

class Aggregator {
public:
    Aggregator(const Options& o, NetLayer* net, const std::vector<int>& owners) : o_(o), net_(net) {
        int flags = o.rs ? FA_SHARD_CLIENT_RS : o.gpus > 1 ? FA_SHARD_RANGE : 0;
        if (o.eager) flags |= FA_ACCUMULATE_ON_ARRIVAL;
        if (o.shared_device) {
            const std::vector<int> zeros((size_t)std::max(1, o.gpus), 0);
            FA_CHECK(fa_create_ex(&ctx_, zeros.data(), o.gpus, flags | FA_TEST_SHARED_DEVICE));
        } else {
            FA_CHECK(fa_create(&ctx_, o.gpus, flags));
        }
        FA_CHECK(fa_set_literal_divisor(ctx_, -1, o.divisor));
        if (o.rs_chunks > 0) {
            fa_tuning t{};
            t.rs_chunks = o.rs_chunks;
            FA_CHECK(fa_ctx_set_tuning(ctx_, &t));
        }
        std::vector<int> order = owners;
        if ((int)order.size() != o.data_owners) {
            order = {0};
            for (int i = 0; i < o.data_owners - 1; ++i) order.push_back(i + o.compute_nodes + 1);
        }
        for (int k = 0; k < (int)order.size(); ++k) slots_.insert({order[k], k});
        expected_ = order;
        claimed_.assign(o.data_owners, 0);
    }
    ~Aggregator() { fa_destroy(ctx_); }

    // Stale receipts across rounds (host/receipts.h): a byte copy of a receipt its owner already had reduced
    // (a late copy of an earlier round's) is dropped -- never counted, never in a slot.
    void end_phase() {
        ledger_.end_phase();
        // frames that ended without a receipt for this phase (a malformed frame, one still queued for the
        // next phase) need no stream any more: their receipts, if any, take the plain path
        streams_.erase(std::remove_if(streams_.begin(), streams_.end(),
                                      [](const Stream& s) { return s.in->ended.load(std::memory_order_acquire); }),
                       streams_.end());
    }

    // ---------------------------------------------------------------- streaming ingest
    //
    // The reference reads a whole frame before anything else happens (network_layer.cpp:48-65) and only then
    // decodes it (aggregator.cpp:63-64); so did this process until round 6, and a phase ended with the H2D
    // copies of the receipts that landed last.  The archive's parameter records (data/<key>) come first in
    // the zip, stored and 64-byte aligned, and every receipt of a bucket is the same module saved again: so
    // the records' places in a frame of a given length are those of the bucket's previous receipt.  A large
    // frame is announced while it arrives (NetLayer::set_streaming); once its owner and bucket are known and
    // the bucket has a layout for its length, each record is DMA'd to the slot as soon as its bytes are in
    // (fa_submit_piece_pinned).  When the frame is complete the archive is parsed as before; if its records
    // are where they were predicted, the slot is committed (fa_submit_commit), else the receipt is submitted
    // the plain way over the streamed bytes.  Only a slot whose owner has no receipt of the bucket yet this
    // phase is streamed into, by one frame at a time, and a receipt that lands whole stops any other frame
    // streaming into its slot -- so a stale copy can never overwrite a receipt taken (the ledger still judges
    // every frame once it is complete; a stream it drops was never committed).
    void set_phase(const std::vector<int>& mps) { phase_mps_ = std::set<int>(mps.begin(), mps.end()); }

    void pump() {
        intake();
        for (auto it = streams_.begin(); it != streams_.end();) {
            Stream& s = *it;
            if (s.in->failed.load(std::memory_order_acquire)) {  // the connection broke: nothing comes of it
                it = streams_.erase(it);
                continue;
            }
            if (s.slot < 0 && !s.cancelled) claim(s);
            if (s.slot >= 0) feed(s, s.in->have.load(std::memory_order_acquire));
            ++it;
        }
    }

    unsigned long long streamed() const { return streamed_; }
    unsigned long long stream_fallbacks() const { return stream_fallbacks_; }
    unsigned long long streamed_bytes() const { return streamed_bytes_; }

    static ReceiptKey key_of(const Receipt& r) {
        return ReceiptKey{r.t_start, r.blob_len, archive_fingerprint(r.blob(), r.blob_len)};
    }

    // A receipt of the other phase is never taken (see main): counted as a stale copy when it is a byte copy
    // of one already reduced, else as ignored (a retransmission of this round's).
    void other_phase(const Receipt& r, int phase) {
        take_stream(r);
        if (ledger_.is_reduced_copy(r.client_id, r.model_part, key_of(r))) {
            std::cerr << "[aggregator] stale part " << r.model_part << " from owner " << r.client_id
                      << " during phase " << phase << " (a byte copy of a receipt already reduced): dropped\n";
            ++stale_dropped_;
        } else {
            std::cerr << "[aggregator] part " << r.model_part << " from owner " << r.client_id << " during phase "
                      << phase << " (a retransmission of this round's): ignored\n";
            ++ignored_;
        }
    }

    // Consumes one receipt of bucket `mp` into its client slot.  Returns whether it is the first receipt of
    // this (owner, bucket) in the round: a retransmission replaces the slot's contents (the newest one wins,
    // as a second torch::load would) but is not another receipt -- the phase waits for D distinct owners.
    // A stale receipt (above) is dropped: returns false without touching the slot.
    bool absorb(const Receipt& r) {
        const Stream st = take_stream(r);  // the frame's own stream, if it was streamed into a slot
        const ReceiptKey key = key_of(r);
        const ReceiptLedger::Verdict v = ledger_.check(r.client_id, r.model_part, key);
        if (v.stale) {
            std::cerr << "[aggregator] stale part " << r.model_part << " from owner " << r.client_id << " (" << v.why
                      << "): dropped\n";
            ++stale_dropped_;
            return false;
        }
        if (!v.note.empty()) {
            std::cerr << "[aggregator] part " << r.model_part << " from owner " << r.client_id << " " << v.note << "\n";
            ++clock_back_;
        }
        const auto t0 = std::chrono::steady_clock::now();
        TorchArchive ar;
        std::string err;
        if (!ar.parse(r.blob(), r.blob_len, &err)) {
            std::cerr << "[aggregator] receipt from " << r.client_id << ": " << err << "\n";
            std::exit(1);
        }
        Bucket& b = buckets_[r.model_part];
        const int es = ar.param_elem_size();  // the bucket dtype: fp32 (the reference) or bf16 (config C3)
        if (!b.defined) {
            if (es == 0) {
                std::cerr << "[aggregator] bucket " << r.model_part << ": parameters not all fp32 or all bf16\n";
                std::exit(1);
            }
            b.numel = (size_t)ar.param_numel();
            b.elem = es;
            const fa_dtype dt = es == 4 ? FA_F32 : FA_BF16;
            FA_CHECK(fa_bucket_define(ctx_, r.model_part, b.numel, dt, dt, o_.data_owners, o_.mode));
            b.defined = true;
        } else if ((size_t)ar.param_numel() != b.numel || es != b.elem) {
            std::cerr << "[aggregator] bucket " << r.model_part << " changed size or dtype\n";
            std::exit(1);
        }
        const int slot = slot_of(r.client_id);
        cancel_streams(r.client_id, r.model_part);  // nothing else writes this slot from here on
        std::vector<const void*> ptrs;
        std::vector<size_t> bytes;
        if (ar.param_segments(&ptrs, &bytes)) {
            auto recs = records_of(r, ptrs, bytes);
            if (st.slot == slot && st.recs && *st.recs == *recs) {
                // streamed: the layout held; the records not sent yet go now, then the slot counts
                Stream done = st;
                feed(done, r.frame->size());
                FA_CHECK(fa_submit_commit(ctx_, r.model_part, slot, weight_of(r.client_id)));
                ++streamed_;
            } else if (r.frame->pinned) {  // DMA from the frame itself; it is held until the bucket is finalized
                if (st.slot >= 0) ++stream_fallbacks_;  // the layout changed: the plain submit overwrites
                FA_CHECK(fa_submit_gather_pinned(ctx_, r.model_part, slot, (int)ptrs.size(), ptrs.data(),
                                                 bytes.data(), weight_of(r.client_id)));
                b.held.push_back(r.frame);
            } else {
                FA_CHECK(fa_submit_gather(ctx_, r.model_part, slot, (int)ptrs.size(), ptrs.data(), bytes.data(),
                                          weight_of(r.client_id)));
            }
        } else {  // strided parameters: flatten first
            std::vector<uint8_t> flat(b.numel * (size_t)b.elem);
            if (!ar.gather_param_bytes(flat.data(), &err)) {
                std::cerr << "[aggregator] " << err << "\n";
                std::exit(1);
            }
            FA_CHECK(fa_submit(ctx_, r.model_part, slot, flat.data(), weight_of(r.client_id)));
        }
        if (r.frame->pinned && !ptrs.empty()) {  // the layout later frames of this length are streamed with
            b.recs = records_of(r, ptrs, bytes);
            b.recs_len = r.blob_len;
        }
        b.bytes_in += r.blob_len;
        ledger_.accept(r.client_id, r.model_part, key);
        const bool first = b.arrived.insert(r.client_id).second;
        b.last = r;  // template of the reply: the last receipt (its buffers travel back, as in the reference)
        st_.absorb_s += secs_since(t0);
        if (!first) {
            std::cerr << "[aggregator] part " << r.model_part << ": owner " << r.client_id << " sent it again\n";
            ++replaced_;
        }
        return first;
    }

    // Reduces bucket mp and returns the framed reply, built once and shared by every destination:
    // the last receipt's archive around the reduced parameters, which the D2H copy writes straight
    // into the frame's parameter records.
    std::shared_ptr<const Bytes> reduce(int mp) {
        Bucket& b = buckets_[mp];
        const auto t0 = std::chrono::steady_clock::now();
        TorchArchive ar;
        std::string err;
        if (!ar.parse(b.last.blob(), b.last.blob_len, &err)) {
            std::cerr << "[aggregator] reply for part " << mp << ": " << err << "\n";
            std::exit(1);
        }
        Message m;  // Task(myid, aggregation_, myid) with model_part, aggregator.cpp:96-101
        m.type = OPERATION;
        m.client_id = o_.id;
        m.prev_node = o_.id;
        m.type_op = AGGREGATION;
        m.model_part = mp;
        m.t_start = now_ms();
        char* values = nullptr;
        auto f = operation_frame(m, ar.size(), &values);
        std::vector<void*> dsts;
        std::vector<size_t> bytes;
        double t_fin;
        if (ar.layout_into((uint8_t*)values, &dsts, &bytes, nullptr)) {
            const auto t1 = std::chrono::steady_clock::now();
            FA_CHECK(fa_finalize_gather(ctx_, mp, (int)dsts.size(), dsts.data(), bytes.data(),
                                        f->pinned ? FA_HOST_PINNED : 0));
            // the records' CRC-32s from the reduced bucket on the GPU (a few us; the host would read the
            // whole reply back); a part read in place into its reply has no device output: the host seals it
            std::vector<uint32_t> crcs(dsts.size());
            const bool gpu_crc = o_.gpu_crc && !bytes.empty() && b.numel * (size_t)b.elem >= kGpuCrcMinBytes &&
                                 fa_output_crc32(ctx_, mp, (int)bytes.size(), bytes.data(), crcs.data()) == FA_OK;
            t_fin = secs_since(t1);
            if (!gpu_crc || !ar.seal_params_with((uint8_t*)values, crcs.data())) ar.seal_params((uint8_t*)values);
        } else {  // strided parameters: through a flat copy
            const auto t1 = std::chrono::steady_clock::now();
            std::vector<uint8_t> out(b.numel * (size_t)b.elem);
            FA_CHECK(fa_finalize(ctx_, mp, out.data()));
            t_fin = secs_since(t1);
            if (!ar.with_param_bytes_into(out.data(), (uint8_t*)values, &err)) {
                std::cerr << "[aggregator] reply for part " << mp << ": " << err << "\n";
                std::exit(1);
            }
        }
        b.held.clear();
        b.arrived.clear();
        b.bytes_in = 0;
        st_.finalize_s += t_fin;
        st_.frame_s += secs_since(t0) - t_fin;
        return f;
    }

    // Fan-out to node 0 and the data owners i + c + 1, i < D - 1 (aggregator.cpp:102-106, :158-164).
    void fan_out(const std::shared_ptr<const Bytes>& f) {
        net_->send(0, f);
        for (int i = 0; i < o_.data_owners - 1; ++i) net_->send(i + o_.compute_nodes + 1, f);
    }

    size_t bytes_in(int mp) { return buckets_[mp].bytes_in; }
    unsigned long long stale_dropped() const { return stale_dropped_; }
    unsigned long long ignored() const { return ignored_; }
    unsigned long long replaced() const { return replaced_; }
    unsigned long long clock_back() const { return clock_back_; }

    // The data owners whose receipt of bucket mp has not arrived this round ("mp 2: 4 7 9").
    std::string missing(const std::vector<int>& mps) {
        std::ostringstream os;
        for (int mp : mps) {
            const auto& got = buckets_[mp].arrived;
            std::ostringstream ids;
            int n = 0;
            for (int c : expected_)
                if (!got.count(c)) ids << (n++ ? " " : "") << c;
            if (n) os << (os.tellp() > 0 ? "; " : "") << "part " << mp << ": " << n << " owner(s) [" << ids.str() << "]";
        }
        return os.str();
    }

    // The reductions of a phase's buckets as one batched launch (fa_reduce_parts: the last-part layers of
    // phase 2, aggregator.cpp:108-150, are one segment table); the following reduce() calls then only
    // copy each result into its reply.  With --eager the chains already ran as the receipts arrived.
    void reduce_all(const std::vector<int>& mps) {
        if (o_.eager || mps.size() < 2) return;
        // parts whose receipts the library keeps to read in place (small pinned receipts, fa_bucket_host_read):
        // each finalize then reduces straight into its reply, one round trip per part instead of a launch here
        // and a copy there.  Asked of the library, which alone knows every condition (the environment, the
        // frames' alignment and pinning); when some part is not kept, the batched launch covers them all.
        if (std::all_of(mps.begin(), mps.end(), [&](int mp) {
                int kept = 0;
                FA_CHECK(fa_bucket_host_read(ctx_, mp, &kept));
                return kept == 1;
            }))
            return;
        const auto t0 = std::chrono::steady_clock::now();
        FA_CHECK(fa_reduce_parts(ctx_, (int)mps.size(), mps.data(), nullptr, nullptr));
        st_.finalize_s += secs_since(t0);
    }

    // Host-side time split since the last call: archive parse + slot staging (absorb), the GPU
    // reduction incl. its D2H copy (finalize), the reply archive + frame (frame).
    struct Stats {
        double absorb_s = 0, finalize_s = 0, frame_s = 0;
    };
    Stats take_stats() {
        Stats s = st_;
        st_ = Stats{};
        return s;
    }

private:
    struct Rec {  // one parameter record: where it lies in the archive, its bytes, where they go in the bucket
        size_t off = 0, bytes = 0, at = 0;
        bool operator==(const Rec& o) const { return off == o.off && bytes == o.bytes && at == o.at; }
    };
    using Recs = std::shared_ptr<const std::vector<Rec>>;
    struct Stream {
        std::shared_ptr<Inflight> in;
        int slot = -1;           // the slot it streams into (-1: none yet)
        bool cancelled = false;  // a receipt of its (owner, bucket) landed whole: never streamed again
        Recs recs;               // the layout it streams by (the bucket's at the time it was claimed)
        size_t next = 0;         // records sent so far
    };

    static Recs records_of(const Receipt& r, const std::vector<const void*>& ptrs, const std::vector<size_t>& bytes) {
        auto v = std::make_shared<std::vector<Rec>>();
        size_t at = 0;
        for (size_t i = 0; i < ptrs.size(); ++i) {
            v->push_back(Rec{(size_t)((const uint8_t*)ptrs[i] - r.blob()), bytes[i], at});
            at += bytes[i];
        }
        return v;
    }

    void intake() {
        for (auto& in : net_->take_new_streams()) streams_.push_back(Stream{in});
    }

    Stream take_stream(const Receipt& r) {
        intake();
        for (auto it = streams_.begin(); it != streams_.end(); ++it)
            if (it->in->buf.get() == r.frame.get()) {
                Stream s = *it;
                streams_.erase(it);
                return s;
            }
        return Stream{};
    }

    void cancel_streams(int owner, int mp) {
        for (auto& s : streams_)
            if (s.in->client_id == owner && s.in->model_part == mp) {
                s.slot = -1;
                s.cancelled = true;
            }
    }

    void claim(Stream& s) {
        const Inflight& in = *s.in;
        if (!phase_mps_.count(in.model_part) || !in.buf->pinned) return;
        auto bi = buckets_.find(in.model_part);
        if (bi == buckets_.end() || !bi->second.defined) return;
        Bucket& b = bi->second;
        if (!b.recs || b.recs->empty() || b.recs_len != in.blob_len || b.arrived.count(in.client_id)) return;
        auto si = slots_.find(in.client_id);
        if (si == slots_.end()) return;  // an owner not seen yet takes its slot when its receipt lands
        for (auto& o : streams_)
            if (&o != &s && o.slot >= 0 && o.in->client_id == in.client_id && o.in->model_part == in.model_part) return;
        s.slot = si->second;
        s.recs = b.recs;
        s.next = 0;
        b.held.push_back(in.buf);  // DMA'd from until the bucket is finalized, whatever becomes of the frame
    }

    void feed(Stream& s, size_t have) {
        const Inflight& in = *s.in;
        while (s.next < s.recs->size()) {
            const Rec& rc = (*s.recs)[s.next];
            if (in.blob_off + rc.off + rc.bytes > have) break;
            FA_CHECK(fa_submit_piece_pinned(ctx_, in.model_part, s.slot, rc.at, in.buf->data() + in.blob_off + rc.off,
                                            rc.bytes));
            streamed_bytes_ += rc.bytes;
            ++s.next;
        }
    }

    struct Bucket {
        bool defined = false;
        size_t numel = 0, bytes_in = 0;
        int elem = 4;  // bytes per parameter element: 4 fp32, 2 bf16
        Recs recs;            // the parameter records of the last pinned receipt (the streaming layout)
        size_t recs_len = 0;  // ... for archives of this length
        Receipt last;
        std::vector<std::shared_ptr<const Bytes>> held;  // pinned frames DMA'd from, until finalize
        std::set<int> arrived;  // client ids received this round
    };

    int slot_of(int client) {
        auto it = slots_.find(client);
        if (it == slots_.end()) {  // an id outside the expected list takes the first slot nobody claimed
            int s = 0;
            while (s < o_.data_owners && claimed_[s]) ++s;
            if (s == o_.data_owners) {
                std::cerr << "[aggregator] more distinct clients than -d " << o_.data_owners << "\n";
                std::exit(1);
            }
            for (auto kv = slots_.begin(); kv != slots_.end();) kv = kv->second == s ? slots_.erase(kv) : std::next(kv);
            it = slots_.insert({client, s}).first;
        }
        claimed_[it->second] = 1;
        return it->second;
    }

    float weight_of(int client) const {
        if (o_.samples.empty()) return 1.0f / (float)o_.data_owners;
        double total = 0;
        for (auto& kv : o_.samples) total += kv.second;
        auto it = o_.samples.find(client);
        return it == o_.samples.end() ? 0.0f : (float)(it->second / total);
    }

    Options o_;
    NetLayer* net_;
    fa_ctx* ctx_ = nullptr;
    std::map<int, Bucket> buckets_;
    std::map<int, int> slots_;  // client id -> slot
    std::vector<char> claimed_;  // slot -> an arrived client holds it
    std::vector<int> expected_;  // the data owners' ids in slot order
    Stats st_;
    ReceiptLedger ledger_;
    // cumulative receipt accounting, printed with every round
    unsigned long long stale_dropped_ = 0, ignored_ = 0, replaced_ = 0, clock_back_ = 0;
    std::vector<Stream> streams_;
    std::set<int> phase_mps_;
    unsigned long long streamed_ = 0, stream_fallbacks_ = 0, streamed_bytes_ = 0;
};

// The next receipt, with the failure detection the reference lacks (its receive loop blocks forever on a
// data owner that died, network_layer.cpp:654-665): every stall_report_s of silence names the owners still
// missing in this phase; after receipt_timeout_s of silence (if set) the aggregator exits with code 3.  Bytes
// of a streamed frame arriving count as activity.  While it waits, the frames still arriving are streamed to
// their slots (Aggregator::pump).
Receipt wait_receipt(NetLayer& net, const Options& o, Aggregator& agg, const std::vector<int>& mps, int round,
                     int phase) {
    static uint64_t gen = 0;  // the network layer's progress counter, as last seen (one consumer)
    Receipt r;
    auto last = std::chrono::steady_clock::now();
    int reports = 0;
    for (;;) {
        agg.pump();
        const double silent = secs_since(last);
        double wait = (reports + 1) * o.stall_report_s - silent;
        if (o.receipt_timeout_s > 0) wait = std::min(wait, o.receipt_timeout_s - silent);
        const int ev = net.wait_event(&r, &gen, std::max(1, (int)(wait * 1000)));
        if (ev == 1) return r;
        if (ev == 2) {  // progress: a frame is arriving
            last = std::chrono::steady_clock::now();
            reports = 0;
            continue;
        }
        const double now_silent = secs_since(last);
        const bool give_up = o.receipt_timeout_s > 0 && now_silent >= o.receipt_timeout_s - 1e-3;
        if (!give_up && now_silent < (reports + 1) * o.stall_report_s - 1e-3) continue;
        ++reports;
        std::cerr << "[aggregator] round " << round << " phase " << phase << ": no receipt for " << now_silent
                  << " s; missing " << agg.missing(mps) << (give_up ? "; giving up (--receipt-timeout)" : "")
                  << "\n";
        if (give_up) {
            net.stop();
            std::exit(3);
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    if (!parse_args(argc, argv, &o)) {
        usage();
        return 2;
    }
    // pinned frame buffers: receipts DMA'd from, replies DMA'd into -- small ones too (from 4 KiB): a small
    // model's receipt then goes to its slot by one DMA instead of a copy into the staging chunks first, and
    // its reply comes back the same way (BASELINE C1)
    std::shared_ptr<BufferPool> pool;
    if (o.pinned) {
        pool = BufferPool::create(
            [](size_t n) -> char* {
                void* p = nullptr;
                return fa_host_alloc(n, &p) == FA_OK ? (char*)p : nullptr;
            },
            [](char* p) { fa_host_free(p); }, true, 4096);
        set_frame_allocator([pool](size_t n) { return pool->get(n); });
    }
    NetLayer net(o.id, RoutingTable(o.port_base), o.senders);
    net.set_link_mbps(o.link_mbps);
    net.set_rx_concurrency(o.rx_concurrency);
    if (o.pinned) net.set_streaming(o.stream_min);  // the records are DMA'd from the pinned frame as it fills
    std::string err;
    if (o.discover && !net.find_init(600, &err)) {
        std::cerr << "[aggregator] discovery failed: " << err << "\n";
        return 1;
    }
    if (!net.start()) {
        std::cerr << "[aggregator] cannot listen on port " << net.routes().port_for(o.id) << "\n";
        return 1;
    }
    std::cerr << "[aggregator] node " << o.id << " listening on " << net.listen_port() << "\n";

    Message refactor = net.next_refactor();  // aggregator.cpp:52-53
    const int L = o.last_layers > 0 ? o.last_layers : last_part_layers(refactor.model_name, refactor.start);
    std::cerr << "[aggregator] refactor: model " << refactor.model_name << "/" << refactor.model_type << " start "
              << refactor.start << " end " << refactor.end << " -> " << L << " last-part layer(s)\n";
    Aggregator agg(o, &net, refactor.data_owners);

    for (int round = 0; o.rounds < 0 || round < o.rounds; ++round) {
        // phase 1: model part 1 from every data owner (aggregator.cpp:59-93)
        // Receipt accounting (the reference counts raw receipts, aggregator.cpp:59-92 / :112-149): a phase
        // ends when every data owner's receipt of every bucket of the phase is in, counted as distinct
        // (owner, bucket) pairs, so a retransmitted receipt replaces its slot instead of ending the phase
        // early with another owner missing.  A receipt of the other phase is always a retransmission of an
        // earlier one: a data owner sends its last-part layers only after it has received the phase-1 reply
        // (data_owner.cpp:228-245), which goes out after phase 1 ends, and its next part 1 only after every
        // phase-2 reply, which goes out after phase 2 ends.  So it is ignored (named in the log), never carried
        // into a later phase, where it would stand for a receipt its owner has not sent yet.  A late copy of
        // the SAME phase's bucket from an earlier round is a byte copy of a receipt already reduced, caught by
        // its (t_start, length, content) key and dropped (ReceiptLedger, host/receipts.h).  The round line
        // counts, cumulatively: stale_dropped (byte copies, either phase), ignored (other-phase receipts that
        // are not copies), replaced (retransmissions within a phase), clock_back (owner clocks that went back).
        auto t0 = std::chrono::steady_clock::now();
        agg.set_phase({1});
        int received = 0;
        while (received < o.data_owners) {
            Receipt r = wait_receipt(net, o, agg, {1}, round, 1);
            if (r.model_part != 1) {
                agg.other_phase(r, 1);
                continue;
            }
            if (agg.absorb(r)) ++received;
        }
        const double recv1 = secs_since(t0);
        const size_t in1 = agg.bytes_in(1);
        agg.end_phase();
        auto t1 = std::chrono::steady_clock::now();
        auto reply1 = agg.reduce(1);
        const double red1 = secs_since(t1);
        const auto s1 = agg.take_stats();
        agg.fan_out(reply1);

        // phase 2: every last-part layer from every data owner (:108-150)
        auto t2 = std::chrono::steady_clock::now();
        int got = 0;
        const int want = o.data_owners * L;
        std::vector<int> mps;
        for (int mp = 2; mp <= L + 1; ++mp) mps.push_back(mp);
        agg.set_phase(mps);
        while (got < want) {
            Receipt r = wait_receipt(net, o, agg, mps, round, 2);
            if (r.model_part == 1) {  // a retransmission of this round's part 1 (above), or a late copy
                agg.other_phase(r, 2);
                continue;
            }
            if (r.model_part < 2 || r.model_part > L + 1) {
                std::cerr << "[aggregator] unexpected model_part " << r.model_part << " in phase 2\n";
                continue;
            }
            if (agg.absorb(r)) ++got;
        }
        const double recv2 = secs_since(t2);
        size_t in2 = 0;
        for (int mp = 2; mp <= L + 1; ++mp) in2 += agg.bytes_in(mp);
        agg.end_phase();
        auto t3 = std::chrono::steady_clock::now();
        std::vector<std::shared_ptr<const Bytes>> replies;
        agg.reduce_all(mps);
        for (int mp : mps) replies.push_back(agg.reduce(mp));
        const double red2 = secs_since(t3);
        const auto s2 = agg.take_stats();
        auto t4 = std::chrono::steady_clock::now();
        for (auto& f : replies) agg.fan_out(f);  // :153-166, in layer order
        net.flush();
        const double send2 = secs_since(t4);
        printf("{\"round\":%d,\"phase1\":{\"receive_s\":%.6f,\"reduce_s\":%.6f,\"bytes_in\":%zu,"
               "\"absorb_s\":%.6f,\"finalize_s\":%.6f,\"frame_s\":%.6f},"
               "\"phase2\":{\"receive_s\":%.6f,\"reduce_s\":%.6f,\"bytes_in\":%zu,\"layers\":%d,"
               "\"absorb_s\":%.6f,\"finalize_s\":%.6f,\"frame_s\":%.6f,\"send_s\":%.6f},"
               "\"send_failures\":%llu,\"stale_dropped\":%llu,\"ignored\":%llu,\"replaced\":%llu,"
               "\"clock_back\":%llu,\"streamed\":%llu,\"stream_fallbacks\":%llu,\"streamed_bytes\":%llu}\n",
               round, recv1, red1, in1, s1.absorb_s, s1.finalize_s, s1.frame_s, recv2, red2, in2, L, s2.absorb_s,
               s2.finalize_s, s2.frame_s, send2, (unsigned long long)net.send_failures(), agg.stale_dropped(), agg.ignored(),
               agg.replaced(), agg.clock_back(), agg.streamed(), agg.stream_fallbacks(), agg.streamed_bytes());
        fflush(stdout);
    }
    net.stop();
    return 0;
}
