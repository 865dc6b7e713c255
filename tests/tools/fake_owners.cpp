// fake_owners.cpp -- TEST TOOL: the init node + D data owners of the reference,
// as far as the aggregator sees them (data_owner.cpp:96-112 refactor, :224-253
// aggregation exchange), in one process.  Each owner sends synthetic model
// parts built from template archives (tests/golden/<cfg>/mp<m>_client0.pt, made
// by the reference's own builders) with parameters from the oracle's generator,
// collects the aggregator's replies and checks them bit-for-bit against the
// oracle (oracle/fa_oracle.c: links the checker, never the product).
//
//   fa_fake_owners --blobs DIR --parts 1,2,3 -d D -c C [--rounds R] [--mode fedavg|literal]
//                  [--port-base P] [--model-name N --model-type T --start S --end E] [--seed X]
//                  [--drop-owner K [--drop-phase P]] [--retransmit K] [--retransmit-late K]
//                  [--clock-skew K,S] [--reply-timeout S] [--rel-tol X] [--routing-table]
//                  [--sequential]   (owners send at once, one connection each, unless --sequential
//                                    or --mode literal, whose result depends on the arrival order)
//                  [--chunked MIN,MAX[,SEED]]  (every frame written in random pieces of MIN..MAX bytes with
//                                    random pauses; owners sending at once then arrive interleaved in random
//                                    order: the aggregator's streaming ingest)
// Every frame is stamped (t_start, network_layer.cpp:761) when it first goes out, on its owner's clock;
// --clock-skew K,S sets owner K's clock back S ms more every round (an NTP step, a VM resume).
// --routing-table: the refactor message carries the owners' addresses (read_table 1, as the init node's
// does, network_layer.cpp:335-359); the reference's own process cannot reach an owner id above 3 without it.
// Prints one JSON line: {"ok": bool, "rounds": R, "checked_elems": ..., "round_ms": [...]}.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <zlib.h>

#include "archive.h"
#include "fa_oracle.h"
#include "net.h"

using namespace fahost;

namespace {

std::string read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

long now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

// Overwrites the t_start field of a length-prefixed OPERATION frame in place (the frame was built with a
// 13-digit placeholder, so a millisecond epoch stamp has the same width).
bool restamp(Bytes& f, long t) {
    static const char kField[] = "\nt_start : ";
    const size_t scan = std::min<size_t>(f.size(), 512);
    const char* b = f.data();
    const char* at = std::search(b, b + scan, kField, kField + sizeof kField - 1);
    if (at == b + scan) return false;
    char* d = f.data() + (at - b) + (sizeof kField - 1);
    size_t w = 0;
    while (d + w < b + scan && d[w] != ',') ++w;
    const std::string v = std::to_string(t);
    if (v.size() != w) return false;
    std::memcpy(d, v.data(), w);
    return true;
}

constexpr long kStampPlaceholder = 1000000000000L;

// The data owners' sending threads, one per owner for the whole run (each owner is a process of its own in
// the reference): a phase hands every owner its job and waits for all of them, with no thread started per
// phase (that cost ~20-40 us per owner on the round's path, a test artifact a deployment does not have).
class OwnerThreads {
public:
    explicit OwnerThreads(int n) {
        for (int k = 0; k < n; ++k) th_.emplace_back([this, k] { loop(k); });
    }
    ~OwnerThreads() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(std::function<void(int)> job) {  // job(k) on owner k's thread, for every owner; returns when all did
        std::unique_lock<std::mutex> lk(m_);
        job_ = std::move(job);
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        done_cv_.wait(lk, [&] { return done_ == (int)th_.size(); });
    }

private:
    void loop(int k) {
        unsigned long seen = 0;
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
            if (quit_) return;
            seen = gen_;
            auto job = job_;
            lk.unlock();
            job(k);
            lk.lock();
            if (++done_ == (int)th_.size()) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::function<void(int)> job_;
    unsigned long gen_ = 0;
    int done_ = 0;
    bool quit_ = false;
};

struct Part {
    int mp;
    std::string blob;
    TorchArchive ar;
    size_t n = 0;
    int es = 4;  // parameter element bytes: 4 fp32, 2 bf16 (the template's dtype)
};

}  // namespace

int main(int argc, char** argv) {
    std::string blobs, parts_s = "1,2,3", mode = "fedavg";
    int D = 2, C = 1, rounds = 1, port_base = 8079, model_name = 2, model_type = 0, start = 6, end = 1;
    uint64_t seed = 0x5EED;
    float divisor = 1000.0f;
    bool concurrent = true;
    int drop_owner = -1, drop_phase = 1;  // failure injection: owner K never sends its phase-P receipts
    int retransmit = -1;                  // owner K sends every receipt twice (a retransmission)
    int retransmit_late = -1;             // owner K re-sends its previous round's receipts during this round
    int skew_owner = -1;                  // --clock-skew K,S: owner K's clock goes back S ms every round
    long skew_ms = 0;
    double rel_tol = 0;                   // > 0: fp32 replies within rel_tol * sum_k |w_k x_k| (the rs layout)
    bool routing_table = false;           // --routing-table: the refactor message carries the owners' addresses
    long reply_timeout_ms = 600000;
    size_t chunk_min = 0, chunk_max = 0;  // --chunked: frames written in random pieces
    uint64_t chunk_seed = 1;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : "";
        if (a == "--blobs") blobs = v, ++i;
        else if (a == "--parts") parts_s = v, ++i;
        else if (a == "-d") D = std::atoi(v), ++i;
        else if (a == "-c") C = std::atoi(v), ++i;
        else if (a == "--rounds") rounds = std::atoi(v), ++i;
        else if (a == "--mode") mode = v, ++i;
        else if (a == "--port-base") port_base = std::atoi(v), ++i;
        else if (a == "--model-name") model_name = std::atoi(v), ++i;
        else if (a == "--model-type") model_type = std::atoi(v), ++i;
        else if (a == "--start") start = std::atoi(v), ++i;
        else if (a == "--end") end = std::atoi(v), ++i;
        else if (a == "--seed") seed = std::strtoull(v, nullptr, 0), ++i;
        else if (a == "--divisor") divisor = (float)std::atof(v), ++i;
        else if (a == "--sequential") concurrent = false;
        else if (a == "--routing-table") routing_table = true;
        else if (a == "--drop-owner") drop_owner = std::atoi(v), ++i;
        else if (a == "--drop-phase") drop_phase = std::atoi(v), ++i;
        else if (a == "--retransmit") retransmit = std::atoi(v), ++i;
        else if (a == "--retransmit-late") retransmit_late = std::atoi(v), ++i;
        else if (a == "--rel-tol") rel_tol = std::atof(v), ++i;
        else if (a == "--clock-skew") {
            const char* c = std::strchr(v, ',');
            if (!c) {
                std::cerr << "--clock-skew K,S\n";
                return 2;
            }
            skew_owner = std::atoi(v), skew_ms = std::atol(c + 1), ++i;
        }
        else if (a == "--reply-timeout") reply_timeout_ms = (long)(std::atof(v) * 1000), ++i;
        else if (a == "--chunked") {
            unsigned long long lo = 0, hi = 0, sd = 1;
            const int got = std::sscanf(v, "%llu,%llu,%llu", &lo, &hi, &sd);
            if (got < 2 || lo < 1 || hi < lo) {
                std::cerr << "--chunked MIN,MAX[,SEED] with 1 <= MIN <= MAX\n";
                return 2;
            }
            chunk_min = lo, chunk_max = hi, chunk_seed = sd, ++i;
        }
        else {
            std::cerr << "unknown argument " << a << "\n";
            return 2;
        }
    }
    if (mode == "literal") concurrent = false;
    if (retransmit_late >= D || retransmit >= D || drop_owner >= D || skew_owner >= D) {
        std::cerr << "owner index out of range (-d " << D << ")\n";
        return 2;
    }
    // template archives
    std::vector<Part> parts;
    {
        std::stringstream ss(parts_s);
        std::string t;
        while (std::getline(ss, t, ',')) {
            Part p;
            p.mp = std::atoi(t.c_str());
            p.blob = read_file(blobs + "/mp" + t + "_client0.pt");
            parts.push_back(std::move(p));
        }
    }
    for (auto& p : parts) {
        std::string err;
        if (!p.ar.parse((const uint8_t*)p.blob.data(), p.blob.size(), &err)) {
            std::cerr << "template mp" << p.mp << ": " << err << "\n";
            return 1;
        }
        p.n = (size_t)p.ar.param_numel();
        p.es = p.ar.param_elem_size();
        if (!p.es) {
            std::cerr << "template mp" << p.mp << ": parameters not all fp32 or all bf16\n";
            return 1;
        }
    }
    // data owner ids: the init node 0 and the ids the aggregator replies to (aggregator.cpp:103-105)
    std::vector<int> ids = {0};
    for (int i = 0; i < D - 1; ++i) ids.push_back(i + C + 1);
    // frame buffers recycled across rounds (the owners' side of a loopback run should not page-fault
    // hundreds of MB per round; separate machines in a real deployment)
    auto pool = BufferPool::create([](size_t n) { return (char*)std::malloc(n); }, [](char* p) { std::free(p); },
                                   false);
    set_frame_allocator([pool](size_t n) { return pool->get(n); });
    RoutingTable routes(port_base);
    std::map<int, std::unique_ptr<NetLayer>> listeners;  // port -> listener
    for (int id : ids) {
        const int port = routes.port_for(id);
        if (listeners.count(port)) continue;
        auto nl = std::make_unique<NetLayer>(id, routes);
        if (!nl->start(port)) {
            std::cerr << "cannot listen on " << port << "\n";
            return 1;
        }
        listeners[port] = std::move(nl);
    }
    NetLayer& tx = *listeners.begin()->second;

    // refactor message from the init node (data_owner.cpp:96-112)
    Message rf;
    rf.type = REFACTOR_DATA_OWNER;
    rf.model_name = model_name;
    rf.model_type = model_type;
    rf.start = start;
    rf.end = end;
    rf.num_classes = 10;
    rf.dataset = 0;
    rf.data_owners = ids;
    rf.read_table = 0;
    if (routing_table) {  // the addresses of owners 4..17 (systemAPI.cpp:212-240): the reference needs them
        for (int id : ids)
            if (id > 3) rf.rooting_table.push_back({id, "127.0.0.1"});
        rf.read_table = 1;
    }
    tx.send(-1, frame_bytes(rf));

    std::vector<float> w(D, 1.0f / (float)D);  // the aggregator's default weights
    bool ok = true;
    size_t checked = 0;
    std::vector<double> round_ms;
    double max_err_over_bound = 0;  // --rel-tol: the worst element against its bound
    std::map<int, std::vector<std::shared_ptr<Bytes>>> prev_frames;  // the previous round's, per mp
    // owner k's clock in round r (--clock-skew)
    auto owner_now = [&](int k, int round) { return now_ms() - (k == skew_owner ? skew_ms * round : 0L); };
    // Replies land on several listeners (one per owner port): poll them all without blocking and nap 20 us
    // when none had anything -- a blocking wait on one listener would add its timeout to every phase (the
    // round time of a small model is a few ms)
    auto collect = [&](int want, std::vector<Receipt>* got) {
        const long t_end = now_ms() + reply_timeout_ms;
        while ((int)got->size() < want && now_ms() < t_end) {
            bool any = false;
            for (auto& kv : listeners) {
                Receipt r;
                while (kv.second->try_next_receipt(&r, 0)) {
                    got->push_back(r);
                    any = true;
                }
            }
            if (!any) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        return (int)got->size() == want;
    };
    const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    OwnerThreads owners(concurrent ? D : 0);
    std::vector<std::mt19937_64> chunk_rng;
    for (int k = 0; k < D; ++k) chunk_rng.emplace_back(chunk_seed * 1000003ull + (uint64_t)k);
    // a frame in random pieces with random pauses (--chunked), else in one write
    auto send_frame = [&](int fd, const Bytes& f, int k) -> bool {
        if (chunk_max == 0) return send_all(fd, f.data(), f.size());
        std::mt19937_64& rng = chunk_rng[(size_t)k];
        for (size_t o = 0; o < f.size();) {
            const size_t c = std::min<size_t>(f.size() - o, chunk_min + rng() % (chunk_max - chunk_min + 1));
            if (!send_all(fd, f.data() + o, c)) return false;
            o += c;
            if (rng() % 32 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
        }
        return true;
    };
    auto fill = [&](uint64_t sd, uint32_t k, size_t n, int es, uint8_t* x) {  // the oracle's generator, in chunks
        std::vector<std::thread> th;
        const size_t per = (n + threads - 1) / threads;
        for (int t = 0; t < threads; ++t) {
            const size_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
            if (lo < hi)
                th.emplace_back([=] {
                    if (es == 4) fa_oracle_fill_f32(sd, k, lo, hi - lo, reinterpret_cast<float*>(x) + lo);
                    else fa_oracle_fill_bf16(sd, k, lo, hi - lo, reinterpret_cast<uint16_t*>(x) + lo);
                });
        }
        for (auto& t : th) t.join();
    };
    for (int round = 0; round < rounds; ++round) {
        // The data owners' side of a round (their training) is not timed: values and frames are made
        // first, then the clock runs from the first phase-1 send to the last phase-2 reply.
        std::map<int, std::vector<std::vector<uint8_t>>> values;  // mp -> per client (the parameters' own dtype)
        std::map<int, std::vector<std::shared_ptr<Bytes>>> frames;
        for (auto& p : parts) {
            for (int k = 0; k < D; ++k) {
                std::vector<uint8_t> x(p.n * (size_t)p.es);
                fill(seed ^ ((uint64_t)round << 48) ^ ((uint64_t)p.mp << 32), (uint32_t)k, p.n, p.es, x.data());
                Message m;  // Task(myID, aggregation_, -1), data_owner.cpp:225-231
                m.type = OPERATION;
                m.client_id = ids[k];
                m.prev_node = -1;
                m.type_op = AGGREGATION;
                m.model_part = p.mp;
                m.t_start = kStampPlaceholder;  // stamped when it goes out
                char* vals = nullptr;
                auto f = operation_frame(m, p.ar.size(), &vals);
                std::string err;
                if (!p.ar.with_param_bytes_into(x.data(), (uint8_t*)vals, &err)) {
                    std::cerr << err << "\n";
                    return 1;
                }
                values[p.mp].push_back(std::move(x));
                frames[p.mp].push_back(std::move(f));
            }
        }
        std::cerr << "[owners] round " << round << ": frames ready, sending\n";
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<Receipt> replies;
        for (int phase = 1; phase <= 2 && ok; ++phase) {
            int sent = 0;
            // (frame, fresh): a fresh frame is stamped on its owner's clock as it goes out; a copy keeps the
            // stamp its original went out with
            std::vector<std::vector<std::pair<std::shared_ptr<Bytes>, bool>>> by_owner(D);
            for (int k = 0; k < D; ++k)
                for (auto& p : parts) {
                    if ((phase == 1) != (p.mp == 1)) continue;
                    if (k == drop_owner && phase == drop_phase) continue;  // this owner "died"
                    // --retransmit-late: the previous round's receipt of this bucket arrives late, once before
                    // and once after this round's (a delayed duplicate; the aggregator must drop both copies,
                    // whichever order they land in)
                    const bool late = k == retransmit_late && prev_frames.count(p.mp);
                    if (late) by_owner[k].push_back({prev_frames[p.mp][k], false});
                    by_owner[k].push_back({frames[p.mp][k], true});
                    if (k == retransmit) by_owner[k].push_back({frames[p.mp][k], false});  // the same receipt again
                    if (late) by_owner[k].push_back({prev_frames[p.mp][k], false});
                    ++sent;  // one reply per bucket and destination, retransmission or not
                }
            std::atomic<bool> send_ok{true};
            auto stamp = [&](int k, std::pair<std::shared_ptr<Bytes>, bool>& f) {
                if (f.second && !restamp(*f.first, owner_now(k, round))) send_ok = false;
            };
            if (concurrent) {  // every owner is its own process in the reference: they send at once
                owners.run([&](int k) {
                    for (auto& f : by_owner[k]) {
                        const int fd = connect_to(routes.host_for(-1), routes.port_for(-1), 100, 200);
                        stamp(k, f);
                        if (fd < 0 || !send_frame(fd, *f.first, k)) send_ok = false;
                        if (fd >= 0) close(fd);
                    }
                });
            } else if (chunk_max > 0) {  // in owner order, each frame in random pieces (--chunked)
                for (int k = 0; k < D && send_ok; ++k)
                    for (auto& f : by_owner[k]) {
                        const int fd = connect_to(routes.host_for(-1), routes.port_for(-1), 100, 200);
                        stamp(k, f);
                        if (fd < 0 || !send_frame(fd, *f.first, k)) send_ok = false;
                        if (fd >= 0) close(fd);
                    }
            } else {  // one after another, in owner order (literal mode: the last receipt is owner D-1's)
                for (int k = 0; k < D; ++k)
                    for (auto& f : by_owner[k]) {
                        stamp(k, f);
                        tx.send(-1, f.first);
                    }
            }
            if (!send_ok) {
                std::cerr << "send to the aggregator failed (or a frame could not be stamped)\n";
                ok = false;
                break;
            }
            std::vector<Receipt> got;
            if (!collect(sent, &got)) {
                std::cerr << "timed out waiting for phase " << phase << " replies\n";
                ok = false;
            }
            for (auto& r : got) replies.push_back(std::move(r));
        }
        // only owner K's frames are kept for the next round (keeping every frame would hold a round of
        // receipts -- 31 GB at C4 -- out of the recycled buffer pool)
        prev_frames.clear();
        if (retransmit_late >= 0)
            for (auto& kv : frames) {
                prev_frames[kv.first].assign(kv.second.size(), nullptr);
                prev_frames[kv.first][retransmit_late] = kv.second[retransmit_late];
            }
        round_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        // every destination of a bucket gets the same reply: the oracle's result (and, with --rel-tol, the
        // bound's sum_k |w_k x_k|) is computed once per bucket and round, not once per reply
        std::map<int, std::vector<uint8_t>> want_of;
        std::map<int, std::vector<double>> sabs_of;
        for (auto& r : replies) {
            const Part* p = nullptr;
            for (auto& q : parts)
                if (q.mp == r.model_part) p = &q;
            TorchArchive ar;
            std::string err;
            if (!p || !ar.parse(r.blob(), r.blob_len, &err) || (size_t)ar.param_numel() != p->n) {
                std::cerr << "bad reply for part " << r.model_part << ": " << err << "\n";
                ok = false;
                continue;
            }
            const size_t es = (size_t)p->es;
            std::vector<uint8_t> got(p->n * es);
            if (ar.param_elem_size() != p->es || !ar.gather_param_bytes(got.data(), &err)) {
                std::cerr << "reply for part " << p->mp << " changed dtype: " << err << "\n";
                ok = false;
                continue;
            }
            const auto& xs = values[p->mp];
            std::vector<uint8_t>& want = want_of[p->mp];
            if (want.empty()) {
                want.resize(p->n * es);
                if (mode == "literal") {
                    if (es == 4) fa_oracle_literal_f32((const float*)xs[D - 1].data(), p->n, divisor, (float*)want.data());
                    else fa_oracle_literal_bf16((const uint16_t*)xs[D - 1].data(), p->n, divisor, want.data(), 1);
                } else if (es == 4) {
                    std::vector<const float*> ptrs;
                    for (auto& x : xs) ptrs.push_back((const float*)x.data());
                    fa_oracle_fedavg_f32(ptrs.data(), w.data(), D, p->n, nullptr, (float*)want.data(), threads);
                } else {  // bf16 buckets: the fp32 chain, rounded once to bf16 (RNE)
                    std::vector<const uint16_t*> ptrs;
                    for (auto& x : xs) ptrs.push_back((const uint16_t*)x.data());
                    fa_oracle_fedavg_bf16(ptrs.data(), w.data(), D, p->n, nullptr, want.data(), 1, threads);
                }
            }
            if (rel_tol > 0 && es == 4 && mode != "literal") {
                // the client-sharded layout sums in the exchange's order: |got - want| <= tol * sum_k |w_k x_k|
                const float* g = (const float*)got.data();
                const float* h = (const float*)want.data();
                std::vector<double>& sabs = sabs_of[p->mp];
                if (sabs.empty()) {
                    sabs.assign(p->n, 0.0);
                    for (size_t i = 0; i < p->n; ++i)
                        for (int k = 0; k < D; ++k) sabs[i] += std::fabs((double)w[k] * ((const float*)xs[k].data())[i]);
                }
                size_t bad = 0;
                double worst = 0;
                for (size_t i = 0; i < p->n; ++i) {
                    const double r = std::fabs((double)g[i] - (double)h[i]) / (rel_tol * sabs[i] + 1e-30);
                    if (!(r <= 1.0)) ++bad;
                    if (r > worst) worst = r;
                }
                if (bad) {
                    std::cerr << "part " << p->mp << ": " << bad << " elements beyond the tolerance (worst " << worst
                              << " of the bound)\n";
                    ok = false;
                }
                max_err_over_bound = std::max(max_err_over_bound, worst);
            } else if (std::memcmp(got.data(), want.data(), p->n * es) != 0) {
                size_t bad = 0;
                while (bad < p->n && std::memcmp(&got[bad * es], &want[bad * es], es) == 0) ++bad;
                std::cerr << "part " << p->mp << " mismatch at element " << bad << " (" << es << "-byte elements)\n";
                ok = false;
            }
            checked += p->n;
            // buffers are the last receipt's (template buffers are identical for every client here)
            if (ar.buffers().size() != p->ar.buffers().size()) ok = false;
            // every parameter record's CRC-32 as torch::load checks it: the central directory's and the local
            // header's (or data descriptor's) against zlib over the record's bytes (the aggregator seals them,
            // from the GPU for large replies: fa_output_crc32)
            for (auto& t : ar.params()) {
                const ZipEntry& z = ar.entries()[(size_t)t.record];
                const uint8_t* rb = r.blob();
                uLong c = ::crc32(0L, Z_NULL, 0);
                for (uint64_t o = 0; o < z.size;) {  // zlib takes uInt lengths
                    const uInt take = (uInt)std::min<uint64_t>(z.size - o, 1u << 30);
                    c = ::crc32(c, rb + z.data_offset + o, take);
                    o += take;
                }
                uint32_t local = 0;
                std::memcpy(&local, rb + (z.desc_offset ? z.desc_offset : z.local_offset + 14), 4);
                if ((uint32_t)c != z.crc || local != z.crc) {
                    std::cerr << "reply for part " << p->mp << ": record " << z.name << " CRC-32 "
                              << std::hex << z.crc << "/" << local << " but its bytes give " << (uint32_t)c << std::dec
                              << "\n";
                    ok = false;
                }
            }
        }
    }
    printf("{\"ok\": %s, \"rounds\": %d, \"data_owners\": %d, \"checked_elems\": %zu, \"round_ms\": [", ok ? "true" : "false",
           rounds, D, checked);
    for (size_t i = 0; i < round_ms.size(); ++i) printf("%s%.3f", i ? ", " : "", round_ms[i]);
    printf("], \"max_err_over_bound\": %.6g}\n", max_err_over_bound);
    for (auto& kv : listeners) kv.second->stop();
    return ok ? 0 : 1;
}
