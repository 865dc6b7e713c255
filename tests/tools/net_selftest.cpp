// net_selftest.cpp -- TEST TOOL (CPU): the aggregator's network layer and frame buffers without a GPU.
//  * D senders push frames at once (one connection each) into one NetLayer; every receipt arrives
//    once, intact, with its header fields (concurrent per-connection readers);
//  * frame buffers come from a BufferPool that recycles them: over all rounds it never holds more
//    buffers than one round can have alive at once (D sender frames + D received frames; without
//    recycling 3 rounds would allocate 3x that), and receipts carry the pool's `pinned` tag;
//  * a frame queued for several destinations reaches each of them (serialize-once fan-out), in
//    order per destination;
//  * streaming (set_streaming): frames written in random pieces are announced while they arrive, their
//    progress is monotonic and true, a complete one is published as the same buffer, a broken one fails;
//  * TorchArchive::layout_into + seal_params == with_params_into on a real archive (optional arg).
// Prints one JSON line {"ok": ..., ...}; exit 0 iff ok.
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <thread>
#include <vector>

#include <zlib.h>

#include "archive.h"
#include "net.h"

using namespace fahost;

static std::shared_ptr<Bytes> make_frame(int client, int part, size_t payload, uint8_t fill) {
    Message m;
    m.type = OPERATION;
    m.client_id = client;
    m.prev_node = -1;
    m.type_op = AGGREGATION;
    m.model_part = part;
    m.t_start = 1700000000000L + client;
    char* v = nullptr;
    auto f = operation_frame(m, payload, &v);
    for (size_t i = 0; i < payload; ++i) v[i] = (char)(fill + i * 7);
    return f;
}

int main(int argc, char** argv) {
    const int D = 6, rounds = 3;
    const size_t payload = 3u << 20;  // > the pool's 1 MiB floor
    bool ok = true;
    std::atomic<size_t> live_allocs{0};
    auto pool = BufferPool::create(
        [&](size_t n) -> char* {
            ++live_allocs;
            return (char*)std::malloc(n);
        },
        [&](char* p) {
            --live_allocs;
            std::free(p);
        },
        true);
    set_frame_allocator([pool](size_t n) { return pool->get(n); });
    const int base = 10000 + (int)(getpid() % 2000) * 10;  // below the ephemeral port range
    RoutingTable routes(base);
    NetLayer agg(-1, routes);
    if (!agg.start()) {
        std::cerr << "bind failed\n";
        return 1;
    }
    for (int r = 0; r < rounds; ++r) {
        std::vector<std::shared_ptr<Bytes>> frames;
        for (int k = 0; k < D; ++k) frames.push_back(make_frame(100 + k, 2 + (k % 2), payload, (uint8_t)(r * 31 + k)));
        std::vector<std::thread> th;
        for (int k = 0; k < D; ++k)
            th.emplace_back([&, k] {
                const int fd = connect_to("127.0.0.1", routes.port_for(-1), 50, 100);
                if (fd < 0 || !send_all(fd, frames[k]->data(), frames[k]->size())) {
                    std::cerr << "sender " << k << " failed\n";
                    ok = false;
                }
                if (fd >= 0) close(fd);
            });
        for (auto& t : th) t.join();
        std::vector<char> seen(D, 0);
        for (int i = 0; i < D; ++i) {
            Receipt rc;
            if (!agg.try_next_receipt(&rc, 20000)) {
                std::cerr << "round " << r << ": receipt " << i << " missing\n";
                ok = false;
                break;
            }
            const int k = rc.client_id - 100;
            if (k < 0 || k >= D || seen[k]) {
                ok = false;
                continue;
            }
            seen[k] = 1;
            if (!(rc.model_part == 2 + (k % 2) && rc.type_op == AGGREGATION && rc.blob_len == payload &&
                  rc.t_start == 1700000000000L + 100 + k && rc.frame->pinned)) {
                std::cerr << "round " << r << ": bad header fields for client " << k << "\n";
                ok = false;
            }
            const char* v = (const char*)rc.blob();
            for (size_t j = 0; j < payload; j += 4099)
                if (v[j] != (char)((uint8_t)(r * 31 + k) + j * 7)) {
                    std::cerr << "payload mismatch client " << k << " at " << j << "\n";
                    ok = false;
                    break;
                }
        }
    }
    // How many buffers round 0 needed depends on timing (a receipt dropped early lends its buffer to a
    // reader still receiving), so the bound is the most a round can hold at once, not round 0's count.
    const size_t allocs = pool->allocations();
    if (allocs > (size_t)(2 * D)) {
        std::cerr << "pool allocated " << allocs << " buffers over " << rounds << " rounds (at most " << 2 * D
                  << " can be alive at once)\n";
        ok = false;
    }

    // fan-out: one frame to three destinations, each one in order
    std::vector<std::unique_ptr<NetLayer>> dests;
    for (int id = 4; id < 7; ++id) {  // 3 < id < 18: port(0) + id + 3
        dests.emplace_back(new NetLayer(id, routes));
        if (!dests.back()->start()) {
            std::cerr << "cannot listen for node " << id << "\n";
            ok = false;
        }
    }
    auto a = make_frame(-1, 2, payload, 1), b = make_frame(-1, 3, 1000, 2);
    for (int id = 4; id < 7; ++id) {
        agg.send(id, a);
        agg.send(id, b);
    }
    agg.flush();
    for (auto& d : dests) {
        Receipt r1, r2;
        if (!(d->try_next_receipt(&r1, 20000) && d->try_next_receipt(&r2, 20000) && r1.model_part == 2 &&
              r2.model_part == 3 && r1.blob_len == payload && r2.blob_len == 1000)) {
            std::cerr << "fan-out: destination missed a frame or got them out of order\n";
            ok = false;
        }
        d->stop();
    }
    // a kept connection whose receiver went away: the next frame goes over a fresh connection to the
    // receiver that took its place (the reference keeps writing into the dead socket)
    uint64_t send_failures = 0;
    {
        auto d7 = std::make_unique<NetLayer>(7, routes);
        if (!d7->start()) ok = false;
        agg.send(7, a, true);
        agg.flush();
        Receipt r1;
        if (!d7->try_next_receipt(&r1, 20000)) ok = false;
        d7->stop();
        d7.reset();
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        auto d7b = std::make_unique<NetLayer>(7, routes);
        if (!d7b->start()) ok = false;
        agg.send(7, b, true);
        agg.flush();
        Receipt r2;
        if (!(d7b->try_next_receipt(&r2, 20000) && r2.model_part == 3 && r2.blob_len == 1000)) {
            std::cerr << "kept connection: the frame after the receiver restarted was lost\n";
            ok = false;
        }
        d7b->stop();
        send_failures = agg.send_failures();
        if (send_failures) ok = false;
    }
    agg.stop();

    // receive gate: 6 owners sending 9 MiB frames at once, at most 2 received at a time, granted in
    // accept order; every frame arrives whole and the FIFO order is the accept order
    {
        RoutingTable groutes(base + 100);
        NetLayer gagg(-1, groutes);
        gagg.set_rx_concurrency(2);
        if (!gagg.start()) {
            std::cerr << "gate: bind failed\n";
            ok = false;
        } else {
            const size_t big = 9u << 20;
            std::vector<std::shared_ptr<Bytes>> gf;
            for (int k = 0; k < D; ++k) gf.push_back(make_frame(200 + k, 2, big, (uint8_t)(77 + k)));
            std::vector<std::thread> th;
            for (int k = 0; k < D; ++k)
                th.emplace_back([&, k] {
                    const int fd = connect_to("127.0.0.1", groutes.port_for(-1), 50, 100);
                    if (fd < 0 || !send_all(fd, gf[k]->data(), gf[k]->size())) ok = false;
                    if (fd >= 0) close(fd);
                });
            std::vector<char> seen(D, 0);
            for (int i = 0; i < D; ++i) {
                Receipt rc;
                if (!gagg.try_next_receipt(&rc, 20000)) {
                    std::cerr << "gate: receipt " << i << " missing\n";
                    ok = false;
                    break;
                }
                const int k = rc.client_id - 200;
                if (k < 0 || k >= D || seen[k] || rc.blob_len != big) {
                    ok = false;
                    continue;
                }
                seen[k] = 1;
                const char* v = (const char*)rc.blob();
                for (size_t j = 0; j < big; j += 65537)
                    if (v[j] != (char)((uint8_t)(77 + k) + j * 7)) {
                        std::cerr << "gate: payload mismatch client " << k << "\n";
                        ok = false;
                        break;
                    }
            }
            for (auto& t : th) t.join();
            gagg.stop();
        }
    }

    // streaming: 4 owners write 3 MiB frames in random pieces (1 B .. 64 KiB) at once; every frame is announced
    // while it arrives with its header fields, its `have` only grows and the bytes below it are the sender's,
    // it ends complete, and the receipt published for it is the same buffer.  One owner hangs up mid-frame:
    // its stream ends failed and no receipt comes of it.
    size_t streamed_checks = 0;
    {
        RoutingTable sroutes(base + 200);
        // on the heap: a NetLayer on the stack where the gate test's stood would reuse its (trivially
        // destroyed) mutexes' addresses, which ThreadSanitizer then takes for the same mutexes
        auto sagg_p = std::make_unique<NetLayer>(-1, sroutes);
        NetLayer& sagg = *sagg_p;
        sagg.set_streaming(1u << 20);
        if (!sagg.start()) {
            std::cerr << "stream: bind failed\n";
            ok = false;
        } else {
            const int S = 5;  // owners 0..3 whole, owner 4 hangs up halfway
            std::vector<std::shared_ptr<Bytes>> sf;
            for (int k = 0; k < S; ++k) sf.push_back(make_frame(300 + k, 2 + (k % 2), payload, (uint8_t)(11 + k)));
            std::vector<std::thread> th;
            for (int k = 0; k < S; ++k)
                th.emplace_back([&, k] {
                    const int fd = connect_to("127.0.0.1", sroutes.port_for(-1), 50, 100);
                    uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1);
                    const size_t end = k == S - 1 ? sf[k]->size() / 2 : sf[k]->size();
                    for (size_t o = 0; fd >= 0 && o < end;) {
                        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                        const size_t c = std::min<size_t>(end - o, 1 + x % 65536);
                        if (!send_all(fd, sf[k]->data() + o, c)) break;
                        o += c;
                        if (x % 16 == 0) std::this_thread::sleep_for(std::chrono::microseconds(x % 200));
                    }
                    if (fd >= 0) close(fd);
                });
            std::map<const Bytes*, std::shared_ptr<Inflight>> streams;
            std::map<const Bytes*, size_t> last_have;
            int receipts = 0;
            uint64_t gen = 0;
            const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(30);
            auto check_progress = [&] {
                for (auto& in : sagg.take_new_streams()) {
                    const int k = in->client_id - 300;
                    if (k < 0 || k >= S || in->model_part != 2 + (k % 2) || in->blob_len != payload) {
                        std::cerr << "stream: bad header fields\n";
                        ok = false;
                        continue;
                    }
                    streams[in->buf.get()] = in;
                }
                for (auto& kv : streams) {
                    Inflight& in = *kv.second;
                    const bool ended = in.ended.load(std::memory_order_acquire);
                    const size_t have = in.have.load(std::memory_order_acquire);
                    if (have < last_have[kv.first]) ok = false;  // never shrinks
                    last_have[kv.first] = have;
                    const int k = in.client_id - 300;
                    // the bytes below `have` are the sender's (the frame text = the sent bytes after the length)
                    for (size_t j = 0; j < have; j += 9973) {
                        ++streamed_checks;
                        if (in.buf->data()[j] != sf[(size_t)k]->data()[4 + j]) {
                            std::cerr << "stream: byte " << j << " of owner " << k << " below have is wrong\n";
                            ok = false;
                            break;
                        }
                    }
                    if (ended && in.failed.load() != (k == S - 1)) {
                        std::cerr << "stream: owner " << k << " ended with the wrong status\n";
                        ok = false;
                    }
                }
            };
            while (receipts < S - 1 && std::chrono::steady_clock::now() < t_end) {
                Receipt rc;
                const int ev = sagg.wait_event(&rc, &gen, 200);
                check_progress();
                if (ev != 1) continue;
                ++receipts;
                auto it = streams.find(rc.frame.get());
                if (it == streams.end() || !it->second->ended.load() || it->second->failed.load() ||
                    it->second->have.load() != rc.frame->size() || rc.client_id == 300 + S - 1) {
                    std::cerr << "stream: receipt of client " << rc.client_id << " does not match its stream\n";
                    ok = false;
                }
            }
            for (auto& t : th) t.join();
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
            check_progress();
            Receipt extra;
            if (receipts != S - 1 || (int)streams.size() != S || sagg.try_next_receipt(&extra, 100)) {
                std::cerr << "stream: " << receipts << " receipts, " << streams.size() << " streams\n";
                ok = false;
            }
            sagg.stop();
        }
    }

    // archive split copy: layout_into + values + seal_params == with_params_into
    size_t checked_archive = 0;
    if (argc > 1) {
        std::ifstream f(argv[1], std::ios::binary);
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string blob = ss.str();
        TorchArchive ar;
        std::string err;
        if (!ar.parse((const uint8_t*)blob.data(), blob.size(), &err)) {
            std::cerr << err << "\n";
            return 1;
        }
        std::vector<float> vals((size_t)ar.param_numel());
        for (size_t i = 0; i < vals.size(); ++i) vals[i] = (float)i * 0.25f - 3.0f;
        std::vector<uint8_t> one(ar.size()), two(ar.size(), 0xAB);
        if (!ar.with_params_into(vals.data(), one.data(), &err)) {
            std::cerr << "with_params_into: " << err << "\n";
            ok = false;
        }
        std::vector<void*> dsts;
        std::vector<size_t> bytes;
        if (!ar.layout_into(two.data(), &dsts, &bytes, &err)) {
            std::cerr << "layout_into: " << err << "\n";
            ok = false;
        }
        const float* src = vals.data();
        for (size_t k = 0; k < dsts.size(); ++k) {
            std::memcpy(dsts[k], src, bytes[k]);
            src += bytes[k] / 4;
        }
        ar.seal_params(two.data());
        if (one != two) {
            std::cerr << "layout_into + seal_params differs from with_params_into\n";
            ok = false;
        }
        // the same seal from CRC-32s computed elsewhere (fa_output_crc32 on the GPU; here zlib's, per parameter)
        std::vector<uint8_t> three(ar.size(), 0xCD);
        std::vector<void*> d3;
        std::vector<size_t> b3;
        if (ar.layout_into(three.data(), &d3, &b3, &err)) {
            std::vector<uint32_t> crcs;
            const float* v = vals.data();
            for (size_t k = 0; k < d3.size(); ++k) {
                std::memcpy(d3[k], v, b3[k]);
                crcs.push_back((uint32_t)::crc32(0, (const Bytef*)v, (uInt)b3[k]));
                v += b3[k] / 4;
            }
            if (!ar.seal_params_with(three.data(), crcs.data()) || three != one) {
                std::cerr << "seal_params_with differs from with_params_into\n";
                ok = false;
            }
        }
        checked_archive = ar.size();
    }
    printf("{\"ok\": %s, \"rounds\": %d, \"senders\": %d, \"pool_allocations\": %zu, \"live_after\": %zu, "
           "\"archive_bytes\": %zu, \"send_failures\": %llu, \"streamed_checks\": %zu}\n",
           ok ? "true" : "false", rounds, D, allocs, (size_t)live_allocs, checked_archive,
           (unsigned long long)send_failures, streamed_checks);
    return ok ? 0 : 1;
}
