// ref_harness.cpp -- golden-vector generator and CPU baseline built against the
// reference's own model builders (compiled from /root/reference by
// oracle/Makefile.ref) and libtorch, the library the reference's arithmetic
// lives in.  TEST INFRASTRUCTURE ONLY: never linked into the product.
//
// It restates, in our own code, the aggregator's state construction and op
// sequence so that the fixtures carry the reference's exact semantics:
//   * systemAPI.cpp:17-38 (init_model_sate): first part = ModelPart(1, end),
//     last part = ModelPart(start, -1); for id -1 the receive slots `parts_`
//     hold the SAME module holders as `parts` (State.h:12 copies the vector of
//     Sequential handles).
//   * aggregator.cpp:63-88 / :117-142: torch::load the received blob into the
//     slot, then per named parameter p <- div(p + p_slot, kTrainSize_10 = 1000)
//     and copy_ back.  Buffers are not reduced (the lookup at :82-86 is dead).
//   * data_owner.cpp:224-244: the producer sends parts[0].layers[0] as
//     model_part 1 and parts[1].layers[i] as model_part i + 2.
//
// Modes (all write JSON to stdout):
//   layout  <name> <type> <start> <end> <nc>
//   golden  <name> <type> <start> <end> <nc> <D> <seed> <wseed> <outdir> [blob_mp; -1 = every bucket <= 200k]
//   bench-fedavg <n> <D> <threads> <reps> [bf16]
//   bench-literal <name> <type> <start> <end> <nc> <D> <threads> <model_part> [arith]
//   bench-round <name> <type> <start> <end> <nc> <D> <threads> <rounds>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <torch/torch.h>

#include "models.h"  // reference: ModelPart, model_name
#include "State.h"   // reference: State
#include "fa_oracle.h"

namespace {

struct AggState {
    std::vector<State> parts, parts_;
};

// systemAPI::init_model_sate for myid == -1, without the SGD optimizers the
// aggregator never steps.
AggState build_state(int name, int type, int start, int end, int nc) {
    ModelPart first((model_name)name, type, 1, end, nc);
    ModelPart last((model_name)name, type, start, -1, nc);
    AggState s;
    State a(-1, first.layers, std::vector<torch::optim::SGD*>(first.layers.size(), nullptr));
    State b(-1, last.layers, std::vector<torch::optim::SGD*>(last.layers.size(), nullptr));
    s.parts.push_back(a);
    s.parts.push_back(b);
    s.parts_.push_back(a);
    s.parts_.push_back(b);
    return s;
}

// model_part id -> (part index, layer index), aggregator.cpp:64 and :118.
struct Bucket {
    int model_part;
    torch::nn::Sequential global, slot;
};

std::vector<Bucket> buckets_of(AggState& s) {
    std::vector<Bucket> out;
    out.push_back({1, s.parts[0].layers[0], s.parts_[0].layers[0]});
    for (size_t i = 0; i < s.parts[1].layers.size(); ++i)
        out.push_back({(int)i + 2, s.parts[1].layers[i], s.parts_[1].layers[i]});
    return out;
}

std::string shape_json(const torch::Tensor& t) {
    std::string r = "[";
    for (int64_t d = 0; d < t.dim(); ++d) r += (d ? "," : "") + std::to_string(t.size(d));
    return r + "]";
}

int64_t param_numel(torch::nn::Sequential m) {
    int64_t n = 0;
    for (auto& p : m->named_parameters(true)) n += p.value().numel();
    return n;
}

std::string layout_json(AggState& s) {
    std::string j = "{\"buckets\":[";
    auto bs = buckets_of(s);
    for (size_t b = 0; b < bs.size(); ++b) {
        j += (b ? "," : "") + std::string("{\"model_part\":") + std::to_string(bs[b].model_part) + ",\"numel\":" +
             std::to_string(param_numel(bs[b].global)) + ",\"params\":[";
        bool first = true;
        for (auto& p : bs[b].global->named_parameters(true)) {
            j += (first ? "" : ",") + std::string("{\"name\":\"") + p.key() + "\",\"shape\":" + shape_json(p.value()) +
                 ",\"numel\":" + std::to_string(p.value().numel()) + "}";
            first = false;
        }
        j += "],\"buffers\":[";
        first = true;
        for (auto& p : bs[b].global->named_buffers(true)) {
            j += (first ? "" : ",") + std::string("{\"name\":\"") + p.key() + "\",\"shape\":" + shape_json(p.value()) +
                 ",\"dtype\":\"" + std::string(c10::toString(p.value().scalar_type())) + "\"}";
            first = false;
        }
        j += "]}";
    }
    return j + "]}";
}

// A data owner's module for one bucket with synthetic parameters: the flattened
// named_parameters() concatenation of client k is fa_oracle_gen_value(seed_b, k, i).
torch::nn::Sequential client_module(int name, int type, int start, int end, int nc, int model_part) {
    AggState s = build_state(name, type, start, end, nc);
    return buckets_of(s)[model_part - 1].global;
}

uint64_t bucket_seed(uint64_t seed, int model_part) { return seed ^ (0x100000001B3ull * (uint64_t)model_part); }

void fill_client(torch::nn::Sequential m, uint64_t seed, int k) {
    torch::NoGradGuard ng;
    uint64_t off = 0;
    for (auto& p : m->named_parameters(true)) {
        auto t = p.value();
        std::vector<float> v((size_t)t.numel());
        fa_oracle_fill_f32(seed, (uint32_t)k, off, v.size(), v.data());
        t.copy_(torch::from_blob(v.data(), t.sizes(), torch::kFloat32));
        off += v.size();
    }
    uint64_t boff = 0;
    for (auto& b : m->named_buffers(true)) {
        auto t = b.value();
        if (t.scalar_type() == torch::kFloat32) {
            std::vector<float> v((size_t)t.numel());
            fa_oracle_fill_f32(seed ^ 0xB0FFE125ull, (uint32_t)k, boff, v.size(), v.data());
            t.copy_(torch::from_blob(v.data(), t.sizes(), torch::kFloat32));
            boff += v.size();
        } else {
            t.fill_(k + 1);  // num_batches_tracked
        }
    }
}

torch::Tensor flat_params(torch::nn::Sequential m) {
    std::vector<torch::Tensor> v;
    for (auto& p : m->named_parameters(true)) v.push_back(p.value().detach().reshape({-1}));
    if (v.empty()) return torch::zeros({0}, torch::kFloat32);
    return torch::cat(v);
}

std::string save_blob(torch::nn::Sequential m) {
    std::ostringstream os;
    torch::save(m, os);
    return os.str();
}

// aggregator.cpp:63-88 restated for one receipt.
void literal_receipt(Bucket& b, const std::string& blob, int64_t k_train) {
    std::istringstream is(blob);
    torch::load(b.slot, is);
    torch::NoGradGuard ng;
    auto g = b.global->named_parameters(true);
    auto r = b.slot->named_parameters(true);
    for (size_t j = 0; j < g.size(); ++j) {
        auto v = torch::div(g[j].value() + r[j].value(), k_train);
        g[j].value().copy_(v);
    }
}

void write_bin(const std::string& path, const void* p, size_t bytes) {
    std::ofstream f(path, std::ios::binary);
    f.write((const char*)p, (std::streamsize)bytes);
}

void write_tensor(const std::string& path, const torch::Tensor& t) {
    auto c = t.contiguous();
    write_bin(path, c.data_ptr(), (size_t)c.numel() * c.element_size());
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int cmd_golden(int argc, char** argv) {
    int name = atoi(argv[2]), type = atoi(argv[3]), start = atoi(argv[4]), end = atoi(argv[5]), nc = atoi(argv[6]);
    int D = atoi(argv[7]);
    uint64_t seed = strtoull(argv[8], nullptr, 0), wseed = strtoull(argv[9], nullptr, 0);
    std::string outdir = argv[10];
    int blob_mp = argc > 11 ? atoi(argv[11]) : 0;

    AggState agg = build_state(name, type, start, end, nc);
    auto bs = buckets_of(agg);
    std::vector<float> w(D);
    fa_oracle_weights(wseed, D, w.data());
    std::string j = "{\"D\":" + std::to_string(D) + ",\"buckets\":[";
    for (size_t bi = 0; bi < bs.size(); ++bi) {
        Bucket& b = bs[bi];
        uint64_t sb = bucket_seed(seed, b.model_part);
        torch::Tensor acc, acc_bf;  // FedAvg restatements in libtorch
        for (int k = 0; k < D; ++k) {
            auto cm = client_module(name, type, start, end, nc, b.model_part);
            fill_client(cm, sb, k);
            std::string blob = save_blob(cm);
            if (k == 0 && (blob_mp == b.model_part || (blob_mp < 0 && param_numel(cm) <= 200000)))
                write_bin(outdir + "/mp" + std::to_string(b.model_part) + "_client0.pt", blob.data(), blob.size());
            auto x = flat_params(cm);
            if (k == 0) {
                acc = torch::zeros_like(x);
                acc_bf = torch::zeros_like(x);
            }
            acc.add_(x, w[k]);
            acc_bf.add_(x.to(torch::kBFloat16).to(torch::kFloat32), w[k]);
            literal_receipt(b, blob, 1000);
        }
        std::string mp = outdir + "/mp" + std::to_string(b.model_part);
        write_tensor(mp + "_literal.f32", flat_params(b.global));
        write_tensor(mp + "_fedavg.f32", acc);
        write_tensor(mp + "_fedavg_bf16.bf16", acc_bf.to(torch::kBFloat16));
        write_tensor(mp + "_fedavg_bf16.f32", acc_bf);
        // buffers of the global module after the round (= last client's, aggregator.cpp:82-86 is dead code)
        std::vector<torch::Tensor> bufs;
        for (auto& t : b.global->named_buffers(true))
            if (t.value().scalar_type() == torch::kFloat32) bufs.push_back(t.value().reshape({-1}));
        if (!bufs.empty()) write_tensor(mp + "_buffers.f32", torch::cat(bufs));
        j += (bi ? "," : "") + std::string("{\"model_part\":") + std::to_string(b.model_part) +
             ",\"numel\":" + std::to_string(acc.numel()) + ",\"seed\":" + std::to_string(sb) + "}";
    }
    j += "],\"weights\":[";
    for (int k = 0; k < D; ++k) {
        char tmp[64];
        snprintf(tmp, sizeof tmp, "%s%.9g", k ? "," : "", w[k]);
        j += tmp;
    }
    printf("%s]}\n", j.c_str());
    return 0;
}

// libtorch CPU FedAvg (acc.add_(x_k, w_k) in client order) over D synthetic
// buckets of n fp32 (or bf16 with `bf16`: the fp32 accumulator takes the bf16
// receipts as they are, type promotion widening them, and the result is rounded
// once to bf16 inside the timed region): the reference's arithmetic library doing
// the intended op.  The inputs are generated on all threads (a C4-sized sample is
// 36 GB), outside the clock.
int cmd_bench_fedavg(int argc, char** argv) {
    int64_t n = atoll(argv[2]);
    int D = atoi(argv[3]), threads = atoi(argv[4]), reps = atoi(argv[5]);
    const bool bf16 = argc > 6 && std::string(argv[6]) == "bf16";
    at::set_num_threads(threads);
    std::vector<torch::Tensor> x(D);
    std::vector<float> w(D);
    fa_oracle_weights(7, D, w.data());
    const double t_fill = now_s();
    for (int k = 0; k < D; ++k) {
        x[k] = torch::empty({n}, bf16 ? torch::kBFloat16 : torch::kFloat32);
        char* base = (char*)x[k].data_ptr();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([=] {
                const int64_t a = n * t / threads, b = n * (t + 1) / threads;
                if (bf16)
                    fa_oracle_fill_bf16(0x5EED, (uint32_t)k, (uint64_t)a, (size_t)(b - a), (uint16_t*)base + a);
                else
                    fa_oracle_fill_f32(0x5EED, (uint32_t)k, (uint64_t)a, (size_t)(b - a), (float*)base + a);
            });
        for (auto& th : pool) th.join();
    }
    const double fill_s = now_s() - t_fill;
    auto acc = torch::zeros({n}, torch::kFloat32);
    torch::Tensor out;
    double best = 1e30, total = 0;
    std::string rep_s;  // every timed rep, so the caller can report the spread
    for (int r = 0; r < reps + 1; ++r) {
        double t0 = now_s();
        acc.zero_();
        for (int k = 0; k < D; ++k) acc.add_(x[k], w[k]);
        if (bf16) out = acc.to(torch::kBFloat16);
        double dt = now_s() - t0;
        if (r == 0) continue;  // warm-up
        total += dt;
        if (dt < best) best = dt;
        char b[32];
        snprintf(b, sizeof b, "%s%.6f", rep_s.empty() ? "" : ",", dt);
        rep_s += b;
    }
    double avg = total / reps, bytes = (double)D * n * (bf16 ? 2 : 4);
    printf("{\"mode\":\"fedavg\",\"dtype\":\"%s\",\"n\":%lld,\"D\":%d,\"threads\":%d,\"reps\":%d,\"avg_s\":%.6f,"
           "\"best_s\":%.6f,\"gib_s\":%.4f,\"fill_s\":%.3f,\"rep_s\":[%s],\"checksum\":%.9g}\n",
           bf16 ? "bf16" : "f32", (long long)n, D, threads, reps, avg, best, bytes / avg / (1ull << 30), fill_s,
           rep_s.c_str(), acc.sum().item<double>());
    return 0;
}

// The reference-literal receive loop (torch::load + (p+p)/1000 + copy_) timed per receipt; with
// `arith` the receipts are decoded before the clock starts and only the arithmetic of aggregator.cpp:72-88
// is timed (p <- div(x + x, 1000), copy_ into the global part, per named parameter).
int cmd_bench_literal(int argc, char** argv) {
    int name = atoi(argv[2]), type = atoi(argv[3]), start = atoi(argv[4]), end = atoi(argv[5]), nc = atoi(argv[6]);
    int D = atoi(argv[7]), threads = atoi(argv[8]), model_part = atoi(argv[9]);
    const bool arith = argc > 10 && std::string(argv[10]) == "arith";
    at::set_num_threads(threads);
    AggState agg = build_state(name, type, start, end, nc);
    Bucket b = buckets_of(agg)[model_part - 1];
    std::vector<std::string> blobs;
    std::vector<torch::nn::Sequential> decoded;
    for (int k = 0; k < D; ++k) {
        auto cm = client_module(name, type, start, end, nc, model_part);
        fill_client(cm, bucket_seed(0x5EED, model_part), k);
        if (arith) decoded.push_back(cm);
        else blobs.push_back(save_blob(cm));
    }
    double t0 = now_s();
    if (arith) {
        torch::NoGradGuard ng;
        auto g = b.global->named_parameters(true);
        for (int k = 0; k < D; ++k) {
            auto x = decoded[(size_t)k]->named_parameters(true);
            for (size_t j = 0; j < g.size(); ++j) g[j].value().copy_(torch::div(x[j].value() + x[j].value(), 1000));
        }
    } else {
        for (int k = 0; k < D; ++k) literal_receipt(b, blobs[k], 1000);
    }
    double dt = now_s() - t0;
    double bytes = (double)D * param_numel(b.global) * 4;
    printf("{\"mode\":\"%s\",\"model_part\":%d,\"numel\":%lld,\"D\":%d,\"threads\":%d,\"s\":%.6f,\"gib_s\":%.4f}\n",
           arith ? "literal-arith" : "literal", model_part, (long long)param_numel(b.global), D, threads, dt,
           bytes / dt / (1ull << 30));
    return 0;
}

// A whole aggregation round of the reference's receive loop, network aside: phase 1 = D receipts of
// model_part 1, phase 2 = D receipts of every last-part layer (aggregator.cpp:59-93, :108-150), each
// receipt torch::load'ed and folded (literal_receipt).  Blobs are made before the clock; `rounds` rounds are
// timed after one warm-up round.  Reports ms per round and GiB/s of parameters received.
int cmd_bench_round(int argc, char** argv) {
    int name = atoi(argv[2]), type = atoi(argv[3]), start = atoi(argv[4]), end = atoi(argv[5]), nc = atoi(argv[6]);
    int D = atoi(argv[7]), threads = atoi(argv[8]), rounds = atoi(argv[9]);
    at::set_num_threads(threads);
    AggState agg = build_state(name, type, start, end, nc);
    auto bs = buckets_of(agg);
    std::vector<std::vector<std::string>> blobs(bs.size());
    int64_t params = 0;
    for (size_t b = 0; b < bs.size(); ++b) {
        params += param_numel(bs[b].global);
        for (int k = 0; k < D; ++k) {
            auto cm = client_module(name, type, start, end, nc, bs[b].model_part);
            fill_client(cm, bucket_seed(0x5EED, bs[b].model_part), k);
            blobs[b].push_back(save_blob(cm));
        }
    }
    std::vector<double> ms;
    for (int r = 0; r < rounds + 1; ++r) {
        const double t0 = now_s();
        for (size_t b = 0; b < bs.size(); ++b)
            for (int k = 0; k < D; ++k) literal_receipt(bs[b], blobs[b][(size_t)k], 1000);
        if (r) ms.push_back((now_s() - t0) * 1e3);
    }
    std::sort(ms.begin(), ms.end());
    double avg = 0;
    for (double x : ms) avg += x / ms.size();
    printf("{\"mode\":\"round\",\"buckets\":%zu,\"params\":%lld,\"D\":%d,\"threads\":%d,\"rounds\":%d,"
           "\"round_ms_avg\":%.4f,\"round_ms_median\":%.4f,\"gib_s\":%.4f}\n",
           bs.size(), (long long)params, D, threads, rounds, avg, ms[ms.size() / 2],
           (double)D * params * 4 / (avg * 1e-3) / (1ull << 30));
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: ref_harness layout|golden|bench-fedavg|bench-literal|bench-round ...\n");
        return 2;
    }
    std::string mode = argv[1];
    // vgg_part prints its arguments to stdout (vgg_help.cpp:249): keep stdout for JSON.
    std::streambuf* saved = std::cout.rdbuf();
    std::ostringstream sink;
    std::cout.rdbuf(sink.rdbuf());
    int rc = 2;
    if (mode == "layout" && argc >= 7) {
        AggState s = build_state(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]));
        printf("%s\n", layout_json(s).c_str());
        rc = 0;
    } else if (mode == "golden" && argc >= 11) {
        rc = cmd_golden(argc, argv);
    } else if (mode == "bench-fedavg" && argc >= 6) {
        rc = cmd_bench_fedavg(argc, argv);
    } else if (mode == "bench-literal" && argc >= 10) {
        rc = cmd_bench_literal(argc, argv);
    } else if (mode == "bench-round" && argc >= 10) {
        rc = cmd_bench_round(argc, argv);
    } else {
        fprintf(stderr, "bad arguments\n");
    }
    std::cout.rdbuf(saved);
    return rc;
}
