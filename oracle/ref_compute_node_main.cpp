// ref_compute_node_main.cpp -- TEST INFRASTRUCTURE (oracle/Makefile.ref, target oracle/_ref/ref_compute_node).
//
// Runs the compute-node binding of INTEGRATION.md section 5 (aggregate_client_states, extracted verbatim into
// oracle/_ref/compute_node_fa.cpp) on the state the reference's own compute node builds: systemAPI(false, id)
// (compute_node.cpp:113) and refactor() of a compute-node refactor message, which calls
// init_state_vector (systemAPI.cpp:3-15, :259-264) -- one State per data owner, each with the model part
// ModelPart(name, model, start, end) makes from the reference's builders (models/models.h:16-43).
// Every client's parameters are then set to the oracle's generator values, the binding aggregates them through
// libfa.so on the GPU, and every client's every layer is compared, bit for bit, with the oracle's ordered
// FedAvg chain (oracle/fa_oracle.c) over the same values with the binding's weights.
//
//   ref_compute_node <data_owners> <model_name> <model_type> <start> <end> [seed]
// prints one JSON line; exit 0 iff every element matched.  The network threads systemAPI starts never
// return (compute_node.cpp joins nothing), so the process ends with _Exit.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <vector>

#include "fa_oracle.h"
#include "fedavg/fa.h"
#include "systemAPI.h"

void aggregate_client_states(systemAPI& sys, fa_ctx* fa, const std::map<int, double>& samples);

int main(int argc, char** argv) {
    if (argc < 6) {
        std::cerr << "usage: ref_compute_node <data_owners> <model_name> <model_type> <start> <end> [seed]\n";
        return 2;
    }
    const int D = std::atoi(argv[1]);
    const uint64_t seed = argc > 6 ? std::strtoull(argv[6], nullptr, 0) : 0xC0DEull;
    systemAPI sys_(false, 1, "main_experiment");  // a compute node, id 1 (compute_node.cpp:113)
    refactoring_data m;                            // what the init node sends a compute node (Task.h:19-28)
    m.to_data_onwer = false;
    m.model_name_ = std::atoi(argv[2]);
    m.model_type_ = std::atoi(argv[3]);
    m.start = std::atoi(argv[4]);
    m.end = std::atoi(argv[5]);
    m.num_class = 10;
    m.prev = -1;
    m.next = -1;
    for (int k = 0; k < D; ++k) m.data_owners.push_back(k == 0 ? 0 : k + 1);  // ids 0, 2, 3, ... (C = 1)
    sys_.refactor(m);  // -> init_state_vector: clients_state[id] = State(id, ModelPart(...).layers, SGD)
    auto& states = sys_.clients_state;
    if ((int)states.size() != D) {
        std::cerr << "init_state_vector built " << states.size() << " states\n";
        std::_Exit(1);
    }
    const size_t L = states.begin()->second.layers.size();
    // the values: client k's layer l = the oracle generator (seed ^ l << 32, client k) over its flattened
    // named_parameters; kept flat for the oracle
    std::map<int, double> samples;
    std::vector<std::vector<std::vector<float>>> x(L);  // [layer][client] flat
    {
        torch::NoGradGuard ng;
        int k = 0;
        for (auto& kv : states) {
            samples[kv.first] = 500.0 + 37.0 * k;  // distinct n_k: the weights matter
            for (size_t l = 0; l < L; ++l) {
                size_t n = 0;
                for (auto& p : kv.second.layers[l]->named_parameters(true)) n += (size_t)p.value().numel();
                x[l].emplace_back(n);
                fa_oracle_fill_f32(seed ^ ((uint64_t)l << 32), (uint32_t)k, 0, n, x[l].back().data());
                size_t o = 0;
                for (auto& p : kv.second.layers[l]->named_parameters(true)) {
                    auto t = p.value();
                    t.copy_(torch::from_blob(x[l].back().data() + o, t.sizes(), torch::kFloat32));
                    o += (size_t)t.numel();
                }
            }
            ++k;
        }
    }
    // the binding's weights, computed as it computes them
    std::vector<float> w;
    double total = 0;
    for (auto& kv : samples) total += kv.second;
    for (auto& kv : samples) w.push_back((float)(kv.second / total));

    fa_ctx* fa = nullptr;
    if (fa_create(&fa, 1, 0) != FA_OK) {
        std::cerr << "fa_create: " << fa_last_error() << "\n";
        std::_Exit(1);
    }
    aggregate_client_states(sys_, fa, samples);  // INTEGRATION.md section 5, verbatim

    size_t elems = 0, mismatches = 0;
    for (size_t l = 0; l < L; ++l) {
        const size_t n = x[l][0].size();
        std::vector<const float*> ptrs;
        for (auto& v : x[l]) ptrs.push_back(v.data());
        std::vector<float> want(n);
        fa_oracle_fedavg_f32(ptrs.data(), w.data(), D, n, nullptr, want.data(), 8);
        for (auto& kv : states) {
            size_t o = 0;
            for (auto& p : kv.second.layers[l]->named_parameters(true)) {
                auto t = p.value().contiguous();
                const size_t c = (size_t)t.numel();
                if (std::memcmp(t.data_ptr<float>(), want.data() + o, c * sizeof(float)) != 0) {
                    for (size_t i = 0; i < c; ++i)
                        if (std::memcmp(t.data_ptr<float>() + i, want.data() + o + i, sizeof(float)) != 0) ++mismatches;
                }
                o += c;
            }
            elems += o;
        }
    }
    fa_destroy(fa);
    std::printf("{\"ok\": %s, \"clients\": %d, \"layers\": %zu, \"checked_elems\": %zu, \"mismatches\": %zu, "
                "\"layer0_elems\": %zu}\n",
                mismatches == 0 && elems > 0 ? "true" : "false", D, L, elems, mismatches, x.empty() ? 0 : x[0][0].size());
    std::fflush(stdout);
    std::_Exit(mismatches == 0 && elems > 0 ? 0 : 1);
}
