// ref_cpu_aggregator.cpp -- TEST INFRASTRUCTURE / CPU BASELINE (oracle/Makefile.ref, target
// oracle/_ref/ref_cpu_aggregator).  Never linked into the product.
//
// BASELINE.json config C1 as the reference runs it: the aggregator process on CPU libtorch, over loopback.
// The process structure is the reference's own code compiled from /root/reference as it lies: systemAPI
// with its receiver and sender threads, network_layer (frames, the per-receipt torch::load input, the
// replies' torch::save in new_message), the model builders behind refactor().  Only aggregator.cpp's main
// is restated here, because aggregator.cpp itself needs third_party/argparse (absent, CMakeLists.txt:15):
//   startup        aggregator.cpp:47-53 (findInit's multicast replaced by its last step, as in
//                  oracle/ref_aggregator_main.cpp: put_internal_task(Task()), network_layer.cpp:289);
//   phase 1        :59-93  D receipts of model part 1, each torch::load'ed into parts_[0].layers[0] and
//                  folded into parts[0].layers[0] as p := (p + r) / kTrainSize_10 per named parameter;
//   reply 1        :96-106 Task(myid, aggregation_, myid), model_part 1, to node 0 and to i + c + 1;
//   phase 2        :108-150 D * L receipts of the last-part layers, loaded into parts[1].layers[mp - 2];
//   replies 2      :153-166 one per layer, same destinations.
// parts and parts_ hold the same module handles for id -1 (systemAPI.cpp:34-37, State.h:12), so r is the
// receipt just loaded and the result is fl(fl(x_last + x_last) / 1000) of the last receipt (the golden
// mp*_literal.f32 fixtures); fake_owners --mode literal checks every reply against exactly that.
//
//   ref_cpu_aggregator <data_owners> <compute_nodes>      (-i -1 -d D -c C; never returns, like the reference)
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>

#include "systemAPI.h"

namespace {

constexpr int kTrainSize10 = 1000;  // aggregator.cpp:48

long epoch_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

// One receipt: decode the archive into `slot`, then every named parameter of `global` becomes
// (global + slot) / kTrainSize10, parameter by parameter in named_parameters() order.
void fold_receipt(const Task& t, torch::nn::Sequential slot, torch::nn::Sequential global) {
    std::stringstream ss(std::string(t.model_parts.begin(), t.model_parts.end()));
    torch::load(slot, ss);
    torch::NoGradGuard no_grad;
    auto g = global->named_parameters(true);
    auto r = slot->named_parameters(true);
    for (size_t j = 0; j < g.size(); ++j) g[j].value().copy_(torch::div(g[j].value() + r[j].value(), kTrainSize10));
}

// The reduced module of `model_part` to node 0 and to the data owners i + c + 1.
void fan_out(systemAPI& sys, int myid, int model_part, torch::nn::Sequential module, int owners, int computes) {
    Task reply(myid, operation::aggregation_, myid);
    reply.model_part = model_part;
    reply.model_part_ = module;
    reply.t_start = epoch_ms();
    sys.my_network_layer.new_message(reply, 0);
    for (int i = 0; i < owners - 1; ++i) {
        reply.t_start = epoch_ms();
        sys.my_network_layer.new_message(reply, i + computes + 1);
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::cerr << "usage: ref_cpu_aggregator <data_owners> <compute_nodes>\n";
        return 2;
    }
    const int myid = -1, owners = std::atoi(argv[1]), computes = std::atoi(argv[2]);
    systemAPI sys(true, myid, "main_experiment");
    sys.my_network_layer.put_internal_task(Task());
    sys.refactor(sys.my_network_layer.check_new_refactor_task());
    const int L = (int)sys.parts[1].layers.size();
    std::cerr << "[ref_cpu_aggregator] refactor done: " << L << " last-part layer(s)\n";
    for (;;) {
        for (int got = 0; got < owners; ++got)
            fold_receipt(sys.my_network_layer.check_new_task(), sys.parts_[0].layers[0], sys.parts[0].layers[0]);
        fan_out(sys, myid, 1, sys.parts[0].layers[0], owners, computes);
        for (int got = 0; got < owners * L; ++got) {
            Task t = sys.my_network_layer.check_new_task();
            const int l = t.model_part - 2;
            fold_receipt(t, sys.parts[1].layers[l], sys.parts[1].layers[l]);
        }
        for (int l = 0; l < L; ++l) fan_out(sys, myid, l + 2, sys.parts[1].layers[l], owners, computes);
    }
}
