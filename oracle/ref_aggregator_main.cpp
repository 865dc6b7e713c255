// ref_aggregator_main.cpp -- TEST INFRASTRUCTURE (oracle/Makefile.ref, target oracle/_ref/ref_aggregator).
//
// Runs the reference-side binding of INTEGRATION.md section 2 (aggregate_rounds, extracted verbatim into
// oracle/_ref/aggregator_fa.cpp) inside the reference's own process structure: systemAPI with its
// receiver / sender threads and network_layer (pipeline_simulation/systemAPI.cpp, network_layer.cpp,
// compiled from /root/reference), the model builders for refactor(), libtorch, and libfa.so for the
// reduction.  This is aggregator.cpp:9-53 without argparse (third_party/argparse is not in the reference
// tree, CMakeLists.txt:15): `ref_aggregator <data_owners> <compute_nodes>` for `-i -1 -d D -c C`.
//
// findInit() (network_layer.cpp:197-291) locates the init node by UDP multicast and then releases the
// receiver thread (put_internal_task(Task()), :289).  On one host the routing table's localhost entries
// (network_layer.h:80-86) already point at the init node, so only that last step runs here -- the bypass
// README.md:77-82 describes.  Everything after it is the reference's code path: check_new_refactor_task,
// refactor -> init_model_sate, then the binding's rounds over check_new_task / new_message.
#include <cstdlib>
#include <iostream>

#include "systemAPI.h"

void aggregate_rounds(systemAPI& sys_, int myid, int num_data_owners, int num_compute_nodes);

int main(int argc, char** argv) {
    if (argc != 3) {
        std::cerr << "usage: ref_aggregator <data_owners> <compute_nodes>\n";
        return 2;
    }
    const int myid = -1, num_data_owners = std::atoi(argv[1]), num_compute_nodes = std::atoi(argv[2]);
    systemAPI sys_(true, myid, "main_experiment");          // aggregator.cpp:47
    sys_.my_network_layer.put_internal_task(Task());       // the end of findInit (aggregator.cpp:51)
    refactoring_data client_message = sys_.my_network_layer.check_new_refactor_task();  // :52
    sys_.refactor(client_message);                         // :53
    std::cerr << "[ref_aggregator] refactor done: " << sys_.parts[1].layers.size() << " last-part layer(s)\n";
    aggregate_rounds(sys_, myid, num_data_owners, num_compute_nodes);  // :55-167 on libfa (never returns)
    return 0;
}
