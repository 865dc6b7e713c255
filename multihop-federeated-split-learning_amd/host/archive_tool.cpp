// archive_tool.cpp -- CLI over host/archive and host/wire for the CPU tests.
//   fa_archive_tool dump <archive>                  JSON: params/buffers (name, storage, shape, numel)
//   fa_archive_tool gather <archive> <out.f32>      parameters in named_parameters order (fp32)
//   fa_archive_tool patch <archive> <in.f32> <out>  archive with new parameters + fixed CRCs
//   fa_archive_tool frame <archive> <out>           a Message.h aggregation frame carrying it
//   fa_archive_tool unframe <frame> <out>           the archive inside a frame (round trip)
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "archive.h"
#include "wire.h"

using namespace fahost;

static std::string slurp(const char* p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static void spit(const char* p, const void* d, size_t n) {
    std::ofstream f(p, std::ios::binary);
    f.write((const char*)d, (std::streamsize)n);
}

static void dump_list(const char* key, const std::vector<TensorView>& v) {
    printf("\"%s\":[", key);
    for (size_t i = 0; i < v.size(); ++i) {
        printf("%s{\"name\":\"%s\",\"storage\":\"%s\",\"numel\":%lld,\"contiguous\":%s,\"shape\":[", i ? "," : "",
               v[i].name.c_str(), v[i].storage_type.c_str(), (long long)v[i].numel, v[i].contiguous ? "true" : "false");
        for (size_t d = 0; d < v[i].sizes.size(); ++d) printf("%s%lld", d ? "," : "", (long long)v[i].sizes[d]);
        printf("]}");
    }
    printf("]");
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::cerr << "usage: fa_archive_tool dump|gather|patch|frame|unframe ...\n";
        return 2;
    }
    const std::string cmd = argv[1];
    const std::string bytes = slurp(argv[2]);
    std::string err;
    if (cmd == "unframe") {
        Message m;
        if (bytes.size() < 4 || !decode(bytes.substr(4), &m, &err)) {
            std::cerr << err << "\n";
            return 1;
        }
        spit(argv[3], m.values.data(), m.values.size());
        printf("{\"client_id\":%d,\"model_part\":%d,\"type_op\":%d,\"bytes\":%zu}\n", m.client_id, m.model_part,
               m.type_op, m.values.size());
        return 0;
    }
    TorchArchive ar;
    if (!ar.parse((const uint8_t*)bytes.data(), bytes.size(), &err)) {
        std::cerr << err << "\n";
        return 1;
    }
    if (cmd == "dump") {
        printf("{\"param_numel\":%lld,", (long long)ar.param_numel());
        dump_list("params", ar.params());
        printf(",");
        dump_list("buffers", ar.buffers());
        printf("}\n");
    } else if (cmd == "gather" && argc > 3) {
        std::vector<float> v((size_t)ar.param_numel());
        if (!ar.gather_params(v.data(), &err)) return std::cerr << err << "\n", 1;
        spit(argv[3], v.data(), v.size() * 4);
    } else if (cmd == "patch" && argc > 4) {
        const std::string in = slurp(argv[3]);
        if (in.size() != (size_t)ar.param_numel() * 4) return std::cerr << "wrong value count\n", 1;
        std::string out;
        if (!ar.with_params((const float*)in.data(), &out, &err)) return std::cerr << err << "\n", 1;
        spit(argv[4], out.data(), out.size());
    } else if (cmd == "frame" && argc > 3) {
        Message m;
        m.type = OPERATION;
        m.client_id = 7;
        m.prev_node = -1;
        m.size_ = 0;
        m.type_op = AGGREGATION;
        m.model_part = 2;
        m.t_start = 1700000000000;
        m.values = bytes;
        const std::string f = frame(m);
        spit(argv[3], f.data(), f.size());
    } else {
        std::cerr << "bad command\n";
        return 2;
    }
    return 0;
}
