// archive_tool.cpp -- CLI over host/archive and host/wire for the CPU tests.
//   fa_archive_tool dump <archive>                  JSON: params/buffers (name, storage, shape, numel)
//   fa_archive_tool gather <archive> <out.f32>      parameters in named_parameters order (fp32)
//   fa_archive_tool patch <archive> <in.f32> <out>  archive with new parameters + fixed CRCs
//   fa_archive_tool frame <archive> <out>           a Message.h aggregation frame carrying it
//   fa_archive_tool unframe <frame> <out>           the archive inside a frame (round trip)
//   fa_archive_tool encode out=<file> key=value ...  any Message.h frame (values=@file, data_owners=0,2,3,
//                                                    rooting_table=0:10.0.0.1,4:10.0.0.5)
//   fa_archive_tool decode <frame>                  JSON of every field (values as length + CRC-32)
// encode/decode take the same arguments as oracle/ref_wire (the reference's own Message.h), so the
// wire tests compare the two byte for byte (tests/golden/frames).
#include <cstdio>
#include <cstring>
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

static int wire_encode(int argc, char** argv) {
    Message m;
    std::string out;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        const size_t eq = a.find('=');
        if (eq == std::string::npos) return std::cerr << "expected key=value: " << a << "\n", 2;
        const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
        auto list = [&](char sep) {
            std::vector<std::string> r;
            std::stringstream ss(v);
            std::string t;
            while (std::getline(ss, t, sep)) r.push_back(t);
            return r;
        };
        if (k == "out") out = v;
        else if (k == "save_connection") m.save_connection = std::stoi(v);
        else if (k == "type") m.type = std::stoi(v);
        else if (k == "client_id") m.client_id = std::stoi(v);
        else if (k == "prev_node") m.prev_node = std::stoi(v);
        else if (k == "size_") m.size_ = std::stoi(v);
        else if (k == "type_op") m.type_op = std::stoi(v);
        else if (k == "model_part") m.model_part = std::stoi(v);
        else if (k == "t_start") m.t_start = std::stol(v);
        else if (k == "batch0") m.batch0 = std::stoi(v);
        else if (k == "values") m.values = !v.empty() && v[0] == '@' ? slurp(v.c_str() + 1) : v;
        else if (k == "start") m.start = std::stoi(v);
        else if (k == "end") m.end = std::stoi(v);
        else if (k == "prev") m.prev = std::stoi(v);
        else if (k == "next") m.next = std::stoi(v);
        else if (k == "dataset") m.dataset = std::stoi(v);
        else if (k == "num_classes") m.num_classes = std::stoi(v);
        else if (k == "model_name") m.model_name = std::stoi(v);
        else if (k == "model_type") m.model_type = std::stoi(v);
        else if (k == "read_table") m.read_table = std::stoi(v);
        else if (k == "data_owners")
            for (auto& t : list(',')) m.data_owners.push_back(std::stoi(t));
        else if (k == "rooting_table")
            for (auto& t : list(',')) {
                const size_t c = t.find(':');
                m.rooting_table.push_back({std::stoi(t.substr(0, c)), t.substr(c + 1)});
            }
        else return std::cerr << "unknown key " << k << "\n", 2;
    }
    const std::string f = frame(m);
    spit(out.c_str(), f.data(), f.size());
    return 0;
}

static int wire_decode(const std::string& raw) {
    int32_t len = 0;
    if (raw.size() < 4) return std::cerr << "short frame\n", 1;
    std::memcpy(&len, raw.data(), 4);
    if (len < 0 || (size_t)len + 4 != raw.size()) return std::cerr << "length prefix does not match\n", 1;
    Message m;
    std::string err;
    if (!decode(raw.substr(4), &m, &err)) return std::cerr << err << "\n", 1;
    printf("{\"save_connection\": %d, \"type\": %d", m.save_connection, m.type);
    if (m.type == OPERATION) {
        printf(", \"client_id\": %d, \"prev_node\": %d, \"size_\": %d, \"type_op\": %d, \"model_part\": %d, "
               "\"t_start\": %ld, \"batch0\": %d, \"values_len\": %zu, \"values_crc32\": %u",
               m.client_id, m.prev_node, m.size_, m.type_op, m.model_part, m.t_start, m.batch0, m.values.size(),
               crc32((const uint8_t*)m.values.data(), m.values.size()));
    } else {
        printf(", \"start\": %d, \"end\": %d, \"prev\": %d, \"next\": %d, \"dataset\": %d, \"num_classes\": %d, "
               "\"model_name\": %d, \"model_type\": %d, \"read_table\": %d, \"data_owners\": [",
               m.start, m.end, m.prev, m.next, m.dataset, m.num_classes, m.model_name, m.model_type, m.read_table);
        for (size_t i = 0; i < m.data_owners.size(); ++i) printf("%s%d", i ? ", " : "", m.data_owners[i]);
        printf("], \"rooting_table\": [");
        for (size_t i = 0; i < m.rooting_table.size(); ++i)
            printf("%s[%d, \"%s\"]", i ? ", " : "", m.rooting_table[i].first, m.rooting_table[i].second.c_str());
        printf("]");
    }
    printf("}\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::string(argv[1]) == "encode") return wire_encode(argc, argv);
    if (argc >= 3 && std::string(argv[1]) == "decode") return wire_decode(slurp(argv[2]));
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
