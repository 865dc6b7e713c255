// ref_wire.cpp -- TEST INFRASTRUCTURE: the reference's own Message.h encoder/parser
// (pipeline_simulation/Message.h, included from where it lies under /root/reference; the
// frame is what network_layer.cpp:764-766 + my_send :6-31 put on the socket: a native-endian
// int length, then fromJson_toStr(toJson(msg))).  Used only by tools/gen_wire_golden.py to
// write tests/golden/frames/; never part of the product.
//
//   ref_wire encode out=<file> key=value ...   (values=@<file> reads the values bytes)
//   ref_wire decode <file>                     -> one JSON line with every field
// Keys: save_connection type client_id prev_node size_ type_op model_part t_start batch0 values
//       start end prev next dataset num_classes model_name model_type data_owners=0,2,3
//       rooting_table=0:10.0.0.1,4:10.0.0.5 read_table
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "Message.h"

static std::string slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static uint32_t crc32_bytes(const std::string& s) {  // IEEE 802.3, bitwise
    uint32_t c = 0xFFFFFFFFu;
    for (unsigned char b : s) {
        c ^= b;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c ^ 0xFFFFFFFFu;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ref_wire encode out=<file> key=value ... | decode <file>\n");
        return 2;
    }
    const std::string cmd = argv[1];
    if (cmd == "encode") {
        Message m{};
        m.save_connection = 0;
        m.type = OPERATION;
        m.dest = 0;
        std::string out;
        for (int i = 2; i < argc; ++i) {
            const std::string a = argv[i];
            const size_t eq = a.find('=');
            const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
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
            else if (k == "values") m.values = v.size() && v[0] == '@' ? slurp(v.substr(1)) : v;
            else if (k == "start") m.start = std::stoi(v);
            else if (k == "end") m.end = std::stoi(v);
            else if (k == "prev") m.prev = std::stoi(v);
            else if (k == "next") m.next = std::stoi(v);
            else if (k == "dataset") m.dataset = std::stoi(v);
            else if (k == "num_classes") m.num_classes = std::stoi(v);
            else if (k == "model_name") m.model_name = std::stoi(v);
            else if (k == "model_type") m.model_type = std::stoi(v);
            else if (k == "read_table") m.read_table = std::stoi(v);
            else if (k == "data_owners") {
                std::stringstream ss(v);
                std::string t;
                while (std::getline(ss, t, ',')) m.data_owners.push_back(std::stoi(t));
            } else if (k == "rooting_table") {
                std::stringstream ss(v);
                std::string t;
                while (std::getline(ss, t, ',')) {
                    const size_t c = t.find(':');
                    m.rooting_table.push_back({std::stoi(t.substr(0, c)), t.substr(c + 1)});
                }
            } else {
                fprintf(stderr, "unknown key %s\n", k.c_str());
                return 2;
            }
        }
        Json::Value j = toJson(m);
        const std::string text = fromJson_toStr<Message>(j);
        const int len = (int)text.size();
        std::ofstream f(out, std::ios::binary);
        f.write((const char*)&len, sizeof(int));
        f.write(text.data(), (std::streamsize)text.size());
        return f ? 0 : 1;
    }
    if (cmd == "decode") {
        const std::string raw = slurp(argv[2]);
        int len = 0;
        std::memcpy(&len, raw.data(), 4);
        const std::string text = raw.substr(4, (size_t)len);
        Json::Value j = fromStr_toJson<Message>(text);
        Message m = fromJson<Message>(j);
        printf("{\"save_connection\": %d, \"type\": %d", m.save_connection, m.type);
        if (m.type == OPERATION) {
            printf(", \"client_id\": %d, \"prev_node\": %d, \"size_\": %d, \"type_op\": %d, \"model_part\": %d, "
                   "\"t_start\": %ld, \"batch0\": %d, \"values_len\": %zu, \"values_crc32\": %u",
                   m.client_id, m.prev_node, m.size_, m.type_op, m.model_part, m.t_start, m.batch0, m.values.size(),
                   crc32_bytes(m.values));
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
    fprintf(stderr, "bad command\n");
    return 2;
}
