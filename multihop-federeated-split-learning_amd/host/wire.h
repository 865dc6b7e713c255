// wire.h -- the reference's message frame, byte-compatible (pipeline_simulation/Message.h).
//
// A frame on the TCP stream is [int32 native-endian length][text] (network_layer.cpp:6-31,
// :33-74).  The text is Message.h's JSON-like dump (fromJson_toStr, Message.h:407-457):
//   "{,\n" + "name : value,\n" for the header properties (save_connection, type)
//   + the operator properties (client_id, prev_node, size_, type_op, model_part,
//     t_start, batch0, values) or the refactor properties (start, end, prev, next,
//     dataset, num_classes, model_name, model_type, data_owners, rooting_table,
//     read_table) + "}".
// `values` is last and binary-safe: the parser takes the rest of the text minus
// the trailing ",\n}" (fromStr_toJson, Message.h:514-518).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace fahost {

enum MsgType { OPERATION = 0, REFACTOR_COMPUTE_NODE = 1, REFACTOR_DATA_OWNER = 2 };  // Message.h:4-6
enum Operation { FORWARD = 1, BACKWARD = 2, OPTIMIZE = 3, REFACTORING = 4, AGGREGATION = 5, NOOP = 6 };  // Task.h:10-17

struct Message {  // Message.h:571-616 field for field
    int save_connection = 0;
    int type = OPERATION;
    int dest = 0;  // not on the wire
    int model_part = 1;
    int start = -1, end = -1, prev = -1, next = -1, dataset = -1, num_classes = -1, model_name = -1, model_type = -1;
    std::vector<int> data_owners;
    std::vector<std::pair<int, std::string>> rooting_table;
    int read_table = 1;
    int client_id = -1, prev_node = -1, size_ = -1, type_op = -1, batch0 = -1;
    long t_start = 0;
    std::string values;
};

// A heap byte buffer that is NOT zero-filled (frames are hundreds of MB).
struct Bytes {
    std::unique_ptr<char[]> p;
    size_t n = 0;
    explicit Bytes(size_t size) : p(new char[size]), n(size) {}
    char* data() { return p.get(); }
    const char* data() const { return p.get(); }
    size_t size() const { return n; }
};

// Text of a frame (without the length prefix).
std::string encode(const Message& m);
// The text of an OPERATION frame up to and including "values : " (the archive follows, then ",\n}").
std::string operation_header(const Message& m);
// Allocates a length-prefixed OPERATION frame with `values_len` bytes reserved for the archive;
// *values points at them (the caller writes the archive in place, e.g. TorchArchive::with_params_into).
std::shared_ptr<Bytes> operation_frame(const Message& m, size_t values_len, char** values);
// Parses the text of a frame; false (with *err) when a field is missing or malformed.
bool decode(const std::string& text, Message* m, std::string* err);
// Length-prefixed frame as it goes on the socket (one copy of m.values).
std::string frame(const Message& m);
std::shared_ptr<Bytes> frame_bytes(const Message& m);

}  // namespace fahost
