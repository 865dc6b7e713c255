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
#include <functional>
#include <map>
#include <memory>
#include <mutex>
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

// A byte buffer that is NOT zero-filled (frames are hundreds of MB).  Heap memory by default; a
// buffer handed out by a pool carries the pool's release function (and `pinned` when the memory is
// page-locked, i.e. a DMA engine can read or write it in place).
struct Bytes {
    char* p = nullptr;
    size_t n = 0;
    bool pinned = false;
    std::function<void(char*)> release;  // empty: delete[]
    explicit Bytes(size_t size) : p(new char[size]), n(size) {}
    Bytes(char* mem, size_t size, bool is_pinned, std::function<void(char*)> rel)
        : p(mem), n(size), pinned(is_pinned), release(std::move(rel)) {}
    ~Bytes() {
        if (release) release(p);
        else delete[] p;
    }
    Bytes(const Bytes&) = delete;
    Bytes& operator=(const Bytes&) = delete;
    char* data() { return p; }
    const char* data() const { return p; }
    size_t size() const { return n; }
};

// Where frame buffers come from (received frames, outgoing frames).  Process-wide; install before
// any network thread starts.  Default: new_frame_buffer == make_shared<Bytes>(n).
using FrameAllocator = std::function<std::shared_ptr<Bytes>(size_t)>;
void set_frame_allocator(FrameAllocator a);
std::shared_ptr<Bytes> new_frame_buffer(size_t n);

// A frame buffer of n bytes whose byte `lead` lies on a 64-byte boundary: the torch::save archive of an
// OPERATION frame starts there, so its tensor records (64-byte aligned within the archive) are 64-byte
// aligned in memory and a kernel can read or write them in place (small receipts).  A view
// into a new_frame_buffer of n + 64 bytes, which goes back to its pool with the view.
std::shared_ptr<Bytes> aligned_frame_buffer(size_t n, size_t lead);
// Where the archive (`values`) of an OPERATION frame's text starts, from its first `have` bytes; 0 when
// they hold no "values : " field (a refactor frame, or a header longer than `have`).
size_t values_offset(const char* text, size_t have);

// A recycling pool of frame buffers over an allocator pair (e.g. fa_host_alloc/fa_host_free for pinned
// memory).  Buffers of at least `min_bytes` are rounded up to a size class (2 MiB multiples from 2 MiB,
// powers of two from 64 KiB below) and return to the pool when their last reference goes; a round's
// frames have the same sizes as the last round's, so the steady state allocates nothing.  Smaller
// requests use the heap.
class BufferPool : public std::enable_shared_from_this<BufferPool> {
public:
    using AllocFn = std::function<char*(size_t)>;
    using FreeFn = std::function<void(char*)>;
    static std::shared_ptr<BufferPool> create(AllocFn alloc, FreeFn free, bool pinned, size_t min_bytes = 1u << 20);
    ~BufferPool();
    std::shared_ptr<Bytes> get(size_t n);
    size_t cached_bytes();
    size_t allocations() const { return allocs_; }

private:
    BufferPool(AllocFn a, FreeFn f, bool pinned, size_t min_bytes)
        : alloc_(std::move(a)), free_fn_(std::move(f)), pinned_(pinned), min_(min_bytes) {}
    AllocFn alloc_;
    FreeFn free_fn_;
    bool pinned_;
    size_t min_;
    std::mutex m_;
    std::multimap<size_t, char*> free_;  // class size -> buffer
    size_t allocs_ = 0;
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
// A received OPERATION frame's text (no length prefix): the header fields decoded into *m, and where
// the torch::save archive (`values`) lies inside it; false for a malformed header.
bool split_receipt(const char* base, size_t size, Message* m, size_t* blob_off, size_t* blob_len, std::string* err);
// The same from the first `have` bytes of a frame text of `size` bytes (a frame still arriving): the header
// must lie within them.
bool split_receipt_head(const char* base, size_t have, size_t size, Message* m, size_t* blob_off, size_t* blob_len,
                        std::string* err);
// Length-prefixed frame as it goes on the socket (one copy of m.values).
std::string frame(const Message& m);
std::shared_ptr<Bytes> frame_bytes(const Message& m);

}  // namespace fahost
