// wire.cpp -- Message.h frame encoder/decoder (see wire.h for the grammar).
#include "wire.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <map>
#include <sstream>

namespace fahost {

namespace {

std::string ints_str(const std::vector<int>& v) {  // getStr<std::vector<int>>, Message.h:181-190
    std::string t = "[ ";
    for (int x : v) t += std::to_string(x) + " ";
    return t + "]";
}

std::string table_str(const std::vector<std::pair<int, std::string>>& v) {  // Message.h:202-211
    std::string t = "[ ";
    for (auto& e : v) t += std::to_string(e.first) + "," + e.second + " ";
    return t + "]";
}

std::vector<int> parse_ints(const std::string& s) {  // getValue<std::vector<int>>, Message.h:268-280
    std::vector<int> out;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ' '))
        if (tok != "[" && tok != "]" && !tok.empty()) out.push_back(std::stoi(tok));
    return out;
}

std::vector<std::pair<int, std::string>> parse_table(const std::string& s) {  // Message.h:296-316
    std::vector<std::pair<int, std::string>> out;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ' ')) {
        if (tok == "[" || tok == "]" || tok.empty()) continue;
        const size_t c = tok.find(',');
        out.emplace_back(std::stoi(tok.substr(0, c)), c == std::string::npos ? "" : tok.substr(c + 1, tok.find(',', c + 1) - c - 1));
    }
    return out;
}

void field(std::string& t, const char* name, const std::string& v) {
    t += name;
    t += " : ";
    t += v;
    t += ",\n";
}

}  // namespace

std::string encode(const Message& m) {
    std::string t = "{,\n";
    field(t, "save_connection", std::to_string(m.save_connection));
    field(t, "type", std::to_string(m.type));
    if (m.type == OPERATION) {
        field(t, "client_id", std::to_string(m.client_id));
        field(t, "prev_node", std::to_string(m.prev_node));
        field(t, "size_", std::to_string(m.size_));
        field(t, "type_op", std::to_string(m.type_op));
        field(t, "model_part", std::to_string(m.model_part));
        field(t, "t_start", std::to_string(m.t_start));
        field(t, "batch0", std::to_string(m.batch0));
        t.reserve(t.size() + m.values.size() + 16);
        field(t, "values", m.values);
    } else {
        field(t, "start", std::to_string(m.start));
        field(t, "end", std::to_string(m.end));
        field(t, "prev", std::to_string(m.prev));
        field(t, "next", std::to_string(m.next));
        field(t, "dataset", std::to_string(m.dataset));
        field(t, "num_classes", std::to_string(m.num_classes));
        field(t, "model_name", std::to_string(m.model_name));
        field(t, "model_type", std::to_string(m.model_type));
        field(t, "data_owners", ints_str(m.data_owners));
        field(t, "rooting_table", table_str(m.rooting_table));
        field(t, "read_table", std::to_string(m.read_table));
    }
    return t + "}";
}

std::string operation_header(const Message& m) {
    std::string t = "{,\n";
    field(t, "save_connection", std::to_string(m.save_connection));
    field(t, "type", std::to_string(m.type));
    field(t, "client_id", std::to_string(m.client_id));
    field(t, "prev_node", std::to_string(m.prev_node));
    field(t, "size_", std::to_string(m.size_));
    field(t, "type_op", std::to_string(m.type_op));
    field(t, "model_part", std::to_string(m.model_part));
    field(t, "t_start", std::to_string(m.t_start));
    field(t, "batch0", std::to_string(m.batch0));
    return t + "values : ";
}

namespace {
FrameAllocator& frame_allocator() {
    static FrameAllocator a;
    return a;
}
}  // namespace

void set_frame_allocator(FrameAllocator a) { frame_allocator() = std::move(a); }

std::shared_ptr<Bytes> new_frame_buffer(size_t n) {
    auto& a = frame_allocator();
    return a ? a(n) : std::make_shared<Bytes>(n);
}

std::shared_ptr<BufferPool> BufferPool::create(AllocFn alloc, FreeFn free, bool pinned, size_t min_bytes) {
    return std::shared_ptr<BufferPool>(new BufferPool(std::move(alloc), std::move(free), pinned, min_bytes));
}

BufferPool::~BufferPool() {
    for (auto& kv : free_) free_fn_(kv.second);
}

std::shared_ptr<Bytes> BufferPool::get(size_t n) {
    if (n < min_) return std::make_shared<Bytes>(n);
    // 2 MiB classes from 2 MiB up; below, powers of two from 64 KiB (a small model's receipts, e.g. LeNet-5's
    // 200 KB parts, then take 256 KiB buffers, not 2 MiB ones)
    size_t cls = (n + (2u << 20) - 1) / (2u << 20) * (2u << 20);
    if (n < (2u << 20)) {
        cls = 64u << 10;
        while (cls < n) cls <<= 1;
    }
    char* p = nullptr;
    {
        std::lock_guard<std::mutex> g(m_);
        auto it = free_.find(cls);
        if (it != free_.end()) {
            p = it->second;
            free_.erase(it);
        }
    }
    if (!p) {
        p = alloc_(cls);
        if (!p) throw std::bad_alloc();
        std::lock_guard<std::mutex> g(m_);
        ++allocs_;
    }
    std::weak_ptr<BufferPool> self = shared_from_this();
    FreeFn fallback = free_fn_;
    return std::make_shared<Bytes>(p, n, pinned_, [self, cls, fallback](char* q) {
        if (auto pool = self.lock()) {
            std::lock_guard<std::mutex> g(pool->m_);
            pool->free_.insert({cls, q});
        } else {
            fallback(q);
        }
    });
}

size_t BufferPool::cached_bytes() {
    std::lock_guard<std::mutex> g(m_);
    size_t t = 0;
    for (auto& kv : free_) t += kv.first;
    return t;
}

std::shared_ptr<Bytes> aligned_frame_buffer(size_t n, size_t lead) {
    auto raw = new_frame_buffer(n + 64);
    const size_t pad = (64 - ((uintptr_t)raw->data() + lead) % 64) % 64;
    char* p = raw->data() + pad;
    const bool pinned = raw->pinned;
    return std::make_shared<Bytes>(p, n, pinned, [raw](char*) {});  // raw returns to its pool with the view
}

size_t values_offset(const char* text, size_t have) {
    static const char kField[] = "\nvalues : ";
    const char* e = text + have;
    const char* at = std::search(text, e, kField, kField + sizeof kField - 1);
    return at == e ? 0 : (size_t)(at - text) + sizeof kField - 1;
}

std::shared_ptr<Bytes> operation_frame(const Message& m, size_t values_len, char** values) {
    const std::string head = operation_header(m);
    const size_t text = head.size() + values_len + 3;
    auto b = aligned_frame_buffer(4 + text, 4 + head.size());  // the archive 64-byte aligned
    const int32_t len = (int32_t)text;
    std::memcpy(b->data(), &len, 4);  // native-endian int, as my_send does (network_layer.cpp:16)
    std::memcpy(b->data() + 4, head.data(), head.size());
    *values = b->data() + 4 + head.size();
    std::memcpy(*values + values_len, ",\n}", 3);
    return b;
}

std::shared_ptr<Bytes> frame_bytes(const Message& m) {
    if (m.type == OPERATION) {
        char* v = nullptr;
        auto b = operation_frame(m, m.values.size(), &v);
        std::memcpy(v, m.values.data(), m.values.size());
        return b;
    }
    const std::string text = encode(m);
    auto b = new_frame_buffer(4 + text.size());
    const int32_t len = (int32_t)text.size();
    std::memcpy(b->data(), &len, 4);
    std::memcpy(b->data() + 4, text.data(), text.size());
    return b;
}

std::string frame(const Message& m) {
    auto b = frame_bytes(m);
    return std::string(b->data(), b->size());
}

namespace {
bool decode_impl(const std::string& text, Message* m, std::string* err);
}

// Integer fields that do not parse (std::stoi / std::stol throw) fail the decode instead of throwing
// out of the receiver thread.
bool decode(const std::string& text, Message* m, std::string* err) {
    try {
        return decode_impl(text, m, err);
    } catch (const std::exception& e) {
        if (err) *err = std::string("bad field value: ") + e.what();
        return false;
    }
}

bool split_receipt(const char* base, size_t size, Message* m, size_t* blob_off, size_t* blob_len, std::string* err) {
    return split_receipt_head(base, size, size, m, blob_off, blob_len, err);
}

bool split_receipt_head(const char* base, size_t have, size_t size, Message* m, size_t* blob_off, size_t* blob_len,
                        std::string* err) {
    // The header is the text before "values : " (at a line start, within the first 4 KiB); the archive
    // runs from there to the closing ",\n}" (Message.h:514-518), parsed without touching its bytes.
    const size_t scan = std::min<size_t>(std::min(have, size), 4096);
    const char* v = nullptr;
    for (size_t i = 0; i + 9 <= scan; ++i)
        if (std::memcmp(base + i, "values : ", 9) == 0 && (i == 0 || base[i - 1] == '\n')) {
            v = base + i;
            break;
        }
    const std::string head = v ? std::string(base, v - base) + "values : ,\n}" : std::string(base, scan);
    if (!decode(head, m, err)) return false;
    *blob_off = *blob_len = 0;
    if (v) {
        *blob_off = (size_t)(v - base) + 9;
        *blob_len = size >= *blob_off + 3 ? size - 3 - *blob_off : 0;
    }
    return true;
}

namespace {
bool decode_impl(const std::string& text, Message* m, std::string* err) {
    // fromStr_toJson (Message.h:499-569): split on ",\n", name/value on " : "; `values`
    // swallows the rest of the text minus the closing ",\n}".
    std::map<std::string, std::string> kv;
    size_t pos = 0;
    while (pos < text.size()) {
        if (text.compare(pos, 6, "values") == 0) {
            const size_t sep = text.find(" : ", pos);
            if (sep == std::string::npos || text.size() < pos + 3) break;
            const size_t vb = sep + 3, ve = text.size() >= 3 ? text.size() - 3 : vb;
            kv["values"] = ve > vb ? text.substr(vb, ve - vb) : std::string();
            break;
        }
        size_t nl = text.find(",\n", pos);
        std::string tok = text.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
        pos = nl == std::string::npos ? text.size() : nl + 2;
        if (tok == "{" || tok == "}" || tok.empty()) continue;
        const size_t sep = tok.find(" : ");
        if (sep == std::string::npos) continue;
        kv[tok.substr(0, sep)] = tok.substr(sep + 3);
    }
    auto geti = [&](const char* k, int* out) -> bool {
        auto it = kv.find(k);
        if (it == kv.end()) {
            if (err) *err = std::string("missing field ") + k;
            return false;
        }
        try {
            *out = std::stoi(it->second);
        } catch (...) {
            if (err) *err = std::string("bad integer in ") + k;
            return false;
        }
        return true;
    };
    Message r;
    if (!geti("save_connection", &r.save_connection) || !geti("type", &r.type)) return false;
    if (r.type == OPERATION) {
        if (!geti("client_id", &r.client_id) || !geti("prev_node", &r.prev_node) || !geti("size_", &r.size_) ||
            !geti("type_op", &r.type_op) || !geti("model_part", &r.model_part) || !geti("batch0", &r.batch0))
            return false;
        auto t = kv.find("t_start");
        if (t == kv.end()) {
            if (err) *err = "missing field t_start";
            return false;
        }
        r.t_start = std::stol(t->second);
        auto v = kv.find("values");
        if (v == kv.end()) {
            if (err) *err = "missing field values";
            return false;
        }
        r.values = std::move(v->second);
    } else {
        if (!geti("start", &r.start) || !geti("end", &r.end) || !geti("prev", &r.prev) || !geti("next", &r.next) ||
            !geti("dataset", &r.dataset) || !geti("num_classes", &r.num_classes) ||
            !geti("model_name", &r.model_name) || !geti("model_type", &r.model_type) ||
            !geti("read_table", &r.read_table))
            return false;
        r.data_owners = parse_ints(kv["data_owners"]);
        r.rooting_table = parse_table(kv["rooting_table"]);
    }
    *m = std::move(r);
    return true;
}
}  // namespace

}  // namespace fahost
