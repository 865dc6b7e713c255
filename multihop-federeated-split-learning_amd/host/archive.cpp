// archive.cpp -- see archive.h.  Zip (stored, zip64-aware) + a minimal pickle
// machine for the protocol-2 `data.pkl` that libtorch's OutputArchive writes.
#include "archive.h"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>

#include <zlib.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace fahost {

// ------------------------------------------------------------------ CRC-32 (IEEE, slicing-by-8)

namespace {
struct CrcTables {
    uint32_t t[8][256];
    CrcTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
};
const CrcTables& crc_tables() {
    static const CrcTables tabs;
    return tabs;
}
}  // namespace

#if defined(__x86_64__)
// Carry-less multiplication folding (PCLMULQDQ) over 16-byte blocks: four 128-bit accumulators fold 64 bytes
// per step, then fold into one, reduce 128 -> 64 -> 32 bits and finish with a Barrett reduction -- the
// method of Intel's "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ" for the reflected IEEE
// polynomial (constants x^(k) mod P for the fold distances, mu = floor(x^64 / P), P' = the polynomial).
// `c` is the running (already inverted) state; n >= 64 and a multiple of 16.  ~10x the table's rate: a
// reply's records are sealed with their CRC-32s (seal_params), which for a small model was the largest
// host cost of a round.
static inline __attribute__((target("pclmul,sse4.1"), always_inline)) __m128i clmul_fold(__m128i x, __m128i k,
                                                                                         __m128i next) {
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), next);
}

static __attribute__((target("pclmul,sse4.1"))) uint32_t crc32_fold(const uint8_t* p, size_t n, uint32_t c) {
    const __m128i k1k2 = _mm_set_epi64x(0x00000001c6e41596LL, 0x0000000154442bd4LL);
    const __m128i k3k4 = _mm_set_epi64x(0x00000000ccaa009eLL, 0x00000001751997d0LL);
    const __m128i k5 = _mm_set_epi64x(0, 0x0000000163cd6124LL);
    const __m128i mu_p = _mm_set_epi64x(0x00000001f7011641LL, 0x00000001db710641LL);
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    auto ld = [](const uint8_t* q) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(q)); };
    __m128i x1 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128((int)c)), x2 = ld(p + 16), x3 = ld(p + 32),
            x4 = ld(p + 48);
    p += 64;
    n -= 64;
    for (; n >= 64; p += 64, n -= 64) {
        x1 = clmul_fold(x1, k1k2, ld(p));
        x2 = clmul_fold(x2, k1k2, ld(p + 16));
        x3 = clmul_fold(x3, k1k2, ld(p + 32));
        x4 = clmul_fold(x4, k1k2, ld(p + 48));
    }
    x1 = clmul_fold(x1, k3k4, x2);
    x1 = clmul_fold(x1, k3k4, x3);
    x1 = clmul_fold(x1, k3k4, x4);
    for (; n >= 16; p += 16, n -= 16) x1 = clmul_fold(x1, k3k4, ld(p));
    // 128 -> 64 bits (also appends 32 zero bits), then 64 -> 32
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), _mm_clmulepi64_si128(k3k4, x1, 0x01));
    __m128i t = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k5, 0x00);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 4), t);
    // Barrett reduction
    t = _mm_and_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), mu_p, 0x10), mask32);
    t = _mm_clmulepi64_si128(t, mu_p, 0x00);
    x1 = _mm_xor_si128(x1, t);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}

static bool have_clmul() {
    static const bool h = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    return h;
}
#endif

uint32_t crc32_table(const uint8_t* p, size_t n, uint32_t crc) {
    const auto& T = crc_tables().t;
    uint32_t c = ~crc;
    while (n >= 8) {
        uint32_t a, b;
        std::memcpy(&a, p, 4);
        std::memcpy(&b, p + 4, 4);
        a ^= c;
        c = T[7][a & 0xFF] ^ T[6][(a >> 8) & 0xFF] ^ T[5][(a >> 16) & 0xFF] ^ T[4][a >> 24] ^ T[3][b & 0xFF] ^
            T[2][(b >> 8) & 0xFF] ^ T[1][(b >> 16) & 0xFF] ^ T[0][b >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = T[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return ~c;
}

uint32_t crc32(const uint8_t* p, size_t n, uint32_t crc) {
#if defined(__x86_64__)
    if (n >= 64 && have_clmul()) {
        const size_t m = n & ~(size_t)15;
        const uint32_t c = crc32_fold(p, m, ~crc);
        return crc32_table(p + m, n - m, ~c);
    }
#endif
    return crc32_table(p, n, crc);
}

// ------------------------------------------------------------------ little-endian helpers

namespace {

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
uint64_t rd64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}
void wr32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }

bool fail(std::string* err, const std::string& m) {
    if (err) *err = m;
    return false;
}

// [off, off + len) lies inside a buffer of `size` bytes (no overflow for any 64-bit inputs).
bool in_bounds(uint64_t off, uint64_t len, uint64_t size) { return off <= size && len <= size - off; }

// Largest decompressed code record accepted (libtorch's code/ records are a few KiB to a few MiB).
constexpr uint64_t kMaxCodeRecord = 64ull << 20;
// Nesting of modules the walk follows (a pickle can make an object its own child through the memo).
constexpr int kMaxModuleDepth = 256;

// ------------------------------------------------------------------ pickle objects

struct PObj;
using P = std::shared_ptr<PObj>;

struct PObj {
    enum Kind { None, Bool, Int, Float, Str, Tuple, List, Dict, Global, Object, Storage, Tensor, Mark } kind = None;
    int64_t i = 0;
    double f = 0;
    std::string s;                          // Str; Global "module name"; Storage: key
    std::string s2;                         // Storage: storage type name
    std::vector<P> items;                   // Tuple / List
    std::vector<std::pair<P, P>> dict;      // Dict (insertion order)
    P cls, state;                           // Object
    // Tensor
    P storage;
    int64_t offset = 0;
    std::vector<int64_t> sizes, strides;
};

P make(PObj::Kind k) {
    auto p = std::make_shared<PObj>();
    p->kind = k;
    return p;
}

// Runs data.pkl; returns the root object.
P unpickle(const uint8_t* p, size_t n, std::string* err) {
    std::vector<P> stack;
    std::vector<size_t> marks;
    std::unordered_map<uint32_t, P> memo;
    size_t i = 0;
    auto need = [&](size_t k) { return i + k <= n; };
    auto pop = [&]() -> P {
        if (stack.empty()) return nullptr;
        P v = stack.back();
        stack.pop_back();
        return v;
    };
    auto pop_mark = [&](std::vector<P>* out) -> bool {
        if (marks.empty()) return false;
        size_t m = marks.back();
        marks.pop_back();
        if (m > stack.size()) return false;
        out->assign(stack.begin() + (long)m, stack.end());
        stack.resize(m);
        return true;
    };
    while (i < n) {
        const uint8_t op = p[i++];
        switch (op) {
            case 0x80:  // PROTO
                if (!need(1)) return fail(err, "pickle: truncated PROTO"), nullptr;
                ++i;
                break;
            case 0x95:  // FRAME
                if (!need(8)) return fail(err, "pickle: truncated FRAME"), nullptr;
                i += 8;
                break;
            case 'c': {  // GLOBAL "module\nname\n"
                const uint8_t* e1 = (const uint8_t*)memchr(p + i, '\n', n - i);
                if (!e1) return fail(err, "pickle: bad GLOBAL"), nullptr;
                const uint8_t* e2 = (const uint8_t*)memchr(e1 + 1, '\n', n - (size_t)(e1 + 1 - p));
                if (!e2) return fail(err, "pickle: bad GLOBAL"), nullptr;
                P g = make(PObj::Global);
                g->s = std::string((const char*)p + i, e1 - (p + i)) + " " + std::string((const char*)e1 + 1, e2 - e1 - 1);
                i = (size_t)(e2 + 1 - p);
                stack.push_back(g);
                break;
            }
            case 'q':  // BINPUT
                if (!need(1) || stack.empty()) return fail(err, "pickle: bad BINPUT"), nullptr;
                memo[p[i++]] = stack.back();
                break;
            case 'r':  // LONG_BINPUT
                if (!need(4) || stack.empty()) return fail(err, "pickle: bad LONG_BINPUT"), nullptr;
                memo[rd32(p + i)] = stack.back();
                i += 4;
                break;
            case 0x94:  // MEMOIZE
                if (stack.empty()) return fail(err, "pickle: bad MEMOIZE"), nullptr;
                memo[(uint32_t)memo.size()] = stack.back();
                break;
            case 'h': {  // BINGET
                if (!need(1)) return fail(err, "pickle: bad BINGET"), nullptr;
                auto it = memo.find(p[i++]);
                if (it == memo.end()) return fail(err, "pickle: BINGET of unknown memo"), nullptr;
                stack.push_back(it->second);
                break;
            }
            case 'j': {  // LONG_BINGET
                if (!need(4)) return fail(err, "pickle: bad LONG_BINGET"), nullptr;
                auto it = memo.find(rd32(p + i));
                i += 4;
                if (it == memo.end()) return fail(err, "pickle: LONG_BINGET of unknown memo"), nullptr;
                stack.push_back(it->second);
                break;
            }
            case '(':
                marks.push_back(stack.size());
                break;
            case ')':
                stack.push_back(make(PObj::Tuple));
                break;
            case ']':
                stack.push_back(make(PObj::List));
                break;
            case '}':
                stack.push_back(make(PObj::Dict));
                break;
            case 'N':
                stack.push_back(make(PObj::None));
                break;
            case 0x88:
            case 0x89: {
                P b = make(PObj::Bool);
                b->i = op == 0x88;
                stack.push_back(b);
                break;
            }
            case 'K':
            case 'M':
            case 'J': {
                const size_t w = op == 'K' ? 1 : op == 'M' ? 2 : 4;
                if (!need(w)) return fail(err, "pickle: truncated int"), nullptr;
                P v = make(PObj::Int);
                v->i = op == 'K' ? p[i] : op == 'M' ? rd16(p + i) : (int32_t)rd32(p + i);
                i += w;
                stack.push_back(v);
                break;
            }
            case 0x8a: {  // LONG1
                if (!need(1)) return fail(err, "pickle: truncated LONG1"), nullptr;
                const size_t w = p[i++];
                if (!need(w) || w > 8) return fail(err, "pickle: unsupported LONG1"), nullptr;
                uint64_t u = 0;
                for (size_t k = 0; k < w; ++k) u |= (uint64_t)p[i + k] << (8 * k);
                if (w && w < 8 && (p[i + w - 1] & 0x80)) u |= ~0ull << (8 * w);  // sign-extend
                i += w;
                P v = make(PObj::Int);
                v->i = (int64_t)u;
                stack.push_back(v);
                break;
            }
            case 'G': {  // BINFLOAT (big-endian double)
                if (!need(8)) return fail(err, "pickle: truncated BINFLOAT"), nullptr;
                uint64_t u = 0;
                for (int k = 0; k < 8; ++k) u = (u << 8) | p[i + k];
                i += 8;
                P v = make(PObj::Float);
                std::memcpy(&v->f, &u, 8);
                stack.push_back(v);
                break;
            }
            case 'X':
            case 0x8c:
            case 'U':
            case 'T': {  // BINUNICODE / SHORT_BINUNICODE / SHORT_BINSTRING / BINSTRING
                const bool shortlen = op == 0x8c || op == 'U';
                if (!need(shortlen ? 1 : 4)) return fail(err, "pickle: truncated string"), nullptr;
                const size_t len = shortlen ? p[i] : rd32(p + i);
                i += shortlen ? 1 : 4;
                if (!need(len)) return fail(err, "pickle: truncated string"), nullptr;
                P v = make(PObj::Str);
                v->s.assign((const char*)p + i, len);
                i += len;
                stack.push_back(v);
                break;
            }
            case 't': {
                P t = make(PObj::Tuple);
                if (!pop_mark(&t->items)) return fail(err, "pickle: TUPLE without MARK"), nullptr;
                stack.push_back(t);
                break;
            }
            case 0x85:
            case 0x86:
            case 0x87: {
                const size_t k = op - 0x84;
                if (stack.size() < k) return fail(err, "pickle: short TUPLEn"), nullptr;
                P t = make(PObj::Tuple);
                t->items.assign(stack.end() - (long)k, stack.end());
                stack.resize(stack.size() - k);
                stack.push_back(t);
                break;
            }
            case 'a': {  // APPEND
                P v = pop();
                if (!v || stack.empty() || stack.back()->kind != PObj::List) return fail(err, "pickle: bad APPEND"), nullptr;
                stack.back()->items.push_back(v);
                break;
            }
            case 'e': {  // APPENDS
                std::vector<P> xs;
                if (!pop_mark(&xs) || stack.empty()) return fail(err, "pickle: bad APPENDS"), nullptr;
                for (auto& x : xs) stack.back()->items.push_back(x);
                break;
            }
            case 's': {  // SETITEM
                P v = pop(), k = pop();
                if (!v || !k || stack.empty() || stack.back()->kind != PObj::Dict) return fail(err, "pickle: bad SETITEM"), nullptr;
                stack.back()->dict.emplace_back(k, v);
                break;
            }
            case 'u': {  // SETITEMS
                std::vector<P> kv;
                if (!pop_mark(&kv) || (kv.size() & 1) || stack.empty() || stack.back()->kind != PObj::Dict)
                    return fail(err, "pickle: bad SETITEMS"), nullptr;
                for (size_t k = 0; k < kv.size(); k += 2) stack.back()->dict.emplace_back(kv[k], kv[k + 1]);
                break;
            }
            case 'Q': {  // BINPERSID: ('storage', <StorageType global>, key, location, numel)
                P pid = pop();
                if (!pid || pid->kind != PObj::Tuple || pid->items.size() < 3 || pid->items[2]->kind != PObj::Str ||
                    pid->items[1]->kind != PObj::Global)
                    return fail(err, "pickle: unsupported persistent id"), nullptr;
                P st = make(PObj::Storage);
                st->s = pid->items[2]->s;
                const std::string& g = pid->items[1]->s;  // "torch FloatStorage"
                st->s2 = g.substr(g.find(' ') + 1);
                stack.push_back(st);
                break;
            }
            case 0x81: {  // NEWOBJ
                P args = pop(), cls = pop();
                if (!cls) return fail(err, "pickle: bad NEWOBJ"), nullptr;
                P o = make(PObj::Object);
                o->cls = cls;
                stack.push_back(o);
                break;
            }
            case 'R': {  // REDUCE
                P args = pop(), fn = pop();
                if (!fn || !args || args->kind != PObj::Tuple) return fail(err, "pickle: bad REDUCE"), nullptr;
                if (fn->kind == PObj::Global && fn->s == "torch._utils _rebuild_tensor_v2") {
                    // (storage, storage_offset, size tuple, stride tuple, ...): every index non-negative
                    if (args->items.size() < 4 || args->items[0]->kind != PObj::Storage ||
                        args->items[1]->kind != PObj::Int || args->items[2]->kind != PObj::Tuple ||
                        args->items[3]->kind != PObj::Tuple ||
                        args->items[2]->items.size() != args->items[3]->items.size() || args->items[1]->i < 0)
                        return fail(err, "pickle: bad _rebuild_tensor_v2"), nullptr;
                    P t = make(PObj::Tensor);
                    t->storage = args->items[0];
                    t->offset = args->items[1]->i;
                    for (auto& x : args->items[2]->items) {
                        if (x->kind != PObj::Int || x->i < 0) return fail(err, "pickle: bad tensor size"), nullptr;
                        t->sizes.push_back(x->i);
                    }
                    for (auto& x : args->items[3]->items) {
                        if (x->kind != PObj::Int || x->i < 0) return fail(err, "pickle: bad tensor stride"), nullptr;
                        t->strides.push_back(x->i);
                    }
                    stack.push_back(t);
                } else if (fn->kind == PObj::Global && fn->s == "collections OrderedDict") {
                    stack.push_back(make(PObj::Dict));
                } else {
                    P o = make(PObj::Object);
                    o->cls = fn;
                    o->state = args;
                    stack.push_back(o);
                }
                break;
            }
            case 'b': {  // BUILD
                P st = pop();
                if (!st || stack.empty()) return fail(err, "pickle: bad BUILD"), nullptr;
                if (stack.back()->kind == PObj::Object) stack.back()->state = st;
                break;
            }
            case '.':
                if (stack.empty()) return fail(err, "pickle: empty at STOP"), nullptr;
                return stack.back();
            default: {
                char b[64];
                snprintf(b, sizeof b, "pickle: unsupported opcode 0x%02x at %zu", op, i - 1);
                fail(err, b);
                return nullptr;
            }
        }
    }
    fail(err, "pickle: no STOP");
    return nullptr;
}

size_t storage_elem_size(const std::string& t) {
    static const std::map<std::string, size_t> m = {
        {"FloatStorage", 4}, {"DoubleStorage", 8}, {"HalfStorage", 2}, {"BFloat16Storage", 2},
        {"LongStorage", 8},  {"IntStorage", 4},    {"ShortStorage", 2}, {"CharStorage", 1},
        {"ByteStorage", 1},  {"BoolStorage", 1}};
    auto it = m.find(t);
    return it == m.end() ? 0 : it->second;
}

// "__parameters__ = ["weight", "bias", ]" inside `class <name>(...)` of a code file.
std::vector<std::string> class_parameters(const std::string& code, const std::string& cls) {
    std::vector<std::string> out;
    size_t c = code.find("class " + cls + "(");
    if (c == std::string::npos) return out;
    size_t end = code.find("\nclass ", c + 1);
    size_t a = code.find("__parameters__ = [", c);
    if (a == std::string::npos || (end != std::string::npos && a > end)) return out;
    size_t b = code.find(']', a);
    std::string lst = code.substr(a, b - a);
    for (size_t q = lst.find('"'); q != std::string::npos; q = lst.find('"', q + 1)) {
        size_t r = lst.find('"', q + 1);
        if (r == std::string::npos) break;
        out.push_back(lst.substr(q + 1, r - q - 1));
        q = r;
    }
    return out;
}

}  // namespace

// ------------------------------------------------------------------ layout cache
//
// Every receipt of a bucket is the same module saved again: the same records at the same offsets, the same
// data.pkl and code records -- only the tensor records' bytes (and their CRCs, and the random
// .data/serialization_id) differ.  The module walk (unpickling data.pkl, inflating the code records) cost
// 20-180 us per receipt on the host (LeNet-5 part 1: 52 us, ResNet-18 part 1: 179 us, in this container),
// once per receipt on the aggregator's one consumer thread.  So the parse keys its result by everything it
// depends on -- the archive size, every record's name, method, sizes and data offsets, and the bytes of
// data.pkl and of the code records -- and a later archive with the same key takes the cached tensor views,
// rebased onto its own bytes.  The key is compared in full (its hash only picks the slot), so a hit is
// exactly what the walk would have produced.

namespace {
struct CachedLayout {
    std::string key;
    std::vector<TensorView> params, buffers;  // data = offset from the archive's first byte
};
constexpr size_t kLayoutSlots = 64, kMaxKeyBytes = 4u << 20;
std::mutex g_layout_mu;
std::vector<CachedLayout> g_layouts(kLayoutSlots);
unsigned long long g_layout_hits = 0;

void rebase(std::vector<TensorView>* out, const std::vector<TensorView>& in, const uint8_t* base, bool to_offsets) {
    *out = in;
    for (auto& t : *out)
        t.data = to_offsets ? reinterpret_cast<const uint8_t*>(t.data - base) : base + reinterpret_cast<uintptr_t>(t.data);
}
}  // namespace

unsigned long long TorchArchive::layout_cache_hits() {
    std::lock_guard<std::mutex> g(g_layout_mu);
    return g_layout_hits;
}

// ------------------------------------------------------------------ TorchArchive

bool TorchArchive::parse(const uint8_t* bytes, size_t size, std::string* err) {
    base_ = bytes;
    size_ = size;
    entries_.clear();
    params_.clear();
    buffers_.clear();
    if (size < 22) return fail(err, "archive too small");
    // end of central directory (+ zip64 records when present)
    size_t eocd = std::string::npos;
    for (size_t i = size - 22 + 1; i-- > 0 && size - i <= 22 + 65535;)
        if (rd32(bytes + i) == 0x06054b50) {
            eocd = i;
            break;
        }
    if (eocd == std::string::npos) return fail(err, "zip: no end-of-central-directory record");
    uint64_t n_entries = rd16(bytes + eocd + 10), cd_off = rd32(bytes + eocd + 16);
    if (eocd >= 20 && rd32(bytes + eocd - 20) == 0x07064b50) {  // zip64 locator
        const uint64_t z64 = rd64(bytes + eocd - 20 + 8);
        if (!in_bounds(z64, 56, size) || rd32(bytes + z64) != 0x06064b50) return fail(err, "zip: bad zip64 record");
        n_entries = rd64(bytes + z64 + 32);
        cd_off = rd64(bytes + z64 + 48);
    }
    uint64_t q = cd_off;
    for (uint64_t e = 0; e < n_entries; ++e) {
        if (!in_bounds(q, 46, size) || rd32(bytes + q) != 0x02014b50) return fail(err, "zip: bad central directory");
        const uint16_t method = rd16(bytes + q + 10), nlen = rd16(bytes + q + 28), xlen = rd16(bytes + q + 30),
                       clen = rd16(bytes + q + 32);
        if (!in_bounds(q, 46ull + nlen + xlen + clen, size)) return fail(err, "zip: central directory entry out of bounds");
        ZipEntry z;
        z.crc = rd32(bytes + q + 16);
        uint64_t csize = rd32(bytes + q + 20), usize = rd32(bytes + q + 24), loff = rd32(bytes + q + 42);
        z.name.assign((const char*)bytes + q + 46, nlen);
        // zip64 extended information: only the fields that are 0xFFFFFFFF are present, in this order
        const uint64_t xend = q + 46 + nlen + xlen;
        for (uint64_t x = q + 46 + nlen; x + 4 <= xend;) {
            const uint16_t id = rd16(bytes + x), len = rd16(bytes + x + 2);
            if (x + 4 + len > xend) return fail(err, "zip: extra field of " + z.name + " out of bounds");
            if (id == 0x0001) {
                uint64_t f = x + 4;
                const uint64_t fend = f + len;
                for (uint64_t* v : {&usize, &csize, &loff}) {
                    if (*v != 0xFFFFFFFFu) continue;
                    if (f + 8 > fend) return fail(err, "zip: short zip64 field in " + z.name);
                    *v = rd64(bytes + f);
                    f += 8;
                }
            }
            x += 4 + len;
        }
        if (method != 0 && method != 8) return fail(err, "zip: record " + z.name + " uses an unsupported method");
        if (method == 0 && csize != usize) return fail(err, "zip: stored record " + z.name + " has mismatched sizes");
        z.method = method;
        z.comp_size = csize;
        if (!in_bounds(loff, 30, size) || rd32(bytes + loff) != 0x04034b50) return fail(err, "zip: bad local header");
        const uint16_t lflags = rd16(bytes + loff + 6);
        z.data_offset = loff + 30 + rd16(bytes + loff + 26) + rd16(bytes + loff + 28);
        z.size = usize;
        z.cd_offset = q;
        z.local_offset = loff;
        if (!in_bounds(z.data_offset, z.comp_size, size)) return fail(err, "zip: record " + z.name + " out of bounds");
        if (lflags & 0x08) {  // data descriptor follows the data, optionally with its signature
            uint64_t d = z.data_offset + z.comp_size;
            if (in_bounds(d, 4, size) && rd32(bytes + d) == 0x08074b50) d += 4;
            if (!in_bounds(d, 4, size)) return fail(err, "zip: data descriptor of " + z.name + " out of bounds");
            z.desc_offset = d;
        }
        entries_.push_back(z);
        q += 46 + nlen + xlen + clen;
    }
    if (entries_.empty()) return fail(err, "zip: empty archive");
    prefix_ = entries_[0].name.substr(0, entries_[0].name.find('/'));
    // the layout key (see "layout cache"): the structure, then data.pkl and the code records' bytes
    std::string key;
    auto put = [&key](uint64_t v) { key.append(reinterpret_cast<const char*>(&v), 8); };
    put(size);
    put(entries_.size());
    const std::string pkl_name = prefix_ + "/data.pkl", code_dir = prefix_ + "/code/";
    for (auto& z : entries_) {
        put(z.name.size());
        key += z.name;
        put(z.method);
        put(z.comp_size);
        put(z.size);
        put(z.data_offset);
        put(z.desc_offset);
    }
    for (auto& z : entries_)
        if ((z.name == pkl_name || z.name.compare(0, code_dir.size(), code_dir) == 0) && key.size() <= kMaxKeyBytes)
            key.append(reinterpret_cast<const char*>(bytes + z.data_offset), (size_t)z.comp_size);
    const bool cacheable = key.size() <= kMaxKeyBytes;
    const size_t slot = cacheable ? crc32(reinterpret_cast<const uint8_t*>(key.data()), key.size()) % kLayoutSlots : 0;
    if (cacheable) {
        std::lock_guard<std::mutex> g(g_layout_mu);
        CachedLayout& c = g_layouts[slot];
        if (c.key == key) {
            rebase(&params_, c.params, bytes, false);
            rebase(&buffers_, c.buffers, bytes, false);
            ++g_layout_hits;
            return true;
        }
    }
    std::map<std::string, int> by_name;
    for (size_t k = 0; k < entries_.size(); ++k) by_name[entries_[k].name] = (int)k;
    auto rec = [&](const std::string& n) -> const ZipEntry* {
        auto it = by_name.find(prefix_ + "/" + n);
        return it == by_name.end() ? nullptr : &entries_[it->second];
    };
    const ZipEntry* pkl = rec("data.pkl");
    if (!pkl) return fail(err, "archive: no data.pkl");
    if (pkl->method != 0) return fail(err, "archive: data.pkl is compressed");
    std::string perr;
    P root = unpickle(bytes + pkl->data_offset, pkl->size, &perr);
    if (!root) return fail(err, perr);

    // Walk the module tree: own attributes in registration order (parameters, buffers), then children
    // -- exactly named_parameters(recurse=true) / named_buffers(recurse=true).
    std::string werr;
    std::map<std::string, std::string> code_cache;
    std::function<bool(const P&, const std::string&, std::vector<TensorView>*, bool, int)> walk;
    auto code_for = [&](const std::string& global) -> std::pair<std::string, std::string> {
        // "__torch__.___torch_mangle_0 Module" -> (code/__torch__/___torch_mangle_0.py, "Module")
        const size_t sp = global.find(' ');
        std::string mod = global.substr(0, sp), cls = global.substr(sp + 1), path = "code/";
        for (char ch : mod) path += ch == '.' ? '/' : ch;
        path += ".py";
        auto it = code_cache.find(path);
        if (it == code_cache.end()) {
            const ZipEntry* z = rec(path);
            std::string text;
            if (z && z->method == 0) {
                text.assign((const char*)bytes + z->data_offset, z->size);
            } else if (z && z->size <= kMaxCodeRecord && z->size / 1032 <= z->comp_size) {
                // raw deflate (libtorch compresses some code records); deflate expands at most ~1032:1
                text.resize(z->size);
                z_stream zs{};
                if (inflateInit2(&zs, -MAX_WBITS) == Z_OK) {
                    zs.next_in = const_cast<Bytef*>(bytes + z->data_offset);
                    zs.avail_in = (uInt)z->comp_size;
                    zs.next_out = (Bytef*)&text[0];
                    zs.avail_out = (uInt)z->size;
                    const int rc = inflate(&zs, Z_FINISH);
                    inflateEnd(&zs);
                    if (rc != Z_STREAM_END) text.clear();
                } else {
                    text.clear();
                }
            }
            it = code_cache.emplace(path, text).first;
        }
        return {it->second, cls};
    };
    walk = [&](const P& obj, const std::string& prefix, std::vector<TensorView>* out, bool want_params,
               int depth) -> bool {
        if (!obj || obj->kind != PObj::Object || !obj->state || obj->state->kind != PObj::Dict) return true;
        if (depth > kMaxModuleDepth) return fail(&werr, "archive: module tree deeper than 256 (a cycle?)");
        auto code = code_for(obj->cls ? obj->cls->s : std::string());
        const std::vector<std::string> pnames = class_parameters(code.first, code.second);
        std::vector<std::pair<P, std::string>> children;
        for (auto& kv : obj->state->dict) {
            if (!kv.first || kv.first->kind != PObj::Str) continue;
            const std::string& key = kv.first->s;
            const P& v = kv.second;
            if (v->kind == PObj::Tensor) {
                const bool is_param = std::find(pnames.begin(), pnames.end(), key) != pnames.end();
                if (is_param != want_params) continue;
                TensorView tv;
                tv.name = prefix + key;
                tv.storage_type = v->storage->s2;
                tv.elem_size = storage_elem_size(tv.storage_type);
                if (!tv.elem_size) return fail(&werr, "archive: unknown storage " + tv.storage_type);
                tv.sizes = v->sizes;
                tv.strides = v->strides;
                tv.storage_offset = v->offset;
                // sizes, strides and the offset are non-negative (unpickle); the element count and the
                // last index are computed in 128 bits and must fit the storage record
                __int128 numel = 1, max_index = tv.storage_offset;
                for (size_t d = 0; d < tv.sizes.size(); ++d) {
                    numel *= tv.sizes[d];
                    if (numel > ((__int128)1 << 50)) return fail(&werr, "archive: tensor " + tv.name + " too large");
                }
                tv.numel = (int64_t)numel;
                for (size_t d = 0; d < tv.sizes.size(); ++d)
                    if (tv.sizes[d] > 0) max_index += (__int128)(tv.sizes[d] - 1) * tv.strides[d];
                int64_t expect = 1;
                tv.contiguous = true;
                for (size_t d = tv.sizes.size(); d-- > 0;) {
                    if (tv.sizes[d] != 1 && tv.strides[d] != expect) tv.contiguous = false;
                    expect *= tv.sizes[d];
                }
                auto it = by_name.find(prefix_ + "/data/" + v->storage->s);
                if (it == by_name.end()) return fail(&werr, "archive: missing storage record " + v->storage->s);
                tv.record = it->second;
                const ZipEntry& z = entries_[tv.record];
                if (z.method != 0) return fail(&werr, "archive: tensor record " + z.name + " is compressed");
                if (tv.numel > 0 && (max_index + 1) * (__int128)tv.elem_size > (__int128)z.size)
                    return fail(&werr, "archive: tensor " + tv.name + " exceeds its storage");
                if (tv.numel == 0 && (__int128)tv.storage_offset * tv.elem_size > (__int128)z.size)
                    return fail(&werr, "archive: tensor " + tv.name + " starts past its storage");
                tv.data = bytes + z.data_offset + (uint64_t)tv.storage_offset * tv.elem_size;
                out->push_back(tv);
            } else if (v->kind == PObj::Object) {
                children.emplace_back(v, prefix + key + ".");
            }
        }
        for (auto& c : children)
            if (!walk(c.first, c.second, out, want_params, depth + 1)) return false;
        return true;
    };
    if (!walk(root, "", &params_, true, 0) || !walk(root, "", &buffers_, false, 0)) return fail(err, werr);
    if (cacheable) {
        CachedLayout c;
        c.key = std::move(key);
        rebase(&c.params, params_, bytes, true);
        rebase(&c.buffers, buffers_, bytes, true);
        std::lock_guard<std::mutex> g(g_layout_mu);
        g_layouts[slot] = std::move(c);
    }
    return true;
}

int64_t TorchArchive::param_numel() const {
    int64_t n = 0;
    for (auto& t : params_) n += t.numel;
    return n;
}

bool TorchArchive::params_are_float() const {
    for (auto& t : params_)
        if (t.storage_type != "FloatStorage") return false;
    return true;
}

int TorchArchive::param_elem_size() const {
    if (params_.empty()) return 4;
    const std::string& st = params_[0].storage_type;
    if (st != "FloatStorage" && st != "BFloat16Storage") return 0;
    for (auto& t : params_)
        if (t.storage_type != st) return 0;
    return st == "FloatStorage" ? 4 : 2;
}

bool TorchArchive::param_segments(std::vector<const void*>* ptrs, std::vector<size_t>* bytes) const {
    ptrs->clear();
    bytes->clear();
    const int es = param_elem_size();
    if (!es) return false;
    for (auto& t : params_) {
        if (!t.contiguous) return false;
        if (t.numel == 0) continue;
        ptrs->push_back(t.data);
        bytes->push_back((size_t)t.numel * (size_t)es);
    }
    return true;
}

// Element-size-agnostic walk of one (possibly strided) parameter in row-major index order:
// fn(e, off) for element e at element offset `off` from the parameter's first element.
template <class Fn>
static void walk_param(const TensorView& t, Fn fn) {
    std::vector<int64_t> idx(t.sizes.size(), 0);
    for (int64_t e = 0; e < t.numel; ++e) {
        int64_t off = 0;
        for (size_t d = 0; d < idx.size(); ++d) off += idx[d] * t.strides[d];
        fn(e, off);
        for (size_t d = idx.size(); d-- > 0;) {
            if (++idx[d] < t.sizes[d]) break;
            idx[d] = 0;
        }
    }
}

bool TorchArchive::gather_param_bytes(uint8_t* dst, std::string* err) const {
    const int es = param_elem_size();
    if (!es) return fail(err, "parameters are not all fp32 or all bf16");
    for (auto& t : params_) {
        if (t.contiguous) {
            std::memcpy(dst, t.data, (size_t)t.numel * (size_t)es);
        } else {
            walk_param(t, [&](int64_t e, int64_t off) { std::memcpy(dst + e * es, t.data + off * es, (size_t)es); });
        }
        dst += (size_t)t.numel * (size_t)es;
    }
    return true;
}

bool TorchArchive::gather_params(float* dst, std::string* err) const {
    if (param_elem_size() != 4) return fail(err, "parameters are not all fp32");
    return gather_param_bytes(reinterpret_cast<uint8_t*>(dst), err);
}

bool TorchArchive::with_params(const float* src, std::string* out, std::string* err) const {
    out->resize(size_);
    return with_params_into(src, (uint8_t*)&(*out)[0], err);
}

namespace {
// Worker threads for the archive's bulk passes (copies, CRC seals), started once and kept: a reply is
// sealed every phase, and starting 15 threads per call cost ~0.5-1 ms of the phase end (C2, r06s04: the
// reply framing took 1.25 ms for 37.7 MB).  One job at a time; the caller runs part 0 itself.  Never
// destroyed (the threads are detached and idle at exit).
class ArchivePool {
public:
    static ArchivePool& get() {
        static ArchivePool* pool = new ArchivePool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        return *pool;
    }
    unsigned size() const { return n_; }
    // fn(i) for i in [0, size()), on the workers and the caller; returns when all have run
    void run(const std::function<void(unsigned)>& fn) {
        std::lock_guard<std::mutex> one(job_mu_);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    explicit ArchivePool(unsigned n) : n_(n) {
        for (unsigned i = 1; i < n_; ++i) std::thread([this, i] { loop(i); }).detach();
    }
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* job;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
                job = job_;
            }
            (*job)(id);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    unsigned n_;
    std::mutex job_mu_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    uint64_t gen_ = 0;
    unsigned pending_ = 0;
};

// Runs fn(lo, hi) over [0, n) split across the pool's threads (inline below `grain` per part).
void parallel_ranges(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
    ArchivePool& pool = ArchivePool::get();
    const size_t parts = std::min<size_t>(pool.size(), std::max<size_t>(1, n / grain));
    if (parts <= 1) {
        fn(0, n);
        return;
    }
    const size_t per = (n + parts - 1) / parts;
    pool.run([&](unsigned p) {
        if (p >= parts) return;
        const size_t lo = std::min(n, p * per), hi = std::min(n, lo + per);
        if (hi > lo) fn(lo, hi);
    });
}
}  // namespace

bool TorchArchive::with_params_into(const float* src, uint8_t* o, std::string* err) const {
    if (param_elem_size() != 4) return fail(err, "parameters are not all fp32");
    return with_param_bytes_into(reinterpret_cast<const uint8_t*>(src), o, err);
}

bool TorchArchive::with_param_bytes_into(const uint8_t* src, uint8_t* o, std::string* err) const {
    const int es = param_elem_size();
    if (!es) return fail(err, "parameters are not all fp32 or all bf16");
    std::vector<void*> dsts;
    std::vector<size_t> bytes;
    if (layout_into(o, &dsts, &bytes, nullptr)) {  // contiguous parameters: copy the gaps, then the values
        for (size_t k = 0; k < dsts.size(); ++k) {
            uint8_t* d = (uint8_t*)dsts[k];
            const uint8_t* s0 = src;
            parallel_ranges(bytes[k], 16u << 20, [&](size_t lo, size_t hi) { std::memcpy(d + lo, s0 + lo, hi - lo); });
            src += bytes[k];
        }
        seal_params(o);
        return true;
    }
    parallel_ranges(size_, 16u << 20, [&](size_t lo, size_t hi) { std::memcpy(o + lo, base_ + lo, hi - lo); });
    for (auto& t : params_) {
        uint8_t* d = o + (t.data - base_);
        walk_param(t, [&](int64_t e, int64_t off) { std::memcpy(d + off * es, src + e * es, (size_t)es); });
        src += (size_t)t.numel * (size_t)es;
    }
    seal_params(o);
    return true;
}

bool TorchArchive::layout_into(uint8_t* o, std::vector<void*>* dsts, std::vector<size_t>* bytes,
                               std::string* err) const {
    std::vector<std::pair<size_t, size_t>> holes;  // [lo, hi) of each parameter's values
    const int es = param_elem_size();
    if (!es) return fail(err, "parameters are not all fp32 or all bf16");
    for (auto& t : params_) {
        if (!t.contiguous) return fail(err, "parameter " + t.name + " is strided");
        holes.push_back({(size_t)(t.data - base_), (size_t)(t.data - base_) + (size_t)t.numel * (size_t)es});
    }
    std::vector<std::pair<size_t, size_t>> sorted = holes;
    std::sort(sorted.begin(), sorted.end());
    for (size_t k = 1; k < sorted.size(); ++k)
        if (sorted[k].first < sorted[k - 1].second) return fail(err, "parameters share storage bytes");
    size_t at = 0;  // everything outside the holes comes from the template
    for (auto& h : sorted) {
        if (h.first > at) std::memcpy(o + at, base_ + at, h.first - at);
        at = std::max(at, h.second);
    }
    if (size_ > at) std::memcpy(o + at, base_ + at, size_ - at);
    dsts->clear();
    bytes->clear();
    for (auto& h : holes) {
        dsts->push_back(o + h.first);
        bytes->push_back(h.second - h.first);
    }
    return true;
}

bool TorchArchive::seal_params_with(uint8_t* o, const uint32_t* crcs) const {
    const int es = param_elem_size();
    if (!es) return false;
    std::vector<char> seen(entries_.size(), 0);
    for (auto& t : params_) {  // one parameter per record, covering all of it
        if (t.record < 0 || seen[t.record]) return false;
        seen[t.record] = 1;
        const ZipEntry& z = entries_[(size_t)t.record];
        if (t.data != base_ + z.data_offset || (uint64_t)t.numel * (uint64_t)es != z.size) return false;
    }
    for (size_t i = 0; i < params_.size(); ++i) {
        const ZipEntry& z = entries_[(size_t)params_[i].record];
        wr32(o + z.cd_offset + 16, crcs[i]);
        if (z.desc_offset) wr32(o + z.desc_offset, crcs[i]);
        else wr32(o + z.local_offset + 14, crcs[i]);
    }
    return true;
}

void TorchArchive::seal_params(uint8_t* o) const {
    // Every parameter record's CRC-32, all records' chunks in one parallel pass: a reply's records are
    // mostly a few MB each (ResNet-18's part 2: 37.7 MB in 2.4-9.4 MB records), so sealing them one after
    // another, each below the parallel threshold, put ~2.6 ms of one core on the end of every C2 phase.
    constexpr size_t kGrain = 1u << 20;
    struct Task {
        int rec;
        size_t lo, len;
    };
    std::vector<char> touched(entries_.size(), 0);
    for (auto& t : params_) touched[t.record] = 1;
    std::vector<Task> tasks;
    size_t total = 0;
    for (size_t k = 0; k < entries_.size(); ++k) {
        if (!touched[k]) continue;
        const uint64_t n = entries_[k].size;
        total += n;
        for (uint64_t lo = 0; lo < n || (n == 0 && lo == 0); lo += kGrain) {
            tasks.push_back(Task{(int)k, (size_t)lo, (size_t)std::min<uint64_t>(kGrain, n - lo)});
            if (n == 0) break;
        }
    }
    std::vector<uint32_t> part(tasks.size());
    auto run = [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) part[i] = crc32(o + entries_[tasks[i].rec].data_offset + tasks[i].lo, tasks[i].len);
    };
    if (total < 4 * kGrain) run(0, tasks.size());  // a small model: no threads
    else parallel_ranges(tasks.size(), 1, run);
    for (size_t i = 0; i < tasks.size();) {  // join each record's chunks in order
        const int k = tasks[i].rec;
        uint32_t c = part[i];
        for (++i; i < tasks.size() && tasks[i].rec == k; ++i)
            c = (uint32_t)crc32_combine(c, part[i], (z_off_t)tasks[i].len);
        const ZipEntry& z = entries_[(size_t)k];
        wr32(o + z.cd_offset + 16, c);
        if (z.desc_offset) wr32(o + z.desc_offset, c);   // flag bit 3: CRC lives in the data descriptor
        else wr32(o + z.local_offset + 14, c);           // otherwise in the local header
    }
}

}  // namespace fahost
