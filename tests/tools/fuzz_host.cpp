// fuzz_host.cpp -- mutation fuzzer for the host-side parsers that read bytes straight off the network:
// the Message frame header (wire.cpp: split_receipt / decode, the grammar of Message.h:499-569) and the
// torch::save archive reader (archive.cpp: zip + zip64 + pickle + module walk).  Built with ASan+UBSan
// (tests/tools/Makefile, target fuzz_host_asan) and run by tests/test_host_sanitizers.py; any
// out-of-bounds access, overflow or uncaught exception aborts the run.  The reference decodes the same
// bytes with torch::load after ~10 string copies (network_layer.cpp:33-74, 622-668; aggregator.cpp:63-64).
//
//   fuzz_host <iterations per file> <seed> <file>...
//   files: *.bin = a frame as sent (int32 length + text), anything else = a torch::save archive.
// Mutations: truncation, bit flips, random bytes, and 16/32/64-bit fields overwritten with extreme values
// (0, -1, 0x7fffffff, 0xffffffff, 2^63, ...), concentrated on the zip headers (PK signatures), the
// data.pkl record and the frame header text.  Prints one JSON line with the counts.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "archive.h"
#include "wire.h"

using namespace fahost;

namespace {

std::vector<uint8_t> read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct Stats {
    long runs = 0, archives_ok = 0, frames_ok = 0, gathered = 0, relaid = 0;
};

// Everything a receipt's bytes go through in the aggregator (aggregator_main.cpp absorb / reduce).
void exercise_archive(const uint8_t* p, size_t n, Stats* st) {
    TorchArchive ar;
    std::string err;
    if (!ar.parse(p, n, &err)) return;
    ++st->archives_ok;
    std::vector<const void*> ptrs;
    std::vector<size_t> bytes;
    if (ar.param_segments(&ptrs, &bytes)) {
        volatile uint8_t sink = 0;
        for (size_t k = 0; k < ptrs.size(); ++k)  // the DMA source ranges must be readable
            if (bytes[k]) sink ^= ((const uint8_t*)ptrs[k])[0] ^ ((const uint8_t*)ptrs[k])[bytes[k] - 1];
        (void)sink;
    }
    const int64_t numel = ar.param_numel();
    if (numel >= 0 && numel <= (64 << 20)) {
        std::vector<float> flat((size_t)numel);
        if (ar.gather_params(flat.data(), &err)) ++st->gathered;
        std::vector<uint8_t> out(ar.size());
        std::vector<void*> dsts;
        if (ar.layout_into(out.data(), &dsts, &bytes, &err)) {
            for (size_t k = 0; k < dsts.size(); ++k) std::memset(dsts[k], 0x3f, bytes[k]);
            ar.seal_params(out.data());
            ++st->relaid;
        }
        std::string copy;
        (void)ar.with_params(flat.data(), &copy, &err);
    }
}

void exercise_frame(const uint8_t* p, size_t n, Stats* st) {
    if (n < 4) return;
    int32_t len;
    std::memcpy(&len, p, 4);
    if (len <= 0 || (size_t)len > n - 4) return;  // net.cpp read_frame drops these before parsing
    Message m;
    size_t off = 0, blen = 0;
    std::string err;
    if (!split_receipt((const char*)p + 4, (size_t)len, &m, &off, &blen, &err)) return;
    ++st->frames_ok;
    if (m.type == OPERATION && blen > 0 && off + blen <= (size_t)len) exercise_archive(p + 4 + off, blen, st);
    Message full;
    (void)decode(std::string((const char*)p + 4, (size_t)len), &full, &err);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: fuzz_host <iterations> <seed> <file>...\n");
        return 2;
    }
    const long iters = std::atol(argv[1]);
    std::mt19937_64 rng(std::strtoull(argv[2], nullptr, 0));
    Stats st;
    for (int f = 3; f < argc; ++f) {
        const std::string path = argv[f];
        const bool is_frame = path.size() > 4 && path.compare(path.size() - 4, 4, ".bin") == 0;
        const std::vector<uint8_t> orig = read_file(argv[f]);
        if (orig.empty()) continue;
        // hot spots: zip signatures, the data.pkl record, the frame's header text
        std::vector<std::pair<size_t, size_t>> hot;
        for (size_t i = 0; i + 4 <= orig.size(); ++i)
            if (orig[i] == 'P' && orig[i + 1] == 'K' && orig[i + 2] < 9 && orig[i + 3] < 9)
                hot.push_back({i, std::min(orig.size(), i + 64)});
        {
            const size_t a0 = is_frame ? 4 : 0;
            TorchArchive ar;
            std::string err;
            size_t off = 0, blen = 0;
            Message m;
            if (is_frame && split_receipt((const char*)orig.data() + 4, orig.size() - 4, &m, &off, &blen, &err))
                hot.push_back({4, std::min(orig.size(), 4 + off)});
            const size_t base = is_frame ? a0 + off : 0;
            if (ar.parse(orig.data() + base, is_frame ? blen : orig.size(), &err))
                for (auto& z : ar.entries())
                    if (z.name.size() >= 8 && z.name.compare(z.name.size() - 8, 8, "data.pkl") == 0)
                        hot.push_back({base + z.data_offset, base + z.data_offset + z.size});
        }
        std::vector<uint8_t> buf;
        for (long it = 0; it < iters; ++it) {
            buf = orig;
            const int nmut = 1 + (int)(rng() % 4);
            for (int k = 0; k < nmut; ++k) {
                size_t pos;
                if (!hot.empty() && rng() % 4 != 0) {
                    const auto& h = hot[rng() % hot.size()];
                    pos = h.first + (h.second > h.first ? rng() % (h.second - h.first) : 0);
                } else {
                    pos = rng() % buf.size();
                }
                if (pos >= buf.size()) pos = buf.size() - 1;
                switch (rng() % 5) {
                    case 0: buf[pos] ^= (uint8_t)(1u << (rng() % 8)); break;
                    case 1: buf[pos] = (uint8_t)rng(); break;
                    case 2: {
                        static const uint64_t vals[] = {0, ~0ull, 0x7fffffffull, 0xffffffffull, 0x80000000ull,
                                                        1ull << 63, 0x7fffffffffffffffull, 0xfffffffeull, 1, 64};
                        const uint64_t v = vals[rng() % (sizeof vals / sizeof vals[0])];
                        const size_t w = (size_t)1 << (1 + rng() % 3);  // 2, 4 or 8 bytes
                        if (pos + w <= buf.size()) std::memcpy(&buf[pos], &v, w);
                        break;
                    }
                    case 3: buf.resize(std::max<size_t>(1, pos)); break;  // truncation
                    default: {  // a digit run in the header text (lengths, ids)
                        const char d = "0123456789-"[rng() % 11];
                        buf[pos] = (uint8_t)d;
                    }
                }
                if (buf.empty()) buf.push_back(0);
            }
            ++st.runs;
            if (is_frame) {
                if (rng() % 2) {  // keep the length prefix consistent with the (mutated) size
                    const int32_t len = (int32_t)std::min<size_t>(buf.size() - std::min<size_t>(4, buf.size()), 0x7fffffff);
                    if (buf.size() >= 4) std::memcpy(buf.data(), &len, 4);
                }
                exercise_frame(buf.data(), buf.size(), &st);
            } else {
                exercise_archive(buf.data(), buf.size(), &st);
            }
        }
        // the unmodified input parses (the seeds are valid)
        if (is_frame) exercise_frame(orig.data(), orig.size(), &st);
        else exercise_archive(orig.data(), orig.size(), &st);
    }
    std::printf("{\"ok\":true,\"runs\":%ld,\"archives_ok\":%ld,\"frames_ok\":%ld,\"gathered\":%ld,\"relaid\":%ld}\n",
                st.runs, st.archives_ok, st.frames_ok, st.gathered, st.relaid);
    return 0;
}
