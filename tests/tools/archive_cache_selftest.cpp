// archive_cache_selftest.cpp -- CPU test of TorchArchive's layout cache (host/archive.cpp): a second archive
// with the same structure, pickle and code records (another receipt of the same bucket) takes the cached
// tensor views, rebased onto its own bytes, and they equal what a fresh walk gives; an archive whose data.pkl
// or code differs is walked afresh.  Args: archives (torch::save blobs).  Prints one JSON line; exit 1 on
// any failure.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "archive.h"

namespace {

int checks = 0, failed = 0;

void expect(bool c, const std::string& what) {
    ++checks;
    if (!c) {
        ++failed;
        std::fprintf(stderr, "FAILED: %s\n", what.c_str());
    }
}

bool same_views(const std::vector<fahost::TensorView>& a, const uint8_t* ba, const std::vector<fahost::TensorView>& b,
                const uint8_t* bb) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
        const auto &x = a[i], &y = b[i];
        if (x.name != y.name || x.storage_type != y.storage_type || x.sizes != y.sizes || x.strides != y.strides ||
            x.numel != y.numel || x.contiguous != y.contiguous || x.record != y.record ||
            x.data - ba != y.data - bb)
            return false;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        std::ifstream f(argv[i], std::ios::binary);
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string blob = ss.str();
        std::string err;
        fahost::TorchArchive a;
        expect(a.parse((const uint8_t*)blob.data(), blob.size(), &err), std::string(argv[i]) + ": " + err);
        // another receipt: the same archive elsewhere in memory, every parameter value changed
        std::vector<uint8_t> other(blob.begin(), blob.end());
        for (auto& t : a.params())
            for (size_t k = 0; k < (size_t)t.numel * t.elem_size; ++k) other[(t.data - (const uint8_t*)blob.data()) + k] ^= 0x5A;
        const unsigned long long h0 = fahost::TorchArchive::layout_cache_hits();
        fahost::TorchArchive b;
        expect(b.parse(other.data(), other.size(), &err), "second receipt parses");
        expect(fahost::TorchArchive::layout_cache_hits() == h0 + 1, "second receipt hits the layout cache");
        expect(same_views(a.params(), (const uint8_t*)blob.data(), b.params(), other.data()) &&
                   same_views(a.buffers(), (const uint8_t*)blob.data(), b.buffers(), other.data()),
               "cached views equal the walk's, rebased");
        std::vector<uint8_t> moved(blob.size() + 64);
        std::memcpy(moved.data() + 64, blob.data(), blob.size());
        fahost::TorchArchive c;
        expect(c.parse(moved.data() + 64, blob.size(), &err) && !c.params().empty() &&
                   c.params()[0].data == moved.data() + 64 + (a.params()[0].data - (const uint8_t*)blob.data()),
               "a hit points into the new bytes");
        // a changed pickle byte (a different module tree, as far as the cache knows): walked afresh
        std::vector<uint8_t> pk(blob.begin(), blob.end());
        for (auto& z : a.entries())
            if (z.name.size() >= 8 && z.name.compare(z.name.size() - 8, 8, "data.pkl") == 0 && z.size > 8)
                pk[z.data_offset + z.size - 2] ^= 0x01;  // a byte before the STOP opcode
        const unsigned long long h1 = fahost::TorchArchive::layout_cache_hits();
        fahost::TorchArchive d;
        (void)d.parse(pk.data(), pk.size(), &err);  // may parse or fail; it must not come from the cache
        expect(fahost::TorchArchive::layout_cache_hits() == h1, "a changed pickle misses the cache");
    }
    std::printf("{\"checks\": %d, \"failed\": %d, \"hits\": %llu}\n", checks, failed,
                fahost::TorchArchive::layout_cache_hits());
    return failed ? 1 : 0;
}
