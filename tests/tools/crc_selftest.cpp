// crc_selftest.cpp -- CPU test of the archive CRC-32 (host/archive.cpp): the PCLMULQDQ folding form against the
// slicing-by-8 table and zlib's crc32 on every length 0..2999 at five misalignments with random seeds, and on
// large buffers; prints the three rates (GB/s).  The reply's zip records are sealed with it (seal_params), so
// a wrong CRC would make the reference's torch::load reject every reply.  Exit code 1 on any mismatch.
#include <zlib.h>

#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "archive.h"

int main() {
    std::mt19937_64 g(1);
    std::vector<uint8_t> buf(1 << 22);
    for (auto& b : buf) b = (uint8_t)g();
    int bad = 0, checks = 0;
    for (size_t n = 0; n < 3000; ++n)
        for (size_t off : {0, 1, 3, 7, 13}) {
            const uint32_t seed = (uint32_t)g();
            const uint32_t a = fahost::crc32(buf.data() + off, n, seed);
            const uint32_t b = fahost::crc32_table(buf.data() + off, n, seed);
            const uint32_t z = (uint32_t)::crc32(seed, buf.data() + off, (uInt)n);
            ++checks;
            if (a != b || a != z) ++bad;
        }
    for (size_t n : {64u, 80u, 1000003u, 4194299u}) {
        ++checks;
        if (fahost::crc32(buf.data() + 5, n) != (uint32_t)::crc32(0, buf.data() + 5, (uInt)n)) ++bad;
    }
    auto rate = [&](auto fn) {
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t x = 0;
        for (int r = 0; r < 20; ++r) x += fn();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return (x == 1 ? 0.0 : 0.0) + 20.0 * buf.size() / dt / 1e9;
    };
    const double fast = rate([&] { return fahost::crc32(buf.data(), buf.size()); });
    const double table = rate([&] { return fahost::crc32_table(buf.data(), buf.size()); });
    const double zl = rate([&] { return (uint32_t)::crc32(0, buf.data(), (uInt)buf.size()); });
    std::printf("{\"checks\": %d, \"bad\": %d, \"crc32_GBs\": %.2f, \"table_GBs\": %.2f, \"zlib_GBs\": %.2f}\n", checks,
                bad, fast, table, zl);
    return bad ? 1 : 0;
}
