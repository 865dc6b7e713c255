// receipts_selftest.cpp -- CPU test of fa_aggregator's receipt ledger (host/receipts.h).
//
// Plays the protocol of data_owner.cpp:224-253 / aggregator.cpp:55-167 with explicit t_start stamps
// (network_layer.cpp:761: the sender stamps its clock when the frame goes out) and checks which receipts
// the ledger calls stale: late copies of earlier rounds before and after the current receipt, copies at
// the floor's own millisecond (decided by content), older copies within a phase, and the receipts that
// must stay current (a frozen part resent with the same bytes in a later round, a retransmission of the
// current receipt).  Prints one JSON line; exit code 1 if any check failed.
#include <cstdio>
#include <string>
#include <vector>

#include "receipts.h"

using fahost::ReceiptLedger;

namespace {

int checks = 0, failed = 0;

void expect(bool cond, const char* what) {
    ++checks;
    if (!cond) {
        ++failed;
        std::fprintf(stderr, "FAILED: %s\n", what);
    }
}

// Content of owner k's receipt of bucket mp in round r (what the fingerprint is taken over).
uint64_t fp_of(int round, int owner, int mp) {
    std::vector<uint8_t> blob(4096 + 13 * mp);
    for (size_t i = 0; i < blob.size(); ++i) blob[i] = (uint8_t)(i * 31 + round * 7 + owner * 3 + mp);
    return fahost::archive_fingerprint(blob.data(), blob.size());
}

}  // namespace

int main() {
    const int D = 4, L = 2;  // owners 0..3, phase 2 = model parts 2..3
    ReceiptLedger led;
    long t = 1000;
    std::vector<std::vector<long>> sent(3, std::vector<long>(D * (L + 2)));  // [round][owner*(L+2)+mp] = t_start
    auto take = [&](int round, int owner, int mp, long ts) {
        const uint64_t fp = fp_of(round, owner, mp);
        const std::string why = led.stale(owner, mp, ts, fp);
        if (why.empty()) led.accept(owner, mp, ts, fp);
        return why;
    };
    for (int round = 0; round < 3; ++round) {
        // phase 1: part 1 from every owner
        for (int k = 0; k < D; ++k) sent[round][k * (L + 2) + 1] = ++t;
        if (round > 0) {  // owner 2's part 1 of the previous round, late, BEFORE its current one
            const std::string why = take(round - 1, 2, 1, sent[round - 1][2 * (L + 2) + 1]);
            expect(!why.empty(), "late copy of last round's part 1 before the current one is stale");
        }
        for (int k = 0; k < D; ++k) expect(take(round, k, 1, sent[round][k * (L + 2) + 1]).empty(), "current part 1");
        if (round > 0) {  // ... and AFTER it: neither counts nor replaces the newer receipt
            expect(!take(round - 1, 2, 1, sent[round - 1][2 * (L + 2) + 1]).empty(),
                   "late copy of last round's part 1 after the current one is stale");
        }
        // a retransmission of this round's own receipt (same stamp, same bytes) is current (it replaces)
        expect(take(round, 3, 1, sent[round][3 * (L + 2) + 1]).empty(), "retransmission of the current receipt");
        led.end_phase();
        // phase 2: the last-part layers, after the phase-1 reply
        t += 5;
        for (int k = 0; k < D; ++k)
            for (int mp = 2; mp <= L + 1; ++mp) sent[round][k * (L + 2) + mp] = ++t;
        if (round > 0)
            expect(!take(round - 1, 1, 3, sent[round - 1][1 * (L + 2) + 3]).empty(),
                   "late copy of last round's phase-2 layer is stale");
        for (int k = 0; k < D; ++k)
            for (int mp = 2; mp <= L + 1; ++mp)
                expect(take(round, k, mp, sent[round][k * (L + 2) + mp]).empty(), "current phase-2 layer");
        led.end_phase();
        t += 5;
    }

    // one millisecond: owner 0's part 1 of the next round stamped in the same ms as its last phase-2 send
    {
        ReceiptLedger l2;
        l2.accept(0, 1, 50, fp_of(0, 0, 1));
        l2.end_phase();
        l2.accept(0, 2, 60, fp_of(0, 0, 2));
        l2.end_phase();
        expect(!l2.stale(0, 1, 60, fp_of(0, 0, 2)).empty(), "a byte copy at the floor's millisecond is stale");
        expect(l2.stale(0, 1, 60, fp_of(1, 0, 1)).empty(), "new content at the floor's millisecond is current");
        expect(!l2.stale(0, 1, 59, fp_of(1, 0, 1)).empty(), "anything sent before the floor is stale");
        // a frozen part: the same bytes as an earlier round, sent later, is current
        expect(l2.stale(0, 1, 70, fp_of(0, 0, 1)).empty(), "same bytes sent after the floor are current");
        // within a phase: an older copy never replaces the newer one; a newer one does
        l2.accept(0, 1, 70, fp_of(1, 0, 1));
        expect(!l2.stale(0, 1, 65, fp_of(9, 0, 1)).empty(), "an older receipt does not replace a newer one");
        expect(l2.stale(0, 1, 71, fp_of(9, 0, 1)).empty(), "a newer receipt replaces");
        // an owner never seen before has no floor
        expect(l2.stale(7, 1, 1, 0).empty(), "an unknown owner's first receipt is current");
    }
    // fingerprints: content and length sensitive, O(1) sampling still sees a change in every word sampled
    {
        std::vector<uint8_t> a(1 << 20, 1), b = a;
        b[8 * ((a.size() / 8) / 1024) * 5] ^= 1;  // a sampled word
        expect(fahost::archive_fingerprint(a.data(), a.size()) != fahost::archive_fingerprint(b.data(), b.size()),
               "fingerprint sees a sampled word change");
        expect(fahost::archive_fingerprint(a.data(), a.size()) != fahost::archive_fingerprint(a.data(), a.size() - 1),
               "fingerprint sees the length");
        expect(fahost::archive_fingerprint(a.data(), 5) == fahost::archive_fingerprint(a.data(), 5), "deterministic");
    }
    std::printf("{\"checks\": %d, \"failed\": %d}\n", checks, failed);
    return failed ? 1 : 0;
}
