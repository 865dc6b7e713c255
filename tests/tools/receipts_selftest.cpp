// receipts_selftest.cpp -- CPU test of fa_aggregator's receipt ledger (host/receipts.h).
//
// Plays the protocol of data_owner.cpp:224-253 / aggregator.cpp:55-167 with explicit t_start stamps
// (network_layer.cpp:761: the sender stamps its clock when the frame goes out) and checks which receipts
// the ledger calls stale: late byte copies of earlier rounds before and after the current receipt, older
// receipts within a phase; and the receipts that must stay current: an owner whose clock stepped back
// between rounds (new content stamped before its previous phase -- the liveness case), a frozen part
// resent with the same bytes under a new stamp, a retransmission of the current receipt.  Prints one JSON
// line; exit code 1 if any check failed.
#include <cstdio>
#include <string>
#include <vector>

#include "receipts.h"

using fahost::ReceiptKey;
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

// Owner k's receipt of bucket mp in round r, stamped ts (the key is what the ledger sees of it).
ReceiptKey key_of(int round, int owner, int mp, long ts) {
    std::vector<uint8_t> blob(4096 + 13 * mp);
    for (size_t i = 0; i < blob.size(); ++i) blob[i] = (uint8_t)(i * 31 + round * 7 + owner * 3 + mp);
    return ReceiptKey{ts, blob.size(), fahost::archive_fingerprint(blob.data(), blob.size())};
}

}  // namespace

int main() {
    // the protocol, three rounds, with owner 2's late copies and owner 1's clock stepping back 10 s a round
    {
        const int D = 4, L = 2;  // owners 0..3, phase 2 = model parts 2..3
        ReceiptLedger led;
        long t = 100000;
        std::vector<std::vector<ReceiptKey>> sent(3, std::vector<ReceiptKey>(D * (L + 2)));
        auto stamp = [&](int round, int k) { return ++t - (k == 1 ? 10000L * round : 0L); };
        auto take = [&](int owner, int mp, const ReceiptKey& k) {
            const ReceiptLedger::Verdict v = led.check(owner, mp, k);
            if (!v.stale) led.accept(owner, mp, k);
            return v;
        };
        for (int round = 0; round < 3; ++round) {
            for (int k = 0; k < D; ++k) sent[round][k * (L + 2) + 1] = key_of(round, k, 1, stamp(round, k));
            if (round > 0)  // owner 2's part 1 of the previous round, late, BEFORE its current one
                expect(take(2, 1, sent[round - 1][2 * (L + 2) + 1]).stale,
                       "late copy of last round's part 1 before the current one is stale");
            for (int k = 0; k < D; ++k) {
                const auto v = take(k, 1, sent[round][k * (L + 2) + 1]);
                expect(!v.stale, "current part 1");
                expect(v.note.empty() == !(k == 1 && round > 0), "the skewed owner's clock is noted, only it");
            }
            if (round > 0) {  // ... and AFTER it: neither counts nor replaces the newer receipt
                expect(take(2, 1, sent[round - 1][2 * (L + 2) + 1]).stale,
                       "late copy of last round's part 1 after the current one is stale");
                expect(led.is_reduced_copy(2, 1, sent[round - 1][2 * (L + 2) + 1]), "other-phase copy is a copy");
            }
            // a retransmission of this round's own receipt (same stamp, same bytes) is current (it replaces)
            expect(!take(3, 1, sent[round][3 * (L + 2) + 1]).stale, "retransmission of the current receipt");
            expect(!led.is_reduced_copy(3, 1, sent[round][3 * (L + 2) + 1]), "not reduced before the phase ends");
            led.end_phase();
            expect(led.is_reduced_copy(3, 1, sent[round][3 * (L + 2) + 1]), "reduced once the phase ends");
            t += 5;
            for (int k = 0; k < D; ++k)
                for (int mp = 2; mp <= L + 1; ++mp) sent[round][k * (L + 2) + mp] = key_of(round, k, mp, stamp(round, k));
            if (round > 0) {
                expect(take(1, 3, sent[round - 1][1 * (L + 2) + 3]).stale,
                       "late copy of the skewed owner's last-round layer is stale (stamped after its current)");
                expect(take(2, 2, sent[round - 1][2 * (L + 2) + 2]).stale, "late copy of last round's layer");
            }
            for (int k = 0; k < D; ++k)
                for (int mp = 2; mp <= L + 1; ++mp)
                    expect(!take(k, mp, sent[round][k * (L + 2) + mp]).stale, "current phase-2 layer");
            led.end_phase();
            t += 5;
        }
        // a copy from two rounds back still matches
        expect(led.check(2, 2, sent[0][2 * (L + 2) + 2]).stale, "a copy two rounds old is stale");
    }
    // single cases
    {
        ReceiptLedger l2;
        l2.accept(0, 1, key_of(0, 0, 1, 50));
        l2.end_phase();
        l2.accept(0, 2, key_of(0, 0, 2, 60));
        l2.end_phase();
        // the same millisecond as the floor: new content is current, a byte copy of a reduced one is stale
        expect(!l2.check(0, 1, key_of(1, 0, 1, 60)).stale, "new content at the floor's millisecond is current");
        expect(l2.check(0, 1, key_of(0, 0, 1, 50)).stale, "a byte copy is stale");
        // the clock went back: new content before the floor is current (noted), never dropped
        const auto back = l2.check(0, 1, key_of(1, 0, 1, 10));
        expect(!back.stale && !back.note.empty(), "new content sent before the floor is current, with a note");
        // a frozen part: the same bytes as an earlier round under a new stamp is current
        expect(!l2.check(0, 1, ReceiptKey{70, key_of(0, 0, 1, 50).len, key_of(0, 0, 1, 50).fp}).stale,
               "same bytes, new stamp: current");
        // ... and a different bucket with the same stamp and content is not a copy of this one
        expect(!l2.check(0, 3, key_of(0, 0, 2, 60)).stale, "copies are per bucket");
        // within a phase: an older receipt never replaces the newer one; a newer one does
        l2.accept(0, 1, key_of(1, 0, 1, 70));
        expect(l2.check(0, 1, key_of(9, 0, 1, 65)).stale, "an older receipt does not replace a newer one");
        expect(!l2.check(0, 1, key_of(9, 0, 1, 71)).stale, "a newer receipt replaces");
        // an owner never seen before
        expect(!l2.check(7, 1, ReceiptKey{1, 0, 0}).stale, "an unknown owner's first receipt is current");
    }
    // a receipt replaced within its phase: a late copy of it in the next round is stale, so it
    // can neither stand in for its owner's receipt of that round nor replace the real one
    {
        ReceiptLedger l4;
        const ReceiptKey first = key_of(0, 5, 1, 100), second = key_of(1, 5, 1, 101);
        expect(!l4.check(5, 1, first).stale, "first receipt of the phase");
        l4.accept(5, 1, first);
        expect(!l4.check(5, 1, second).stale, "a newer receipt with other content replaces it");
        l4.accept(5, 1, second);
        expect(l4.is_reduced_copy(5, 1, first), "the replaced receipt is remembered at once");
        l4.end_phase();  // phase 1 reduced with `second`
        l4.accept(5, 2, key_of(0, 5, 2, 102));
        l4.end_phase();
        const auto late = l4.check(5, 1, first);
        expect(late.stale, "a late copy of the replaced receipt in the next round is stale");
        expect(l4.check(5, 1, second).stale, "a late copy of the reduced receipt is stale");
        expect(!l4.check(5, 1, key_of(2, 5, 1, 103)).stale, "the next round's own receipt is current");
        // a retransmission (the same key) does not push its own key: it stays current within its phase
        ReceiptLedger l5;
        l5.accept(6, 1, first);
        l5.accept(6, 1, first);
        expect(!l5.is_reduced_copy(6, 1, first), "a retransmission is not remembered as replaced");
    }
    // the memory is bounded: kKeep phases of a bucket
    {
        ReceiptLedger l3;
        for (long r = 0; r < (long)ReceiptLedger::kKeep + 2; ++r) {
            l3.accept(0, 1, ReceiptKey{1000 + r, 8, (uint64_t)r});
            l3.end_phase();
        }
        expect(!l3.is_reduced_copy(0, 1, ReceiptKey{1000, 8, 0}), "the oldest key was forgotten");
        expect(l3.is_reduced_copy(0, 1, ReceiptKey{1002, 8, 2}), "the last kKeep keys are kept");
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
