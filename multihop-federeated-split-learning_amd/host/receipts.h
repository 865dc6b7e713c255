// receipts.h -- which receipts of a round are current (fa_aggregator's receipt ledger).
//
// The reference aggregator counts raw receipts and consumes whatever arrives (aggregator.cpp:59-92,
// :112-149).  The wire carries no round number, so a delayed copy of an earlier round's receipt would be
// reduced as if it were this round's.  What a late copy is, though, is a BYTE copy of a frame its owner
// already sent -- header included, so it carries the very t_start its original carried (stamped on the
// owner's clock by its sender thread when the frame went out, network_layer.cpp:761).  So the ledger
// keys every receipt it reduced by (owner, bucket, t_start, archive length, content fingerprint) and:
//   * drops a receipt whose key matches one its owner already had reduced (the last kKeep phases of that
//     bucket): a late copy or a retransmission that arrived after its phase ended;
//   * accepts everything else, including a receipt stamped before its owner's previous phase (an owner
//     clock that stepped back: an NTP step, a VM resume) -- logged, never dropped, since dropping a genuine
//     receipt would leave the phase waiting forever for an owner that will not resend;
//   * within a phase, a second receipt of (owner, bucket) replaces the one taken unless it was sent before
//     it (the newest wins, whichever arrives last); the replaced receipt's key is remembered as if it had
//     been reduced, so a late copy of it in a later round is stale too.
// A genuine receipt is only ever mistaken for a copy if it carries the exact millisecond stamp, length and
// sampled content of an earlier receipt of the same owner and bucket: a clock stepped back onto that very
// millisecond with the sampled words unchanged.
// Header-only and free of HIP, so the CPU suite tests it (tests/tools/receipts_selftest.cpp).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <utility>

namespace fahost {

// FNV-1a over the length and 1024 evenly spaced 8-byte words of an archive (and its ragged tail): two
// rounds' receipts of a bucket differ in (nearly) every parameter, so the sampled words tell them apart; a
// copy matches.  O(1) in the archive size; the ledger never relies on it alone (the exact t_start too).
inline uint64_t archive_fingerprint(const uint8_t* b, size_t len) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)len;
    const size_t words = len / 8;
    const size_t step = std::max<size_t>(1, words / 1024);
    for (size_t i = 0; i < words; i += step) {
        uint64_t v;
        std::memcpy(&v, b + i * 8, 8);
        h = (h ^ v) * 1099511628211ull;
    }
    for (size_t i = words * 8; i < len; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

// What a receipt is, as far as the ledger knows it.
struct ReceiptKey {
    long t_start = 0;
    size_t len = 0;
    uint64_t fp = 0;
    bool operator==(const ReceiptKey& o) const { return t_start == o.t_start && len == o.len && fp == o.fp; }
};

class ReceiptLedger {
public:
    static constexpr size_t kKeep = 64;  // reduced receipts remembered per (owner, bucket): 64 rounds back

    struct Verdict {
        bool stale = false;
        std::string why;   // stale: why it is dropped
        std::string note;  // current but worth a log line (the owner's clock went back)
    };

    Verdict check(int owner, int model_part, const ReceiptKey& k) const {
        Verdict v;
        auto c = consumed_.find({owner, model_part});
        if (c != consumed_.end() && std::find(c->second.begin(), c->second.end(), k) != c->second.end()) {
            v.stale = true;
            v.why = "a byte copy of the receipt sent at " + std::to_string(k.t_start) + ", already reduced or replaced";
            return v;
        }
        auto a = accepted_.find({owner, model_part});
        if (a != accepted_.end() && k.t_start < a->second.t_start) {
            v.stale = true;
            v.why = "sent at " + std::to_string(k.t_start) + ", before the receipt already taken (" +
                    std::to_string(a->second.t_start) + ")";
            return v;
        }
        auto fl = floor_.find(owner);
        if (fl != floor_.end() && k.t_start < fl->second)
            v.note = "sent at " + std::to_string(k.t_start) + ", before its owner's receipts of the previous phase (" +
                     std::to_string(fl->second) + "): the owner's clock went back; new content, accepted";
        return v;
    }

    // Whether the receipt is a byte copy of one already reduced (a receipt of the other phase is never
    // taken; this tells a late copy from a retransmission of the current round's).
    bool is_reduced_copy(int owner, int model_part, const ReceiptKey& k) const {
        auto c = consumed_.find({owner, model_part});
        return c != consumed_.end() && std::find(c->second.begin(), c->second.end(), k) != c->second.end();
    }

    // The receipt was consumed into its slot.  When it replaces an earlier one of the same (owner, bucket)
    // with different content, that one joins the reduced keys now: it was taken, so a late copy of it is
    // never current again (it would otherwise count as its owner's receipt of a later phase).
    void accept(int owner, int model_part, const ReceiptKey& k) {
        auto it = accepted_.find({owner, model_part});
        if (it != accepted_.end() && !(it->second == k)) remember({owner, model_part}, it->second);
        accepted_[{owner, model_part}] = k;
    }

    // The phase's buckets are reduced: their receipts join the reduced ones, and the newest stamp of each
    // owner becomes its floor (what a later phase's stamps are compared with, for the clock note).
    void end_phase() {
        for (auto& kv : accepted_) remember(kv.first, kv.second);
        std::map<int, long> fl;
        for (auto& kv : accepted_) {
            const int owner = kv.first.first;
            auto it = fl.find(owner);
            fl[owner] = it == fl.end() ? kv.second.t_start : std::max(it->second, kv.second.t_start);
        }
        for (auto& kv : fl) floor_[kv.first] = kv.second;
        accepted_.clear();
    }

private:
    void remember(const std::pair<int, int>& ob, const ReceiptKey& k) {
        auto& q = consumed_[ob];
        q.push_back(k);
        if (q.size() > kKeep) q.pop_front();
    }

    std::map<int, long> floor_;                                      // owner -> newest stamp of its last phase
    std::map<std::pair<int, int>, std::deque<ReceiptKey>> consumed_;  // (owner, bucket) -> reduced receipts
    std::map<std::pair<int, int>, ReceiptKey> accepted_;              // (owner, bucket) -> taken this phase
};

}  // namespace fahost
