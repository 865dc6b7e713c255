// receipts.h -- which receipts of a round are current (fa_aggregator's receipt ledger).
//
// The reference aggregator counts raw receipts and consumes whatever arrives (aggregator.cpp:59-92,
// :112-149).  The wire carries no round number, so a delayed copy of an earlier round's receipt would be
// reduced as if it were this round's.  What the wire does carry is t_start, stamped on the owner's clock by
// its sender thread when the frame goes out (network_layer.cpp:761), and an owner's sends follow the
// protocol (data_owner.cpp:224-253): its part 1 of round r+1 only after the phase-2 replies of round r,
// which go out after its phase-2 receipts of round r arrived; its phase-2 receipts only after the phase-1
// reply, i.e. after its part 1.  So, per owner:
//   * the floor of a phase = the newest t_start among the owner's receipts the previous phase reduced; a
//     receipt sent before it (t_start < floor) belongs to an earlier phase: stale;
//   * t_start == floor (one millisecond) is decided by content: a byte copy of a receipt the last two phases
//     reduced (archive_fingerprint) is stale, anything else is new;
//   * within a phase, a second receipt of (owner, bucket) sent before the one already taken does not
//     replace it (the newest wins, whichever arrives last).
// Header-only and free of HIP, so the CPU suite tests it (tests/tools/receipts_selftest.cpp).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace fahost {

// FNV-1a over the length and 1024 evenly spaced 8-byte words of an archive (and its ragged tail): two
// rounds' receipts of a bucket differ in (nearly) every parameter, so the sampled words tell them apart; a
// copy matches.  O(1) in the archive size.
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

class ReceiptLedger {
public:
    // Empty when the receipt is current; else why it is stale.
    std::string stale(int owner, int model_part, long t_start, uint64_t fp) const {
        auto fl = floor_.find(owner);
        if (fl != floor_.end()) {
            if (t_start < fl->second)
                return "sent at " + std::to_string(t_start) + ", before its owner's receipts of the previous phase (" +
                       std::to_string(fl->second) + ")";
            auto c = consumed_.find(owner);
            if (t_start == fl->second && c != consumed_.end() &&
                std::find(c->second.begin(), c->second.end(), fp) != c->second.end())
                return "a copy of a receipt an earlier phase already reduced";
        }
        auto a = accepted_.find({owner, model_part});
        if (a != accepted_.end() && t_start < a->second.first)
            return "sent at " + std::to_string(t_start) + ", before the receipt already taken (" +
                   std::to_string(a->second.first) + ")";
        return std::string();
    }

    // The receipt was consumed into its slot (it replaces an earlier one of the same (owner, bucket)).
    void accept(int owner, int model_part, long t_start, uint64_t fp) { accepted_[{owner, model_part}] = {t_start, fp}; }

    // The phase's buckets are reduced: its receipts set every owner's floor for the next phase, and their
    // fingerprints join the last two phases' (what a late copy at the floor's millisecond is matched against).
    void end_phase() {
        std::map<int, long> fl;
        std::map<int, std::vector<uint64_t>> fps;
        for (auto& kv : accepted_) {
            const int owner = kv.first.first;
            auto it = fl.find(owner);
            fl[owner] = it == fl.end() ? kv.second.first : std::max(it->second, kv.second.first);
            fps[owner].push_back(kv.second.second);
        }
        for (auto& kv : fl) floor_[kv.first] = kv.second;
        for (auto& kv : fps) {
            auto& prev = last_phase_fps_[kv.first];
            std::vector<uint64_t> both = prev;
            both.insert(both.end(), kv.second.begin(), kv.second.end());
            consumed_[kv.first] = both;
            prev = kv.second;
        }
        accepted_.clear();
    }

private:
    std::map<int, long> floor_;                                   // owner -> t_start floor of this phase
    std::map<int, std::vector<uint64_t>> consumed_, last_phase_fps_;  // owner -> the last two / last phase's
    std::map<std::pair<int, int>, std::pair<long, uint64_t>> accepted_;  // (owner, bucket) -> (t_start, fp)
};

}  // namespace fahost
