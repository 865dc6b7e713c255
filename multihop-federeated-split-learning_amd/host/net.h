// net.h -- the aggregator's side of the reference's task-delivery layer
// (pipeline_simulation/network_layer.{h,cpp}), wire-compatible.
//
// Threading model kept from the reference (network_layer.h:49-63, .cpp:372-480):
// a receiver thread (accept, frames -> FIFO task queue under a mutex + condvar),
// sender threads (queue of outgoing frames, connect with retries, close unless
// save_connection), and the main thread as the single consumer.
// Differences, all deliberate:
//  * every accepted connection is read by a reader thread of its own (from a pool of
//    reusable readers), so D data owners
//    sending at once are received in parallel (the reference reads one frame at
//    a time in its select loop, :372-480).  The FIFO still holds frames in the
//    reference's order -- the order their connections were accepted (or, on a
//    kept-open connection, the order the frames began): each frame takes a
//    sequence number there and a reorder buffer publishes them in that order, so
//    frames one node sends back to back are consumed in the order it sent them;
//  * frame buffers come from new_frame_buffer (wire.h): the aggregator installs
//    a pool of pinned buffers, so a receipt's records go to the GPU by DMA
//    straight from the bytes they arrived in;
//  * a receipt keeps the frame bytes it arrived in (read once, not zero-filled)
//    and points at the archive inside them -- the reference makes ~10 full
//    copies of every blob;
//  * an outgoing frame is built once and shared by every destination (the
//    reference re-serializes per destination, network_layer.cpp:305-313), and
//    destinations are served by several sender threads (the reference has one,
//    :742-829); frames to one destination keep their order;
//  * the 8 Mbit/s link emulation (network_layer.cpp:654-665) is opt-in.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "wire.h"

namespace fahost {

// network_layer.h:80-86 plus the port rules of network_layer.cpp:510-538 and systemAPI.cpp:222-251.
// `base` shifts every default port (reference: base 8079 -> id -2 on 8079, -1 on 8080, 0 on 8081).
class RoutingTable {
public:
    explicit RoutingTable(int base = 8079);
    int port_for(int id) const;
    std::string host_for(int id) const;
    void set_host(int id, const std::string& host);
    // systemAPI::refactor's update from the refactor message's rooting table.
    void apply(const std::vector<std::pair<int, std::string>>& table);

private:
    std::map<int, std::pair<std::string, int>> t_;
};

struct Receipt {  // Task.h:30-51, the fields the aggregation path uses
    int client_id = -1, prev_node = -1, model_part = 1, type_op = -1;
    long t_start = 0;
    std::shared_ptr<const Bytes> frame;  // owns the bytes (the frame text, without the length prefix)
    size_t blob_off = 0, blob_len = 0;   // the torch::save archive inside `frame`
    const uint8_t* blob() const { return (const uint8_t*)frame->data() + blob_off; }
};

// A large OPERATION frame while it is still arriving (NetLayer::set_streaming): its header fields, the buffer
// it is being received into and how much of the frame text is in.  The reader stores `have` (release) after
// the bytes below it have landed, and sets `ended` (with `failed` when the connection broke) last.  The
// complete frame is then published as a Receipt whose `frame` is this same buffer.
struct Inflight {
    int client_id = -1, model_part = 0;
    long t_start = 0;
    std::shared_ptr<Bytes> buf;
    size_t blob_off = 0, blob_len = 0;
    std::atomic<size_t> have{0};
    std::atomic<bool> ended{false}, failed{false};
};

class NetLayer {
public:
    NetLayer(int my_id, RoutingTable routes, int senders = 8)
        : my_id_(my_id), routes_(std::move(routes)), n_senders_(senders < 1 ? 1 : senders) {}
    ~NetLayer();

    // Receiver thread on routes.port_for(my_id) (or `port` when >= 0).  Returns false if bind fails.
    bool start(int port = -1);
    void stop();
    int listen_port() const { return port_; }

    // findInit (network_layer.cpp:197-291): announce my id on 224.0.0.0:4321 and accept the init
    // node's TCP connection on my port to learn its address.  Optional (loopback runs skip it).
    bool find_init(int timeout_s, std::string* err);

    // Link emulation: receipts are held until t_start + bytes*8/(mbps*1e6) s (0 = off).
    void set_link_mbps(double mbps) { link_mbps_ = mbps; }
    // Receive at most k frames of >= kGateBytes at a time, granted in FIFO order (0 = no limit).  Owners
    // that send at once share the link and, unlimited, all finish together at the end of the phase -- so
    // every receipt's H2D copy would start then.  Gated, receipts complete one after another and their
    // copies overlap the rest of the phase.  A gated receive that makes no progress for kGateStallMs gives
    // its turn up (a stalled owner does not hold the others back).
    void set_rx_concurrency(int k) { gate_limit_ = k; }
    static constexpr size_t kGateBytes = 8u << 20;
    static constexpr int kGateStallMs = 2000;

    // Streaming ingest: frames of at least min_bytes (0 = off) are announced as Inflight while they arrive, so
    // the consumer can start on the parts already in (the reference reads a whole frame first,
    // network_layer.cpp:48-65).  Readers report progress every kStreamStep bytes and at the end.
    void set_streaming(size_t min_bytes) { stream_min_ = min_bytes; }
    static constexpr size_t kStreamStep = 256u << 10;
    // Inflight frames announced since the last call.
    std::vector<std::shared_ptr<Inflight>> take_new_streams();
    // Waits up to timeout_ms for a receipt (1, *r set) or for stream progress since *gen (2); 0 on timeout.
    int wait_event(Receipt* r, uint64_t* gen, int timeout_ms);

    Receipt next_receipt();      // blocking FIFO pop (check_new_task for a data owner, :392-409)
    Message next_refactor();     // blocking (check_new_refactor_task, :481-493)
    bool try_next_receipt(Receipt* r, int timeout_ms);

    // Queue a length-prefixed frame for `dest`; the same frame may be queued for many destinations.
    void send(int dest, std::shared_ptr<const Bytes> framed, bool keep_open = false);
    void flush();                // wait until every queued frame has been sent

    RoutingTable& routes() { return routes_; }
    uint64_t bytes_received() const { return bytes_rx_; }
    // Frames that could not be delivered (no connection after the retries, or a send that failed again on
    // a fresh connection); the reference ignores send errors (network_layer.cpp:19-24).
    uint64_t send_failures() const { return send_failures_; }

private:
    struct Out {
        int dest;
        std::shared_ptr<const Bytes> bytes;
        bool keep;
    };
    struct Sender {
        std::thread th;
        std::deque<Out> q;
        bool busy = false;
        std::map<int, int> open;  // dest -> socket kept open (save_connection)
    };
    struct Conn {
        std::atomic<bool> done{false};
        std::mutex m;
        int fd = -1;         // -1 once the reader closed it
        uint64_t seq0 = 0;   // sequence number of the connection's first frame (taken at accept)
    };
    struct Item {  // a parsed frame waiting for its turn in the FIFO
        int kind = 0;  // 0 nothing (closed without a frame / malformed), 1 receipt, 2 refactor
        Receipt r;
        Message m;
    };
    uint64_t take_seq();
    void publish(uint64_t seq, Item item);
    void receiver_loop();
    void reader_loop(Conn* c);
    void reader_worker();
    void sender_loop(int i);
    Item parse_frame(std::shared_ptr<Bytes> text, bool* keep);
    std::shared_ptr<Bytes> recv_frame_gated(int fd, uint64_t seq);
    std::shared_ptr<Inflight> announce(const std::shared_ptr<Bytes>& b, size_t have, size_t len);
    void progress(Inflight* in, size_t have, bool end, bool failed);
    bool gate_enter(uint64_t seq);
    void gate_leave();

    int my_id_;
    RoutingTable routes_;
    int n_senders_;
    int port_ = -1, listen_fd_ = -1;
    double link_mbps_ = 0;
    std::atomic<bool> running_{false};
    int gate_limit_ = 0;
    std::mutex m_gate_;
    std::condition_variable cv_gate_;
    int gate_active_ = 0;            // under m_gate_
    std::set<uint64_t> gate_wait_;   // under m_gate_: FIFO positions waiting for a turn
    std::atomic<uint64_t> bytes_rx_{0};
    std::atomic<uint64_t> send_failures_{0};
    std::thread rx_;
    // Reader threads, reused from connection to connection: the protocol opens a connection per frame (the
    // reference's save_connection 0), and a thread started per connection put ~20-40 us of thread creation
    // on every frame's path (a small model's round is a dozen frames).  An accepted connection waits in
    // rd_q_ for an idle reader; when none is idle a new one starts, so concurrent owners are still read in
    // parallel.  Idle readers stay for the next connections until stop().
    std::mutex m_rd_;
    std::condition_variable cv_rd_;
    std::deque<Conn*> rd_q_;            // under m_rd_
    int rd_idle_ = 0;                   // under m_rd_
    bool rd_stop_ = false;              // under m_rd_
    std::vector<std::thread> readers_;  // started by the receiver thread, joined by stop()
    std::mutex m_rx_;
    std::condition_variable cv_rx_;
    std::deque<Receipt> receipts_;
    std::deque<Message> refactors_;
    size_t stream_min_ = 0;
    uint64_t progress_gen_ = 0;                         // under m_rx_
    std::vector<std::shared_ptr<Inflight>> new_streams_;  // under m_rx_
    uint64_t next_seq_ = 0, next_pub_ = 0;  // under m_rx_
    std::map<uint64_t, Item> pending_;       // finished frames waiting for an earlier one
    std::mutex m_tx_;
    std::condition_variable cv_tx_, cv_tx_idle_;
    std::vector<std::unique_ptr<Sender>> senders_;
    std::map<int, int> sender_of_;  // destination -> sender index (under m_tx_)
    std::mutex m_routes_;  // routes_ is updated by readers (refactor) and read by senders
};

// Blocking helpers shared with the test tools.
bool send_all(int fd, const void* p, size_t n);
std::shared_ptr<Bytes> recv_frame(int fd);  // [int32 len][len bytes] -> the len bytes; null on EOF / error
int connect_to(const std::string& host, int port, int tries, int wait_ms);

}  // namespace fahost
