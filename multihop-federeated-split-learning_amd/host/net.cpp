// net.cpp -- see net.h.
#include "net.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <iostream>
#include <list>

namespace fahost {

namespace {
long now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

void big_buffers(int fd) {
    int sz = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
}
}  // namespace

// ------------------------------------------------------------------ routing

RoutingTable::RoutingTable(int base) {
    const int d = base - 8079;
    t_[-2] = {"localhost", 8079 + d};
    t_[-1] = {"localhost", 8080 + d};
    t_[0] = {"localhost", 8081 + d};
    t_[1] = {"localhost", 8082 + d};
    t_[2] = {"localhost", 8083 + d};
    t_[3] = {"localhost", 8083 + d};
    t_[18] = {"localhost", 8081 + d};
}

int RoutingTable::port_for(int id) const {
    if (id > 3 && id < 18) return t_.at(0).second + id + 3;   // network_layer.cpp:510-514
    if (id >= 18) return t_.at(18).second + (id - 18);         // :530-534
    auto it = t_.find(id);
    return it == t_.end() ? -1 : it->second.second;
}

std::string RoutingTable::host_for(int id) const {
    auto it = t_.find(id);
    return it == t_.end() ? std::string("localhost") : it->second.first;
}

void RoutingTable::set_host(int id, const std::string& host) {
    auto it = t_.find(id);
    if (it == t_.end()) t_[id] = {host, port_for(id)};
    else it->second.first = host;
}

void RoutingTable::apply(const std::vector<std::pair<int, std::string>>& table) {
    for (auto& e : table) {  // systemAPI.cpp:200-255
        if (e.first > 3 && e.first < 18) t_[e.first] = {e.second, t_.at(0).second + e.first + 3};
        else if (e.first >= 18) t_[e.first] = {e.second, t_.at(18).second + (e.first - 18)};
        else t_[e.first].first = e.second;
    }
}

// ------------------------------------------------------------------ socket helpers

bool send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
        ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

// A kept connection whose peer has closed it (FIN or reset already seen): writing would succeed into the
// socket buffer and lose the frame, so the sender reconnects instead.  The receivers never send data back,
// so anything readable on a sender's socket means end of stream or an error.
static bool peer_closed(int fd) {
    char c;
    const ssize_t k = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    return k == 0 || (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK);
}

static bool recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n > 0) {
        ssize_t k = ::recv(fd, c, n, 0);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

// The frame's buffer, from its first bytes (already read into `head`): sized `len`, with the archive of an
// OPERATION frame 64-byte aligned in memory (aligned_frame_buffer), the head copied in.
std::shared_ptr<Bytes> frame_buffer_for(const char* head, size_t have, size_t len) {
    auto b = aligned_frame_buffer(len, values_offset(head, have));
    std::memcpy(b->data(), head, have);
    return b;
}

constexpr size_t kHeadBytes = 1024;  // an OPERATION header is ~150 bytes

std::shared_ptr<Bytes> recv_frame(int fd) {
    int32_t len = 0;
    if (!recv_all(fd, &len, 4) || len <= 0) return nullptr;
    char head[kHeadBytes];
    const size_t have = std::min<size_t>(kHeadBytes, (size_t)len);
    if (!recv_all(fd, head, have)) return nullptr;
    auto b = frame_buffer_for(head, have, (size_t)len);
    if (!recv_all(fd, b->data() + have, (size_t)len - have)) return nullptr;
    return b;
}

int connect_to(const std::string& host, int port, int tries, int wait_ms) {
    for (int t = 0; t < tries; ++t) {
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        if (getaddrinfo(host == "localhost" ? "127.0.0.1" : host.c_str(), std::to_string(port).c_str(), &hints,
                        &res) == 0) {
            int fd = socket(AF_INET, SOCK_STREAM, 0);
            if (fd >= 0) big_buffers(fd);
            if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
                freeaddrinfo(res);
                int one = 1;
                setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
                return fd;
            }
            if (fd >= 0) close(fd);
            freeaddrinfo(res);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(wait_ms));  // the reference retries every 4 s
    }
    return -1;
}

// ------------------------------------------------------------------ NetLayer

NetLayer::~NetLayer() { stop(); }

bool NetLayer::start(int port) {
    port_ = port >= 0 ? port : routes_.port_for(my_id_);
    listen_fd_ = socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd_ < 0) return false;
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    big_buffers(listen_fd_);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons((uint16_t)port_);
    if (bind(listen_fd_, (sockaddr*)&a, sizeof a) < 0 || listen(listen_fd_, 64) < 0) {
        close(listen_fd_);
        listen_fd_ = -1;
        return false;
    }
    running_ = true;
    rx_ = std::thread(&NetLayer::receiver_loop, this);
    for (int i = 0; i < n_senders_; ++i) {
        senders_.emplace_back(new Sender());
    }
    for (int i = 0; i < n_senders_; ++i) senders_[i]->th = std::thread(&NetLayer::sender_loop, this, i);
    return true;
}

void NetLayer::stop() {
    if (!running_.exchange(false)) return;
    {
        std::lock_guard<std::mutex> lk(m_tx_);
    }
    cv_tx_.notify_all();
    {
        std::lock_guard<std::mutex> lk(m_gate_);
    }
    cv_gate_.notify_all();  // readers waiting for a receive turn
    // wake the receiver's poll/accept, and close the socket only after it has left: closing under it
    // raced its reads of listen_fd_ (TSan, tests/test_host_sanitizers.py) and could hand it a reused fd
    if (listen_fd_ >= 0) shutdown(listen_fd_, SHUT_RDWR);
    if (rx_.joinable()) rx_.join();  // it has waited for every connection's reader to finish
    {
        std::lock_guard<std::mutex> lk(m_rd_);
        rd_stop_ = true;
    }
    cv_rd_.notify_all();
    for (auto& t : readers_)
        if (t.joinable()) t.join();
    readers_.clear();
    if (listen_fd_ >= 0) {
        close(listen_fd_);
        listen_fd_ = -1;
    }
    for (auto& s : senders_) {
        if (s->th.joinable()) s->th.join();
        for (auto& kv : s->open) close(kv.second);
    }
    senders_.clear();
}

NetLayer::Item NetLayer::parse_frame(std::shared_ptr<Bytes> text, bool* keep) {
    Item it;
    // Parse the header without touching the archive (split_receipt, wire.h).
    Message m;
    std::string err;
    size_t blob_off = 0, blob_len = 0;
    if (!split_receipt(text->data(), text->size(), &m, &blob_off, &blob_len, &err)) {
        std::cerr << "[net] dropping malformed frame: " << err << "\n";
        return it;
    }
    *keep = m.save_connection == 1;
    if (m.type == OPERATION) {
        Receipt& r = it.r;
        it.kind = 1;
        r.client_id = m.client_id;
        r.prev_node = m.prev_node;
        r.model_part = m.model_part;
        r.type_op = m.type_op;
        r.t_start = m.t_start;
        r.blob_off = blob_off;
        r.blob_len = blob_len;
        if (link_mbps_ > 0) {  // network_layer.cpp:654-665, opt-in
            const long due = r.t_start + (long)(text->size() * 8.0 / (link_mbps_ * 1e6) * 1000.0);
            const long now = now_ms();
            if (due > now) std::this_thread::sleep_for(std::chrono::milliseconds(due - now));
        }
        r.frame = std::move(text);
    } else {
        it.kind = 2;
        if (m.read_table == 1) {
            std::lock_guard<std::mutex> g(m_routes_);
            routes_.apply(m.rooting_table);
        }
        it.m = std::move(m);
    }
    return it;
}

uint64_t NetLayer::take_seq() {
    std::lock_guard<std::mutex> lk(m_rx_);
    return next_seq_++;
}

void NetLayer::publish(uint64_t seq, Item item) {
    {
        std::lock_guard<std::mutex> lk(m_rx_);
        pending_.emplace(seq, std::move(item));
        for (auto it = pending_.find(next_pub_); it != pending_.end(); it = pending_.find(next_pub_)) {
            if (it->second.kind == 1) receipts_.push_back(std::move(it->second.r));
            else if (it->second.kind == 2) refactors_.push_back(std::move(it->second.m));
            pending_.erase(it);
            ++next_pub_;
        }
    }
    cv_rx_.notify_all();
}

// A reader thread: takes accepted connections from rd_q_ and reads each to its end (reader_loop).
void NetLayer::reader_worker() {
    std::unique_lock<std::mutex> lk(m_rd_);
    for (;;) {
        ++rd_idle_;
        cv_rd_.wait(lk, [&] { return rd_stop_ || !rd_q_.empty(); });
        --rd_idle_;
        if (rd_q_.empty()) return;  // stopping, nothing left to read
        Conn* c = rd_q_.front();
        rd_q_.pop_front();
        lk.unlock();
        reader_loop(c);  // sets c->done last
        lk.lock();
    }
}

void NetLayer::receiver_loop() {
    std::list<std::unique_ptr<Conn>> conns;
    auto reap = [&](bool all) {
        if (all) {  // unblock every reader inside recv, then wait for each connection to be done
            for (auto& c : conns) {
                std::lock_guard<std::mutex> g(c->m);
                if (c->fd >= 0) shutdown(c->fd, SHUT_RDWR);
            }
            for (auto& c : conns)
                while (!c->done) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        for (auto it = conns.begin(); it != conns.end();) it = (*it)->done ? conns.erase(it) : std::next(it);
    };
    const int lfd = listen_fd_;  // stop() closes it only after this thread has been joined
    while (running_) {
        pollfd p{lfd, POLLIN, 0};
        if (poll(&p, 1, 200) <= 0) {
            reap(false);
            continue;
        }
        int fd = accept(lfd, nullptr, nullptr);
        if (fd < 0) continue;
        big_buffers(fd);
        conns.emplace_back(new Conn());
        Conn* c = conns.back().get();
        c->fd = fd;
        c->seq0 = take_seq();  // accept order fixes the FIFO position of the connection's first frame
        {
            std::lock_guard<std::mutex> lk(m_rd_);
            rd_q_.push_back(c);
            if (rd_idle_ < (int)rd_q_.size()) readers_.emplace_back(&NetLayer::reader_worker, this);
        }
        cv_rd_.notify_one();
        reap(false);
    }
    reap(true);
}

bool NetLayer::gate_enter(uint64_t seq) {
    std::unique_lock<std::mutex> lk(m_gate_);
    gate_wait_.insert(seq);
    cv_gate_.wait(lk, [&] { return !running_ || (gate_active_ < gate_limit_ && *gate_wait_.begin() == seq); });
    gate_wait_.erase(seq);
    if (!running_) {
        cv_gate_.notify_all();
        return false;
    }
    ++gate_active_;
    cv_gate_.notify_all();  // the next position may be admitted too
    return true;
}

void NetLayer::gate_leave() {
    {
        std::lock_guard<std::mutex> lk(m_gate_);
        --gate_active_;
    }
    cv_gate_.notify_all();
}

// A large OPERATION frame whose head is in: announced to the consumer as Inflight (set_streaming).
std::shared_ptr<Inflight> NetLayer::announce(const std::shared_ptr<Bytes>& b, size_t have, size_t len) {
    Message m;
    size_t off = 0, blen = 0;
    if (!split_receipt_head(b->data(), have, len, &m, &off, &blen, nullptr) || m.type != OPERATION || off == 0)
        return nullptr;
    auto in = std::make_shared<Inflight>();
    in->client_id = m.client_id;
    in->model_part = m.model_part;
    in->t_start = m.t_start;
    in->buf = b;
    in->blob_off = off;
    in->blob_len = blen;
    in->have.store(have, std::memory_order_release);
    {
        std::lock_guard<std::mutex> lk(m_rx_);
        new_streams_.push_back(in);
        ++progress_gen_;
    }
    cv_rx_.notify_all();
    return in;
}

void NetLayer::progress(Inflight* in, size_t have, bool end, bool failed) {
    in->have.store(have, std::memory_order_release);
    if (end) {
        in->failed.store(failed, std::memory_order_release);
        in->ended.store(true, std::memory_order_release);
    }
    {
        std::lock_guard<std::mutex> lk(m_rx_);
        ++progress_gen_;
    }
    cv_rx_.notify_all();
}

std::vector<std::shared_ptr<Inflight>> NetLayer::take_new_streams() {
    std::lock_guard<std::mutex> lk(m_rx_);
    std::vector<std::shared_ptr<Inflight>> out;
    out.swap(new_streams_);
    return out;
}

int NetLayer::wait_event(Receipt* r, uint64_t* gen, int timeout_ms) {
    // on the system clock, as try_next_receipt (libstdc++'s steady-clock wait_for is invisible to TSan)
    const auto until = std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms);
    std::unique_lock<std::mutex> lk(m_rx_);
    cv_rx_.wait_until(lk, until, [&] { return !receipts_.empty() || progress_gen_ != *gen; });
    const bool moved = progress_gen_ != *gen;
    *gen = progress_gen_;
    if (!receipts_.empty()) {
        *r = std::move(receipts_.front());
        receipts_.pop_front();
        return 1;
    }
    return moved ? 2 : 0;
}

// recv_frame with the receive gate (set_rx_concurrency): the length first, then -- for a large frame,
// once its turn has come -- the body.  A turn is given up when the sender stalls.  A frame of at least
// stream_min_ bytes is announced to the consumer while it arrives (set_streaming).
std::shared_ptr<Bytes> NetLayer::recv_frame_gated(int fd, uint64_t seq) {
    int32_t len = 0;
    if (!recv_all(fd, &len, 4) || len <= 0) return nullptr;
    // the header first, outside the gate: a sender that stalls inside it holds up only its own reader
    char head[kHeadBytes];
    const size_t have = std::min<size_t>(kHeadBytes, (size_t)len);
    if (!recv_all(fd, head, have)) return nullptr;
    bool gated = gate_limit_ > 0 && (size_t)len >= kGateBytes;
    if (gated && !gate_enter(seq)) return nullptr;
    auto b = frame_buffer_for(head, have, (size_t)len);
    std::shared_ptr<Inflight> in;
    if (stream_min_ > 0 && (size_t)len >= stream_min_ && have < (size_t)len) in = announce(b, have, (size_t)len);
    size_t told = have;  // bytes reported to the consumer so far
    char* c = reinterpret_cast<char*>(b->data()) + have;
    size_t n = (size_t)len - have;
    auto last = std::chrono::steady_clock::now();
    while (n > 0) {
        pollfd p{fd, POLLIN, 0};
        const int r = poll(&p, 1, 200);
        if (r < 0 && errno != EINTR) break;
        if (r <= 0) {
            if (!running_) break;
            if (gated && std::chrono::steady_clock::now() - last > std::chrono::milliseconds(kGateStallMs)) {
                gate_leave();  // the owner stalled: let the others through
                gated = false;
            }
            continue;
        }
        const ssize_t k = ::recv(fd, c, n, 0);
        if (k <= 0) break;
        c += k;
        n -= (size_t)k;
        last = std::chrono::steady_clock::now();
        if (in && n > 0 && (size_t)len - n - told >= kStreamStep) {
            told = (size_t)len - n;
            progress(in.get(), told, false, false);
        }
    }
    if (gated) gate_leave();
    if (in) progress(in.get(), (size_t)len - n, true, n != 0);
    return n == 0 ? b : nullptr;
}

// One connection: one frame (the reference's default, save_connection 0), or frames until EOF when
// the sender keeps the connection open (save_connection 1).
void NetLayer::reader_loop(Conn* c) {
    const int fd = c->fd;
    uint64_t seq = c->seq0;
    for (;;) {
        auto text = gate_limit_ > 0 || stream_min_ > 0 ? recv_frame_gated(fd, seq) : recv_frame(fd);
        if (!text) {
            publish(seq, Item{});  // release the FIFO position
            break;
        }
        bytes_rx_ += text->size() + 4;
        bool keep = false;
        // hand the frame over: once published, the consumer holds the only reference, so the buffer
        // returns to the pool as soon as the receipt is dropped (not when this thread gets to run again)
        publish(seq, parse_frame(std::move(text), &keep));
        if (!keep) break;
        bool ready = false;
        while (running_ && !ready) {
            pollfd p{fd, POLLIN, 0};
            ready = poll(&p, 1, 200) > 0;
        }
        if (!ready) break;
        seq = take_seq();  // the next frame on a kept-open connection queues from when it begins
    }
    {
        std::lock_guard<std::mutex> g(c->m);
        close(fd);
        c->fd = -1;
    }
    c->done = true;
}

void NetLayer::sender_loop(int i) {
    Sender& me = *senders_[i];
    while (true) {
        Out o;
        {
            std::unique_lock<std::mutex> lk(m_tx_);
            cv_tx_.wait(lk, [&] { return !me.q.empty() || !running_; });
            if (me.q.empty()) break;
            o = me.q.front();
            me.q.pop_front();
            me.busy = true;
        }
        int fd = -1;
        auto it = me.open.find(o.dest);
        if (it != me.open.end()) {
            fd = it->second;
            if (peer_closed(fd)) {
                close(fd);
                me.open.erase(it);
                fd = -1;
            }
        }
        std::string host;
        int port;
        {
            std::lock_guard<std::mutex> g(m_routes_);
            host = routes_.host_for(o.dest);
            port = routes_.port_for(o.dest);
        }
        const bool reused = fd >= 0;
        if (fd < 0) fd = connect_to(host, port, 100, 200);
        bool sent = fd >= 0 && send_all(fd, o.bytes->data(), o.bytes->size());
        if (!sent && reused) {
            // the kept connection broke (the peer restarted or closed it): one fresh connection, the whole
            // frame again -- the receiver drops the partial frame with the dead connection
            close(fd);
            me.open.erase(o.dest);
            fd = connect_to(host, port, 100, 200);
            sent = fd >= 0 && send_all(fd, o.bytes->data(), o.bytes->size());
        }
        if (fd < 0) {
            ++send_failures_;
            std::cerr << "[net] cannot reach node " << o.dest << " at " << host << ":" << port << "\n";
        } else if (!sent) {
            ++send_failures_;
            std::cerr << "[net] send to node " << o.dest << " failed\n";
            close(fd);
            me.open.erase(o.dest);
        } else if (o.keep) {
            me.open[o.dest] = fd;
        } else {
            close(fd);
            me.open.erase(o.dest);
        }
        {
            std::lock_guard<std::mutex> lk(m_tx_);
            me.busy = false;
        }
        cv_tx_idle_.notify_all();
    }
}

void NetLayer::send(int dest, std::shared_ptr<const Bytes> framed, bool keep_open) {
    {
        std::lock_guard<std::mutex> lk(m_tx_);
        // one sender per destination keeps that destination's frames in order; destinations are dealt
        // to the senders round-robin at first use, so a fan-out to S destinations uses S senders
        auto it = sender_of_.find(dest);
        if (it == sender_of_.end()) it = sender_of_.insert({dest, (int)(sender_of_.size() % senders_.size())}).first;
        senders_[(size_t)it->second]->q.push_back({dest, std::move(framed), keep_open});
    }
    cv_tx_.notify_all();
}

void NetLayer::flush() {
    std::unique_lock<std::mutex> lk(m_tx_);
    cv_tx_idle_.wait(lk, [&] {
        for (auto& s : senders_)
            if (!s->q.empty() || s->busy) return false;
        return true;
    });
}

Receipt NetLayer::next_receipt() {
    std::unique_lock<std::mutex> lk(m_rx_);
    cv_rx_.wait(lk, [&] { return !receipts_.empty(); });
    Receipt r = std::move(receipts_.front());
    receipts_.pop_front();
    return r;
}

bool NetLayer::try_next_receipt(Receipt* r, int timeout_ms) {
    std::unique_lock<std::mutex> lk(m_rx_);
    // wait_until on the system clock (pthread_cond_timedwait): libstdc++'s steady-clock wait_for goes
    // through pthread_cond_clockwait, which ThreadSanitizer (gcc 11) does not intercept -- it then
    // misses the unlock inside the wait and reports the receiver's next lock as a double lock.
    const auto until = std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms);
    if (!cv_rx_.wait_until(lk, until, [&] { return !receipts_.empty(); })) return false;
    *r = std::move(receipts_.front());
    receipts_.pop_front();
    return true;
}

Message NetLayer::next_refactor() {
    std::unique_lock<std::mutex> lk(m_rx_);
    cv_rx_.wait(lk, [&] { return !refactors_.empty(); });
    Message m = std::move(refactors_.front());
    refactors_.pop_front();
    return m;
}

bool NetLayer::find_init(int timeout_s, std::string* err) {
    // Announce (network_layer.cpp:215-227).
    int u = socket(AF_INET, SOCK_DGRAM, 0);
    if (u < 0) return *err = "udp socket", false;
    sockaddr_in g{};
    g.sin_family = AF_INET;
    g.sin_addr.s_addr = inet_addr("224.0.0.0");
    g.sin_port = htons(4321);
    int id = my_id_;
    sendto(u, &id, sizeof id, 0, (sockaddr*)&g, sizeof g);
    close(u);
    // The init node connects to my port and sends "ACK" (findPeers, :164-186); its address is the init's.
    int s = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons((uint16_t)routes_.port_for(my_id_));
    if (bind(s, (sockaddr*)&a, sizeof a) < 0 || listen(s, 4) < 0) {
        close(s);
        return *err = "bind for discovery", false;
    }
    fd_set rs;
    FD_ZERO(&rs);
    FD_SET(s, &rs);
    timeval tv{timeout_s, 0};
    if (select(s + 1, &rs, nullptr, nullptr, &tv) <= 0) {
        close(s);
        return *err = "no init node connected", false;
    }
    sockaddr_in c{};
    socklen_t cl = sizeof c;
    int fd = accept(s, (sockaddr*)&c, &cl);
    if (fd >= 0) {
        char ip[INET_ADDRSTRLEN];
        inet_ntop(AF_INET, &c.sin_addr, ip, sizeof ip);
        routes_.set_host(0, ip);
        char buf[256];
        (void)::recv(fd, buf, sizeof buf, 0);
        close(fd);
    }
    close(s);
    return fd >= 0;
}

}  // namespace fahost
