// refnet_driver.cpp -- runs the REFERENCE's net_manager (compiled from
// /root/reference/src where it lies, oracle/refnet/build.py) with and without
// the CRC-32C layer spliced into its socket calls (refnet_wrap.cpp).  Test
// infrastructure: tests/test_refnet.py drives it; nothing here ships.
//
//   refnet_driver connect       should_connect_ipv4, recreated without gtest
//                               (/root/reference/tests/net_manager_tests.cpp:6-55)
//   refnet_driver send_receive  should_send_and_receive (:57-138)
//   refnet_driver echo          the reference example's traffic
//                               (example/client.cpp:14-47 against the echo of
//                               example/server.cpp:10-31): 5 x 5 typed messages
//                               over the five delivery methods + the
//                               13,218-byte fragmented message
//   refnet_driver mtu           the MTU probe (net_peer.cpp:664-698): after it
//                               settles, a fragmented send fills datagrams to
//                               the MTU; the widest datagram on the wire minus
//                               the layer's 4 bytes is the MTU it settled on
//   refnet_driver flip [n]      a link that flips one bit of every n-th
//                               datagram: 300 RELIABLE_ORDERED messages must
//                               all arrive, in order; the layer counts drops
//   refnet_driver lose [n]      the same with every n-th datagram lost (any
//                               variant: the reference's own loss handling)
//   refnet_driver bench         1000 x 256 B echoes, UNRELIABLE and
//                               RELIABLE_ORDERED
//   refnet_driver merged IN OUT crafted MERGED containers (file IN, written by
//                               tests/golden/make_dispatch_ref.py) sent one by
//                               one from the client's own endpoint (the wrapper
//                               replaces one outgoing datagram, refnet_inject):
//                               the server's net_peer::process_packet cuts them
//                               (net_peer.cpp:164-187); every packet it
//                               delivers to the listener (method, payload) is
//                               written to OUT as JSON, per container
//
// Each mode prints one JSON line and exits 0 when its checks pass.
#include <lnl/lnl.h>
#include <lnl/net_event_based_listener.h>
#include <lnl/net_manager.h>

#include "../../include/lnl_crc32c.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int refnet_crc_on(void);
uint64_t refnet_sent(void);
uint64_t refnet_dropped(void);
uint64_t refnet_flipped(void);
int64_t refnet_max_sent(void);
void refnet_reset_max_sent(void);
void refnet_set_flip_every(uint32_t n);
void refnet_set_lose_every(uint32_t n);
uint64_t refnet_lost(void);
void refnet_inject(const uint8_t* p, size_t n, uint16_t port_be);
uint64_t refnet_injected(void);
}

namespace {

using clk = std::chrono::steady_clock;

double since(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

// poll both managers until done() or the time runs out
bool pump(lnl::net_manager& a, lnl::net_manager& b, double seconds, const std::function<bool()>& done,
          int sleep_us = 1000) {
    const auto t0 = clk::now();
    while (since(t0) < seconds) {
        a.poll_events();
        b.poll_events();
        if (done()) return true;
        std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    }
    return done();
}

struct Pair {
    lnl::net_event_based_listener sl, cl;
    lnl::net_manager server{&sl};
    lnl::net_manager client{&cl};
    std::shared_ptr<lnl::net_peer> client_peer;  // the client's view of the server
    bool connected = false;

    Pair() {
        sl.connection_request().subscribe([](auto& request) { request->accept(); });
        cl.peer_connected().subscribe([this](auto& peer) {
            connected = true;
            client_peer = peer;
        });
        server.name = "server";
        client.name = "client";
    }
    bool connect(double seconds = 5.0) {
        static lnl::net_data_writer writer;
        if (!server.start() || !client.start()) return false;
        lnl::net_address addr(server.address());
        addr.set_address("localhost");
        client.connect(addr, writer);
        return pump(client, server, seconds, [this] {
            return connected && client.first_peer() &&
                   client.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED &&
                   server.first_peer() &&
                   server.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED;
        });
    }
    // the example server's echo (example/server.cpp:10-31)
    void echo_server() {
        sl.network_receive().subscribe([](auto& peer, lnl::net_data_reader& reader, auto, auto method) {
            std::vector<uint8_t> buf(reader.remaining());
            if (!reader.try_read(buf.data(), buf.size())) return;
            peer->send(buf, method);
        });
    }
};

void print_counters(std::string& js) {
    char b[256];
    snprintf(b, sizeof b, "\"crc\": %d, \"datagrams_sent\": %llu, \"dropped\": %llu, \"flipped\": %llu, \"max_wire\": %lld",
             refnet_crc_on(), (unsigned long long)refnet_sent(), (unsigned long long)refnet_dropped(),
             (unsigned long long)refnet_flipped(), (long long)refnet_max_sent());
    js += b;
}

int finish(bool ok, std::string js) {
    js = "{\"ok\": " + std::string(ok ? "true" : "false") + ", " + js + ", ";
    print_counters(js);
    js += "}";
    printf("%s\n", js.c_str());
    fflush(stdout);
    return ok ? 0 : 1;
}

// ---- should_connect_ipv4 / should_send_and_receive ------------------------
// Same steps and retry budget as the reference's tests (15 polls, 10 ms
// apart); the only change is gtest's ASSERT_* becoming the exit status.
int t_connect() {
    static lnl::net_data_writer writer;
    constexpr int kRetries = 15;
    bool is_connected = false;
    lnl::net_event_based_listener sl, cl;
    sl.connection_request().subscribe([](auto& request) { request->accept(); });
    cl.peer_connected().subscribe([&](auto&) { is_connected = true; });
    sl.peer_disconnected().subscribe([&](auto&, auto&) { is_connected = false; });
    lnl::net_manager server(&sl), client(&cl);
    server.name = "server";
    client.name = "client";
    server.start();
    client.start();
    lnl::net_address addr(server.address());
    addr.set_address("localhost");
    client.connect(addr, writer);
    for (int i = 0; i < kRetries; ++i) {
        client.poll_events();
        server.poll_events();
        if (is_connected && client.first_peer() &&
            client.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED)
            break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    const bool ok = is_connected && client.first_peer() &&
                    client.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED;
    return finish(ok, "\"test\": \"should_connect_ipv4\"");
}

int t_send_receive() {
    static thread_local lnl::net_data_writer writer;
    constexpr int kRetries = 15;
    bool is_received = false, is_sent = false;
    const uint32_t data = 0xDEADBEEF;
    lnl::net_event_based_listener sl, cl;
    sl.connection_request().subscribe([](auto& request) { request->accept(); });
    cl.peer_connected().subscribe([&](auto& peer) {
        writer.reset();
        writer.write(data);
        peer->send(writer, lnl::DELIVERY_METHOD::RELIABLE_ORDERED);
        is_sent = true;
    });
    sl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto method) {
        if (method != lnl::DELIVERY_METHOD::RELIABLE_ORDERED) return;
        is_received = reader.read<uint32_t>() == data;
    });
    lnl::net_manager server(&sl), client(&cl);
    server.name = "server";
    client.name = "client";
    server.start();
    client.start();
    lnl::net_address addr(server.address());
    addr.set_address("localhost");
    client.connect(addr, writer);
    for (int i = 0; i < kRetries; ++i) {
        client.poll_events();
        server.poll_events();
        if (server.first_peer() && server.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    bool ok = server.first_peer() && server.first_peer()->connection_state() == lnl::CONNECTION_STATE::CONNECTED;
    for (int i = 0; i < kRetries; ++i) {
        client.poll_events();
        server.poll_events();
        if (is_sent && is_received) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    ok = ok && is_sent && is_received;
    return finish(ok, "\"test\": \"should_send_and_receive\"");
}

// ---- the reference example's echo -------------------------------------------
int t_echo() {
    Pair P;
    P.echo_server();
    int typed[5][5] = {};  // [delivery type][num]
    int frag_ok = 0, frag_seen = 0;
    P.cl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto) {
        if (reader.size() == 13218) {
            ++frag_seen;
            frag_ok += reader.data()[reader.position()] == 192 && reader.data()[reader.position() + 13217] == 31;
            return;
        }
        const int32_t type = reader.read<int32_t>(), num = reader.read<int32_t>();
        if (type >= 0 && type < 5 && num >= 0 && num < 5) ++typed[type][num];
    });
    if (!P.connect()) return finish(false, "\"test\": \"echo\", \"stage\": \"connect\"");
    // example/client.cpp:14-47, sent from the connected callback's peer
    lnl::net_data_writer w;
    const lnl::DELIVERY_METHOD methods[5] = {
        lnl::DELIVERY_METHOD::RELIABLE_UNORDERED, lnl::DELIVERY_METHOD::RELIABLE_ORDERED,
        lnl::DELIVERY_METHOD::SEQUENCED, lnl::DELIVERY_METHOD::UNRELIABLE,
        lnl::DELIVERY_METHOD::RELIABLE_SEQUENCED};
    for (int i = 0; i < 5; ++i)
        for (int t = 0; t < 5; ++t) {
            w.reset();
            w.write(t);
            w.write(i);
            P.client_peer->send(w, methods[t]);
        }
    std::vector<uint8_t> frag(13218, 0);
    frag[0] = 192;
    frag[13217] = 31;
    P.client_peer->send(frag, lnl::DELIVERY_METHOD::RELIABLE_ORDERED);
    auto count = [&] {
        int c = 0;
        for (auto& r : typed)
            for (int v : r) c += v > 0;
        return c;
    };
    pump(P.client, P.server, 10.0, [&] { return count() == 25 && frag_ok == 1; });
    char b[160];
    snprintf(b, sizeof b, "\"test\": \"echo\", \"typed_echoed\": %d, \"fragment_echoed\": %d", count(), frag_ok);
    // the reliable kinds must all come back; loopback loses nothing in practice
    return finish(count() == 25 && frag_ok == 1 && frag_seen == 1, b);
}

// ---- MTU probe ----------------------------------------------------------------
int t_mtu() {
    Pair P;
    P.echo_server();
    int got = 0;
    P.cl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto) {
        got += reader.size() == 13218;
    });
    if (!P.connect()) return finish(false, "\"test\": \"mtu\", \"stage\": \"connect\"");
    // one probe per MTU_CHECK_DELAY (1 s, net_peer.h:20); up to 6 steps, then
    // MAX_MTU_CHECK_ATTEMPTS (4) failures end it
    pump(P.client, P.server, 11.0, [] { return false; }, 2000);
    refnet_reset_max_sent();
    std::vector<uint8_t> big(13218, 7);
    P.client_peer->send(big, lnl::DELIVERY_METHOD::RELIABLE_ORDERED);
    pump(P.client, P.server, 5.0, [&] { return got == 1; });
    const int64_t wire = refnet_max_sent();
    const int64_t mtu = wire - (refnet_crc_on() ? LNL_CRC32C_LAYER_EXTRA : 0);
    char b[160];
    snprintf(b, sizeof b, "\"test\": \"mtu\", \"echoed\": %d, \"mtu\": %lld, \"max_packet_size\": %d", got,
             (long long)mtu, (int)lnl::net_constants::MAX_PACKET_SIZE);
    return finish(got == 1 && wire <= lnl::net_constants::MAX_PACKET_SIZE, b);
}

// ---- a bit-flipping (or lossy) link ---------------------------------------------
int t_flip(uint32_t every, bool lose) {
    Pair P;
    constexpr int kMsgs = 300;
    std::vector<int32_t> seen;
    P.sl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto method) {
        if (method != lnl::DELIVERY_METHOD::RELIABLE_ORDERED) return;
        const int32_t v = reader.read<int32_t>();
        if (v >= 0) seen.push_back(v);
    });
    if (!P.connect()) return finish(false, "\"test\": \"flip\", \"stage\": \"connect\"");
    if (lose)
        refnet_set_lose_every(every);
    else
        refnet_set_flip_every(every);
    // Messages go out one every 2 ms, then a filler (-1) every 5 ms until all
    // have arrived.  The steady traffic matters: the reference's reliable
    // channel leaves the peer's send queue as soon as a pass sends nothing new
    // (pending_packet::try_send returns false for a packet that is sent and not
    // yet due, net_reliable_channel.cpp:192-204, where upstream LiteNetLib
    // returns true), so after a loss it resends only when new data wakes the
    // channel -- with or without the layer (mode "lose" shows the same).
    lnl::net_data_writer w;
    auto send = [&](int32_t v) {
        w.reset();
        w.write(v);
        w.write(std::string(40 + (v < 0 ? 0 : v % 50), 'x'));
        P.client_peer->send(w, lnl::DELIVERY_METHOD::RELIABLE_ORDERED);
    };
    for (int32_t i = 0; i < kMsgs; ++i) {
        send(i);
        pump(P.client, P.server, 0.002, [] { return false; }, 500);
    }
    const auto t0 = clk::now();
    while ((int)seen.size() < kMsgs && since(t0) < 30.0) {
        send(-1);
        pump(P.client, P.server, 0.005, [] { return false; }, 500);
    }
    refnet_set_flip_every(0);
    refnet_set_lose_every(0);
    bool in_order = (int)seen.size() == kMsgs;
    for (int i = 0; in_order && i < kMsgs; ++i) in_order = seen[i] == i;
    char b[160];
    snprintf(b, sizeof b, "\"test\": \"%s\", \"every\": %u, \"received\": %d, \"in_order\": %s, \"lost\": %llu",
             lose ? "lose" : "flip", every, (int)seen.size(), in_order ? "true" : "false",
             (unsigned long long)refnet_lost());
    return finish(in_order && (lose || !refnet_crc_on() || refnet_dropped() > 0), b);
}

// ---- 1000 x 256 B echo timing -------------------------------------------------
int t_bench() {
    Pair P;
    P.echo_server();
    int echoed = 0;
    P.cl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto) {
        echoed += reader.remaining() == 256;
    });
    if (!P.connect()) return finish(false, "\"test\": \"bench\", \"stage\": \"connect\"");
    std::string js = "\"test\": \"bench\"";
    bool ok = true;
    const struct {
        const char* name;
        lnl::DELIVERY_METHOD m;
        double timeout;
    } kinds[2] = {{"unreliable", lnl::DELIVERY_METHOD::UNRELIABLE, 2.0},
                  {"reliable_ordered", lnl::DELIVERY_METHOD::RELIABLE_ORDERED, 20.0}};
    std::vector<uint8_t> msg(256, 0x5A);
    for (const auto& k : kinds) {
        std::vector<double> secs;
        int min_echoed = 1000;
        for (int rep = 0; rep < 5; ++rep) {
            echoed = 0;
            const auto t0 = clk::now();
            for (int i = 0; i < 1000; ++i) P.client_peer->send(msg, k.m);
            pump(P.client, P.server, k.timeout, [&] { return echoed >= 1000; }, 50);
            secs.push_back(since(t0));
            min_echoed = std::min(min_echoed, echoed);
            pump(P.client, P.server, 0.2, [] { return false; });  // drain stragglers
        }
        std::sort(secs.begin(), secs.end());
        char b[200];
        snprintf(b, sizeof b, ", \"%s_s_median\": %.5f, \"%s_s_min\": %.5f, \"%s_min_echoed\": %d", k.name, secs[2],
                 k.name, secs[0], k.name, min_echoed);
        js += b;
        if (k.m == lnl::DELIVERY_METHOD::RELIABLE_ORDERED) ok = ok && min_echoed == 1000;
    }
    return finish(ok, js);
}

// ---- MERGED containers through the reference's process_packet ------------------
// Input: "LNLM", u32 count, u32 connection number, then per container u32 length
// + bytes (header byte first, no CRC field: the layer adds it on the way).  Each
// one replaces the client's next datagram to the server (a TRIG message makes
// one); a MARK message sent after it closes the container's deliveries (UDP
// loopback and the server's single receive thread keep the order).
int t_merged(const char* in_path, const char* out_path) {
    FILE* f = fopen(in_path, "rb");
    if (!f) return finish(false, "\"test\": \"merged\", \"stage\": \"open input\"");
    char magic[4];
    uint32_t count = 0, conn = 0;
    bool ok = fread(magic, 1, 4, f) == 4 && memcmp(magic, "LNLM", 4) == 0 && fread(&count, 4, 1, f) == 1 &&
              fread(&conn, 4, 1, f) == 1;
    std::vector<std::vector<uint8_t>> cont(ok ? count : 0);
    for (auto& c : cont) {
        uint32_t n = 0;
        ok = ok && fread(&n, 4, 1, f) == 1 && n <= 65507;
        c.resize(ok ? n : 0);
        ok = ok && fread(c.data(), 1, c.size(), f) == c.size();
    }
    fclose(f);
    if (!ok) return finish(false, "\"test\": \"merged\", \"stage\": \"read input\"");
    Pair P;
    static const uint8_t kTrig[4] = {'T', 'R', 'I', 'G'}, kMark[4] = {'M', 'A', 'R', 'K'};
    std::vector<std::pair<int, std::vector<uint8_t>>> got;  // (method, payload)
    int marks = 0;
    P.sl.network_receive().subscribe([&](auto&, lnl::net_data_reader& reader, auto, auto method) {
        std::vector<uint8_t> b(reader.remaining());
        if (!b.empty() && !reader.try_read(b.data(), b.size())) return;
        if (b.size() == 8 && memcmp(b.data(), kMark, 4) == 0) {
            ++marks;
            return;
        }
        if (b.size() == 4 && memcmp(b.data(), kTrig, 4) == 0) return;  // a trigger the injection did not replace
        got.emplace_back((int)method, std::move(b));
    });
    if (!P.connect()) return finish(false, "\"test\": \"merged\", \"stage\": \"connect\"");
    const auto server_peer = P.server.first_peer();
    if (!server_peer || server_peer->connect_number() != conn || P.client_peer->connect_number() != conn) {
        char b[160];
        snprintf(b, sizeof b, "\"test\": \"merged\", \"stage\": \"connection number\", \"expected\": %u", conn);
        return finish(false, b);
    }
    lnl::net_address sa(P.server.address());
    const uint16_t port_be = sa.raw.sin_port;
    FILE* o = fopen(out_path, "w");
    if (!o) return finish(false, "\"test\": \"merged\", \"stage\": \"open output\"");
    fprintf(o, "{\"containers\": %u, \"connection_number\": %u, \"delivered\": [\n", count, conn);
    const std::vector<uint8_t> trig(kTrig, kTrig + 4);
    uint32_t done_ok = 0;
    for (uint32_t i = 0; i < count; ++i) {
        got.clear();
        const uint64_t before = refnet_injected();
        refnet_inject(cont[i].data(), cont[i].size(), port_be);
        P.client_peer->send(trig, lnl::DELIVERY_METHOD::UNRELIABLE);
        bool sent = pump(P.client, P.server, 3.0, [&] { return refnet_injected() > before; }, 200);
        const int want = marks + 1;
        std::vector<uint8_t> mark(kMark, kMark + 4);
        for (int k = 0; k < 4; ++k) mark.push_back((uint8_t)(i >> (8 * k)));
        P.client_peer->send(mark, lnl::DELIVERY_METHOD::UNRELIABLE);
        bool closed = sent && pump(P.client, P.server, 3.0, [&] { return marks >= want; }, 200);
        if (!closed) break;
        ++done_ok;
        fprintf(o, "%s[", i ? ",\n" : "");
        for (size_t k = 0; k < got.size(); ++k) {
            fprintf(o, "%s[%d, \"", k ? ", " : "", got[k].first);
            for (uint8_t v : got[k].second) fprintf(o, "%02x", v);
            fprintf(o, "\"]");
        }
        fprintf(o, "]");
    }
    fprintf(o, "\n]}\n");
    fclose(o);
    char b[160];
    snprintf(b, sizeof b, "\"test\": \"merged\", \"containers\": %u, \"closed\": %u", count, done_ok);
    return finish(done_ok == count, b);
}

}  // namespace

int main(int argc, char** argv) {
    lnl::initialize();
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "connect") return t_connect();
    if (mode == "send_receive") return t_send_receive();
    if (mode == "echo") return t_echo();
    if (mode == "mtu") return t_mtu();
    if (mode == "flip") return t_flip(argc > 2 ? (uint32_t)atoi(argv[2]) : 5u, false);
    if (mode == "lose") return t_flip(argc > 2 ? (uint32_t)atoi(argv[2]) : 5u, true);
    if (mode == "bench") return t_bench();
    if (mode == "merged" && argc > 3) return t_merged(argv[2], argv[3]);
    fprintf(stderr, "usage: %s connect|send_receive|echo|mtu|flip [n]|bench|merged IN OUT\n", argv[0]);
    return 2;
}
