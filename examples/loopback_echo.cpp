// loopback_echo.cpp -- BASELINE config 1 with the CRC-32C packet layer on.
//
// A clean-room, minimal stand-in for the reference's example/server.cpp +
// example/client.cpp pair (/root/reference/example/server.cpp:10-31,
// client.cpp:10-48): a client sends N messages of 256 bytes (payload byte i =
// i) to an echo server over UDP loopback, UNRELIABLE or RELIABLE_ORDERED, and
// counts the echoes.  It is NOT the reference's net_manager (no connection
// handshake, MTU discovery, merging or fragments -- out of scope here); it
// exists to run the packet layer exactly where a net_manager would
// (INTEGRATION.md):
//
//   send_raw     (net_manager.cpp:515-521): lnl::crc32c_layer::process_outbound_packet
//                into a scratch buffer, sendto the scratch;
//   receive_logic (net_manager.cpp:218-222): recvfrom, process_inbound_packet,
//                drop on mismatch (counted), else strip the CRC and dispatch.
//
// Wire format (LiteNetLib-style header byte, property in bits 0-4):
//   UNRELIABLE (0):  [0][payload]
//   CHANNELED  (1):  [1][seq u16 LE][channel u8][payload]      reliable ordered
//   ACK        (2):  [2][seq u16 LE][channel u8]
// followed on the wire by LE32 CRC-32C of everything before it.
//
// --corrupt K flips one bit of every K-th datagram AFTER the CRC was appended
// (a corrupted link): the receiving layer must drop exactly those, and the
// reliable mode must still deliver every message through retransmission.
//
// --crc 0 turns the layer off (the baseline for its cost).  Prints one JSON
// line.  CPU only; links the product library for the layer.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../include/lnl_crc32c_layer.hpp"

namespace {

enum : uint8_t { kUnreliable = 0, kChanneled = 1, kAck = 2 };
constexpr size_t kMtu = 1432;  // net_constants.h:29-39 POSSIBLE_MTU.back()
using clk = std::chrono::steady_clock;

struct Endpoint {
    int fd = -1;
    sockaddr_in addr{};
    lnl::crc32c_layer layer;
    uint64_t sent = 0, corrupted = 0;
    uint32_t corrupt_every = 0;
    bool crc = true;  // false: the layer is off (baseline for its cost)

    void open() {
        fd = socket(AF_INET, SOCK_DGRAM, 0);
        if (fd < 0) {
            perror("socket");
            exit(2);
        }
        addr.sin_family = AF_INET;
        addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        addr.sin_port = 0;
        if (bind(fd, (sockaddr*)&addr, sizeof addr) != 0) {
            perror("bind");
            exit(2);
        }
        socklen_t len = sizeof addr;
        getsockname(fd, (sockaddr*)&addr, &len);
        fcntl(fd, F_SETFL, O_NONBLOCK);
        int buf = 8 << 20;
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
    }

    // the send_raw hook: append the CRC into scratch, never into `data`
    void send_raw(const uint8_t* data, size_t length, const sockaddr_in& to) {
        uint8_t wire[kMtu + lnl::crc32c_layer::extra_packet_size_for_layer];
        size_t n = length;
        if (crc)
            n = layer.process_outbound_packet(data, length, wire, sizeof wire);
        else
            memcpy(wire, data, length);
        ++sent;
        if (corrupt_every && sent % corrupt_every == 0) {
            wire[(sent * 7) % n] ^= (uint8_t)(1u << (sent % 8));
            ++corrupted;
        }
        sendto(fd, wire, n, 0, (const sockaddr*)&to, sizeof to);
    }

    // the receive_logic hook: false = nothing (more) to read
    bool receive(std::vector<uint8_t>& out, sockaddr_in& from) {
        uint8_t buf[kMtu + 64];
        while (true) {
            socklen_t len = sizeof from;
            ssize_t r = recvfrom(fd, buf, sizeof buf, 0, (sockaddr*)&from, &len);
            if (r <= 0) return false;
            size_t size = (size_t)r;
            if (crc && !layer.process_inbound_packet(buf, size)) continue;  // dropped, counted by the layer
            out.assign(buf, buf + size);
            return true;
        }
    }
};

// Reliable-ordered channel state (one direction each way).
struct ReliableOut {
    uint16_t next_seq = 0;
    std::map<uint16_t, std::pair<std::vector<uint8_t>, clk::time_point>> unacked;
    uint64_t retransmits = 0;
};
struct ReliableIn {
    uint16_t expected = 0;
    std::map<uint16_t, std::vector<uint8_t>> early;
};

std::vector<uint8_t> channeled(uint16_t seq, const uint8_t* payload, size_t n) {
    std::vector<uint8_t> p(4 + n);
    p[0] = kChanneled;
    p[1] = (uint8_t)seq;
    p[2] = (uint8_t)(seq >> 8);
    p[3] = 0;
    memcpy(p.data() + 4, payload, n);
    return p;
}

void send_ack(Endpoint& e, uint16_t seq, const sockaddr_in& to) {
    const uint8_t a[4] = {kAck, (uint8_t)seq, (uint8_t)(seq >> 8), 0};
    e.send_raw(a, sizeof a, to);
}

// In-order delivery of a CHANNELED packet; calls deliver(payload) per message.
template <class F>
void on_channeled(Endpoint& e, ReliableIn& in, const std::vector<uint8_t>& p, const sockaddr_in& from, F deliver) {
    const uint16_t seq = (uint16_t)(p[1] | (p[2] << 8));
    send_ack(e, seq, from);
    if ((int16_t)(seq - in.expected) < 0) return;  // duplicate
    in.early.emplace(seq, std::vector<uint8_t>(p.begin() + 4, p.end()));
    for (auto it = in.early.find(in.expected); it != in.early.end(); it = in.early.find(in.expected)) {
        deliver(it->second);
        in.early.erase(it);
        ++in.expected;
    }
}

}  // namespace

int main(int argc, char** argv) {
    std::string mode = "unreliable";
    uint32_t count = 1000, size = 256, corrupt = 0, window = 64;
    bool crc_on = true;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--mode") mode = argv[i + 1];
        else if (k == "--count") count = (uint32_t)atoi(argv[i + 1]);
        else if (k == "--size") size = (uint32_t)atoi(argv[i + 1]);
        else if (k == "--corrupt") corrupt = (uint32_t)atoi(argv[i + 1]);
        else if (k == "--crc") crc_on = atoi(argv[i + 1]) != 0;
    }
    const bool reliable = mode == "reliable_ordered";
    if (size + 4 > kMtu - lnl::crc32c_layer::extra_packet_size_for_layer) {
        fprintf(stderr, "message too large for the layer MTU\n");
        return 2;
    }
    Endpoint server, client;
    server.open();
    client.open();
    server.corrupt_every = client.corrupt_every = corrupt;
    server.crc = client.crc = crc_on;

    std::vector<uint8_t> payload(size);
    for (uint32_t i = 0; i < size; ++i) payload[i] = (uint8_t)i;

    ReliableOut c_out, s_out;
    ReliableIn c_in, s_in;
    uint32_t next_msg = 0, echoed = 0, bad_payload = 0;
    const auto t0 = clk::now();
    const auto rto = std::chrono::milliseconds(5);
    std::vector<uint8_t> pkt;
    sockaddr_in from{};

    auto check_echo = [&](const std::vector<uint8_t>& msg) {
        if (msg.size() != size || memcmp(msg.data(), payload.data(), size) != 0) ++bad_payload;
        ++echoed;
    };

    while (true) {
        const auto now = clk::now();
        // client: send as the window allows
        while (next_msg < count && (!reliable || c_out.unacked.size() < window)) {
            if (reliable) {
                auto p = channeled(c_out.next_seq, payload.data(), size);
                client.send_raw(p.data(), p.size(), server.addr);
                c_out.unacked[c_out.next_seq++] = {std::move(p), now};
            } else {
                std::vector<uint8_t> p(1 + size);
                p[0] = kUnreliable;
                memcpy(p.data() + 1, payload.data(), size);
                client.send_raw(p.data(), p.size(), server.addr);
            }
            ++next_msg;
        }
        // server: echo everything (same delivery method)
        while (server.receive(pkt, from)) {
            if (pkt.empty()) continue;
            if (pkt[0] == kUnreliable) {
                server.send_raw(pkt.data(), pkt.size(), from);
            } else if (pkt[0] == kChanneled && pkt.size() >= 4) {
                on_channeled(server, s_in, pkt, from, [&](const std::vector<uint8_t>& m) {
                    auto p = channeled(s_out.next_seq, m.data(), m.size());
                    server.send_raw(p.data(), p.size(), from);
                    s_out.unacked[s_out.next_seq++] = {std::move(p), clk::now()};
                });
            } else if (pkt[0] == kAck && pkt.size() >= 4) {
                s_out.unacked.erase((uint16_t)(pkt[1] | (pkt[2] << 8)));
            }
        }
        // client: collect echoes and acks
        while (client.receive(pkt, from)) {
            if (pkt.empty()) continue;
            if (pkt[0] == kUnreliable) {
                check_echo(std::vector<uint8_t>(pkt.begin() + 1, pkt.end()));
            } else if (pkt[0] == kChanneled && pkt.size() >= 4) {
                on_channeled(client, c_in, pkt, from, check_echo);
            } else if (pkt[0] == kAck && pkt.size() >= 4) {
                c_out.unacked.erase((uint16_t)(pkt[1] | (pkt[2] << 8)));
            }
        }
        // retransmissions
        auto resend = [&](Endpoint& e, ReliableOut& o, const sockaddr_in& to) {
            for (auto& kv : o.unacked)
                if (clk::now() - kv.second.second > rto) {
                    e.send_raw(kv.second.first.data(), kv.second.first.size(), to);
                    kv.second.second = clk::now();
                    ++o.retransmits;
                }
        };
        if (reliable) {
            resend(client, c_out, server.addr);
            resend(server, s_out, client.addr);
        }
        const bool done = reliable ? (echoed == count && c_out.unacked.empty() && s_out.unacked.empty())
                                   : next_msg == count;
        if (done && (reliable || echoed + client.layer.dropped() + server.layer.dropped() >= count)) break;
        if (clk::now() - t0 > std::chrono::seconds(20)) break;  // unreliable: losses are final
        if (!reliable && next_msg == count && clk::now() - t0 > std::chrono::milliseconds(500)) break;
    }
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    printf("{\"mode\": \"%s\", \"crc\": %s, \"messages\": %u, \"size\": %u, \"echoed\": %u, \"bad_payload\": %u, "
           "\"datagrams_sent\": %llu, \"corrupted\": %llu, \"dropped_by_crc\": %llu, \"retransmits\": %llu, "
           "\"elapsed_ms\": %.3f, \"echoes_per_s\": %.1f}\n",
           mode.c_str(), crc_on ? "true" : "false", count, size, echoed, bad_payload, (unsigned long long)(client.sent + server.sent),
           (unsigned long long)(client.corrupted + server.corrupted),
           (unsigned long long)(client.layer.dropped() + server.layer.dropped()),
           (unsigned long long)(c_out.retransmits + s_out.retransmits), ms, echoed / (ms / 1000.0));
    close(server.fd);
    close(client.fd);
    return 0;
}
