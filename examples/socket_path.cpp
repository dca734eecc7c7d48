// socket_path.cpp -- BASELINE config 5 over real sockets: the receive side of
// a net_manager with the CRC layer on, batched.
//
// A sender thread blasts wire datagrams (LiteNetLib header byte, payload,
// LE32 CRC-32C from the layer; every --corrupt-th one with a flipped bit, some
// with headers net_packet::verify rejects) over UDP loopback with sendmmsg.
// The receiver replaces the reference's one-recvfrom-per-datagram loop
// (/root/reference/src/lnl/net_manager.cpp:199-223) with
//
//   lnl_ingress_recv_batch   one recvmmsg burst -> pinned CSR buffer
//   lnl_inbound_filter_host  H2D -> CRC + verify() on the GPU -> status D2H
//
// and checks every status against the CPU form (lnl_inbound_status).  Prints
// one JSON line: datagrams and bytes received, the ingress-only rate and the
// rate with the GPU filter, and the status counts.
//
//   hipcc -O2 -std=c++17 examples/socket_path.cpp -Llitenetlibpp_amd -llnl_crc32c \
//         -Wl,-rpath,$PWD/litenetlibpp_amd -o socket_path
//   ./socket_path [--count N] [--burst B] [--corrupt K] [--device D] [--receivers R]
//
// --egress 1 (the send half): the senders hold PAYLOAD
// bursts (no CRC) and run the product's send side per burst --
// lnl_crc32c_append_host (pinned payloads -> H2D -> CRC + append on the GPU ->
// D2H wire burst) then one lnl_egress_send_batch (sendmmsg) -- so every byte
// goes host -> GPU -> socket -> host -> GPU.  The line then also carries the
// send side's times and its PCIe-inclusive append rate.
//
// --receivers R: R receive sockets bound to
// one port with SO_REUSEPORT, one receiver thread each with its own pinned
// burst buffer, fed by R sender sockets (the kernel spreads flows over the
// sockets by 4-tuple hash).  The host filter serialises GPU use per device,
// so while one thread's burst is on the GPU the others keep receiving.
#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../include/lnl_crc32c.h"

namespace {

using clk = std::chrono::steady_clock;

struct Opts {
    uint32_t count = 200000;
    uint32_t burst = 1024;
    uint32_t corrupt = 50;
    int device = 0;
    uint32_t receivers = 1;
    uint32_t egress = 0;
};

Opts parse(int argc, char** argv) {
    Opts o;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        const long v = strtol(argv[i + 1], nullptr, 10);
        if (k == "--count") o.count = (uint32_t)v;
        else if (k == "--burst") o.burst = (uint32_t)v;
        else if (k == "--corrupt") o.corrupt = (uint32_t)v;
        else if (k == "--device") o.device = (int)v;
        else if (k == "--receivers") o.receivers = (uint32_t)std::max(1L, std::min(v, 64L));
        else if (k == "--egress") o.egress = (uint32_t)v;
    }
    return o;
}

// wire datagrams: header byte (mostly UNRELIABLE / CHANNELED, some property
// bytes verify() rejects), payload, LE32 CRC from the layer
std::vector<std::vector<uint8_t>> make_wire(uint32_t n, uint32_t corrupt) {
    std::mt19937_64 rng(7);
    std::vector<std::vector<uint8_t>> w(n);
    std::vector<uint8_t> body;
    for (uint32_t i = 0; i < n; ++i) {
        const size_t len = 1 + rng() % (LNL_INGRESS_SLOT - LNL_CRC32C_LAYER_EXTRA);
        body.resize(len);
        for (auto& b : body) b = (uint8_t)rng();
        const uint32_t r = (uint32_t)(rng() % 100);
        body[0] = r < 60 ? 0x00 : r < 95 ? 0x01 : (uint8_t)(0x12 + r % 14);  // 18..31: unknown property
        w[i].resize(len + LNL_CRC32C_LAYER_EXTRA);
        lnl_crc32c_layer_outbound(body.data(), 0, len, w[i].data(), w[i].size());
        if (corrupt && i % corrupt == corrupt - 1) w[i][rng() % w[i].size()] ^= (uint8_t)(1u << (rng() % 8));
    }
    return w;
}

// payloads only (header byte + body, no CRC field): the egress mode's input
std::vector<std::vector<uint8_t>> make_payloads(uint32_t n) {
    std::mt19937_64 rng(11);
    std::vector<std::vector<uint8_t>> p(n);
    for (uint32_t i = 0; i < n; ++i) {
        p[i].resize(1 + rng() % (LNL_INGRESS_SLOT - LNL_CRC32C_LAYER_EXTRA));
        for (auto& b : p[i]) b = (uint8_t)rng();
        const uint32_t r = (uint32_t)(rng() % 100);
        p[i][0] = r < 60 ? 0x00 : r < 95 ? 0x01 : (uint8_t)(0x12 + r % 14);
    }
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    const Opts o = parse(argc, argv);
    const auto wire = o.egress ? std::vector<std::vector<uint8_t>>() : make_wire(o.count, o.corrupt);
    const auto payloads = o.egress ? make_payloads(o.count) : std::vector<std::vector<uint8_t>>();

    const uint32_t R = o.receivers;
    std::vector<int> rx(R), tx(R);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    for (uint32_t r = 0; r < R; ++r) {
        rx[r] = socket(AF_INET, SOCK_DGRAM, 0);
        int one = 1, rcvbuf = 1 << 26;
        setsockopt(rx[r], SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof rcvbuf);
        if (R > 1) setsockopt(rx[r], SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
        if (bind(rx[r], (sockaddr*)&a, sizeof a) != 0) return perror("bind"), 1;
        if (r == 0) {  // the others join the port the first one got
            socklen_t al = sizeof a;
            getsockname(rx[0], (sockaddr*)&a, &al);
        }
    }
    for (uint32_t r = 0; r < R; ++r) {
        tx[r] = socket(AF_INET, SOCK_DGRAM, 0);
        if (connect(tx[r], (sockaddr*)&a, sizeof a) != 0) return perror("connect"), 1;
    }
    if (hipSetDevice(o.device) != hipSuccess) {
        fprintf(stderr, "no HIP device for the pinned burst buffers\n");
        return 2;
    }

    std::atomic<uint32_t> senders_left{R};
    std::atomic<int> tx_fail{0};
    std::vector<double> t_append(R, 0.0), t_egress(R, 0.0);
    std::vector<uint64_t> tx_payload(R, 0);
    std::vector<std::thread> senders;
    for (uint32_t r = 0; r < R; ++r)
        senders.emplace_back(o.egress ? std::function<void()>([&, r] {
            // the product's send side per burst of 64: payloads -> pinned burst
            // -> lnl_crc32c_append_host -> lnl_egress_send_batch
            constexpr uint32_t kB = 64;
            const size_t pcap = (size_t)kB * LNL_INGRESS_SLOT;
            uint8_t *pay = nullptr, *wb = nullptr;
            if (hipSetDevice(o.device) != hipSuccess || hipHostMalloc((void**)&pay, pcap) != hipSuccess ||
                hipHostMalloc((void**)&wb, pcap + kB * LNL_CRC32C_LAYER_EXTRA) != hipSuccess) {
                tx_fail = 2;
                --senders_left;
                return;
            }
            std::vector<uint64_t> poff(kB + 1), woff(kB + 1), rel(kB + 1);
            std::vector<int64_t> st(kB);
            std::vector<uint32_t> mine;
            for (uint32_t i = r; i < o.count; i += R) mine.push_back(i);
            std::mt19937 flip(r + 1);
            for (size_t i = 0; i < mine.size() && !tx_fail;) {
                const uint32_t k = (uint32_t)std::min<size_t>(kB, mine.size() - i);
                poff[0] = woff[0] = 0;
                for (uint32_t j = 0; j < k; ++j) {
                    const auto& p = payloads[mine[i + j]];
                    memcpy(pay + poff[j], p.data(), p.size());
                    poff[j + 1] = poff[j] + p.size();
                    woff[j + 1] = poff[j + 1] + (uint64_t)(j + 1) * LNL_CRC32C_LAYER_EXTRA;
                }
                const auto a0 = clk::now();
                if (lnl_crc32c_append_host(pay, poff.data(), k, wb, nullptr, o.device) != 0) {
                    fprintf(stderr, "append_host: %s\n", lnl_crc32c_last_error());
                    tx_fail = 1;
                    break;
                }
                const auto a1 = clk::now();
                if (o.corrupt)  // a flipped bit on the wire now and then: the receiver's filter drops it
                    for (uint32_t j = 0; j < k; ++j)
                        if (mine[i + j] % o.corrupt == o.corrupt - 1) wb[woff[j] + flip() % (woff[j + 1] - woff[j])] ^= 0x08;
                uint32_t done = 0;
                while (done < k) {  // paced by the socket buffer
                    for (uint32_t j = done; j <= k; ++j) rel[j - done] = woff[j] - woff[done];
                    const int64_t m = lnl_egress_send_batch(tx[r], wb + woff[done], rel.data(), k - done, nullptr, 0,
                                                            st.data(), 200);
                    if (m < 0) {
                        fprintf(stderr, "egress: %lld\n", (long long)m);
                        tx_fail = 1;
                        break;
                    }
                    done += (uint32_t)m;
                }
                t_append[r] += std::chrono::duration<double>(a1 - a0).count();
                t_egress[r] += std::chrono::duration<double>(clk::now() - a1).count();
                tx_payload[r] += poff[k];
                i += k;
            }
            (void)hipHostFree(pay);
            (void)hipHostFree(wb);
            --senders_left;
        }) : std::function<void()>([&, r] {  // sendmmsg bursts of 64 (datagrams r, r + R, ...), paced by the socket buffer
            std::vector<mmsghdr> m(64);
            std::vector<iovec> iov(64);
            std::vector<uint32_t> mine;
            for (uint32_t i = r; i < o.count; i += R) mine.push_back(i);
            for (size_t i = 0; i < mine.size();) {
                const uint32_t k = (uint32_t)std::min<size_t>(64, mine.size() - i);
                for (uint32_t j = 0; j < k; ++j) {
                    const auto& w = wire[mine[i + j]];
                    iov[j] = {(void*)w.data(), w.size()};
                    memset(&m[j].msg_hdr, 0, sizeof m[j].msg_hdr);
                    m[j].msg_hdr.msg_iov = &iov[j];
                    m[j].msg_hdr.msg_iovlen = 1;
                }
                const int n = sendmmsg(tx[r], m.data(), k, 0);
                if (n > 0) i += (size_t)n;
                else std::this_thread::yield();
            }
            --senders_left;
        }));

    std::atomic<uint64_t> got{0}, bytes{0}, c0{0}, c1{0}, c2{0}, mismatch{0};
    std::atomic<int> fail{0};
    std::vector<double> t_ingress(R, 0.0), t_filter(R, 0.0);
    const auto t0 = clk::now();
    std::vector<std::thread> receivers;
    for (uint32_t r = 0; r < R; ++r)
        receivers.emplace_back([&, r] {
            uint8_t* buf = nullptr;  // this thread's pinned burst buffer
            const size_t cap = (size_t)o.burst * LNL_INGRESS_SLOT;
            if (hipSetDevice(o.device) != hipSuccess || hipHostMalloc((void**)&buf, cap) != hipSuccess) {
                fail = 2;
                return;
            }
            std::vector<uint64_t> off(o.burst + 1);
            std::vector<uint8_t> status(o.burst);
            while (true) {
                const bool done = senders_left.load() == 0;
                const auto a0 = clk::now();
                const int n = lnl_ingress_recv_batch(rx[r], buf, cap, off.data(), o.burst, nullptr, done ? 50 : 200);
                const auto a1 = clk::now();
                if (n < 0) {
                    fprintf(stderr, "ingress: %d\n", n);
                    fail = 1;
                    break;
                }
                if (n == 0) {
                    if (done) break;
                    continue;
                }
                t_ingress[r] += std::chrono::duration<double>(a1 - a0).count();
                const int rc = lnl_inbound_filter_host(buf, off.data(), (uint32_t)n, status.data(), o.device);
                t_filter[r] += std::chrono::duration<double>(clk::now() - a1).count();
                if (rc) {
                    fprintf(stderr, "filter: %d %s\n", rc, lnl_crc32c_last_error());
                    fail = 1;
                    break;
                }
                uint64_t cnt[3] = {0, 0, 0}, bad = 0;
                for (int i = 0; i < n; ++i) {
                    const uint8_t s = status[i];
                    if (s <= 2) ++cnt[s];
                    if (s != (uint8_t)lnl_inbound_status(buf + off[i], off[i + 1] - off[i])) ++bad;
                }
                c0 += cnt[0];
                c1 += cnt[1];
                c2 += cnt[2];
                mismatch += bad;
                got += (uint64_t)n;
                bytes += off[n];
            }
            (void)hipHostFree(buf);
        });
    for (auto& t : receivers) t.join();
    const double wall = std::chrono::duration<double>(clk::now() - t0).count();
    for (auto& t : senders) t.join();
    if (fail) return fail.load();
    if (tx_fail) return 10 + tx_fail.load();
    double ti = 0, tf = 0, tboth = 0;  // slowest receiver
    for (uint32_t r = 0; r < R; ++r)
        ti = std::max(ti, t_ingress[r]), tf = std::max(tf, t_filter[r]), tboth = std::max(tboth, t_ingress[r] + t_filter[r]);
    // single receiver: ingress-only and ingress + filter rates from the per-burst
    // times; several: the aggregate over the wall time of the whole run
    printf("{\"sent\": %u, \"received\": %llu, \"bytes\": %llu, \"burst\": %u, \"receivers\": %u, "
           "\"ingress_s\": %.4f, \"filter_s\": %.4f, \"wall_s\": %.4f, "
           "\"ingress_gbps\": %.3f, \"ingress_plus_gpu_filter_gbps\": %.3f, \"aggregate_wall_gbps\": %.3f, "
           "\"accept\": %llu, \"drop_crc\": %llu, \"malformed\": %llu, \"gpu_cpu_mismatch\": %llu",
           o.count, (unsigned long long)got.load(), (unsigned long long)bytes.load(), o.burst, R, ti, tf, wall,
           bytes.load() / ti / 1e9, bytes.load() / tboth / 1e9, bytes.load() / wall / 1e9,
           (unsigned long long)c1.load(), (unsigned long long)c0.load(), (unsigned long long)c2.load(),
           (unsigned long long)mismatch.load());
    if (o.egress) {
        double ta = 0, te = 0;
        uint64_t pb = 0;
        for (uint32_t r = 0; r < R; ++r) ta = std::max(ta, t_append[r]), te = std::max(te, t_egress[r]), pb += tx_payload[r];
        printf(", \"egress\": true, \"tx_payload_bytes\": %llu, \"append_host_s\": %.4f, \"egress_send_s\": %.4f, "
               "\"append_host_gbps\": %.3f, \"egress_send_gbps\": %.3f",
               (unsigned long long)pb, ta, te, pb / (double)R / ta / 1e9, pb / (double)R / te / 1e9);
    }
    printf("}\n");
    for (uint32_t r = 0; r < R; ++r) close(rx[r]), close(tx[r]);
    return mismatch.load() ? 3 : 0;
}
