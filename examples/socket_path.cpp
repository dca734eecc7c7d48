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
//   ./socket_path [--count N] [--burst B] [--corrupt K] [--device D]
#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

}  // namespace

int main(int argc, char** argv) {
    const Opts o = parse(argc, argv);
    const auto wire = make_wire(o.count, o.corrupt);

    int rx = socket(AF_INET, SOCK_DGRAM, 0), tx = socket(AF_INET, SOCK_DGRAM, 0);
    int rcvbuf = 1 << 26;
    setsockopt(rx, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof rcvbuf);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(rx, (sockaddr*)&a, sizeof a) != 0) return perror("bind"), 1;
    socklen_t al = sizeof a;
    getsockname(rx, (sockaddr*)&a, &al);
    if (connect(tx, (sockaddr*)&a, sizeof a) != 0) return perror("connect"), 1;

    uint8_t* buf = nullptr;  // pinned burst buffer
    const size_t cap = (size_t)o.burst * LNL_INGRESS_SLOT;
    if (hipSetDevice(o.device) != hipSuccess || hipHostMalloc((void**)&buf, cap) != hipSuccess) {
        fprintf(stderr, "no HIP device for the pinned burst buffer\n");
        return 2;
    }
    std::vector<uint64_t> off(o.burst + 1);
    std::vector<uint8_t> status(o.burst);

    std::atomic<bool> done{false};
    std::thread sender([&] {  // sendmmsg bursts of 64, paced by the socket buffer
        std::vector<mmsghdr> m(64);
        std::vector<iovec> iov(64);
        for (uint32_t i = 0; i < o.count;) {
            const uint32_t k = std::min<uint32_t>(64, o.count - i);
            for (uint32_t j = 0; j < k; ++j) {
                iov[j] = {(void*)wire[i + j].data(), wire[i + j].size()};
                memset(&m[j].msg_hdr, 0, sizeof m[j].msg_hdr);
                m[j].msg_hdr.msg_iov = &iov[j];
                m[j].msg_hdr.msg_iovlen = 1;
            }
            const int r = sendmmsg(tx, m.data(), k, 0);
            if (r > 0) i += (uint32_t)r;
            else std::this_thread::yield();
        }
        done = true;
    });

    uint64_t got = 0, bytes = 0, counts[3] = {0, 0, 0}, mismatch = 0;
    double t_ingress = 0, t_filter = 0;
    const auto t0 = clk::now();
    while (true) {
        const auto a0 = clk::now();
        const int n = lnl_ingress_recv_batch(rx, buf, cap, off.data(), o.burst, nullptr, done ? 50 : 200);
        const auto a1 = clk::now();
        if (n < 0) return fprintf(stderr, "ingress: %d\n", n), 1;
        if (n == 0) {
            if (done) break;
            continue;
        }
        t_ingress += std::chrono::duration<double>(a1 - a0).count();
        const int rc = lnl_inbound_filter_host(buf, off.data(), (uint32_t)n, status.data(), o.device);
        t_filter += std::chrono::duration<double>(clk::now() - a1).count();
        if (rc) return fprintf(stderr, "filter: %d %s\n", rc, lnl_crc32c_last_error()), 1;
        for (int i = 0; i < n; ++i) {
            const uint8_t s = status[i];
            if (s <= 2) ++counts[s];
            if (s != (uint8_t)lnl_inbound_status(buf + off[i], off[i + 1] - off[i])) ++mismatch;
        }
        got += (uint64_t)n;
        bytes += off[n];
    }
    const double wall = std::chrono::duration<double>(clk::now() - t0).count();
    sender.join();
    printf("{\"sent\": %u, \"received\": %llu, \"bytes\": %llu, \"burst\": %u, "
           "\"ingress_s\": %.4f, \"filter_s\": %.4f, \"wall_s\": %.4f, "
           "\"ingress_gbps\": %.3f, \"ingress_plus_gpu_filter_gbps\": %.3f, "
           "\"accept\": %llu, \"drop_crc\": %llu, \"malformed\": %llu, \"gpu_cpu_mismatch\": %llu}\n",
           o.count, (unsigned long long)got, (unsigned long long)bytes, o.burst, t_ingress, t_filter, wall,
           bytes / t_ingress / 1e9, bytes / (t_ingress + t_filter) / 1e9, (unsigned long long)counts[1],
           (unsigned long long)counts[0], (unsigned long long)counts[2], (unsigned long long)mismatch);
    (void)hipHostFree(buf);
    close(rx);
    close(tx);
    return mismatch ? 3 : 0;
}
