// refnet_wrap.cpp -- the CRC-32C layer spliced into the REFERENCE's own
// net_manager at link time (test infrastructure; built by oracle/refnet/build.py
// into oracle/_ref/net/, never shipped).
//
// The reference sources are compiled where they lie; their two socket calls
// are routed here with -Wl,--wrap=sendto -Wl,--wrap=recvfrom, which is the
// same edit INTEGRATION.md describes, applied without touching their text:
//
//  * send_raw (/root/reference/src/lnl/net_manager.cpp:515-521) sends
//    data[offset .. offset+length); the wrapper writes payload || LE32(crc)
//    into a per-thread scratch buffer with lnl_crc32c_layer_outbound (the
//    product library, include/lnl_crc32c.h) and sends that.  The caller's
//    buffer is const and may be shared (net_peer.cpp:482, 534, 575): it is
//    never written.
//  * receive_logic (net_manager.cpp:202-223) receives into a
//    MAX_PACKET_SIZE buffer; the wrapper checks the trailing CRC with
//    lnl_crc32c_layer_inbound and returns the stripped length, or counts the
//    datagram as dropped and waits for the next one itself (the INTEGRATION.md
//    edit recycles the packet and goes back to the loop's poll instead; the
//    caller sees the same sequence of accepted datagrams).
//
// REFNET_CRC=0 builds the same wrappers as pass-through observers (the CRC-off
// baseline measured with identical plumbing).  REFNET_CRC=2 (the crc_src
// variant) also leaves the layer to the caller: there send_raw and
// receive_logic themselves are rewritten to INTEGRATION.md's snippets
// (build.py), so the wrappers only observe, corrupt, lose and inject; an
// injected datagram gets its CRC here, since it replaces one that send_raw
// had already checksummed.  Every variant records the
// largest datagram it put on the wire, which is how the tests read the MTU the
// probe settled on (net_peer keeps m_mtu private).  refnet_set_flip_every(n)
// corrupts one bit of every n-th outgoing datagram after the CRC was written:
// a bit-flipping link.  refnet_inject(bytes, port) replaces the next datagram
// sent to that (network-order) port with the given bytes, before the layer:
// crafted datagrams then reach the other manager from a connected peer's own
// endpoint (the MERGED-cut fixture, refnet_driver merged).
#include <errno.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>

#include <netinet/in.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/lnl_crc32c.h"

#ifndef REFNET_CRC
#define REFNET_CRC 1
#endif
#if REFNET_CRC == 2
#include "refnet_layer.hpp"
#endif

extern "C" {
ssize_t __real_sendto(int fd, const void* buf, size_t len, int flags, const struct sockaddr* addr, socklen_t alen);
ssize_t __real_recvfrom(int fd, void* buf, size_t len, int flags, struct sockaddr* addr, socklen_t* alen);
}

namespace {
std::atomic<uint64_t> g_sent{0}, g_received{0}, g_dropped{0}, g_flipped{0};
std::atomic<int64_t> g_max_sent{0};
std::atomic<uint32_t> g_flip_every{0};
std::atomic<uint64_t> g_flip_ctr{0};
std::atomic<uint32_t> g_lose_every{0};
std::atomic<uint64_t> g_lose_ctr{0}, g_lost{0};

// a lossy link (any variant): every n-th datagram never leaves
bool lose() {
    const uint32_t every = g_lose_every.load(std::memory_order_relaxed);
    if (!every || g_lose_ctr.fetch_add(1, std::memory_order_relaxed) % every != every - 1) return false;
    g_lost.fetch_add(1, std::memory_order_relaxed);
    return true;
}

// one pending injection: bytes and the destination port it replaces a datagram to
std::mutex g_inj_mu;
std::vector<uint8_t> g_inj;
bool g_inj_pending = false;
uint16_t g_inj_port = 0;
std::atomic<uint64_t> g_inj_done{0};

// the datagram to send instead of buf, or null (keeps buf)
bool take_injection(const struct sockaddr* addr, socklen_t alen, std::vector<uint8_t>& out) {
    if (!addr || alen < (socklen_t)sizeof(sockaddr_in) || addr->sa_family != AF_INET) return false;
    std::lock_guard<std::mutex> lk(g_inj_mu);
    if (!g_inj_pending || ((const sockaddr_in*)addr)->sin_port != g_inj_port) return false;
    out.swap(g_inj);
    g_inj_pending = false;
    return true;
}

void note_sent(int64_t n) {
    g_sent.fetch_add(1, std::memory_order_relaxed);
    int64_t m = g_max_sent.load(std::memory_order_relaxed);
    while (n > m && !g_max_sent.compare_exchange_weak(m, n, std::memory_order_relaxed)) {
    }
}
}  // namespace

extern "C" {

ssize_t __wrap_sendto(int fd, const void* buf, size_t len, int flags, const struct sockaddr* addr, socklen_t alen) {
    thread_local std::vector<uint8_t> inj;
    const size_t caller_len = len;
    const bool injected = take_injection(addr, alen, inj);
    if (injected) {
        buf = inj.data();
        len = inj.size();
    }
    struct Done {  // count the injection once it has gone out (or was lost)
        bool on;
        ~Done() {
            if (on) g_inj_done.fetch_add(1);
        }
    } done{injected};
#if REFNET_CRC
    thread_local uint8_t scratch[65536 + LNL_CRC32C_LAYER_EXTRA];
#if REFNET_CRC == 2
    // the caller's datagram already carries its CRC; copied (the buffer is the
    // caller's) so that a corrupting link can flip a bit of it
    int64_t wire;
    if (injected) {
        wire = lnl_crc32c_layer_outbound((const uint8_t*)buf, 0, len, scratch, sizeof scratch);
    } else {
        wire = len <= sizeof scratch ? (int64_t)len : -1;
        if (wire >= 0) memcpy(scratch, buf, len);
    }
#else
    const int64_t wire = lnl_crc32c_layer_outbound((const uint8_t*)buf, 0, len, scratch, sizeof scratch);
#endif
    if (wire < 0) {
        errno = EMSGSIZE;
        return -1;
    }
    const uint32_t every = g_flip_every.load(std::memory_order_relaxed);
    if (every) {
        const uint64_t c = g_flip_ctr.fetch_add(1, std::memory_order_relaxed);
        if (c % every == every - 1) {
            const uint64_t k = (c + 1) * 2654435761ull;
            scratch[k % (uint64_t)wire] ^= (uint8_t)(1u << ((k >> 32) % 8u));
            g_flipped.fetch_add(1, std::memory_order_relaxed);
        }
    }
    note_sent(wire);
    if (lose()) return wire;
    const ssize_t r = __real_sendto(fd, scratch, (size_t)wire, flags, addr, alen);
    return injected && r >= 0 ? (ssize_t)caller_len : r;
#else
    note_sent((int64_t)len);
    if (lose()) return (ssize_t)len;
    const ssize_t r = __real_sendto(fd, buf, len, flags, addr, alen);
    return injected && r >= 0 ? (ssize_t)caller_len : r;
#endif
}

ssize_t __wrap_recvfrom(int fd, void* buf, size_t len, int flags, struct sockaddr* addr, socklen_t* alen) {
    for (;;) {
        socklen_t al = alen ? *alen : 0;
        const ssize_t n = __real_recvfrom(fd, buf, len, flags, addr, alen ? &al : nullptr);
        if (n < 0) return n;
        if (alen) *alen = al;
#if REFNET_CRC == 1
        const int64_t payload = lnl_crc32c_layer_inbound((const uint8_t*)buf, (size_t)n);
        if (payload < 0) {  // a checksum failure looks like loss to the reliability layer
            g_dropped.fetch_add(1, std::memory_order_relaxed);
            continue;
        }
        g_received.fetch_add(1, std::memory_order_relaxed);
        return (ssize_t)payload;
#else
        g_received.fetch_add(1, std::memory_order_relaxed);
        return n;
#endif
    }
}

// observers for the test driver
int refnet_crc_on(void) { return REFNET_CRC ? 1 : 0; }
uint64_t refnet_sent(void) { return g_sent.load(); }
uint64_t refnet_received(void) { return g_received.load(); }
#if REFNET_CRC == 2
uint64_t refnet_dropped(void) { return refnet_layers_dropped(); }  // the rewritten receive_logic's layers
#else
uint64_t refnet_dropped(void) { return g_dropped.load(); }
#endif
uint64_t refnet_flipped(void) { return g_flipped.load(); }
int64_t refnet_max_sent(void) { return g_max_sent.load(); }
void refnet_reset_max_sent(void) { g_max_sent.store(0); }
void refnet_set_flip_every(uint32_t n) { g_flip_every.store(n); }
void refnet_set_lose_every(uint32_t n) { g_lose_every.store(n); }
uint64_t refnet_lost(void) { return g_lost.load(); }
void refnet_inject(const uint8_t* p, size_t n, uint16_t port_be) {
    std::lock_guard<std::mutex> lk(g_inj_mu);
    g_inj.assign(p, p + n);
    g_inj_port = port_be;
    g_inj_pending = true;
}
uint64_t refnet_injected(void) { return g_inj_done.load(); }

}  // extern "C"
