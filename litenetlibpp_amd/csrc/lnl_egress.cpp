// lnl_egress.cpp -- batched socket egress of a CSR wire burst (SURVEY.md 8(f)
// item 2, the send half; the host step after lnl_crc32c_append_host / _csr_dev).
//
// The reference sends one datagram per syscall: net_manager::send_raw is one
// sendto of data[offset .. offset + length) to the peer's sockaddr_in
// (/root/reference/src/lnl/net_manager.cpp:515-523).  Here one sendmmsg call
// hands the kernel up to kMaxVec datagrams of a CSR wire burst -- datagram
// i = wire[off[i] .. off[i+1]), e.g. lnl_crc32c_append_host's output with
// off[i] = h_off[i] - h_off[0] + 4 i -- each to its own endpoint, one
// endpoint for all, or none (a connected socket).
//
// Error behaviour follows send_raw per datagram (:525-567): a datagram the
// kernel refuses gets its negative errno in status[i] (send_raw returns -1 for
// host / network unreachable and raises a NETWORK_ERROR event, 0 for other
// errors: the caller maps status to that) and the burst goes on with the next
// one; that includes ENOBUFS (the interface queue, not the socket buffer, is
// full: poll would report POLLOUT at once and the call would spin).  A full
// socket buffer (EAGAIN) is not a per-datagram error: with wait_ms != 0 the
// call polls for POLLOUT and continues, until one deadline of wait_ms from the
// call's start (-1: no deadline); with 0, or once the deadline has passed, it
// returns early and the datagrams from the returned count on were not
// attempted.
//
// CPU only (no HIP): it is the socket side of the path.
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>

#include <chrono>
#include <vector>

#include "../../include/lnl_crc32c.h"

namespace {
constexpr unsigned kMaxVec = 1024;  // UIO_MAXIOV: sendmmsg's per-call limit
}

extern "C" int64_t lnl_egress_send_batch(int fd, const uint8_t* wire, const uint64_t* off, uint32_t n,
                                         const void* addrs, uint32_t naddrs, int64_t* status, int wait_ms) {
    if (fd < 0 || !off || (!wire && n && off[n] != 0)) return -EINVAL;
    if (addrs && naddrs != 1 && naddrs != n) return -EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return -EINVAL;
    const sockaddr_in* sa = static_cast<const sockaddr_in*>(addrs);
    thread_local std::vector<mmsghdr> msgs;
    thread_local std::vector<iovec> iov;
    if (msgs.size() < kMaxVec) {
        msgs.resize(kMaxVec);
        iov.resize(kMaxVec);
    }
    using clock = std::chrono::steady_clock;
    const clock::time_point deadline = clock::now() + std::chrono::milliseconds(wait_ms > 0 ? wait_ms : 0);
    uint32_t i = 0;
    while (i < n) {
        const uint32_t k = n - i < kMaxVec ? n - i : kMaxVec;
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t d = i + j;
            iov[j].iov_base = const_cast<uint8_t*>(wire) + off[d];
            iov[j].iov_len = off[d + 1] - off[d];
            memset(&msgs[j].msg_hdr, 0, sizeof msgs[j].msg_hdr);
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
            if (sa) {
                msgs[j].msg_hdr.msg_name = const_cast<sockaddr_in*>(naddrs == 1 ? sa : sa + d);
                msgs[j].msg_hdr.msg_namelen = sizeof(sockaddr_in);
            }
        }
        const int r = sendmmsg(fd, msgs.data(), k, MSG_DONTWAIT);
        if (r > 0) {
            if (status)
                for (int j = 0; j < r; ++j) status[i + j] = (int64_t)msgs[j].msg_len;
            i += (uint32_t)r;
            continue;
        }
        // r < 0: the first datagram of this call failed (sendmmsg reports an
        // error only when nothing was sent)
        const int err = r < 0 ? errno : EAGAIN;
        if (err == EINTR) continue;
        if (err == EAGAIN || err == EWOULDBLOCK) {
            if (wait_ms == 0) return (int64_t)i;
            int left = -1;  // wait_ms < 0: no deadline
            if (wait_ms > 0) {
                const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
                if (ms <= 0) return (int64_t)i;  // deadline passed: datagrams i.. not attempted
                left = (int)ms;
            }
            pollfd p{fd, POLLOUT, 0};
            const int pr = poll(&p, 1, left);
            if (pr < 0 && errno != EINTR) return -errno;
            if (pr == 0) return (int64_t)i;  // wait expired: datagrams i.. not attempted
            continue;
        }
        if (err == EBADF || err == ENOTSOCK) return -err;  // the call itself is wrong, not a datagram
        // a per-datagram failure (EHOSTUNREACH, ENETUNREACH, EMSGSIZE, ENOBUFS,
        // ECONNREFUSED from an earlier ICMP, ...): send_raw's error case for
        // this datagram, then the next one
        if (status) status[i] = -(int64_t)err;
        ++i;
    }
    return (int64_t)n;
}
