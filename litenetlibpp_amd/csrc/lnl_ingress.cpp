// lnl_ingress.cpp -- batched socket ingress into a CSR burst (SURVEY.md 8(f)
// item 2; the host step before lnl_inbound_filter_host / _csr_dev).
//
// The reference receives one datagram per syscall: poll, then recvfrom into a
// pooled MAX_PACKET_SIZE (1432-byte) packet, resize to the returned length
// (/root/reference/src/lnl/net_manager.cpp:199-223).  Here one recvmmsg call
// pulls up to max_n datagrams into fixed 1432-byte slots of the caller's
// buffer (pinned memory gives the full PCIe rate for the batch that follows),
// and the burst is then compacted in place into the CSR layout the batch entry
// points take: datagram i = buf[off[i] .. off[i+1]).  Compaction only moves
// data towards the front (off[i] <= i * slot), so memmove in order is safe.
// Datagrams longer than a slot are truncated to it, as recvfrom into the
// reference's 1432-byte packet truncates them.
//
// CPU only (no HIP): it is the socket side of the path.
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>

#include <vector>

#include "../../include/lnl_crc32c.h"

extern "C" int lnl_ingress_recv_batch(int fd, uint8_t* buf, size_t cap, uint64_t* off, uint32_t max_n,
                                      void* addrs, int wait_ms) {
    if (fd < 0 || !buf || !off) return -EINVAL;
    const size_t slot = LNL_INGRESS_SLOT;
    const size_t fit = cap / slot;
    const uint32_t k = (uint32_t)(fit < max_n ? fit : max_n);
    off[0] = 0;
    if (k == 0) return max_n == 0 ? 0 : -ENOSPC;
    if (wait_ms != 0) {  // the reference's poll before its receive loop (net_manager.cpp:202-207)
        pollfd p{fd, POLLIN, 0};
        const int r = poll(&p, 1, wait_ms);
        if (r < 0) return -errno;
        if (r == 0) return 0;
    }
    thread_local std::vector<mmsghdr> msgs;
    thread_local std::vector<iovec> iov;
    if (msgs.size() < k) {
        msgs.resize(k);
        iov.resize(k);
    }
    sockaddr_in* sa = static_cast<sockaddr_in*>(addrs);
    for (uint32_t i = 0; i < k; ++i) {
        iov[i].iov_base = buf + (size_t)i * slot;
        iov[i].iov_len = slot;
        memset(&msgs[i].msg_hdr, 0, sizeof msgs[i].msg_hdr);
        msgs[i].msg_hdr.msg_iov = &iov[i];
        msgs[i].msg_hdr.msg_iovlen = 1;
        if (sa) {
            msgs[i].msg_hdr.msg_name = &sa[i];
            msgs[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
        }
    }
    const int r = recvmmsg(fd, msgs.data(), k, MSG_DONTWAIT, nullptr);
    if (r < 0) return errno == EAGAIN || errno == EWOULDBLOCK ? 0 : -errno;
    for (int i = 0; i < r; ++i) {
        const size_t len = msgs[i].msg_len;
        if (off[i] != (uint64_t)i * slot) memmove(buf + off[i], buf + (size_t)i * slot, len);
        off[i + 1] = off[i] + len;
    }
    return r;
}
