/*
 * lnl_crc32c.h -- C ABI of the MI355X-native CRC-32C packet-layer path.
 *
 * Drop-in boundary.  The reference (Revan600/LiteNetLibPP) has no packet
 * layers and no checksum (/root/reference/README.MD:35); its upstream C#
 * original exposes CRC-32C as a PacketLayerBase subclass
 * (ExtraPacketSizeForLayer = 4, ProcessOutBoundPacket, ProcessInboundPacket).
 * These entry points are what a net_manager would bind at its two datagram
 * choke points:
 *
 *   outbound  net_manager::send_raw, before sendto
 *             /root/reference/src/lnl/net_manager.cpp:515-523
 *   inbound   net_manager::receive_logic, after recvfrom + packet->resize and
 *             before on_message_received / packet->verify()
 *             /root/reference/src/lnl/net_manager.cpp:210-222, :342-343
 *
 * over the bytes net_packet::data()[0 .. size())
 * (/root/reference/include/lnl/net_packet.h:112-118), with every MTU of
 * net_constants::POSSIBLE_MTU (/root/reference/include/lnl/net_constants.h:29-39)
 * reduced by LNL_CRC32C_LAYER_EXTRA when the layer is on.
 *
 * CRC-32C: Castagnoli, reflected polynomial 0x82F63B78, init and xorout
 * 0xFFFFFFFF; CRC("123456789") = 0xE3069283; CRC of 0 bytes = 0.
 *
 * Conventions
 *   - Callers own every buffer.  d_* pointers are device memory of the
 *     current HIP device; h_* pointers are host memory.
 *   - *_dev calls are asynchronous and ordered on `hip_stream` (a hipStream_t,
 *     NULL = the null stream).  They never synchronise.  *_host calls block.
 *   - Return 0 on success or a negative errno-style code:
 *       -EINVAL (-22) bad argument, -ENODEV (-19) no usable gfx950 device,
 *       -ENOMEM (-12) allocation failure, -EIO (-5) a HIP runtime error.
 *     lnl_crc32c_last_error() returns this thread's message for the last
 *     failure.  No C++ exception crosses this ABI.
 *   - Empty batches (n == 0) are valid and launch nothing.
 *   - No batch entry point ever computes on the CPU: without a usable GPU
 *     they fail with -ENODEV.
 *   - Device kernels fetch whole 128-byte-aligned memory lines: they may READ
 *     (never write) bytes of the same 128-byte line before the first / after
 *     the last datagram.  Such a line never crosses a page, so this cannot
 *     fault; the bytes are masked out of every CRC.
 */
#ifndef LNL_CRC32C_H
#define LNL_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LNL_CRC32C_ABI_VERSION 10

/* Bytes the layer adds to every datagram (upstream ExtraPacketSizeForLayer). */
#define LNL_CRC32C_LAYER_EXTRA 4

/* ---- per-datagram CPU path (send_raw / receive_logic hooks) -------------- */

/* CRC-32C of p[0..n).  Stateless, reentrant, thread-safe: send_raw runs on the
 * receive, logic and user threads (/root/reference/src/lnl/net_manager.cpp:106-107).
 * Uses the SSE4.2 crc32 instruction when the host has it. */
uint32_t lnl_crc32c(const uint8_t* p, size_t n);

/* Incremental form: lnl_crc32c_extend(lnl_crc32c(a), b) == lnl_crc32c(a || b);
 * lnl_crc32c_extend(0, p, n) == lnl_crc32c(p, n). */
uint32_t lnl_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);

/* Outbound layer step (upstream Crc32cLayer.ProcessOutBoundPacket): writes
 * data[offset .. offset+length) followed by LE32(crc32c of those bytes) into
 * dst (dst may not alias data; data is const and may be a shared per-peer
 * buffer, see /root/reference/src/lnl/net_peer.cpp:482, :575).  Returns the
 * new length (length + 4) or a negative code if dst_cap is too small. */
int64_t lnl_crc32c_layer_outbound(const uint8_t* data, size_t offset, size_t length,
                                  uint8_t* dst, size_t dst_cap);

/* Inbound layer step (upstream Crc32cLayer.ProcessInboundPacket): returns the
 * payload length (length - 4) if length >= 5 and the trailing LE32 matches the
 * CRC-32C of the preceding bytes, else -1 (drop silently: a checksum failure
 * looks like packet loss to the reliability layer). */
int64_t lnl_crc32c_layer_inbound(const uint8_t* data, size_t length);

/* net_packet::verify() (/root/reference/include/lnl/net_packet.h:120-131) of a
 * packet data[0..size) after the layer has stripped its CRC: 1 if the property
 * (data[0] & 0x1F) is a known one and size covers its header (plus the 6-byte
 * fragment header when data[0] & 0x80), else 0.  size 0 gives 0. */
int lnl_packet_verify(const uint8_t* data, size_t size);

/* The whole inbound acceptance test of one wire datagram, as net_manager would
 * apply it with the layer on (receive_logic :218-222, then
 * on_message_received :343): LNL_INBOUND_DROP_CRC (length < 5 or CRC
 * mismatch), LNL_INBOUND_MALFORMED (CRC fine, verify() fails) or
 * LNL_INBOUND_ACCEPT (strip 4 bytes and dispatch). */
#define LNL_INBOUND_DROP_CRC 0
#define LNL_INBOUND_ACCEPT 1
#define LNL_INBOUND_MALFORMED 2
int lnl_inbound_status(const uint8_t* data, size_t length);

/* ---- batched GPU path (gfx950 kernels) ----------------------------------- */

/* out[i] = CRC32C(d_base + i*stride, len), i < n.  stride >= len. */
int lnl_crc32c_batch_fixed_dev(const uint8_t* d_base, size_t stride, uint32_t len,
                               uint32_t n, uint32_t* d_out, void* hip_stream);

/* out[i] = CRC32C(d_base + d_off[i], d_off[i+1] - d_off[i]), i < n.
 * d_off holds n+1 non-decreasing byte offsets; any byte alignment. */
int lnl_crc32c_batch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                             uint32_t* d_out, void* hip_stream);

/* Batched outbound layer (the send side over a CSR burst): datagram i,
 * d_base[d_off[i] .. d_off[i+1]), goes to d_dst + (d_off[i] - d_off[0]) + 4 i
 * as payload || LE32(CRC32C(payload)) -- the bytes lnl_crc32c_layer_outbound
 * gives for it -- so the wire burst is back to back, d_off[n] - d_off[0] + 4 n
 * bytes.  d_crc (optional, may be NULL) also receives the CRCs.  d_dst must not
 * overlap the source bytes.  Stream-ordered; returns 0 or a negative errno. */
int lnl_crc32c_append_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, uint8_t* d_dst,
                              uint32_t* d_crc, void* hip_stream);

/* Batched inbound verification (the layer's receive side over a CSR batch of
 * whole datagrams, trailing LE32 CRC included): d_ok[i] = 1 if datagram i has
 * length >= 5 and its trailing CRC matches, else 0.  d_crc (optional, may be
 * NULL) receives the CRC computed over the first length-4 bytes. */
int lnl_crc32c_verify_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                              uint8_t* d_ok, uint32_t* d_crc, void* hip_stream);

/* Batched inbound filter: lnl_inbound_status of every
 * datagram of a CSR batch of wire datagrams, in one pass -- d_status[i] is
 * LNL_INBOUND_DROP_CRC, LNL_INBOUND_ACCEPT or LNL_INBOUND_MALFORMED. */
int lnl_inbound_filter_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                               uint8_t* d_status, void* hip_stream);

/* Host-resident batch (the socket path): copies h_base/h_off to `device`
 * in chunks over LNL_HOST_DEFAULT_STREAMS HIP streams (H2D -> kernel -> D2H
 * overlapped; lnl_crc32c_batch_host_ex below sets the count), writes
 * h_out[i], blocks until done.  h_off as in batch_csr_dev (h_off[0] may be
 * nonzero).  Pinned (hipHostMalloc / hipHostRegister) buffers give the full
 * PCIe rate; pageable ones work but copy through a staging buffer.  (A
 * pageable h_out -- CRCs here, statuses for lnl_inbound_filter_host, h_crc for
 * lnl_crc32c_append_host -- goes through the library's own pinned staging,
 * chunk by chunk, so it does not slow the pipeline.) */
int lnl_crc32c_batch_host(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                          uint32_t* h_out, int device);

/* The packets a filtered burst delivers: for every
 * datagram with d_status[i] == LNL_INBOUND_ACCEPT, either the datagram itself
 * without its CRC, or -- for a MERGED container (property 12) -- the packets
 * it carries, cut as net_peer::process_packet does
 * (/root/reference/src/lnl/net_peer.cpp:164-187: [u16 LE size][packet]...,
 * stopping at the first packet net_packet::verify rejects or that runs past
 * the datagram; lnl_dispatch_csr_dev_ex below can walk as the reference's
 * own buffer does instead).  Packet k: base[d_pkt_start[k] .. + d_pkt_len[k])
 * from datagram d_pkt_parent[k], in datagram order.  *d_total (device)
 * receives the number of packets; only the first `cap` are written.
 * Stream-ordered. */
int lnl_dispatch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, const uint8_t* d_status,
                         uint64_t* d_pkt_start, uint32_t* d_pkt_len, uint32_t* d_pkt_parent, uint32_t cap,
                         uint32_t* d_total, void* hip_stream);

/* lnl_inbound_filter_csr_dev followed by lnl_dispatch_csr_dev, same outputs
 * (d_status[i] for every datagram, then the delivered packets), with the
 * MERGED walk done in the filter's pass over the bytes: the dispatch step
 * reads no datagram bytes again for batches the span path takes.  This is
 * the receive_logic -> process_packet chain (net_manager.cpp:218-222 -> :343
 * -> net_peer.cpp:164-187) for a whole burst.  Stream-ordered. */
int lnl_inbound_filter_dispatch_csr_dev(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                        uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                        uint32_t* d_pkt_parent, uint32_t cap, uint32_t* d_total,
                                        void* hip_stream);

/* Where the MERGED walk may read (lnl_dispatch_opts.tail).  The reference
 * bounds its walk by the received packet's buffer capacity, not by the
 * datagram (/root/reference/src/lnl/net_peer.cpp:167-183, buffer_size() at
 * :171), and that buffer is always a fresh zero-filled 2048-byte one
 * (net_packet() -> ensure(1432), include/lnl/net_packet.h:46-49, 194-208;
 * pool_recycle deletes every buffer over MAX_PACKET_SIZE,
 * src/lnl/net_manager.cpp:290-292).  So a size field in a container's last
 * byte, or an entry that runs past the datagram, is cut from the bytes after
 * it, and the reference delivers a zero-padded packet.
 *   LNL_DISPATCH_TAIL_DATAGRAM  stop at the datagram's end (the default of
 *                               lnl_dispatch_csr_dev; identical for every
 *                               container net_peer::send_merged builds)
 *   LNL_DISPATCH_TAIL_ZERO      the reference handed the stripped datagram:
 *                               zeros right after it, the walk bounded by the
 *                               2048-byte capacity
 *   LNL_DISPATCH_TAIL_LAYER     the reference with INTEGRATION.md's
 *                               receive_logic edit: the layer shrinks the
 *                               packet, so the 4 stripped CRC bytes stay in
 *                               the buffer after it, then zeros
 * Under the two tail rules a packet may extend past the bytes its datagram
 * holds: d_pkt_len[k] is the reference's length, d_pkt_avail[k] (optional)
 * how many of its bytes, from d_pkt_start[k], are the wire burst's (the
 * datagram, or the datagram and its CRC field); the caller zero-fills the
 * remaining d_pkt_len[k] - d_pkt_avail[k].  (Under the datagram rule
 * d_pkt_avail[k] == d_pkt_len[k].)  A nested container is one packet under
 * every rule: the caller's process_packet cuts it again (with a zero tail, as
 * the reference's fresh pool packet has). */
#define LNL_DISPATCH_TAIL_DATAGRAM 0
#define LNL_DISPATCH_TAIL_ZERO 1
#define LNL_DISPATCH_TAIL_LAYER 2
typedef struct lnl_dispatch_opts {
    uint32_t size;        /* sizeof(lnl_dispatch_opts) */
    uint32_t tail;        /* LNL_DISPATCH_TAIL_* */
    uint32_t reserved[2]; /* 0 */
} lnl_dispatch_opts;

/* lnl_dispatch_csr_dev / lnl_inbound_filter_dispatch_csr_dev with options
 * (opts NULL: the datagram rule) and the per-packet in-burst byte counts
 * (d_pkt_avail, cap entries, may be NULL).  -EINVAL for a bad size, tail or
 * reserved field. */
int lnl_dispatch_csr_dev_ex(const uint8_t* d_base, const uint64_t* d_off, uint32_t n, const uint8_t* d_status,
                            uint64_t* d_pkt_start, uint32_t* d_pkt_len, uint32_t* d_pkt_parent,
                            uint32_t* d_pkt_avail, uint32_t cap, uint32_t* d_total, const lnl_dispatch_opts* opts,
                            void* hip_stream);
int lnl_inbound_filter_dispatch_csr_dev_ex(const uint8_t* d_base, const uint64_t* d_off, uint32_t n,
                                           uint8_t* d_status, uint64_t* d_pkt_start, uint32_t* d_pkt_len,
                                           uint32_t* d_pkt_parent, uint32_t* d_pkt_avail, uint32_t cap,
                                           uint32_t* d_total, const lnl_dispatch_opts* opts, void* hip_stream);

/* Upstream LiteNetLib's XOR-encryption layer (XorEncryptLayer; SURVEY.md 8(f)
 * item 4), in place: data[i] ^= key[i % key_len] for i < length, the key phase
 * restarting at every datagram.  Both directions are the same map; the layer
 * adds no bytes.  key_len 1 .. LNL_XOR_MAX_KEY. */
#define LNL_XOR_MAX_KEY 256
int lnl_xor_layer(uint8_t* data, size_t length, const uint8_t* key, size_t key_len);
/* The same over every datagram of a device batch (stream-ordered). */
int lnl_xor_layer_csr_dev(uint8_t* d_base, const uint64_t* d_off, uint32_t n, const uint8_t* key,
                          size_t key_len, void* hip_stream);
int lnl_xor_layer_fixed_dev(uint8_t* d_base, size_t stride, uint32_t len, uint32_t n, const uint8_t* key,
                            size_t key_len, void* hip_stream);

/* Host-resident inbound filter (lnl_inbound_filter_csr_dev over a pinned host
 * burst, the same chunked pipeline as lnl_crc32c_batch_host): writes
 * h_status[i] (LNL_INBOUND_*), blocks until done. */
int lnl_inbound_filter_host(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                            uint8_t* h_status, int device);

/* Batched socket ingress (CPU): one recvmmsg call pulls up to max_n datagrams
 * from the UDP socket fd into LNL_INGRESS_SLOT-byte slots of buf (cap bytes;
 * pinned memory for the GPU batch that follows), then compacts them in place
 * to a CSR burst: datagram i = buf[off[i] .. off[i+1]), off[0] = 0 (off has
 * max_n + 1 entries).  addrs (optional) receives max_n struct sockaddr_in
 * senders.  wait_ms != 0 polls first (-1: forever), like the reference's
 * receive loop (/root/reference/src/lnl/net_manager.cpp:202-223); 0 never
 * blocks.  Returns the number of datagrams (0: none ready), or a negative
 * errno.  Longer datagrams are truncated to the slot, as recvfrom into the
 * reference's MAX_PACKET_SIZE packet truncates them. */
#define LNL_INGRESS_SLOT 1432
int lnl_ingress_recv_batch(int fd, uint8_t* buf, size_t cap, uint64_t* off, uint32_t max_n, void* addrs,
                           int wait_ms);

/* Host-resident outbound layer (the send side of the socket path; SURVEY.md
 * 8(f) item 2): the payload burst, datagram i = h_payload[h_off[i] ..
 * h_off[i+1]) as in lnl_crc32c_batch_host (pinned
 * memory gives the full PCIe rate) goes H2D in chunks over four HIP streams,
 * through lnl_crc32c_append_csr_dev on `device`, and back D2H as the wire
 * burst: datagram i at h_wire + (h_off[i] - h_off[0]) + 4 i as
 * payload || LE32(CRC32C(payload)) -- the bytes lnl_crc32c_layer_outbound
 * gives for it, back to back (h_off[n] - h_off[0] + 4 n bytes; its offsets are
 * h_off[i] - h_off[0] + 4 i).  h_crc (optional, may be NULL) receives the
 * CRCs.  h_wire must not overlap h_payload.  Blocks until done.  This is
 * net_manager::send_raw's layer step for a whole burst
 * (/root/reference/src/lnl/net_manager.cpp:515-521). */
int lnl_crc32c_append_host(const uint8_t* h_payload, const uint64_t* h_off, uint32_t n, uint8_t* h_wire,
                           uint32_t* h_crc, int device);

/* Batched socket egress (CPU): sendmmsg of the wire
 * burst's datagrams -- datagram i = wire[off[i] .. off[i+1]), the CSR layout
 * lnl_ingress_recv_batch produces (for lnl_crc32c_append_host's wire burst,
 * off[i] = h_off[i] - h_off[0] + 4 i) -- in calls of up to 1024, replacing
 * one sendto per datagram
 * (/root/reference/src/lnl/net_manager.cpp:515-523).  addrs: NULL for a
 * connected socket, else naddrs (1: one endpoint for all, or n: one per
 * datagram) struct sockaddr_in.  status (optional, n entries) receives, for
 * every datagram attempted, the bytes sent or a negative errno for a datagram
 * the kernel refused (send_raw's error case, :525-567, ENOBUFS included; the
 * burst goes on).  When the socket buffer is full (EAGAIN), wait_ms > 0 polls
 * for room until one deadline wait_ms after the call started, -1 polls
 * without a deadline, and 0 returns at once.  Returns the number of datagrams attempted, from the
 * front (the rest were not: buffer full and the wait expired), or a negative
 * errno when the call itself is invalid (bad fd, arguments). */
int64_t lnl_egress_send_batch(int fd, const uint8_t* wire, const uint64_t* off, uint32_t n, const void* addrs,
                              uint32_t naddrs, int64_t* status, int wait_ms);

/* Multi-device form of lnl_crc32c_batch_host: the batch
 * is split into ndev contiguous datagram ranges of ceil(n / ndev) (the last
 * possibly shorter or empty), range r runs on devices[r] through
 * lnl_crc32c_batch_host on its own host thread, all ranges concurrently; no
 * data crosses between devices.  Blocks until every range is done.  A device
 * may appear more than once (its ranges then run one after the other).
 * Returns 0, or the first failing range's code (message via
 * lnl_crc32c_last_error on the calling thread). */
int lnl_crc32c_batch_host_multi(const uint8_t* h_base, const uint64_t* h_off, uint32_t n,
                                uint32_t* h_out, const int* devices, int ndev);

/* ---- host pipelines with explicit options -------------------------------- */

/* Options of the host-resident pipelines (lnl_crc32c_batch_host,
 * lnl_inbound_filter_host, lnl_crc32c_append_host take the defaults).  A zero
 * field takes its default; `size` must be sizeof(lnl_host_opts) (a larger
 * struct from a newer header is accepted, its extra fields ignored).
 *   streams          HIP streams the chunks go round-robin over, each with its
 *                    own device staging slot: 1 .. LNL_HOST_MAX_STREAMS
 *                    (default LNL_HOST_DEFAULT_STREAMS).  Two is BASELINE
 *                    config 5 ("overlapped on 2 HIP streams"); with two, a
 *                    stream's next H2D waits behind its own D2H, which costs
 *                    the send side (a D2H as large as its H2D), not the CRC
 *                    and filter paths.
 *   chunk_datagrams  datagrams per chunk at most (default 65536)
 *   chunk_bytes      bytes per chunk at most (default 64 MiB; a single longer
 *                    datagram gets a chunk of its own) */
#define LNL_HOST_MAX_STREAMS 8
#define LNL_HOST_DEFAULT_STREAMS 4
typedef struct lnl_host_opts {
    uint32_t size;
    uint32_t streams;
    uint32_t chunk_datagrams;
    uint32_t reserved; /* 0 */
    uint64_t chunk_bytes;
} lnl_host_opts;

/* lnl_crc32c_batch_host / lnl_inbound_filter_host / lnl_crc32c_append_host
 * with options (opts may be NULL: every default).  -EINVAL for a bad size,
 * streams > LNL_HOST_MAX_STREAMS or a nonzero reserved field. */
int lnl_crc32c_batch_host_ex(const uint8_t* h_base, const uint64_t* h_off, uint32_t n, uint32_t* h_out,
                             int device, const lnl_host_opts* opts);
int lnl_inbound_filter_host_ex(const uint8_t* h_base, const uint64_t* h_off, uint32_t n, uint8_t* h_status,
                               int device, const lnl_host_opts* opts);
int lnl_crc32c_append_host_ex(const uint8_t* h_payload, const uint64_t* h_off, uint32_t n, uint8_t* h_wire,
                              uint32_t* h_crc, int device, const lnl_host_opts* opts);

/* ---- misc ---------------------------------------------------------------- */

/* Releases the device scratch the library keeps for `hip_stream` on the
 * current device (the CSR span path's control and exchange blocks, the XOR
 * chunk map), stream-ordered.  Call it before destroying a stream the batch
 * entry points were given; the library also bounds what it keeps (the least
 * recently used streams' scratch is freed beyond LNL_STREAM_CACHE per device,
 * stream-ordered behind its last use; an entry last used while at most
 * LNL_STREAM_CACHE / 2 streams held scratch is freed after a device
 * synchronise).
 * Returns 0 (also when nothing was kept for the stream). */
#define LNL_STREAM_CACHE 32
int lnl_stream_release(void* hip_stream);

/* Diagnostics (tests): fills every wave-batch exchange arrival word of the span
 * scratch kept for `hip_stream` with `value`, as an aborted call could leave
 * it.  Synchronises the stream first; blocking.  -ENOENT when no CSR call has
 * run on the stream yet; -EINVAL (nothing written) for a value no earlier call
 * could have left: an epoch (value >> 2) past the calls made on the stream.
 * Later calls must be unaffected (the arrival words pair by per-call epoch,
 * crc32c_span.h). */
int lnl_diag_fill_span_arrivals(void* hip_stream, uint64_t value);

/* Message for the last failure on the calling thread ("" if none). */
const char* lnl_crc32c_last_error(void);

/* LNL_CRC32C_ABI_VERSION of the loaded library. */
int lnl_crc32c_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LNL_CRC32C_H */
