// lnl_dispatch.hip -- the packets a filtered burst delivers (SURVEY.md 8(f)
// item 3): every accepted datagram is one packet (its CRC stripped), except a
// MERGED container, which is cut into the packets it carries.
//
// The container walk restates net_peer::process_packet's MERGED case
// (/root/reference/src/lnl/net_peer.cpp:164-187), the sender side being
// net_peer::send_user_data / send_merged (:446-486): after the 1-byte header,
// [u16 LE size][packet of `size` bytes] repeated; each packet must pass
// net_packet::verify() (lnl_packet.h) or the walk stops there.
//
//   pos = HEADER_SIZE (1)
//   while pos < size:
//       if pos + 2 > size: stop                       (*)
//       L = u16 at pos; pos += 2
//       if L > size - pos: stop                       (*)
//       if !verify(packet[pos .. pos+L)): stop         (L = 0 fails: no header byte)
//       emit [pos, pos+L); pos += L
//
// (*) The default rule (LNL_DISPATCH_TAIL_DATAGRAM).  The reference bounds
// its walk by the pooled buffer's capacity instead (net_peer.cpp:171,
// buffer_size()), and that buffer is deterministic: every received packet is
// a fresh net_packet() -- ensure(1432) zero-fills 2048 bytes
// (net_packet.h:46-49, 194-208) -- because pool_recycle deletes any packet
// whose buffer exceeds MAX_PACKET_SIZE (net_manager.cpp:290-292), which is
// every one.  So past the datagram it reads zeros (or, with the layer's
// receive_logic edit of INTEGRATION.md, the 4 stripped CRC bytes and then
// zeros) and delivers zero-padded packets.  The tail modes reproduce that:
//
//   pos = 1
//   while pos < size:
//       L = u16 at pos (tail bytes past the datagram); pos += 2
//       if cap - pos < L: stop                        (cap = 2048)
//       if !verify(tail byte at pos, L): stop
//       emit [pos, pos+L) with avail = the bytes of it inside the datagram
//       (+ the CRC field, LNL_DISPATCH_TAIL_LAYER); pos += L
//
// Well-formed containers -- all send_merged produces -- split identically
// under every rule.
//
// A nested container is delivered as one packet (the reference's
// process_packet would cut it again); send_merged never nests.
//
// Two launches: walk and count the packets of every datagram (recording the
// first kDispatchRec), then emit them in datagram order from the records.  A
// walk step is one dependent round trip to a random 64-B sector, so walking
// each container once (not once per pass) halves the latency-bound part of
// the call.  The emit pass finds datagram i's first output slot itself: the
// counting pass leaves each workgroup's packet total, and an emit workgroup
// adds up its predecessors' totals (at most kDispatchPrefixWgs of them, read
// from L2) and scans its own counts.  Larger batches run a hipCUB exclusive
// scan of the counts between the two launches instead.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "crc32c_kernels.h"
#include "crc32c_span.h"
#include "lnl_packet.h"

#ifndef LNL_EXPERIMENTS
#define LNL_EXPERIMENTS 0
#endif

namespace lnl {

namespace {

constexpr uint32_t kMergedProperty = 12;  // PACKET_PROPERTY::MERGED, net_enums.h:60

// Bytes q[0..2] (u16 LE size, then the packet's header byte) with two aligned
// dword loads instead of three byte loads.  Safe whenever q[0..1] lie inside
// the datagram: the walk only reads at pos with pos + 2 <= size, and the wire
// datagram carries 4 more CRC bytes, so both dwords hold at least one byte of
// the batch and never touch another page.
__device__ inline uint32_t load3(const uint8_t* q) {
    const uintptr_t a = (uintptr_t)q;
    const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return (uint32_t)(v >> ((a & 3u) * 8u));
}

// Bytes pos .. pos + 2 of a datagram of `size` bytes (CRC stripped) under a
// tail rule: the datagram's own bytes below lim (size, or size + 4 with the
// CRC field), zeros from there on.  Only the first byte of each lies past
// the wire datagram: byte loads, so nothing outside the batch is touched.
__device__ inline uint32_t tail_load3(const uint8_t* p, uint32_t pos, uint32_t size, uint32_t lim) {
    if (pos + 3u <= size) return load3(p + pos);
    uint32_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 3u; ++j)
        if (pos + j < lim) v |= (uint32_t)p[pos + j] << (8u * j);
    return v;
}

// Walk datagram i; for each delivered packet call emit(start, len) (start
// relative to the datagram).  Returns the number of packets.
template <typename F>
__device__ inline uint32_t walk(const DispatchArgs& a, uint64_t s, uint32_t size, F&& emit) {
    const uint8_t* p = a.base + s;
    // the header byte and the first entry of a container share a round trip
    uint32_t v = size >= 3u ? load3(p + 1) : 0u;
    if ((p[0] & 0x1Fu) != kMergedProperty) {
        emit(0u, size);
        return 1;
    }
    uint32_t pos = 1, c = 0;
    if (a.tail) {  // the reference's buffer: capacity-bounded, tail bytes past the datagram
        const uint32_t lim = size + (a.tail == kDispatchTailLayer ? 4u : 0u);
        const uint32_t cap = dispatch_ref_capacity(size + 4u);
        while (pos < size) {
            v = tail_load3(p, pos, size, lim);
            const uint32_t L = v & 0xFFFFu;
            pos += 2;
            if (cap - pos < L) break;
            if (L == 0u || !lnl_packet_verify_hdr((uint8_t)(v >> 16), L)) break;
            emit(pos, L);
            pos += L;
            ++c;
        }
        return c;
    }
    while (pos < size) {
        if (pos + 2u > size) break;
        if (pos != 1u) v = load3(p + pos);
        const uint32_t L = v & 0xFFFFu;
        pos += 2;
        if (L > size - pos) break;
        if (L == 0u || !lnl_packet_verify_hdr((uint8_t)(v >> 16), L)) break;
        emit(pos, L);
        pos += L;
        ++c;
    }
    return c;
}

// Sum of v over the 256-thread workgroup (every thread calls it; uses a
// barrier).
__device__ inline uint32_t block_sum(uint32_t v, uint32_t* s_part) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    if (lane == 0u) s_part[w] = v;
    __syncthreads();
    return s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// Pass 1: walk every accepted datagram once; count its packets and keep the
// first kDispatchRec as (pos << 16 | len) records, slot-major so a wave's
// stores are coalesced.
__global__ __launch_bounds__(256) void dispatch_count_kernel(DispatchArgs a) {
    __shared__ uint32_t s_part[4];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    uint32_t c = 0;
    if (i < a.n) {
        const uint8_t st = a.status[i];  // issued together with the offsets
        const uint64_t o0 = a.off[i], o1 = a.off[i + 1];
        if (st == 1u) {  // LNL_INBOUND_ACCEPT only
            const uint64_t s = o0 - a.off0;
            const uint32_t size = (uint32_t)(o1 - o0) - 4u;  // CRC stripped
            uint32_t k = 0;
            c = walk(a, s, size, [&](uint32_t pos, uint32_t len) {
                if (k < kDispatchRec) a.rec[(size_t)k * a.n + i] = (pos << 16) | len;
                ++k;
            });
        }
        a.counts[i] = c;
    }
    if (a.wgsum) {
        const uint32_t t = block_sum(c, s_part);
        if (threadIdx.x == 0u) a.wgsum[blockIdx.x] = t;
    }
}

// Pass 1 of the fused path: the span kernel left one block per datagram
// ([count, records 0 .. 6], written by the lane that owns the datagram; a
// block per datagram keeps those scattered writes to one 32-byte sector).
// Keep the counts of accepted datagrams, zero the rest, move the records to
// the slot-major layout the emit pass reads (coalesced here), and walk again
// what a block cannot hold (8 or more packets) or what the span kernel did not
// see (a batch it does not take: its control block says so).
__global__ __launch_bounds__(256) void dispatch_fix_kernel(DispatchArgs a) {
    __shared__ uint32_t s_part[4];
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint8_t st = i < a.n ? a.status[i] : 0u;
    uint32_t c = 0;
    if (st == 1u) {
        const bool walked = a.span_ctl[2] != 0u;  // (written by the span kernel of this call)
        const uint4* blk = reinterpret_cast<const uint4*>(a.blk + (size_t)i * kWalkBlock);
        const uint4 b0 = walked ? blk[0] : make_uint4(kWalkBlock, 0u, 0u, 0u);
        c = b0.x;
        bool again = c >= kWalkBlock && c != kWalkPlain;
        if (c == kWalkPlain) {  // the datagram itself, CRC stripped
            a.rec[i] = (uint32_t)(a.off[i + 1] - a.off[i]) - 4u;
            c = 1;
        } else if (c < kWalkBlock) {
            const uint4 b1 = blk[1];
            const uint32_t r[7] = {b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            // the span kernel walks by the datagram rule; under a tail rule a
            // container it stopped short of its end may read on past it, so
            // that one is walked again here (well-formed ones end exactly)
            if (a.tail) {
                uint32_t last = 0;
#pragma unroll
                for (uint32_t k = 0; k < 7; ++k)
                    if (k + 1u == c) last = r[k];
                const uint32_t next = c ? (last >> 16) + (last & 0xFFFFu) : 1u;
                again = next < (uint32_t)(a.off[i + 1] - a.off[i]) - 4u;
            }
            if (!again) {
#pragma unroll
                for (uint32_t k = 0; k < 7; ++k)
                    if (k < c) a.rec[(size_t)k * a.n + i] = r[k];
            }
        }
        if (again) {
            const uint64_t o0 = a.off[i], o1 = a.off[i + 1];
            const uint32_t size = (uint32_t)(o1 - o0) - 4u;
            uint32_t k = 0;
            c = walk(a, o0 - a.off0, size, [&](uint32_t pos, uint32_t len) {
                if (k < kDispatchRec) a.rec[(size_t)k * a.n + i] = (pos << 16) | len;
                ++k;
            });
        }
    }
    if (i < a.n) a.counts[i] = c;
    if (a.wgsum) {
        const uint32_t t = block_sum(c, s_part);
        if (threadIdx.x == 0u) a.wgsum[blockIdx.x] = t;
    }
}

// Pass 2: datagram i's packets go to [first[i], first[i] + counts[i]).  A
// wave owns 64 consecutive datagrams, whose packets form one contiguous range
// of the output.  Datagrams whose packets all sit in pass 1's records (at most
// kDispatchRec, positions < 64 KiB) are written cooperatively: lane l takes
// packet F0 + l + 64t, finds its datagram by binary search over the wave's
// `first` values in LDS, and the stores of consecutive lanes are consecutive.
// Longer containers are walked again by their own lane.
constexpr uint32_t kEmitMaxSteps = 16;  // cooperative only while the range is <= 16 x 64 packets

// packet bytes [pos, pos + len) of a datagram whose own bytes end at lim
__device__ inline uint32_t pkt_avail(uint32_t pos, uint32_t len, uint32_t lim) {
    const uint32_t in = lim > pos ? lim - pos : 0u;
    return in < len ? in : len;
}

__global__ __launch_bounds__(256) void dispatch_emit_kernel(DispatchArgs a) {
    __shared__ uint32_t s_first[4][65];
    __shared__ uint32_t s_fast[4][64];
    __shared__ uint32_t s_lim[4][64];
    __shared__ uint64_t s_start[4][64];
    __shared__ uint32_t s_rec[4][kDispatchRec][64];
    __shared__ uint32_t s_part[4], s_wsum[4];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t i0 = blockIdx.x * 256u + w * 64u;
    const uint32_t i = i0 + lane;
    uint32_t c = 0, f = 0, size = 0;
    uint64_t s = 0;
    if (a.wgsum) {
        // first slot = the predecessors' totals + this workgroup's scan
        uint32_t pre = 0;  // (8 loads in flight per thread: <= 4 round trips for 8192 workgroups)
        for (uint32_t t = threadIdx.x; t < blockIdx.x; t += 8u * 256u) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t j = 0; j < 8u; ++j) v[j] = t + 256u * j < blockIdx.x ? a.wgsum[t + 256u * j] : 0u;
#pragma unroll
            for (uint32_t j = 0; j < 8u; ++j) pre += v[j];
        }
        c = i < a.n ? a.counts[i] : 0u;
        uint32_t incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= (uint32_t)d) incl += o;
        }
        if (lane == 63u) s_wsum[w] = incl;
        pre = block_sum(pre, s_part);  // (its barrier also publishes s_wsum)
        for (uint32_t v = 0; v < w; ++v) pre += s_wsum[v];
        f = pre + incl - c;  // lanes past n: c = 0, f = the total
        if (i < a.n) {
            if (i + 1u == a.n) *a.total = f + c;
            s = a.off[i] - a.off0;
            if (c) size = (uint32_t)(a.off[i + 1] - a.off[i]) - 4u;
        }
    } else if (i < a.n) {
        c = a.counts[i];
        f = a.first[i];
        if (i + 1u == a.n) *a.total = f + c;
        s = a.off[i] - a.off0;
        if (c) size = (uint32_t)(a.off[i + 1] - a.off[i]) - 4u;
    } else if (i0 < a.n) {
        f = a.first[a.n - 1] + a.counts[a.n - 1];  // past the end: empty, first = total
    }
    // (positions are 16-bit in the records: a tail walk's reach past its
    // datagram stays below size + 2)
    const bool fast = c <= kDispatchRec && size < 65534u;
    // bytes of the datagram a packet may take as its own: the rest of a
    // packet cut under a tail rule is the caller's zero fill (pkt_avail)
    const uint32_t lim = a.tail ? size + (a.tail == kDispatchTailLayer ? 4u : 0u) : 0xFFFFFFFFu;
    s_first[w][lane] = f;
    if (lane == 63u) s_first[w][64] = f + c;
    s_fast[w][lane] = fast;
    s_start[w][lane] = s;
    s_lim[w][lane] = lim;
    for (uint32_t k = 0; k < kDispatchRec; ++k)
        if (fast && k < c) s_rec[w][k][lane] = a.rec[(size_t)k * a.n + i];
    __syncthreads();
    if (i0 >= a.n) return;
    const uint32_t F0 = s_first[w][0], F1 = s_first[w][64];
    const bool coop = F1 - F0 <= kEmitMaxSteps * 64u;
    if (coop) {
        const uint32_t end = F1 < a.cap ? F1 : a.cap;
        for (uint32_t j = F0 + lane; j < end; j += 64u) {
            uint32_t lo = 0;  // last datagram d of the wave with first[d] <= j
            for (uint32_t step = 32; step; step >>= 1)
                if (s_first[w][lo + step] <= j && lo + step < 64u) lo += step;
            if (!s_fast[w][lo]) continue;
            const uint32_t r = s_rec[w][j - s_first[w][lo]][lo];
            if (a.nt) {
                __builtin_nontemporal_store(s_start[w][lo] + (r >> 16), a.pkt_start + j);
                __builtin_nontemporal_store(r & 0xFFFFu, a.pkt_len + j);
                __builtin_nontemporal_store(i0 + lo, a.pkt_parent + j);
            } else {
                a.pkt_start[j] = s_start[w][lo] + (r >> 16);
                a.pkt_len[j] = r & 0xFFFFu;
                a.pkt_parent[j] = i0 + lo;
            }
            if (a.pkt_avail) a.pkt_avail[j] = pkt_avail(r >> 16, r & 0xFFFFu, s_lim[w][lo]);
        }
    }
    if (c == 0u || f >= a.cap || (coop && fast)) return;
    auto put = [&](uint32_t k, uint32_t pos, uint32_t len) {
        if (f + k < a.cap) {
            a.pkt_start[f + k] = s + pos;
            a.pkt_len[f + k] = len;
            a.pkt_parent[f + k] = i;
            if (a.pkt_avail) a.pkt_avail[f + k] = pkt_avail(pos, len, lim);
        }
    };
    if (fast) {
        for (uint32_t k = 0; k < c; ++k) {
            const uint32_t r = s_rec[w][k][lane];
            put(k, r >> 16, r & 0xFFFFu);
        }
    } else {
        uint32_t k = 0;
        walk(a, s, size, [&](uint32_t pos, uint32_t len) { put(k++, pos, len); });
    }
}

#if LNL_EXPERIMENTS
// One pass (experiments build only, LNL_DISPATCH_ONEPASS=1): walk, count and write in one launch.  The workgroup's
// packet offset comes from a decoupled look-back over per-workgroup flags
// (a.look[b] = flag << 32 | value; flag 1: this workgroup's own count,
// 2: inclusive prefix), so there is no device-wide scan launch and the
// records never leave the chip.  Wave 0 reads 64 predecessors' flags per
// round trip and stops at the nearest inclusive prefix.  Workgroups are
// dispatched in order, so a predecessor a workgroup waits on is resident or
// done; the spin is bounded anyway, and a timeout reports total = 0xFFFFFFFF
// instead of hanging.
constexpr uint32_t kLookSpin = 1u << 22;

__device__ inline uint64_t look_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void look_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void dispatch_onepass_kernel(DispatchArgs a) {
    __shared__ uint32_t s_first[4][65];
    __shared__ uint32_t s_fast[4][64];
    __shared__ uint64_t s_start[4][64];
    __shared__ uint32_t s_rec[4][kDispatchRec][64];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_prefix, s_bad;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t i0 = blockIdx.x * 256u + w * 64u;
    const uint32_t i = i0 + lane;
    uint32_t c = 0, size = 0;
    uint64_t s = 0;
    if (i < a.n) {
        const uint8_t st = a.status[i];
        const uint64_t o0 = a.off[i], o1 = a.off[i + 1];
        s = o0 - a.off0;
        if (st == 1u) {  // LNL_INBOUND_ACCEPT only
            size = (uint32_t)(o1 - o0) - 4u;  // CRC stripped
            uint32_t k = 0;
            c = walk(a, s, size, [&](uint32_t pos, uint32_t len) {
                if (k < kDispatchRec) s_rec[w][k][lane] = (pos << 16) | len;
                ++k;
            });
        }
    }
    const bool fast = c <= kDispatchRec && size < 65536u;
    // workgroup scan of the counts: waves by shuffles, then the 4 wave sums
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
    if (lane == 63u) s_wsum[w] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (uint32_t v = 0; v < 4u; ++v) {
        wbase += v < w ? s_wsum[v] : 0u;
        total += s_wsum[v];
    }
    if (w == 0u) {  // wave 0 looks back 64 predecessors per round trip
        const uint32_t b = blockIdx.x;
        uint32_t prefix = 0, bad = 0;
        if (b == 0) {
            if (lane == 0u) look_store(&a.look[0], (2ull << 32) | total);
        } else {
            if (lane == 0u) look_store(&a.look[b], (1ull << 32) | total);
            int64_t j = (int64_t)b - 1;
            uint32_t spin = 0;
            while (true) {
                const int64_t idx = j - (int64_t)lane;
                const uint64_t v = idx >= 0 ? look_load(&a.look[idx]) : (2ull << 32);  // before 0: prefix 0
                const uint32_t flag = (uint32_t)(v >> 32);
                const uint64_t m2 = __ballot(flag == 2u), m0 = __ballot(flag == 0u);
                const uint32_t first2 = m2 ? (uint32_t)__builtin_ctzll(m2) : 64u;
                const uint64_t need = first2 >= 63u ? ~0ull : ((2ull << first2) - 1ull);
                if (m0 & need) {  // a predecessor this window needs has not published yet
                    if (++spin > kLookSpin) {
                        bad = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t part = lane <= first2 ? (uint32_t)v : 0u;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) part += (uint32_t)__shfl_xor((int)part, d, 64);
                prefix += part;
                if (first2 < 64u) break;
                j -= 64;
            }
            if (lane == 0u && !bad) look_store(&a.look[b], (2ull << 32) | (prefix + total));
        }
        if (lane == 0u) {
            s_prefix = prefix;
            s_bad = bad;
        }
    }
    __syncthreads();
    const uint32_t f = s_prefix + wbase + incl - c;  // first output slot of datagram i
    if (i + 1u == a.n) *a.total = s_bad ? 0xFFFFFFFFu : f + c;
    if (s_bad) return;
    // cooperative, coalesced write of the wave's packets (as dispatch_emit_kernel)
    s_first[w][lane] = f;  // lanes past n: c = 0, f = the running total
    if (lane == 63u) s_first[w][64] = f + c;
    s_fast[w][lane] = fast;
    s_start[w][lane] = s;
    __syncthreads();
    if (i0 >= a.n) return;
    const uint32_t F0 = s_first[w][0], F1 = s_first[w][64];
    const bool coop = F1 - F0 <= kEmitMaxSteps * 64u;
    if (coop) {
        const uint32_t end = F1 < a.cap ? F1 : a.cap;
        for (uint32_t j = F0 + lane; j < end; j += 64u) {
            uint32_t lo = 0;
            for (uint32_t step = 32; step; step >>= 1)
                if (s_first[w][lo + step] <= j && lo + step < 64u) lo += step;
            if (!s_fast[w][lo]) continue;
            const uint32_t r = s_rec[w][j - s_first[w][lo]][lo];
            if (a.nt) {
                __builtin_nontemporal_store(s_start[w][lo] + (r >> 16), a.pkt_start + j);
                __builtin_nontemporal_store(r & 0xFFFFu, a.pkt_len + j);
                __builtin_nontemporal_store(i0 + lo, a.pkt_parent + j);
            } else {
                a.pkt_start[j] = s_start[w][lo] + (r >> 16);
                a.pkt_len[j] = r & 0xFFFFu;
                a.pkt_parent[j] = i0 + lo;
            }
        }
    }
    if (c == 0u || f >= a.cap || (coop && fast)) return;
    auto put = [&](uint32_t k, uint32_t pos, uint32_t len) {
        if (f + k < a.cap) {
            a.pkt_start[f + k] = s + pos;
            a.pkt_len[f + k] = len;
            a.pkt_parent[f + k] = i;
        }
    };
    if (fast) {
        for (uint32_t k = 0; k < c; ++k) {
            const uint32_t r = s_rec[w][k][lane];
            put(k, r >> 16, r & 0xFFFFu);
        }
    } else {
        uint32_t k = 0;
        walk(a, s, size, [&](uint32_t pos, uint32_t len) { put(k++, pos, len); });
    }
}

#endif  // LNL_EXPERIMENTS

}  // namespace

size_t dispatch_scan_bytes(uint32_t n) {
    size_t bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n) !=
        hipSuccess)
        return 0;
    return bytes;
}

hipError_t launch_dispatch(const DispatchArgs& a, void* scan_tmp, size_t scan_bytes, hipStream_t stream) {
    const dim3 grid((a.n + 255u) / 256u);
    if (a.wgsum && grid.x > kDispatchPrefixWgs) return hipErrorInvalidValue;
#if LNL_EXPERIMENTS
    if (a.look) {  // one pass (flags zeroed by the caller; the datagram rule only)
        if (a.tail || a.pkt_avail) return hipErrorInvalidValue;
        hipLaunchKernelGGL(dispatch_onepass_kernel, grid, dim3(256), 0, stream, a);
        return hipGetLastError();
    }
#else
    if (a.look) return hipErrorInvalidValue;  // the one-pass form is not in the product build
#endif
    hipLaunchKernelGGL(dispatch_count_kernel, grid, dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (!a.wgsum) {
        e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, a.counts, a.first, (int)a.n, stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dispatch_emit_kernel, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_dispatch_walked(const DispatchArgs& a, void* scan_tmp, size_t scan_bytes, hipStream_t stream) {
    const dim3 grid((a.n + 255u) / 256u);
    if (a.wgsum && grid.x > kDispatchPrefixWgs) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dispatch_fix_kernel, grid, dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (!a.wgsum) {
        e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, a.counts, a.first, (int)a.n, stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dispatch_emit_kernel, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
