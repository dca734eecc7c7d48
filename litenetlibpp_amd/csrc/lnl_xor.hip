// lnl_xor.hip -- upstream LiteNetLib's XOR-encryption packet layer over a
// batch (unported by the reference, README.MD:35).
//
// Upstream XorEncryptLayer (C#, not available offline; restated):
// ExtraPacketSizeForLayer = 0, and both directions do, per datagram,
//
//   for i in 0 .. length-1:  data[offset + i] ^= key[i % key.Length]
//
// i.e. the key phase restarts at every datagram's first byte.  The batch form
// applies it in place to every datagram of a CSR or fixed-stride batch.
//
// HBM-bound byte map (reads and writes every datagram byte once): a group of
// 32 lanes owns a datagram and walks its 16-byte pieces (aligned to the
// buffer, so loads and stores are whole dwordx4, four per lane in flight,
// except the partial first and last piece of each datagram: their other bytes
// belong to the neighbouring datagrams, updated concurrently by other lanes,
// so those pieces are read whole and written back byte by byte, own bytes
// only.  One workgroup per 8 datagrams, no persistent cap.  Measured on the
// config-2 batch (tools/kvariants.py xor_*): 16 lanes / nt / 8 workgroups per
// CU 1.04 ms, default policy 0.81, 64 lanes x 2 pieces 0.67, 32 lanes x 4
// pieces uncapped 0.59 ms = 5.0 TB/s read + write; masked atomicXor per word
// for the edge pieces 1.73 ms.
//
// Key bytes come from LDS: four copies of the periodic key stream shifted by
// 0..3 bytes, so the 16 key bytes of any phase m are four aligned dword reads
// from copy m & 3.
//
// Fixed strides >= 16 over a 16-byte aligned base take the flat kernel below
// instead (whole pieces per lane, no shared edges): 0.502 ms on the config-2
// batch, 5.86 TB/s read + write, with 2 pieces in flight and nt loads/stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_kernels.h"

#ifndef LNL_EXPERIMENTS
#define LNL_EXPERIMENTS 0
#endif

namespace lnl {

namespace {

constexpr int kThreads = 256;
// build knobs (tools/kvariants.py): lanes per datagram (LNL_XOR_GROUP,
// crc32c_kernels.h), pieces per lane in flight, nt (1) or default (0) policy
// for the whole-piece loads and stores
#ifndef LNL_XOR_UNROLL
#define LNL_XOR_UNROLL 4
#endif
#ifndef LNL_XOR_NT
#define LNL_XOR_NT 0
#endif
constexpr int kGroup = LNL_XOR_GROUP;
constexpr int kUnroll = LNL_XOR_UNROLL;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kKeyWords = (kXorMaxKey + 20 + 3) / 4;

// key stream copies: ks[s][i] bytes = key[(i + s) % K], i < K + 20, s = 0..3
__device__ inline void stage_key(const XorArgs& a, uint32_t (*ks)[kKeyWords]) {
    const uint32_t K = a.key_len;
    const uint32_t words = (K + 20 + 3) / 4;
    for (uint32_t t = threadIdx.x; t < 4 * words; t += kThreads) {
        const uint32_t s = t / words, w = t - s * words;
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; ++b) v |= (uint32_t)a.key[(4 * w + b + s) % K] << (8 * b);
        ks[s][w] = v;
    }
}

// the 16 key-stream bytes starting at phase m (< K)
__device__ inline u32x4 key_at(const uint32_t (*ks)[kKeyWords], uint32_t m) {
    const uint32_t* kw = &ks[m & 3u][m >> 2];
    return u32x4{kw[0], kw[1], kw[2], kw[3]};
}

// bytes [lo, hi) of a 16-byte piece, as four dword masks
__device__ inline u32x4 byte_range(int lo, int hi) {
    u32x4 m;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int l = min(max(lo - 4 * w, 0), 4), h = min(max(hi - 4 * w, 0), 4);
        m[w] = h > l ? (uint32_t)((1ull << (8 * h)) - (1ull << (8 * l))) : 0u;
    }
    return m;
}

__global__ __launch_bounds__(kThreads) void xor_layer_kernel(XorArgs a) {
    // key stream copies: S_s[i] = key[(i + s) % K], i < K + 20 (bytes), s = 0..3
    __shared__ uint32_t ks[4][kKeyWords];
    const uint32_t K = a.key_len;
    stage_key(a, ks);
    __syncthreads();

    const uint32_t groups = gridDim.x * (kThreads / kGroup);
    const uint32_t sub = threadIdx.x % kGroup;
    const uint32_t adv = (16u * kGroup) % K;  // key phase advance between a lane's pieces
    for (uint32_t d = blockIdx.x * (kThreads / kGroup) + threadIdx.x / kGroup; d < a.n; d += groups) {
        uint64_t start;
        uint32_t len;
        if (a.off) {
            start = a.off[d] - a.off0;
            len = (uint32_t)(a.off[d + 1] - a.off[d]);
        } else {
            start = (uint64_t)d * a.stride;
            len = a.len;
        }
        if (len == 0) continue;
        const uint64_t p0 = (uint64_t)(uintptr_t)(a.base + start), p1 = p0 + len;  // datagram bytes
        const uint64_t q0 = p0 & ~(uint64_t)15;
        const uint32_t head = (uint32_t)(p0 - q0);                  // bytes of piece 0 before p0
        const uint32_t pieces = (uint32_t)((p1 - q0 + 15) >> 4);
        // key phase of this lane's first piece's byte 0 (datagram offset 16 sub - head >= -15)
        uint32_t m = (16u * sub + 15u * K - head) % K;
        // four pieces per lane in flight: loads first, then XOR and stores
        for (uint32_t k0 = sub; k0 < pieces; k0 += kUnroll * kGroup) {
            u32x4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t k = k0 + (uint32_t)u * kGroup;
                const uint64_t q = q0 + 16u * (uint64_t)k;
                if (k < pieces && q >= p0 && q + 16u <= p1) {
#if LNL_XOR_NT
                    v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>((uintptr_t)q));
#else
                    v[u] = *reinterpret_cast<const u32x4*>((uintptr_t)q);
#endif
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t k = k0 + (uint32_t)u * kGroup;
                if (k >= pieces) break;
                const uint64_t q = q0 + 16u * (uint64_t)k;
                const uint32_t* kw = &ks[m & 3u][(m - (m & 3u)) >> 2];
                const u32x4 key4 = {kw[0], kw[1], kw[2], kw[3]};
                if (q >= p0 && q + 16u <= p1) {  // whole piece inside the datagram
#if LNL_XOR_NT
                    __builtin_nontemporal_store(v[u] ^ key4, reinterpret_cast<u32x4*>((uintptr_t)q));
#else
                    *reinterpret_cast<u32x4*>((uintptr_t)q) = v[u] ^ key4;
#endif
                } else {
                    // first / last piece: its other bytes belong to neighbouring
                    // datagrams, updated concurrently by other lanes with byte
                    // stores of their own -- read the piece, store this
                    // datagram's bytes one by one
                    const u32x4 pv = *reinterpret_cast<const u32x4*>((uintptr_t)q);
                    const u32x4 x = pv ^ key4;
                    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
                    uint8_t* bp = reinterpret_cast<uint8_t*>((uintptr_t)q);
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const uint64_t at = q + (uint64_t)j;
                        if (at >= p0 && at < p1) bp[j] = (uint8_t)(xw[j >> 2] >> (8 * (j & 3)));
                    }
                }
                m += adv;
                if (m >= K) m -= K;
            }
        }
    }
}


// Flat fixed-stride kernel (stride >= 16, len <= stride, 16-byte aligned base):
// the batch is one byte range, cut into 16-byte pieces that consecutive lanes
// own whole -- every load and store is a coalesced dwordx4, and no piece is
// shared, so there are no byte-store edges.  A lane tracks, for its piece at
// byte 16k, the datagram d, the offset r = 16k - d*stride and the key phase
// r % K incrementally over its grid-stride steps (no division in the loop).
// The key of a piece is the key stream at phase r % K up to the datagram's end
// (or the gap after it), then the stream at phase 0 for the next datagram.
struct FlatState {
    uint32_t d, r, ph;
};

__device__ inline void flat_step(FlatState& st, const FlatArgs& f) {
    st.d += f.sd;
    st.r += f.sr;
    st.ph += f.srk;
    if (st.ph >= f.K) st.ph -= f.K;
    if (st.r >= f.S) {
        st.r -= f.S;
        st.d += 1u;
        st.ph = st.ph >= f.SK ? st.ph - f.SK : st.ph + f.K - f.SK;
    }
}

__device__ inline u32x4 flat_key(const uint32_t (*ks)[kKeyWords], const FlatArgs& f, const FlatState& st) {
    const uint32_t L = f.L;
    if (st.d < f.n && st.r + 16u <= L) return key_at(ks, st.ph);  // whole piece in one datagram
    // bytes [0, ca) belong to datagram d (offsets r.. < L), bytes [bc, hb) to d + 1
    int ca = 0, bc = 16, hb = 16;
    if (st.d < f.n && st.r < L) ca = (int)min(L - st.r, 16u);
    if (f.S - st.r < 16u && st.d + 1u < f.n) {
        bc = (int)(f.S - st.r);
        hb = (int)min((uint32_t)bc + L, 16u);
    }
    const u32x4 mA = byte_range(0, ca), mB = byte_range(bc, hb);
    u32x4 k = key_at(ks, st.ph) & mA;
    if (hb > bc) {
        const uint32_t m2 = (f.K - (uint32_t)bc % f.K) % f.K;  // byte b >= bc: key[(b - bc) % K]
        k |= key_at(ks, m2) & mB;
    }
    return k;
}

// kTile: workgroup b takes the kU x 256 consecutive pieces from b x kU x 256 on
// (one pass, grid sized to the batch: the dispatcher hands out the batch in
// order); otherwise a persistent grid strides over it, kU pieces per lane per step
template <int kU, bool kNT, bool kTile = false>
__global__ __launch_bounds__(kThreads) void xor_flat_kernel(XorArgs a, FlatArgs f) {
    __shared__ uint32_t ks[4][kKeyWords];
    stage_key(a, ks);
    __syncthreads();
    const uint32_t T = kTile ? kThreads : gridDim.x * kThreads;
    const uint32_t k0 = blockIdx.x * kThreads * (kTile ? kU : 1) + threadIdx.x;
    if (k0 >= f.pieces) return;
    FlatState st;
    {
        const uint64_t o = 16ull * k0;
        st.d = (uint32_t)(o / f.S);
        st.r = (uint32_t)(o - (uint64_t)st.d * f.S);
        st.ph = st.r % f.K;
    }
    u32x4* const base = reinterpret_cast<u32x4*>(a.base);
    for (uint32_t k = k0; k < f.pieces; k += kU * T) {
        u32x4 v[kU];
        FlatState sts[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            sts[u] = st;
            if (k + u * T < f.whole) {
                if constexpr (kNT)
                    v[u] = __builtin_nontemporal_load(base + k + u * T);
                else
                    v[u] = base[k + u * T];
            }
            flat_step(st, f);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t q = k + u * T;
            if (q >= f.pieces) break;
            const u32x4 key = flat_key(ks, f, sts[u]);
            if (q < f.whole) {
                if constexpr (kNT)
                    __builtin_nontemporal_store(v[u] ^ key, base + q);
                else
                    base[q] = v[u] ^ key;
            } else {  // the last piece runs past the batch: its own bytes only
                uint8_t* bp = a.base + 16ull * q;
                const uint32_t kw[4] = {key.x, key.y, key.z, key.w};
                for (uint32_t j = 0; j < 16u && 16ull * q + j < f.span; ++j)
                    bp[j] ^= (uint8_t)(kw[j >> 2] >> (8 * (j & 3)));
            }
        }
        if (kTile) break;
    }
}

// ---- flat CSR kernel -----------------------------------------------------
// A CSR batch's bytes [off[0], off[n]) are one range with no gaps, so the flat
// form carries over: 16-byte pieces of the range (aligned to the buffer); a
// wave takes CHUNKS of kCsrChunkPieces consecutive pieces (lane l: pieces l,
// l + 64, ..., coalesced dwordx4 loads and stores, nontemporal) from a contiguous
// run of chunks, and every piece has exactly one owner -- whole-piece stores,
// byte stores only for the batch's two edge pieces (their outside bytes are
// not the batch's).  The key phase of a piece needs its datagram: a wave finds
// the datagram holding its first chunk's first byte by a 64-ary search of the
// offsets (4 rounds for 2^20 datagrams), loads the next 64 datagram starts per
// chunk into LDS, and each lane places its piece among them by a 6-step
// search; the next chunk's datagram follows from the count of starts.  A piece
// with datagram starts inside it gets its key by segments (the key stream at
// phase 0 from each start on).  A chunk holding 64 starts or more (datagrams
// of < 32 bytes on average) reads the starts from global memory instead.
#ifndef LNL_XOR_CSR_U
#define LNL_XOR_CSR_U 2  // pieces per lane and chunk (1: 445 us per config-3 batch, 2: 368, 4: 382, 8: 444)
#endif
constexpr uint32_t kCsrU = LNL_XOR_CSR_U;
constexpr uint32_t kCsrChunkPieces = 64 * kCsrU;  // 2 KiB per wave and chunk
constexpr uint32_t kCsrChunkBytes = 16 * kCsrChunkPieces;

// x % K for x < 2^32, M = ceil(2^32 / K) (64-bit: 2^32 for K = 1): the
// quotient estimate is floor(x / K) or one more
__device__ inline uint32_t mod_k(uint64_t x, uint32_t K, uint64_t M) {
    const uint32_t x32 = (uint32_t)x;
    const uint32_t q = (uint32_t)(((uint64_t)x32 * M) >> 32);
    int64_t r = (int64_t)x32 - (int64_t)q * K;
    if (r < 0) r += K;
    if (r >= (int64_t)K) r -= K;
    return (uint32_t)r;
}

// max{d <= n : pos(off[d]) <= P} by a 64-ary search over the wave (P inside
// the batch: the result is < n); pos(x) = x - off0 + ab
__device__ inline uint32_t wave_datagram_of(const XorArgs& a, uint64_t ab, uint64_t P) {
    const uint32_t lane = __lane_id();
    uint32_t lo = 0, hi = a.n;  // pos(off[lo]) <= P; answer in [lo, hi)
    while (hi - lo > 1u) {
        const uint32_t step = (hi - lo + 63u) >> 6;
        const uint32_t idx = lo + lane * step;
        const bool le = idx < hi && a.off[idx] - a.off0 + ab <= P;
        const uint64_t m = __ballot(le);                  // lane 0 is always set
        const uint32_t last = 63u - (uint32_t)__builtin_clzll(m);
        lo += last * step;
        const uint32_t nh = lo + step;
        hi = nh < hi ? nh : hi;
    }
    return lo;
}

#ifndef LNL_XOR_CSR_NT
#define LNL_XOR_CSR_NT 1  // nontemporal whole-piece loads and stores (experiments: 0 = default policy)
#endif
__device__ inline u32x4 csr_load(const u32x4* p) {
#if LNL_XOR_CSR_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ inline void csr_store(u32x4 v, u32x4* p) {
#if LNL_XOR_CSR_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

__global__ __launch_bounds__(256) void xor_csr_flat_kernel(XorArgs a, uint64_t M) {
    __shared__ uint32_t ks[4][kKeyWords];
    __shared__ uint32_t bnd[4][64];  // per wave: the chunk's next 64 datagram starts, chunk-relative
    stage_key(a, ks);
    __syncthreads();
    const uint32_t K = a.key_len;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t ab = (uint64_t)((uintptr_t)a.base & 15u);  // buffer misalignment
    uint8_t* const abase = a.base - ab;                       // 16-byte aligned
    const uint64_t B0 = a.off[0] - a.off0 + ab, B1 = a.off[a.n] - a.off0 + ab;  // the batch, from abase
    if (B1 <= B0) return;
    const uint64_t S = B0 & ~(uint64_t)15;
    const uint64_t chunks = (B1 - S + kCsrChunkBytes - 1u) / kCsrChunkBytes;
    const uint64_t waves = (uint64_t)gridDim.x * 4u, gw = (uint64_t)blockIdx.x * 4u + w;
    const uint64_t per = (chunks + waves - 1u) / waves;
    const uint64_t c_begin = gw * per, c_end = c_begin + per < chunks ? c_begin + per : chunks;
    if (c_begin >= c_end) return;
    auto pos = [&](uint32_t d) -> uint64_t { return a.off[d] - a.off0 + ab; };
    uint64_t C0 = S + c_begin * kCsrChunkBytes;
    uint32_t d0 = wave_datagram_of(a, ab, C0 < B0 ? B0 : C0);  // holds the chunk's first batch byte
    for (uint64_t c = c_begin; c < c_end; ++c, C0 += kCsrChunkBytes) {
        const uint64_t Cend = C0 + kCsrChunkBytes;
        u32x4 v[kCsrU];
        uint64_t q[kCsrU];
#pragma unroll
        for (int u = 0; u < (int)kCsrU; ++u) {
            q[u] = C0 + 16u * (lane + 64u * u);
            if (q[u] >= B0 && q[u] + 16u <= B1)
                v[u] = csr_load(reinterpret_cast<const u32x4*>(abase + q[u]));
        }
        const uint64_t st0 = pos(d0);  // start of the datagram holding the chunk's first batch byte
        const uint32_t dj = d0 + 1u + lane;
        const uint64_t sj = dj <= a.n ? pos(dj) : ~0ull;
        bnd[w][lane] = sj < Cend ? (uint32_t)(sj - C0) : kCsrChunkBytes + 1u;
        const uint64_t in_chunk = __ballot(sj < Cend);
        const bool many = (in_chunk >> 63) != 0ull;  // the 64th start is still inside: read starts globally
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < (int)kCsrU; ++u) {
            const uint64_t qa = q[u];
            if (qa >= B1 || qa + 16u <= B0) continue;  // piece outside the batch
            const uint64_t first_byte = qa < B0 ? B0 : qa;
            // datagram d of the piece's first batch byte, its start, and the
            // starts after it (LDS when the chunk has < 64 of them)
            uint32_t d;
            if (!many) {
                const uint32_t r = (uint32_t)(first_byte - C0);
                uint32_t lo = 0;  // starts <= r among bnd[0..63] (sorted; beyond-chunk ones are > any r)
#pragma unroll
                for (uint32_t step = 32; step; step >>= 1)
                    if (bnd[w][lo + step - 1u] <= r) lo += step;
                d = d0 + lo;
            } else {  // this lane's own binary search of the offsets
                uint32_t lo = 0, hi = a.n;
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pos(mid) <= first_byte) lo = mid; else hi = mid;
                }
                d = lo;
            }
            auto start_of = [&](uint32_t dd) -> uint64_t {  // dd in (d0, d0 + 64]: LDS, else global
                if (!many && dd > d0 && dd <= d0 + 64u) {
                    const uint32_t rel = bnd[w][dd - d0 - 1u];
                    return rel <= kCsrChunkBytes ? C0 + rel : (dd <= a.n ? pos(dd) : ~0ull);
                }
                return dd <= a.n ? pos(dd) : ~0ull;
            };
            const uint64_t sd = d == d0 ? st0 : start_of(d);
            // key by segments: bytes before the next start at d's phase, then
            // each further datagram from phase 0
            uint32_t ph = qa >= sd ? mod_k(qa - sd, K, M) : (K - mod_k(sd - qa, K, M)) % K;
            u32x4 key = {0u, 0u, 0u, 0u};
            int lo_b = 0;
            uint32_t dd = d;
            while (true) {
                const uint64_t nb = start_of(dd + 1u);
                const int hi_b = nb >= qa + 16u ? 16 : (int)(nb - qa);
                if (hi_b > lo_b) key |= key_at(ks, ph) & byte_range(lo_b, hi_b);
                if (hi_b >= 16 || dd + 1u >= a.n) break;
                lo_b = hi_b > lo_b ? hi_b : lo_b;
                ph = (K - (uint32_t)lo_b % K) % K;  // byte lo_b gets key[0]
                ++dd;
            }
            if (qa >= B0 && qa + 16u <= B1) {
                csr_store(v[u] ^ key, reinterpret_cast<u32x4*>(abase + qa));
            } else {  // the batch's edge piece: its own bytes only
                uint8_t* bp = abase + qa;
                for (uint32_t j = 0; j < 16u; ++j) {
                    const uint64_t at = qa + j;
                    if (at >= B0 && at < B1) bp[j] ^= (uint8_t)(key[j >> 2] >> (8 * (j & 3)));
                }
            }
        }
        // the next chunk's first datagram: the last start <= Cend
        if (!many)
            d0 += (uint32_t)__popcll(__ballot(sj <= Cend));
        else if (c + 1u < c_end)
            d0 = wave_datagram_of(a, ab, Cend);
        __builtin_amdgcn_wave_barrier();  // bnd[w] is rewritten by the next chunk
    }
}

// (x mod K) for any 64-bit x: the 32-bit multiply path when x < 2^32 (every
// datagram shorter than 4 GiB), a 64-bit remainder otherwise
__device__ inline uint32_t mod_k64(uint64_t x, uint32_t K, uint64_t M) {
    return (x >> 32) == 0u ? mod_k(x, K, M) : (uint32_t)(x % K);
}

// ---- streaming CSR kernel (the product's CSR path) ------------------------
// The flat CSR kernel above places every piece among the next 64 starts with
// a 6-step LDS search and loads those 64 starts once per chunk, after the
// chunk before it has counted its own: a dependent round trip per 2 KiB.
// Here a wave streams a contiguous run of 2 KiB chunks (2 pieces per lane,
// coalesced dwordx4, the loads of the two chunks after it issued before this
// chunk's stores), and keeps the next 64 datagram starts in registers (one per lane),
// reloaded only when a chunk reaches the 64th.  A chunk's pieces take their key
// phase from the datagram start at or before them: a wave-uniform loop over
// the few starts that fall inside the chunk (~3 per 2 KiB at config 3) -- no
// per-piece search.  A start inside a piece splits its key into segments, as
// in the flat kernels.
#ifndef LNL_XOR_STREAM_U
#define LNL_XOR_STREAM_U 2  // pieces per lane and chunk
#endif
#ifndef LNL_XOR_STREAM_AHEAD
#define LNL_XOR_STREAM_AHEAD 2  // chunks loaded ahead of the one being processed (1 or 2)
#endif
constexpr uint32_t kStreamU = LNL_XOR_STREAM_U;
constexpr uint32_t kStreamChunk = 64u * kStreamU * 16u;  // bytes per wave and chunk

__global__ __launch_bounds__(256) void xor_csr_stream_kernel(XorArgs a, uint64_t M) {
    __shared__ uint32_t ks[4][kKeyWords];
    stage_key(a, ks);
    __syncthreads();
    const uint32_t K = a.key_len;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t ab = (uint64_t)((uintptr_t)a.base & 15u);  // buffer misalignment
    uint8_t* const abase = a.base - ab;                       // 16-byte aligned
    const uint64_t B0 = a.off[0] - a.off0 + ab, B1 = a.off[a.n] - a.off0 + ab;  // the batch, from abase
    if (B1 <= B0) return;
    const uint64_t S = B0 & ~(uint64_t)15;
    const uint64_t chunks = (B1 - S + kStreamChunk - 1u) / kStreamChunk;
    const uint64_t waves = (uint64_t)gridDim.x * 4u, gw = (uint64_t)blockIdx.x * 4u + w;
    const uint64_t per = (chunks + waves - 1u) / waves;
    const uint64_t c_begin = gw * per, c_end = c_begin + per < chunks ? c_begin + per : chunks;
    if (c_begin >= c_end) return;
    auto pos = [&](uint32_t d) -> uint64_t { return a.off[d] - a.off0 + ab; };
    uint64_t C0 = S + c_begin * kStreamChunk;
    // the datagram holding the run's first batch byte, its start, and the
    // window of the next 64 starts (lane j: datagram dw + 1 + j; ~0 past n)
    uint32_t dw = wave_datagram_of(a, ab, C0 < B0 ? B0 : C0);
    uint64_t st_cur = pos(dw);
    auto load_window = [&](uint32_t d) -> uint64_t {
        const uint32_t dj = d + 1u + lane;
        return dj <= a.n ? pos(dj) : ~0ull;
    };
    uint64_t sv = load_window(dw);
    u32x4 v[kStreamU], nv[kStreamU], nv2[kStreamU];
    auto load_chunk = [&](uint64_t c0, u32x4* dst) {
#pragma unroll
        for (int u = 0; u < (int)kStreamU; ++u) {
            const uint64_t q = c0 + 16u * (lane + 64u * u);
            if (q >= B0 && q + 16u <= B1) dst[u] = csr_load(reinterpret_cast<const u32x4*>(abase + q));
        }
    };
    load_chunk(C0, v);
    if (LNL_XOR_STREAM_AHEAD == 2 && c_begin + 1u < c_end) load_chunk(C0 + kStreamChunk, nv);
    for (uint64_t c = c_begin; c < c_end; ++c, C0 += kStreamChunk) {
        const uint64_t Cend = C0 + kStreamChunk;
        if (LNL_XOR_STREAM_AHEAD == 2) {
            if (c + 2u < c_end) load_chunk(Cend + kStreamChunk, nv2);
        } else if (c + 1u < c_end) {
            load_chunk(Cend, nv);
        }
        // the window must hold every start up to the chunk's last byte (and
        // one past it): slide it to the first start after C0 when it does not
        // (re-anchored by a search when all 64 are behind C0)
        {
            const uint64_t top = __shfl(sv, 63, 64);
            if (top != ~0ull && top < Cend) {
                const uint64_t done = __ballot(sv <= C0);  // starts already behind: a prefix of lanes
                if (done == ~0ull) {
                    dw = wave_datagram_of(a, ab, C0 < B0 ? B0 : C0);
                    st_cur = pos(dw);
                } else {
                    const uint32_t k = (uint32_t)__popcll(done);
                    if (k > 0u) st_cur = __shfl(sv, (int)k - 1, 64);
                    dw += k;
                }
                sv = load_window(dw);
            }
        }
        // more than 64 starts in one chunk (datagrams under 64 bytes on
        // average): the pieces search the offsets themselves (below)
        const bool dense = __shfl(sv, 63, 64) != ~0ull && __shfl(sv, 63, 64) < Cend;
        uint64_t q[kStreamU], sq[kStreamU];  // piece address, start at or before it
        u32x4 key[kStreamU];
        uint32_t seg[kStreamU];  // first byte of the piece's open key segment (0: none started inside)
        // (a piece before the batch's first byte -- only the run's first
        // piece, an edge piece -- starts its segment at that byte)
        auto begin_piece = [&](int u, uint64_t start) {
            sq[u] = start;
            seg[u] = start > q[u] ? (uint32_t)(start - q[u] < 16u ? start - q[u] : 16u) : 0u;
        };
#pragma unroll
        for (int u = 0; u < (int)kStreamU; ++u) {
            q[u] = C0 + 16u * (lane + 64u * u);
            key[u] = u32x4{0u, 0u, 0u, 0u};
            begin_piece(u, st_cur);
        }
        if (!dense) {
            // the starts inside (C0, Cend + 15]: ascending, a run of lanes
            uint64_t in = __ballot(sv > C0 && sv < Cend + 16u);
            while (in) {
                const int j = __builtin_ctzll(in);
                in &= in - 1u;
                const uint64_t s = __shfl(sv, j, 64);
#pragma unroll
                for (int u = 0; u < (int)kStreamU; ++u) {
                    if (s <= q[u]) {
                        sq[u] = s;
                    } else if (s < q[u] + 16u) {  // a datagram starts inside the piece
                        const uint32_t b = (uint32_t)(s - q[u]);
                        const uint32_t ph = seg[u] == 0u ? mod_k64(q[u] - sq[u], K, M)
                                                         : (K - mod_k(seg[u], K, M)) % K;
                        key[u] |= key_at(ks, ph) & byte_range((int)seg[u], (int)b);
                        seg[u] = b;
                    }
                }
            }
        } else {
            // dense chunk: each piece finds its own datagram (binary search)
#pragma unroll
            for (int u = 0; u < (int)kStreamU; ++u) {
                if (q[u] + 16u <= B0 || q[u] >= B1) continue;
                const uint64_t first_byte = q[u] < B0 ? B0 : q[u];
                uint32_t lo = 0, hi = a.n;
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pos(mid) <= first_byte) lo = mid; else hi = mid;
                }
                begin_piece(u, pos(lo));
                for (uint32_t d = lo + 1u; d <= a.n; ++d) {
                    const uint64_t s = pos(d);
                    if (s >= q[u] + 16u) break;
                    if (s <= q[u]) { sq[u] = s; continue; }
                    const uint32_t b = (uint32_t)(s - q[u]);
                    const uint32_t ph = seg[u] == 0u ? mod_k64(q[u] - sq[u], K, M) : (K - mod_k(seg[u], K, M)) % K;
                    key[u] |= key_at(ks, ph) & byte_range((int)seg[u], (int)b);
                    seg[u] = b;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < (int)kStreamU; ++u) {
            const uint64_t qa = q[u];
            if (qa >= B1 || qa + 16u <= B0) continue;  // piece outside the batch
            const uint32_t ph = seg[u] == 0u ? mod_k64(qa - sq[u], K, M) : (K - mod_k(seg[u], K, M)) % K;
            key[u] |= key_at(ks, ph) & byte_range((int)seg[u], 16);
            if (qa >= B0 && qa + 16u <= B1) {
                csr_store(v[u] ^ key[u], reinterpret_cast<u32x4*>(abase + qa));
            } else {  // the batch's edge piece: its own bytes only
                uint8_t* bp = abase + qa;
                for (uint32_t j = 0; j < 16u; ++j) {
                    const uint64_t at = qa + j;
                    if (at >= B0 && at < B1) bp[j] ^= (uint8_t)(key[u][j >> 2] >> (8 * (j & 3)));
                }
            }
        }
        // the next chunk's current start: the last start <= Cend (after a
        // dense chunk the window does not reach it: search again)
        if (!dense) {
            const uint64_t done = __ballot(sv <= Cend);
            if (done) st_cur = __shfl(sv, 63 - __builtin_clzll(done), 64);
        } else if (c + 1u < c_end) {
            dw = wave_datagram_of(a, ab, Cend);
            st_cur = pos(dw);
            sv = load_window(dw);
        }
#pragma unroll
        for (int u = 0; u < (int)kStreamU; ++u) {
            v[u] = nv[u];
            if (LNL_XOR_STREAM_AHEAD == 2) nv[u] = nv2[u];
        }
    }
}

// ---- grid-interleaved CSR kernel (the product's CSR path) -----------------
// The run kernels above give each wave its own contiguous run of the batch:
// ~6000 read+write streams hundreds of KiB apart, which the DRAM serves with
// page misses and read/write turnarounds (both measured at 4.1-4.2 TB/s on the
// config-3 batch, against 5.86 for the grid-stride fixed-stride kernel over
// the same bytes).  Here chunk c goes to wave c mod W, so at any moment the
// whole grid works inside one window of W x 2 KiB, as the fixed kernel does.
// A wave's chunks are then W chunks apart, with nothing to carry between them:
// chunk c's datagram comes from a chunk map, first[c] = the datagram holding
// the chunk's first batch byte, written by a small map kernel launched before
// (one thread per datagram marks the chunks whose first byte it holds).  The
// 64 starts from first[c] on are one coalesced load (lane j: start of
// first[c] + j).  A wave loads the next chunk's data, the next window and the
// map word two chunks ahead before it keys and stores this chunk.  Waves are
// numbered XCD-major, so neighbouring chunks -- which share offsets lines --
// run under one L2.
#ifndef LNL_XOR_GRID_U
#define LNL_XOR_GRID_U 2  // pieces per lane and chunk (2 KiB chunks)
#endif
constexpr uint32_t kGridU = LNL_XOR_GRID_U;
constexpr uint32_t kGridChunk = 64u * kGridU * 16u;  // 2 KiB per wave and chunk

// map granularity: 2 KiB chunks, coarsened 2^k-fold until the map fits `cap`
// words (batches averaging over 2 KiB per datagram)
__device__ inline uint32_t map_shift(uint64_t chunks, uint32_t cap) {
    uint32_t k = 0;
    while (((chunks + (1ull << k) - 1u) >> k) > cap) ++k;
    return k;
}

__global__ __launch_bounds__(256) void xor_chunk_map_kernel(XorArgs a, uint32_t* first, uint32_t cap) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ab = (uint64_t)((uintptr_t)a.base & 15u);
    const uint64_t B0 = a.off[0] - a.off0 + ab, B1 = a.off[a.n] - a.off0 + ab;
    if (B1 <= B0) return;
    const uint64_t S = B0 & ~(uint64_t)15;
    const uint64_t chunks = (B1 - S + kGridChunk - 1u) / kGridChunk;
    const uint32_t k = map_shift(chunks, cap);
    const uint64_t G = (uint64_t)kGridChunk << k, blocks = (chunks + (1ull << k) - 1u) >> k;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    uint64_t c_lo = 0, c_hi = 0;
    if (i < a.n) {
        const uint64_t Pi = a.off[i] - a.off0 + ab, Pj = a.off[i + 1] - a.off0 + ab;
        if (Pj > Pi) {  // map blocks whose first byte S + m G lies in [Pi, Pj)
            c_lo = Pi <= B0 ? 0u : (Pi - S + G - 1u) / G;
            c_hi = (Pj - S + G - 1u) / G;
            c_hi = c_hi < blocks ? c_hi : blocks;
        }
    }
    // a datagram over 16 blocks: the whole wave writes its marks
    const bool big = c_hi > c_lo + 16u;
    uint64_t bigs = __ballot(big);
    while (bigs) {
        const int j = __builtin_ctzll(bigs);
        bigs &= bigs - 1u;
        const uint64_t lo = __shfl(c_lo, j, 64), hi = __shfl(c_hi, j, 64);
        const uint32_t d = (uint32_t)__shfl((int)i, j, 64);
        for (uint64_t c = lo + lane; c < hi; c += 64u) first[c] = d;
    }
    if (!big)
        for (uint64_t c = c_lo; c < c_hi; ++c) first[c] = i;
}

__global__ __launch_bounds__(256) void xor_csr_grid_kernel(XorArgs a, uint64_t M, const uint32_t* first, uint32_t cap) {
    __shared__ uint32_t ks[4][kKeyWords];
    __shared__ u32x4 below[17];    // below[b]: bytes [0, b) of a piece
    __shared__ uint32_t neg[16];   // neg[b] = -b mod K: the phase that puts key[0] on byte b
    const uint64_t ab = (uint64_t)((uintptr_t)a.base & 15u);  // buffer misalignment
    uint8_t* const abase = a.base - ab;                       // 16-byte aligned
    const uint64_t B0 = a.off[0] - a.off0 + ab, B1 = a.off[a.n] - a.off0 + ab;  // the batch, from abase
    if (B1 <= B0) return;
    const uint64_t S = B0 & ~(uint64_t)15;
    const uint64_t chunks = (B1 - S + kGridChunk - 1u) / kGridChunk;
#ifndef LNL_XOR_GRID_XCD
#define LNL_XOR_GRID_XCD 0  // 1: waves numbered XCD-major (neighbouring chunks under one L2)
#endif
    const uint32_t G = gridDim.x;
    const uint32_t vb = LNL_XOR_GRID_XCD && (G & 7u) == 0u ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    // (the grid is sized from n, not from the bytes: a workgroup past the
    // batch's chunks leaves before it stages anything)
    if ((uint64_t)vb * 4u >= chunks) return;
    stage_key(a, ks);
    const uint32_t K = a.key_len;
    if (threadIdx.x < 17u) {
        const int bb = (int)threadIdx.x;
        u32x4 m;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int h = min(max(bb - 4 * w, 0), 4);
            m[w] = (uint32_t)((1ull << (8 * h)) - 1u);
        }
        below[bb] = m;
        if (bb < 16) neg[bb] = (K - (uint32_t)bb % K) % K;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t mk = map_shift(chunks, cap);  // chunk c's map word: first[c >> mk]
    const uint64_t W = (uint64_t)G * 4u, gw = (uint64_t)vb * 4u + w;
    if (gw >= chunks) return;
    auto pos = [&](uint32_t d) -> uint64_t { return a.off[d] - a.off0 + ab; };
    auto load_chunk = [&](uint64_t c0, u32x4* dst) {
#pragma unroll
        for (int u = 0; u < (int)kGridU; ++u) {
            const uint64_t q = c0 + 16u * (lane + 64u * u);
            if (q >= B0 && q + 16u <= B1) dst[u] = csr_load(reinterpret_cast<const u32x4*>(abase + q));
        }
    };
    // lane j: start of datagram d + j (~0 past the batch); lane 0 is d's own
    auto window = [&](uint32_t d) -> uint64_t {
        const uint32_t dj = d + lane;
        return dj <= a.n ? pos(dj) : ~0ull;
    };
    // the key stream from byte b of a piece on, over bytes [b, 16)
    auto restart = [&](u32x4 key, uint32_t b) -> u32x4 {
        const u32x4 keep = below[b];
        return (key & keep) | (key_at(ks, neg[b]) & ~keep);
    };
    uint64_t c = gw;
    uint32_t d1 = c + W < chunks ? first[(c + W) >> mk] : 0u;
    u32x4 v[kGridU], nv[kGridU];
    load_chunk(S + c * kGridChunk, v);
    uint64_t sv = window(first[c >> mk]);
    for (; c < chunks; c += W) {
        const uint64_t C0 = S + c * kGridChunk, Cend = C0 + kGridChunk;
        const bool more = c + W < chunks;
        uint64_t nsv = ~0ull;
        uint32_t d2 = 0u;
        if (more) {
            load_chunk(C0 + W * kGridChunk, nv);
            if (c + 2u * W < chunks) d2 = first[(c + 2u * W) >> mk];
            nsv = window(d1);
        }
        // the window's datagram holds C0, or (coarse map) precedes it: the
        // last of its starts <= C0 (none: the batch's first chunk, whose C0
        // may precede the batch -- its first start counts as inside)
        const uint64_t behind = __ballot(sv <= C0);
        const int k0 = behind ? 63 - __builtin_clzll(behind) : 0;
        const uint64_t st0 = __shfl(sv, k0, 64), top = __shfl(sv, 63, 64);
        // the window ends inside the chunk (63 starts or more in it: datagrams
        // under 32 bytes on average, or a coarse map far behind)
        const bool dense = top != ~0ull && top < Cend;
        u32x4 key[kGridU];
        if (!dense) {
            // chunk-relative starts inside (C0, Cend), ascending lanes; piece u
            // of the lane covers chunk bytes [qr, qr + 16).  Pass 1: each
            // piece's phase reference from the last start at or before it
            // (phase = (qr + ref) mod K); pass 2: each start inside a piece
            // restarts the key stream there.
            const bool inside = sv > C0 && sv < Cend;
            const uint32_t srel = inside ? (uint32_t)(sv - C0) : 0u;
            const uint64_t ins = __ballot(inside);
            const uint64_t lead = st0 <= C0 ? C0 - st0 : 0u;
            const uint32_t base0 = mod_k64(lead, K, M);
            uint32_t ref[kGridU];
#pragma unroll
            for (int u = 0; u < (int)kGridU; ++u) ref[u] = base0;
            for (uint64_t in = ins; in; in &= in - 1u) {
                const uint32_t sr = __builtin_amdgcn_readlane(srel, __builtin_ctzll(in));
#pragma unroll
                for (int u = 0; u < (int)kGridU; ++u)
                    if (sr <= 16u * (lane + 64u * u)) ref[u] = 0u - sr;
            }
#pragma unroll
            for (int u = 0; u < (int)kGridU; ++u) key[u] = key_at(ks, mod_k(16u * (lane + 64u * u) + ref[u], K, M));
            for (uint64_t in = ins; in; in &= in - 1u) {
                const uint32_t sr = __builtin_amdgcn_readlane(srel, __builtin_ctzll(in));
#pragma unroll
                for (int u = 0; u < (int)kGridU; ++u) {
                    const uint32_t b = sr - 16u * (lane + 64u * u);  // start's byte in the piece
                    if (b - 1u < 15u) key[u] = restart(key[u], b);
                }
            }
        } else {
            // dense chunk: each piece finds its own datagram (binary search)
#pragma unroll
            for (int u = 0; u < (int)kGridU; ++u) {
                const uint64_t q = C0 + 16u * (lane + 64u * u);
                key[u] = u32x4{0u, 0u, 0u, 0u};
                if (q + 16u <= B0 || q >= B1) continue;
                const uint64_t first_byte = q < B0 ? B0 : q;
                uint32_t lo = 0, hi = a.n;
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pos(mid) <= first_byte) lo = mid; else hi = mid;
                }
                const uint64_t s0 = pos(lo);
                key[u] = key_at(ks, s0 <= q ? mod_k64(q - s0, K, M) : 0u);
                if (s0 > q) key[u] = restart(key[u], (uint32_t)(s0 - q));
                for (uint32_t d = lo + 1u; d <= a.n; ++d) {
                    const uint64_t s = pos(d);
                    if (s >= q + 16u) break;
                    if (s > q) key[u] = restart(key[u], (uint32_t)(s - q));
                }
            }
        }
        if (C0 >= B0 && Cend <= B1) {  // every piece whole inside the batch
#pragma unroll
            for (int u = 0; u < (int)kGridU; ++u)
                csr_store(v[u] ^ key[u], reinterpret_cast<u32x4*>(abase + C0 + 16u * (lane + 64u * u)));
        } else {
#pragma unroll
            for (int u = 0; u < (int)kGridU; ++u) {
                const uint64_t qa = C0 + 16u * (lane + 64u * u);
                if (qa >= B1 || qa + 16u <= B0) continue;  // piece outside the batch
                if (qa >= B0 && qa + 16u <= B1) {
                    csr_store(v[u] ^ key[u], reinterpret_cast<u32x4*>(abase + qa));
                } else {  // the batch's edge piece: its own bytes only
                    uint8_t* bp = abase + qa;
                    for (uint32_t j = 0; j < 16u; ++j) {
                        const uint64_t at = qa + j;
                        if (at >= B0 && at < B1) bp[j] ^= (uint8_t)(key[u][j >> 2] >> (8 * (j & 3)));
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < (int)kGridU; ++u) v[u] = nv[u];
        sv = nsv;
        d1 = d2;
    }
}

}  // namespace

hipError_t launch_xor_csr_grid(const XorArgs& a, uint32_t* first, uint32_t cap, int grid, hipStream_t stream) {
    const uint64_t M = ((1ull << 32) + a.key_len - 1u) / a.key_len;
    hipLaunchKernelGGL(xor_chunk_map_kernel, dim3((a.n + 255u) / 256u), dim3(256), 0, stream, a, first, cap);
    hipLaunchKernelGGL(xor_csr_grid_kernel, dim3(grid), dim3(kThreads), 0, stream, a, M, (const uint32_t*)first, cap);
    return hipGetLastError();
}

hipError_t launch_xor_csr_stream(const XorArgs& a, int grid, hipStream_t stream) {
    const uint64_t M = ((1ull << 32) + a.key_len - 1u) / a.key_len;
    hipLaunchKernelGGL(xor_csr_stream_kernel, dim3(grid), dim3(kThreads), 0, stream, a, M);
    return hipGetLastError();
}

hipError_t launch_xor_csr_flat(const XorArgs& a, int grid, hipStream_t stream) {
    const uint64_t M = ((1ull << 32) + a.key_len - 1u) / a.key_len;
    hipLaunchKernelGGL(xor_csr_flat_kernel, dim3(grid), dim3(kThreads), 0, stream, a, M);
    return hipGetLastError();
}

hipError_t launch_xor_flat(const XorArgs& a, const FlatArgs& f, int grid, int variant, hipStream_t stream) {
#if !LNL_EXPERIMENTS
    (void)variant;  // product: tiles of 2 x 256 pieces, nontemporal
    hipLaunchKernelGGL((xor_flat_kernel<2, true, true>), dim3(grid), dim3(kThreads), 0, stream, a, f);
#else
    switch (variant) {  // pieces in flight per lane x cache policy (measured in DESIGN 4.8); 11..14: tiles
        case 11: hipLaunchKernelGGL((xor_flat_kernel<1, true, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 12: hipLaunchKernelGGL((xor_flat_kernel<2, true, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 13: hipLaunchKernelGGL((xor_flat_kernel<4, true, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 14: hipLaunchKernelGGL((xor_flat_kernel<2, false, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 15: hipLaunchKernelGGL((xor_flat_kernel<1, false, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 2: hipLaunchKernelGGL((xor_flat_kernel<4, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 3: hipLaunchKernelGGL((xor_flat_kernel<8, false>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 4: hipLaunchKernelGGL((xor_flat_kernel<8, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 5: hipLaunchKernelGGL((xor_flat_kernel<2, false>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        case 6: hipLaunchKernelGGL((xor_flat_kernel<2, true>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
        default: hipLaunchKernelGGL((xor_flat_kernel<4, false>), dim3(grid), dim3(kThreads), 0, stream, a, f); break;
    }
#endif
    return hipGetLastError();
}

hipError_t launch_xor_layer(const XorArgs& a, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(xor_layer_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace lnl
