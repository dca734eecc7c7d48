"""ctypes loader for the CPU oracle (oracle/build/libcrc32c_oracle.so).

Test infrastructure: used only by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  Builds the oracle with make if
the shared object is missing (gcc only; no GPU needed).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libcrc32c_oracle.so")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    L = ctypes.CDLL(ORACLE_SO)
    for f in ("oracle_crc32c_bitwise", "oracle_crc32c_sliced", "oracle_crc32c_hw"):
        getattr(L, f).restype = ctypes.c_uint32
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for f in ("oracle_crc32c_bitwise_extend", "oracle_crc32c_sliced_extend", "oracle_crc32c_hw_extend"):
        getattr(L, f).restype = ctypes.c_uint32
        getattr(L, f).argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_has_sse42.restype = ctypes.c_int
    L.oracle_batch_fixed.restype = ctypes.c_int
    L.oracle_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    L.oracle_batch_csr.restype = ctypes.c_int
    L.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_int]
    L.oracle_batch_csr_bitwise.restype = None
    L.oracle_batch_csr_bitwise.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p]
    _lib = L
    return L


def mt19937_64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """SURVEY.md 8(d) synthetic input: mt19937_64(seed) outputs, little-endian."""
    words = np.empty((nbytes + 7) // 8, dtype=np.uint64)
    L = load()
    L.oracle_fill_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_fill_mt19937_64.restype = None
    L.oracle_fill_mt19937_64(seed, words.ctypes.data, words.size)
    return words.view(np.uint8)[:nbytes]


def _buf(b):
    arr = np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)
    return arr


def crc(data, kind: str = "hw") -> int:
    a = _buf(data)
    return int(getattr(load(), f"oracle_crc32c_{kind}")(a.ctypes.data, a.nbytes))


def batch_fixed(data: np.ndarray, stride: int, length: int, n: int, threads: int = 0) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint32)
    load().oracle_batch_fixed(data.ctypes.data, stride, length, n, out.ctypes.data, threads)
    return out


def batch_csr(data: np.ndarray, offsets: np.ndarray, threads: int = 0, bitwise: bool = False) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets).astype(np.uint64, copy=False)
    n = off.size - 1
    out = np.empty(n, dtype=np.uint32)
    if bitwise:
        load().oracle_batch_csr_bitwise(data.ctypes.data, off.ctypes.data, n, out.ctypes.data)
    else:
        load().oracle_batch_csr(data.ctypes.data, off.ctypes.data, n, out.ctypes.data, threads)
    return out


# ---- packet acceptance after the CRC layer ----------------------------------
# net_packet::verify() (/root/reference/include/lnl/net_packet.h:120-131) over
# HEADER_SIZES (:20-38: 17 initialisers for 18 properties, so index 17 is 0)
# with net_constants.h:16-20 (HEADER_SIZE 1, CHANNELED 4, CONNECT_REQUEST 18,
# CONNECT_ACCEPT 15, FRAGMENT_HEADER_SIZE 6).  Pinned to the reference's own
# compiled header by tests/golden/packet_verify.bin.
HEADER_SIZES = [1, 4, 4, 3, 11, 18, 15, 9, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0]
FRAGMENT_HEADER_SIZE = 6
INBOUND_DROP_CRC, INBOUND_ACCEPT, INBOUND_MALFORMED = 0, 1, 2


def packet_verify(b0: int, size: int) -> bool:
    """verify() of a packet whose byte 0 is b0 and whose size is `size` (size 0:
    the reference reads byte 0 of its zeroed pool buffer, property 0 -> False)."""
    if size == 0:
        b0 = 0
    prop = b0 & 0x1F
    if prop >= len(HEADER_SIZES):
        return False
    hs = HEADER_SIZES[prop]
    return size >= hs and (not (b0 & 0x80) or size >= hs + FRAGMENT_HEADER_SIZE)


def inbound_status(wire: np.ndarray) -> int:
    """Layer check (length >= 5, trailing LE32 == CRC-32C of the rest), then
    verify() of the stripped packet (net_manager.cpp:218-222, :343)."""
    w = np.ascontiguousarray(wire, dtype=np.uint8)
    if w.size < 5:
        return INBOUND_DROP_CRC
    if crc(w[:-4]) != int(w[-4:].view("<u4")[0]):
        return INBOUND_DROP_CRC
    return INBOUND_ACCEPT if packet_verify(int(w[0]), w.size - 4) else INBOUND_MALFORMED


REF_PACKET_SO = os.path.join(ORACLE_DIR, "_ref", "libref_packet.so")


def load_ref_packet():
    """The reference's own net_packet compiled by `make -C oracle ref`
    (oracle/_ref/libref_packet.so), or None where it was not built."""
    if not os.path.exists(REF_PACKET_SO):
        return None
    L = ctypes.CDLL(REF_PACKET_SO)
    L.ref_packet_verify.restype = ctypes.c_int
    L.ref_packet_verify.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.ref_packet_header_size.restype = ctypes.c_int
    L.ref_packet_header_size.argtypes = [ctypes.c_uint8]
    return L


MERGED_PROPERTY = 12  # PACKET_PROPERTY::MERGED (net_enums.h:60)


DISPATCH_TAIL_DATAGRAM, DISPATCH_TAIL_ZERO, DISPATCH_TAIL_LAYER = 0, 1, 2  # include/lnl_crc32c.h


def ref_capacity(nbytes: int) -> int:
    """buffer_size() of the reference's packet holding nbytes: net_packet()
    allocates 2048 zero-filled bytes (ensure(1432), net_packet.h:46-49,
    194-208) and resize() doubles it while it is short."""
    cap = 2048
    while cap < nbytes:
        cap *= 2
    return cap


def dispatch_ex(wire_list, status, tail=DISPATCH_TAIL_DATAGRAM):
    """Packets a filtered burst delivers: (datagram index, offset within the
    datagram, length, avail) per packet.  Accepted datagrams are one packet
    (CRC stripped); a MERGED container is cut as net_peer::process_packet does
    (/root/reference/src/lnl/net_peer.cpp:164-187).

    tail DISPATCH_TAIL_DATAGRAM: the walk stops at the datagram's end.  The
    other two walk the reference's own received buffer: bounded by its
    capacity (:171, buffer_size() = 2048), with the bytes after the datagram
    read as zeros (DISPATCH_TAIL_ZERO) or as the stripped CRC field and then
    zeros (DISPATCH_TAIL_LAYER: INTEGRATION.md's receive_logic edit shrinks
    the packet, the field stays in the buffer).  avail = the packet's bytes
    that lie in the wire datagram; the rest are those zeros."""
    out = []
    for i, (w, st) in enumerate(zip(wire_list, status)):
        if st != INBOUND_ACCEPT:
            continue
        size = len(w) - 4
        if w[0] & 0x1F != MERGED_PROPERTY:
            out.append((i, 0, size, size))
            continue
        if tail == DISPATCH_TAIL_DATAGRAM:
            pos = 1
            while pos < size:
                if pos + 2 > size:
                    break
                L = int(w[pos]) | (int(w[pos + 1]) << 8)
                pos += 2
                if L > size - pos or L == 0 or not packet_verify(int(w[pos]), L):
                    break
                out.append((i, pos, L, L))
                pos += L
            continue
        lim = size + (4 if tail == DISPATCH_TAIL_LAYER else 0)
        cap = ref_capacity(len(w))
        buf = bytes(w[:lim]) + bytes(cap - lim)
        pos = 1
        while pos < size:
            L = buf[pos] | (buf[pos + 1] << 8)
            pos += 2
            if cap - pos < L:
                break
            if L == 0 or not packet_verify(buf[pos], L):
                break
            out.append((i, pos, L, max(0, min(L, lim - pos))))
            pos += L
    return out


def dispatch(wire_list, status):
    """dispatch_ex under the datagram rule, as (datagram, offset, length)."""
    return [(i, o, L) for i, o, L, _ in dispatch_ex(wire_list, status)]


def cut_merged(pkt, ref_tail=False):
    """The entries of one MERGED packet: [(offset, length)].  Bounded by the
    packet itself (dispatch()'s datagram rule), or with ref_tail as the
    reference cuts a packet it got from its pool (a fresh zero-filled buffer
    of ref_capacity bytes, net_peer.cpp:175-176; offsets past the packet then
    read zeros)."""
    if ref_tail:
        size = len(pkt)
        cap = ref_capacity(size)
        buf = bytes(pkt) + bytes(cap - size)
        out, pos = [], 1
        while pos < size:
            L = buf[pos] | (buf[pos + 1] << 8)
            pos += 2
            if cap - pos < L or L == 0 or not packet_verify(buf[pos], L):
                break
            out.append((pos, L))
            pos += L
        return out
    out, pos, size = [], 1, len(pkt)
    while pos + 2 <= size:
        L = int(pkt[pos]) | (int(pkt[pos + 1]) << 8)
        pos += 2
        if L > size - pos or L == 0 or not packet_verify(int(pkt[pos]), L):
            break
        out.append((pos, L))
        pos += L
    return out


def deliver(pkt, conn, ref_tail=False):
    """What net_peer::process_packet hands the user for one dispatched packet
    (/root/reference/src/lnl/net_peer.cpp:138-243), for the properties the
    dispatch fixture uses: dropped unless its connection number is conn (:156);
    UNRELIABLE -> [payload after the 1-byte header] (:240-243); MERGED -> its
    entries (cut_merged: the datagram-bounded rule, or the reference's own
    with ref_tail), each delivered the same way; anything else -> nothing."""
    pkt = bytes(pkt)
    if not pkt or ((pkt[0] & 0x60) >> 5) != conn:
        return []
    prop = pkt[0] & 0x1F
    if prop == 0:
        return [pkt[1:]]
    if prop != MERGED_PROPERTY:
        return []
    buf = pkt + bytes(ref_capacity(len(pkt)) - len(pkt)) if ref_tail else pkt
    out = []
    for o, L in cut_merged(pkt, ref_tail):
        out += deliver(buf[o:o + L], conn, ref_tail)
    return out


def xor_layer(data: np.ndarray, key: bytes) -> np.ndarray:
    """Upstream LiteNetLib XorEncryptLayer on one datagram (restated; the C#
    source is not available offline -- parity unpinned):
    data[i] ^= key[i % len(key)], the phase restarting at each datagram."""
    d = np.asarray(data, dtype=np.uint8)
    k = np.frombuffer(key, np.uint8)
    return d ^ np.resize(k, d.size) if d.size else d.copy()
