"""Host-side mirror of the CRC-32C packet-layer path.

Two halves, both thin wrappers over the C ABI (include/lnl_crc32c.h):

* per-datagram (CPU, product code in csrc/crc32c_host.cpp): ``crc32c``,
  ``crc32c_extend`` and ``Crc32cLayer`` -- the packet layer the reference's
  ``net_manager`` would call at its two datagram choke points
  (/root/reference/src/lnl/net_manager.cpp:515-523 outbound before ``sendto``;
  :210-222 inbound after ``recvfrom``/``resize``, before ``verify()`` at :343).
  It mirrors upstream LiteNetLib's ``Crc32cLayer``: 4 extra bytes per datagram,
  append LE32(crc) outbound, drop silently inbound when the datagram is shorter
  than header + CRC or the CRC does not match.
* batched (gfx950 kernels): ``batch_fixed``, ``batch_csr``, ``verify_csr`` on
  device tensors, ``batch_host`` on host buffers.  These never compute on the
  CPU; without the library or a gfx950 GPU they raise.

Device buffers are torch tensors (torch is plumbing here: device memory and
streams).  CRC results are returned as ``torch.int32`` tensors holding the
uint32 bit patterns (use ``.cpu().numpy().view(np.uint32)``).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from ._lib import (DISPATCH_TAIL_DATAGRAM, DISPATCH_TAIL_LAYER, DISPATCH_TAIL_ZERO, HOST_DEFAULT_STREAMS,
                   HOST_MAX_STREAMS, Crc32cError, DispatchOpts, HostOpts, check, lib)

EXTRA_PACKET_SIZE = 4  # LNL_CRC32C_LAYER_EXTRA / upstream ExtraPacketSizeForLayer
HEADER_SIZE = 1        # net_constants::HEADER_SIZE (/root/reference/include/lnl/net_constants.h:16)

__all__ = [
    "Crc32cError", "EXTRA_PACKET_SIZE", "crc32c", "crc32c_extend", "Crc32cLayer",
    "batch_fixed", "batch_csr", "verify_csr", "batch_host", "batch_host_multi", "mtu_with_layer",
    "packet_verify", "inbound_status", "inbound_filter", "filter_dispatch", "inbound_filter_host", "ingress_recv_batch",
    "dispatch", "DISPATCH_TAIL_DATAGRAM", "DISPATCH_TAIL_ZERO", "DISPATCH_TAIL_LAYER", "xor_layer", "xor_layer_csr", "xor_layer_fixed",
    "INGRESS_SLOT", "HOST_DEFAULT_STREAMS", "HOST_MAX_STREAMS", "stream_release",
    "INBOUND_DROP_CRC", "INBOUND_ACCEPT", "INBOUND_MALFORMED",
]


def _addr(buf) -> tuple[int, int, object]:
    """(address, length, keepalive) of a bytes-like or numpy buffer."""
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            buf = np.ascontiguousarray(buf)
        return buf.ctypes.data, buf.nbytes, buf
    mv = memoryview(buf).cast("B")
    if mv.readonly:
        arr = np.frombuffer(mv, dtype=np.uint8)
        return arr.ctypes.data, arr.nbytes, arr
    c = (ctypes.c_uint8 * len(mv)).from_buffer(mv)
    return ctypes.addressof(c), len(mv), c


# ---------------------------------------------------------------- CPU path
def crc32c(data) -> int:
    """CRC-32C of a bytes-like object (CRC('123456789') = 0xE3069283)."""
    a, n, _k = _addr(data)
    return int(lib().lnl_crc32c(a, n))


def crc32c_extend(crc: int, data) -> int:
    """crc32c_extend(crc32c(a), b) == crc32c(a + b)."""
    a, n, _k = _addr(data)
    return int(lib().lnl_crc32c_extend(crc & 0xFFFFFFFF, a, n))


def mtu_with_layer(mtu: int) -> int:
    """Effective MTU with the CRC layer on: every POSSIBLE_MTU entry loses 4
    bytes (/root/reference/include/lnl/net_constants.h:29-39)."""
    return mtu - EXTRA_PACKET_SIZE


class Crc32cLayer:
    """Packet layer with upstream ``PacketLayerBase`` semantics.

    ``process_outbound(data, offset, length)`` returns the bytes to hand to
    ``sendto`` (payload + LE32 CRC) without touching ``data`` (send_raw's buffer
    is const and may be shared, /root/reference/src/lnl/net_peer.cpp:482).
    ``process_inbound(datagram)`` returns the payload with the CRC stripped, or
    None to drop the datagram (it then looks like loss to the reliable channel).
    """

    extra_packet_size = EXTRA_PACKET_SIZE

    def __init__(self):
        self.dropped = 0  # "checksum: bad" counter (upstream logs it)

    def process_outbound(self, data, offset: int = 0, length: Optional[int] = None) -> bytes:
        a, n, _k = _addr(data)
        if length is None:
            length = n - offset
        if offset < 0 or length < 0 or offset + length > n:
            raise ValueError("offset/length outside data")
        out = ctypes.create_string_buffer(length + EXTRA_PACKET_SIZE)
        r = lib().lnl_crc32c_layer_outbound(a, offset, length, ctypes.addressof(out), len(out))
        if r < 0:
            raise Crc32cError(int(r), "lnl_crc32c_layer_outbound", "bad arguments")
        return out.raw[:r]

    def process_inbound(self, datagram) -> Optional[bytes]:
        a, n, _k = _addr(datagram)
        r = lib().lnl_crc32c_layer_inbound(a, n)
        if r < 0:
            self.dropped += 1
            return None
        return bytes(memoryview(datagram).cast("B")[:r])


# ---------------------------------------------------------------- GPU path
def _torch():
    import torch
    return torch


def _stream_handle(stream) -> int:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def _check_dev_u8(t, name):
    torch = _torch()
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous()):
        raise TypeError(f"{name} must be a contiguous torch.uint8 CUDA tensor")


def _out_u32(out, n, device):
    torch = _torch()
    if out is None:
        return torch.empty(n, dtype=torch.int32, device=device)
    if not (out.is_cuda and out.dtype in (torch.int32, torch.uint32) and out.is_contiguous()
            and out.numel() >= n):
        raise TypeError("out must be a contiguous int32/uint32 CUDA tensor with >= n elements")
    return out


def batch_fixed(data, stride: int, length: int, n: int, out=None, stream=None):
    """out[i] = CRC32C(data[i*stride : i*stride + length]) on the GPU."""
    _check_dev_u8(data, "data")
    if n < 0 or length < 0 or stride < 0:
        raise ValueError("negative size")
    if n and (n - 1) * stride + length > data.numel():
        raise ValueError("batch exceeds data")
    out = _out_u32(out, n, data.device)
    check(lib().lnl_crc32c_batch_fixed_dev(data.data_ptr(), stride, length, n, out.data_ptr(),
                                           _stream_handle(stream)), "lnl_crc32c_batch_fixed_dev")
    return out


def _check_off(offsets, data):
    torch = _torch()
    if not (offsets.is_cuda and offsets.dtype in (torch.int64, torch.uint64) and offsets.is_contiguous()):
        raise TypeError("offsets must be a contiguous int64 CUDA tensor (n + 1 entries)")


def batch_csr(data, offsets, out=None, stream=None):
    """out[i] = CRC32C(data[off[i]:off[i+1]]) on the GPU (offsets: n+1 int64)."""
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    out = _out_u32(out, max(n, 0), data.device)
    if n > 0:
        check(lib().lnl_crc32c_batch_csr_dev(data.data_ptr(), offsets.data_ptr(), n, out.data_ptr(),
                                             _stream_handle(stream)), "lnl_crc32c_batch_csr_dev")
    return out


def append_csr(data, offsets, out=None, want_crc: bool = False, stream=None):
    """Batched outbound layer: the wire burst of a CSR burst of payloads --
    datagram i at (off[i] - off[0]) + 4 i as payload || LE32(crc) (what
    lnl_crc32c_layer_outbound writes for it).  Returns the uint8 wire tensor
    (off[n] - off[0] + 4 n bytes; ``out`` may supply it) [, crc (int32)]."""
    torch = _torch()
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    size = int(offsets[-1].item() - offsets[0].item()) + 4 * n if n > 0 else 0
    if out is None:
        out = torch.empty(size, dtype=torch.uint8, device=data.device)
    else:
        _check_dev_u8(out, "out")
        if out.numel() < size:
            raise ValueError(f"out holds {out.numel()} bytes, the wire burst needs {size}")
    crc = torch.empty(max(n, 0), dtype=torch.int32, device=data.device) if want_crc else None
    if n > 0:
        check(lib().lnl_crc32c_append_csr_dev(data.data_ptr(), offsets.data_ptr(), n, out.data_ptr(),
                                              crc.data_ptr() if crc is not None else None,
                                              _stream_handle(stream)), "lnl_crc32c_append_csr_dev")
    return (out, crc) if want_crc else out


def verify_csr(data, offsets, want_crc: bool = False, stream=None):
    """Batched inbound layer: ok[i] = datagram i (trailing LE32 CRC included)
    is >= 5 bytes and its CRC matches.  Returns ok (uint8) [, crc (int32)]."""
    torch = _torch()
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    ok = torch.empty(max(n, 0), dtype=torch.uint8, device=data.device)
    crc = torch.empty(max(n, 0), dtype=torch.int32, device=data.device) if want_crc else None
    if n > 0:
        check(lib().lnl_crc32c_verify_csr_dev(data.data_ptr(), offsets.data_ptr(), n, ok.data_ptr(),
                                              crc.data_ptr() if crc is not None else None,
                                              _stream_handle(stream)), "lnl_crc32c_verify_csr_dev")
    return (ok, crc) if want_crc else ok


INBOUND_DROP_CRC, INBOUND_ACCEPT, INBOUND_MALFORMED = 0, 1, 2  # include/lnl_crc32c.h


def packet_verify(packet) -> bool:
    """net_packet::verify() of a packet (CRC already stripped), on the CPU."""
    addr, n, _keep = _addr(packet)
    return bool(lib().lnl_packet_verify(addr, n))


def inbound_status(wire) -> int:
    """INBOUND_DROP_CRC / INBOUND_ACCEPT / INBOUND_MALFORMED for one wire
    datagram (layer check, then verify() of the stripped packet), on the CPU."""
    addr, n, _keep = _addr(wire)
    return int(lib().lnl_inbound_status(addr, n))


def inbound_filter(data, offsets, out=None, stream=None):
    """Batched inbound filter on the GPU: status[i] of every wire datagram of a
    CSR batch (uint8: INBOUND_DROP_CRC / INBOUND_ACCEPT / INBOUND_MALFORMED)."""
    torch = _torch()
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    status = out if out is not None else torch.empty(max(n, 0), dtype=torch.uint8, device=data.device)
    if status.dtype != torch.uint8 or status.numel() < max(n, 0) or status.device != data.device:
        raise ValueError("out must be a uint8 tensor of n entries on the data's device")
    if n > 0:
        check(lib().lnl_inbound_filter_csr_dev(data.data_ptr(), offsets.data_ptr(), n, status.data_ptr(),
                                               _stream_handle(stream)), "lnl_inbound_filter_csr_dev")
    return status


def _dispatch_opts(tail: int):
    if tail not in (DISPATCH_TAIL_DATAGRAM, DISPATCH_TAIL_ZERO, DISPATCH_TAIL_LAYER):
        raise ValueError(f"tail must be one of DISPATCH_TAIL_* (0, 1, 2), got {tail}")
    return ctypes.byref(DispatchOpts.make(tail))


def dispatch(data, offsets, status, cap: Optional[int] = None, stream=None, tail: int = DISPATCH_TAIL_DATAGRAM,
             avail: bool = False):
    """Packets a filtered burst delivers, on the GPU: accepted datagrams (CRC
    stripped) and the packets of MERGED containers (lnl_dispatch_csr_dev_ex).
    Returns (start int64, length int32, parent int32) tensors of the delivered
    packets (all of them when cap is None: a first call counts, a second
    fills), plus the in-burst byte counts (int32) when avail is set.  tail:
    the walk's bound past the datagram (DISPATCH_TAIL_DATAGRAM: stop there;
    DISPATCH_TAIL_ZERO / DISPATCH_TAIL_LAYER: the reference's zero-filled
    2048-byte buffer, net_peer.cpp:167-183; see include/lnl_crc32c.h)."""
    torch = _torch()
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    dev = data.device
    if not (isinstance(status, torch.Tensor) and status.is_cuda and status.dtype == torch.uint8
            and status.is_contiguous() and status.numel() >= max(n, 0) and status.device == dev):
        raise TypeError("status must be a contiguous uint8 CUDA tensor of >= n entries on the data's device")
    opts = _dispatch_opts(tail)
    total = torch.zeros(1, dtype=torch.int32, device=dev)

    def run(c):
        start = torch.empty(max(c, 1), dtype=torch.int64, device=dev)
        length = torch.empty(max(c, 1), dtype=torch.int32, device=dev)
        parent = torch.empty(max(c, 1), dtype=torch.int32, device=dev)
        av = torch.empty(max(c, 1), dtype=torch.int32, device=dev) if avail else None
        check(lib().lnl_dispatch_csr_dev_ex(data.data_ptr(), offsets.data_ptr(), max(n, 0), status.data_ptr(),
                                            start.data_ptr(), length.data_ptr(), parent.data_ptr(),
                                            av.data_ptr() if avail else None, c, total.data_ptr(), opts,
                                            _stream_handle(stream)), "lnl_dispatch_csr_dev_ex")
        return start, length, parent, av

    start, length, parent, av = run(cap if cap is not None else 0)
    t = int(total.item()) & 0xFFFFFFFF  # u32 count
    if cap is None:
        start, length, parent, av = run(t)
        cap = t
    k = min(t, cap)
    if avail:
        return start[:k], length[:k], parent[:k], av[:k]
    return start[:k], length[:k], parent[:k]


def filter_dispatch(data, offsets, cap: Optional[int] = None, out=None, stream=None,
                    tail: int = DISPATCH_TAIL_DATAGRAM, avail: bool = False):
    """inbound_filter + dispatch in one pass over the bytes
    (lnl_inbound_filter_dispatch_csr_dev_ex).  Returns (status uint8, start
    int64, length int32, parent int32[, avail int32]); the packets as dispatch()
    returns them."""
    torch = _torch()
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    n = offsets.numel() - 1
    dev = data.device
    status = out if out is not None else torch.empty(max(n, 0), dtype=torch.uint8, device=dev)
    if status.dtype != torch.uint8 or status.numel() < max(n, 0) or status.device != dev \
            or not status.is_contiguous():
        raise ValueError("out must be a contiguous uint8 tensor of n entries on the data's device")
    opts = _dispatch_opts(tail)
    total = torch.zeros(1, dtype=torch.int32, device=dev)

    def run(c):
        start = torch.empty(max(c, 1), dtype=torch.int64, device=dev)
        length = torch.empty(max(c, 1), dtype=torch.int32, device=dev)
        parent = torch.empty(max(c, 1), dtype=torch.int32, device=dev)
        av = torch.empty(max(c, 1), dtype=torch.int32, device=dev) if avail else None
        check(lib().lnl_inbound_filter_dispatch_csr_dev_ex(
            data.data_ptr(), offsets.data_ptr(), max(n, 0), status.data_ptr(), start.data_ptr(),
            length.data_ptr(), parent.data_ptr(), av.data_ptr() if avail else None, c, total.data_ptr(), opts,
            _stream_handle(stream)), "lnl_inbound_filter_dispatch_csr_dev_ex")
        return start, length, parent, av

    start, length, parent, av = run(cap if cap is not None else 0)
    t = int(total.item()) & 0xFFFFFFFF  # u32 count
    if cap is None:
        start, length, parent, av = run(t)
        cap = t
    k = min(t, cap)
    if avail:
        return status, start[:k], length[:k], parent[:k], av[:k]
    return status, start[:k], length[:k], parent[:k]


def _key(key) -> bytes:
    k = key.encode("utf-8") if isinstance(key, str) else bytes(key)   # upstream SetKey(string): UTF-8
    if not 1 <= len(k) <= 256:
        raise ValueError("key must be 1..256 bytes")
    return k


def xor_layer(data: np.ndarray, key) -> None:
    """Upstream XorEncryptLayer on one datagram, in place, on the CPU."""
    k = _key(key)
    if data.dtype != np.uint8 or not data.flags["C_CONTIGUOUS"]:
        raise ValueError("data must be a contiguous uint8 array")
    check(lib().lnl_xor_layer(data.ctypes.data, data.nbytes, k, len(k)), "lnl_xor_layer")


def xor_layer_csr(data, offsets, key, stream=None) -> None:
    """XorEncryptLayer over every datagram of a device CSR batch, in place."""
    _check_dev_u8(data, "data")
    _check_off(offsets, data)
    k = _key(key)
    n = offsets.numel() - 1
    if n > 0:
        check(lib().lnl_xor_layer_csr_dev(data.data_ptr(), offsets.data_ptr(), n, k, len(k),
                                          _stream_handle(stream)), "lnl_xor_layer_csr_dev")


def xor_layer_fixed(data, stride: int, length: int, n: int, key, stream=None) -> None:
    """XorEncryptLayer over n datagrams at a fixed stride on the device, in place."""
    _check_dev_u8(data, "data")
    k = _key(key)
    if n and (n - 1) * stride + length > data.numel():
        raise ValueError("batch exceeds data")
    if n > 0:
        check(lib().lnl_xor_layer_fixed_dev(data.data_ptr(), stride, length, n, k, len(k),
                                            _stream_handle(stream)), "lnl_xor_layer_fixed_dev")


def _host_csr(data, offsets):
    """Contiguous uint8 bytes and uint64 offsets of a host CSR batch, checked
    the way the C ABI cannot (it never sees the buffer's size): offsets start
    at >= 0, never decrease and end inside data.  A negative int64 offset
    would otherwise wrap to a huge uint64 and the H2D copy read out of bounds."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets)
    if off.ndim != 1 or off.size == 0:
        raise ValueError("offsets must be a 1-D array of n + 1 entries")
    if off.dtype.kind not in "iu":
        raise TypeError("offsets must be an integer array")
    if off.dtype.kind == "i" and off.size and int(off.min()) < 0:
        raise ValueError("negative offset")
    off = off.astype(np.uint64, copy=False)
    if off.size > 1 and bool((off[1:] < off[:-1]).any()):
        raise ValueError("offsets decrease")
    if int(off[-1]) > data.size:
        raise ValueError(f"offsets end at {int(off[-1])}, past the {data.size}-byte buffer")
    return data, off


def _host_opts(streams, chunk_datagrams, chunk_bytes):
    """ctypes pointer to an lnl_host_opts (None: every default)."""
    if not (streams or chunk_datagrams or chunk_bytes):
        return None
    if streams and not 1 <= streams <= HOST_MAX_STREAMS:
        raise ValueError(f"streams must be 1..{HOST_MAX_STREAMS}")
    return ctypes.pointer(HostOpts.make(streams or 0, chunk_datagrams or 0, chunk_bytes or 0))


def inbound_filter_host(data: np.ndarray, offsets: np.ndarray, device: int = 0, streams: Optional[int] = None,
                        chunk_datagrams: Optional[int] = None, chunk_bytes: Optional[int] = None) -> np.ndarray:
    """Host-resident burst through the GPU inbound filter (H2D -> filter ->
    D2H, chunks over ``streams`` HIP streams, default HOST_DEFAULT_STREAMS).
    Blocking.  Returns uint8 status codes.  Mirrors lnl_inbound_filter_host_ex."""
    data, offsets = _host_csr(data, offsets)
    opts = _host_opts(streams, chunk_datagrams, chunk_bytes)
    n = offsets.size - 1
    out = np.empty(max(n, 0), dtype=np.uint8)
    if n > 0:
        check(lib().lnl_inbound_filter_host_ex(data.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, device,
                                               opts), "lnl_inbound_filter_host_ex")
    return out


INGRESS_SLOT = 1432  # LNL_INGRESS_SLOT: bytes per datagram slot (the reference's MAX_PACKET_SIZE)


def ingress_recv_batch(fd: int, buf: np.ndarray, max_n: int, wait_ms: int = 0):
    """One recvmmsg burst from UDP socket fd into buf (uint8, ideally pinned),
    compacted to CSR.  Returns (n, offsets[n + 1]); n = 0 when nothing was ready."""
    if buf.dtype != np.uint8 or not buf.flags["C_CONTIGUOUS"]:
        raise ValueError("buf must be a contiguous uint8 array")
    off = np.zeros(max_n + 1, dtype=np.uint64)
    r = lib().lnl_ingress_recv_batch(fd, buf.ctypes.data, buf.nbytes, off.ctypes.data, max_n, None, wait_ms)
    if r < 0:
        raise Crc32cError(r, "lnl_ingress_recv_batch", os.strerror(-r))
    return r, off[: r + 1]


def append_host(data: np.ndarray, offsets: np.ndarray, device: int = 0, want_crc: bool = False, out=None,
                streams: Optional[int] = None, chunk_datagrams: Optional[int] = None,
                chunk_bytes: Optional[int] = None):
    """Host-resident outbound layer over the GPU (H2D -> CRC + append -> D2H,
    chunks over ``streams`` HIP streams, default HOST_DEFAULT_STREAMS).  Blocking.  Returns (wire, wire_offsets[, crc]): datagram i is
    wire[wire_offsets[i] .. wire_offsets[i + 1]) = payload || LE32(CRC), the
    bytes Crc32cLayer.process_outbound gives for it.  ``out``: a uint8 array of
    at least the wire burst's size to write it into -- pinned memory (as for
    ``data``) gives the full PCIe rate; a fresh pageable array otherwise.
    Mirrors lnl_crc32c_append_host_ex."""
    data, offsets = _host_csr(data, offsets)
    opts = _host_opts(streams, chunk_datagrams, chunk_bytes)
    n = offsets.size - 1
    wire_off = (offsets - offsets[0]) + EXTRA_PACKET_SIZE * np.arange(n + 1, dtype=np.uint64)
    if out is not None:
        if out.dtype != np.uint8 or not out.flags["C_CONTIGUOUS"] or out.size < int(wire_off[-1]):
            raise ValueError("out must be a contiguous uint8 array of at least the wire burst's size")
        wire = out[: int(wire_off[-1])]
    else:
        wire = np.empty(int(wire_off[-1]), dtype=np.uint8)
    crc = np.empty(max(n, 0), dtype=np.uint32) if want_crc else None
    if n > 0:
        check(lib().lnl_crc32c_append_host_ex(data.ctypes.data, offsets.ctypes.data, n, wire.ctypes.data,
                                              None if crc is None else crc.ctypes.data, device, opts),
              "lnl_crc32c_append_host_ex")
    return (wire, wire_off, crc) if want_crc else (wire, wire_off)


def egress_send_batch(fd: int, wire: np.ndarray, offsets: np.ndarray, addrs=None, wait_ms: int = -1):
    """One sendmmsg burst (in calls of <= 1024) of the CSR wire burst to UDP
    socket fd.  addrs: None (connected socket), one (host, port) pair, or one
    per datagram.  Returns (attempted, status): status[i] = bytes sent or a
    negative errno for datagrams the kernel refused.  Mirrors
    lnl_egress_send_batch."""
    import socket
    import struct
    wire, offsets = _host_csr(wire, offsets)
    n = offsets.size - 1
    if n > 0 and int(offsets[0]) != 0:
        raise ValueError("wire offsets must start at 0")
    packed, naddrs = None, 0
    if addrs is not None:
        pairs = [addrs] if isinstance(addrs, tuple) else list(addrs)
        if len(pairs) not in (1, n):
            raise ValueError("addrs: one endpoint, or one per datagram")
        # struct sockaddr_in: family (host order), port and address (network order), 8 pad bytes
        raw = b"".join(struct.pack("=H", socket.AF_INET) + struct.pack("!H", p) + socket.inet_aton(h) + bytes(8)
                       for h, p in pairs)
        packed = np.frombuffer(raw, dtype=np.uint8).copy()
        naddrs = len(pairs)
    status = np.zeros(max(n, 0), dtype=np.int64)
    r = lib().lnl_egress_send_batch(fd, wire.ctypes.data, offsets.ctypes.data, n,
                                    None if packed is None else packed.ctypes.data, naddrs,
                                    status.ctypes.data, wait_ms)
    if r < 0:
        raise Crc32cError(int(r), "lnl_egress_send_batch", os.strerror(int(-r)))
    return int(r), status


def batch_host(data: np.ndarray, offsets: np.ndarray, device: int = 0, streams: Optional[int] = None,
               chunk_datagrams: Optional[int] = None, chunk_bytes: Optional[int] = None) -> np.ndarray:
    """Host-resident batch over the GPU (H2D -> kernel -> D2H, chunks over
    ``streams`` HIP streams, default HOST_DEFAULT_STREAMS; BASELINE config 5 is
    streams=2).  Blocking.  ``data`` uint8, ``offsets`` uint64/int64 with n+1
    entries.  Mirrors lnl_crc32c_batch_host_ex."""
    data, offsets = _host_csr(data, offsets)
    opts = _host_opts(streams, chunk_datagrams, chunk_bytes)
    n = offsets.size - 1
    out = np.empty(max(n, 0), dtype=np.uint32)
    if n > 0:
        check(lib().lnl_crc32c_batch_host_ex(data.ctypes.data, offsets.ctypes.data, n, out.ctypes.data,
                                             device, opts), "lnl_crc32c_batch_host_ex")
    return out


def stream_release(stream=None) -> None:
    """Frees the scratch the library keeps for ``stream`` (a torch stream,
    a raw hipStream_t handle or None) on the current device; call it before
    the stream goes away.  Mirrors lnl_stream_release."""
    lib().lnl_stream_release(stream if isinstance(stream, int) else _stream_handle(stream))


def batch_host_multi(data: np.ndarray, offsets: np.ndarray, devices) -> np.ndarray:
    """Host-resident batch split over several GPUs (contiguous datagram ranges
    of ceil(n / len(devices)), one host thread per range, no data exchanged
    between devices).  Blocking.  Mirrors lnl_crc32c_batch_host_multi."""
    data, offsets = _host_csr(data, offsets)
    devs = np.ascontiguousarray(list(devices), dtype=np.int32)
    if devs.size == 0:
        raise ValueError("empty device list")
    n = offsets.size - 1
    out = np.empty(max(n, 0), dtype=np.uint32)
    if n > 0:
        check(lib().lnl_crc32c_batch_host_multi(data.ctypes.data, offsets.ctypes.data, n, out.ctypes.data,
                                                devs.ctypes.data, int(devs.size)),
              "lnl_crc32c_batch_host_multi")
    return out
