"""ctypes binding of the in-tree product library ``liblnl_crc32c.so``.

This is the Python mirror of the C ABI in ``include/lnl_crc32c.h`` (the same
entry points a cgo/JNI/ctypes maintainer would bind).  It
loads ONLY the in-tree library and raises if it is missing: there is no
Python or CPU fallback for the batch entry points.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblnl_crc32c.so")

_c_u8p = ctypes.c_void_p  # raw addresses (host bytes or device pointers)


class Crc32cError(RuntimeError):
    """A negative return code from the C ABI (errno-style) plus its message."""

    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"{what} failed ({code}): {msg}")
        self.code = code


class HostOpts(ctypes.Structure):
    """struct lnl_host_opts (include/lnl_crc32c.h): zero fields take the defaults."""
    _fields_ = [("size", ctypes.c_uint32), ("streams", ctypes.c_uint32), ("chunk_datagrams", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("chunk_bytes", ctypes.c_uint64)]

    @classmethod
    def make(cls, streams: int = 0, chunk_datagrams: int = 0, chunk_bytes: int = 0) -> "HostOpts":
        return cls(ctypes.sizeof(cls), streams, chunk_datagrams, 0, chunk_bytes)


class DispatchOpts(ctypes.Structure):
    """struct lnl_dispatch_opts (include/lnl_crc32c.h)."""
    _fields_ = [("size", ctypes.c_uint32), ("tail", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 2)]

    @classmethod
    def make(cls, tail: int = 0) -> "DispatchOpts":
        return cls(ctypes.sizeof(cls), tail)


DISPATCH_TAIL_DATAGRAM, DISPATCH_TAIL_ZERO, DISPATCH_TAIL_LAYER = 0, 1, 2  # LNL_DISPATCH_TAIL_*

HOST_MAX_STREAMS = 8       # LNL_HOST_MAX_STREAMS
HOST_DEFAULT_STREAMS = 4   # LNL_HOST_DEFAULT_STREAMS

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
            "or `make -C litenetlibpp_amd` (no fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    L.lnl_crc32c.restype = ctypes.c_uint32
    L.lnl_crc32c.argtypes = [_c_u8p, ctypes.c_size_t]
    L.lnl_crc32c_extend.restype = ctypes.c_uint32
    L.lnl_crc32c_extend.argtypes = [ctypes.c_uint32, _c_u8p, ctypes.c_size_t]
    L.lnl_crc32c_layer_outbound.restype = ctypes.c_int64
    L.lnl_crc32c_layer_outbound.argtypes = [_c_u8p, ctypes.c_size_t, ctypes.c_size_t, _c_u8p,
                                            ctypes.c_size_t]
    L.lnl_crc32c_layer_inbound.restype = ctypes.c_int64
    L.lnl_crc32c_layer_inbound.argtypes = [_c_u8p, ctypes.c_size_t]
    L.lnl_crc32c_batch_fixed_dev.restype = ctypes.c_int
    L.lnl_crc32c_batch_fixed_dev.argtypes = [_c_u8p, ctypes.c_size_t, ctypes.c_uint32,
                                             ctypes.c_uint32, _c_u8p, ctypes.c_void_p]
    L.lnl_crc32c_batch_csr_dev.restype = ctypes.c_int
    L.lnl_crc32c_batch_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p,
                                           ctypes.c_void_p]
    L.lnl_crc32c_append_csr_dev.restype = ctypes.c_int
    L.lnl_crc32c_append_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, ctypes.c_void_p]
    L.lnl_crc32c_verify_csr_dev.restype = ctypes.c_int
    L.lnl_crc32c_verify_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p,
                                            ctypes.c_void_p]
    L.lnl_crc32c_batch_host.restype = ctypes.c_int
    L.lnl_crc32c_batch_host.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_int]
    L.lnl_crc32c_batch_host_multi.restype = ctypes.c_int
    L.lnl_crc32c_batch_host_multi.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, ctypes.c_int]
    L.lnl_packet_verify.restype = ctypes.c_int
    L.lnl_packet_verify.argtypes = [_c_u8p, ctypes.c_size_t]
    L.lnl_inbound_status.restype = ctypes.c_int
    L.lnl_inbound_status.argtypes = [_c_u8p, ctypes.c_size_t]
    L.lnl_inbound_filter_csr_dev.restype = ctypes.c_int
    L.lnl_inbound_filter_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_void_p]
    L.lnl_inbound_filter_host.restype = ctypes.c_int
    L.lnl_inbound_filter_host.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_int]
    L.lnl_ingress_recv_batch.restype = ctypes.c_int
    L.lnl_ingress_recv_batch.argtypes = [ctypes.c_int, _c_u8p, ctypes.c_size_t, _c_u8p, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_int]
    L.lnl_crc32c_append_host.restype = ctypes.c_int
    L.lnl_crc32c_append_host.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, ctypes.c_int]
    L.lnl_egress_send_batch.restype = ctypes.c_int64
    L.lnl_egress_send_batch.argtypes = [ctypes.c_int, _c_u8p, _c_u8p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_uint32, _c_u8p, ctypes.c_int]
    L.lnl_dispatch_csr_dev.restype = ctypes.c_int
    L.lnl_dispatch_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, _c_u8p, _c_u8p,
                                       ctypes.c_uint32, _c_u8p, ctypes.c_void_p]
    L.lnl_inbound_filter_dispatch_csr_dev.restype = ctypes.c_int
    L.lnl_inbound_filter_dispatch_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, _c_u8p,
                                                      _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_void_p]
    dopts_p = ctypes.POINTER(DispatchOpts)
    L.lnl_dispatch_csr_dev_ex.restype = ctypes.c_int
    L.lnl_dispatch_csr_dev_ex.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, _c_u8p, _c_u8p, _c_u8p,
                                          ctypes.c_uint32, _c_u8p, dopts_p, ctypes.c_void_p]
    L.lnl_inbound_filter_dispatch_csr_dev_ex.restype = ctypes.c_int
    L.lnl_inbound_filter_dispatch_csr_dev_ex.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, _c_u8p,
                                                         _c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, dopts_p,
                                                         ctypes.c_void_p]
    L.lnl_xor_layer.restype = ctypes.c_int
    L.lnl_xor_layer.argtypes = [_c_u8p, ctypes.c_size_t, _c_u8p, ctypes.c_size_t]
    L.lnl_xor_layer_csr_dev.restype = ctypes.c_int
    L.lnl_xor_layer_csr_dev.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_size_t, ctypes.c_void_p]
    L.lnl_xor_layer_fixed_dev.restype = ctypes.c_int
    L.lnl_xor_layer_fixed_dev.argtypes = [_c_u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _c_u8p,
                                          ctypes.c_size_t, ctypes.c_void_p]
    opts_p = ctypes.POINTER(HostOpts)
    L.lnl_crc32c_batch_host_ex.restype = ctypes.c_int
    L.lnl_crc32c_batch_host_ex.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_int, opts_p]
    L.lnl_inbound_filter_host_ex.restype = ctypes.c_int
    L.lnl_inbound_filter_host_ex.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, ctypes.c_int, opts_p]
    L.lnl_crc32c_append_host_ex.restype = ctypes.c_int
    L.lnl_crc32c_append_host_ex.argtypes = [_c_u8p, _c_u8p, ctypes.c_uint32, _c_u8p, _c_u8p, ctypes.c_int, opts_p]
    L.lnl_stream_release.restype = ctypes.c_int
    L.lnl_stream_release.argtypes = [ctypes.c_void_p]
    L.lnl_diag_fill_span_arrivals.restype = ctypes.c_int
    L.lnl_diag_fill_span_arrivals.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.lnl_crc32c_last_error.restype = ctypes.c_char_p
    L.lnl_crc32c_last_error.argtypes = []
    L.lnl_crc32c_abi_version.restype = ctypes.c_int
    L.lnl_crc32c_abi_version.argtypes = []
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().lnl_crc32c_last_error().decode(errors="replace")
        raise Crc32cError(rc, what, msg)
