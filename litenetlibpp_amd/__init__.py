"""litenetlibpp_amd -- MI355X-native CRC-32C packet-layer path for a
LiteNetLibPP-style reliable-UDP stack.

The product is ``liblnl_crc32c.so`` (gfx950 HIP kernels + a C ABI,
``include/lnl_crc32c.h``); this package is its Python mirror.
"""
from .crc32c import (  # noqa: F401
    EXTRA_PACKET_SIZE,
    Crc32cError,
    Crc32cLayer,
    append_csr,
    append_host,
    batch_csr,
    batch_fixed,
    batch_host,
    batch_host_multi,
    dispatch,
    DISPATCH_TAIL_DATAGRAM,
    DISPATCH_TAIL_LAYER,
    DISPATCH_TAIL_ZERO,
    egress_send_batch,
    filter_dispatch,
    xor_layer,
    xor_layer_csr,
    xor_layer_fixed,
    inbound_filter,
    inbound_filter_host,
    ingress_recv_batch,
    INGRESS_SLOT,
    inbound_status,
    packet_verify,
    INBOUND_ACCEPT,
    INBOUND_DROP_CRC,
    INBOUND_MALFORMED,
    crc32c,
    crc32c_extend,
    mtu_with_layer,
    verify_csr,
    stream_release,
    HOST_DEFAULT_STREAMS,
    HOST_MAX_STREAMS,
)
from ._lib import LIB_PATH, HostOpts, lib  # noqa: F401

__version__ = "0.1.0"
