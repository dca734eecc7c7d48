"""The C-ABI boundary without a GPU: the library loads, exports every entry
point include/lnl_crc32c.h declares, the per-datagram CPU half matches the
oracle, and the batch half refuses to run (no CPU fallback) when no gfx950
device is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lnl_crc32c.h")


@pytest.fixture(scope="module")
def pkg():
    import litenetlibpp_amd as P
    if not os.path.exists(P.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "litenetlibpp_amd")], check=True,
                       capture_output=True)
    return P


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*[\w ]+?\**\s*\**(lnl_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("lnl_crc32c", "lnl_crc32c_extend", "lnl_crc32c_batch_fixed_dev",
              "lnl_crc32c_batch_csr_dev", "lnl_crc32c_batch_host", "lnl_crc32c_verify_csr_dev",
              "lnl_crc32c_layer_outbound", "lnl_crc32c_layer_inbound", "lnl_crc32c_last_error",
              "lnl_crc32c_batch_host_multi", "lnl_packet_verify", "lnl_inbound_status",
              "lnl_inbound_filter_csr_dev", "lnl_inbound_filter_host", "lnl_ingress_recv_batch",
              "lnl_dispatch_csr_dev", "lnl_inbound_filter_dispatch_csr_dev", "lnl_xor_layer", "lnl_xor_layer_csr_dev", "lnl_xor_layer_fixed_dev",
              "lnl_crc32c_append_host", "lnl_egress_send_batch", "lnl_crc32c_batch_host_ex",
              "lnl_inbound_filter_host_ex", "lnl_crc32c_append_host_ex", "lnl_stream_release",
              "lnl_diag_fill_span_arrivals", "lnl_dispatch_csr_dev_ex", "lnl_inbound_filter_dispatch_csr_dev_ex"):
        assert s in syms


def test_library_exports_every_declared_symbol(pkg):
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (lnl_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    assert pkg.lib().lnl_crc32c_abi_version() == 10


def test_ctypes_bindings_match_the_header(pkg):
    """Every entry point the Python mirror binds takes as many arguments as
    include/lnl_crc32c.h declares."""
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    L = pkg.lib()
    checked = 0
    for name, params in re.findall(r"\b(lnl_\w+)\s*\(([^)]*)\)\s*;", txt):
        argtypes = getattr(getattr(L, name), "argtypes", None)
        if argtypes is None:
            continue
        count = 0 if params.strip() in ("", "void") else params.count(",") + 1
        assert len(argtypes) == count, (name, len(argtypes), count)
        checked += 1
    assert checked >= 15


def test_cpu_crc_matches_oracle(pkg):
    rng = np.random.default_rng(11)
    assert pkg.crc32c(b"123456789") == 0xE3069283
    assert pkg.crc32c(b"") == 0
    for L in list(range(0, 200)) + [1399, 1400, 1432, 9000, 65507]:
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert pkg.crc32c(d) == oracle.crc(d, "bitwise"), L


def test_cpu_extend(pkg):
    rng = np.random.default_rng(12)
    a = rng.integers(0, 256, 1001, dtype=np.uint8).tobytes()
    b = rng.integers(0, 256, 433, dtype=np.uint8).tobytes()
    assert pkg.crc32c_extend(pkg.crc32c(a), b) == pkg.crc32c(a + b)
    assert pkg.crc32c_extend(0, a) == pkg.crc32c(a)
    assert pkg.crc32c_extend(pkg.crc32c(a), b"") == pkg.crc32c(a)


def test_layer_roundtrip_and_drop(pkg):
    layer = pkg.Crc32cLayer()
    payload = bytes([0x0B]) + bytes(range(200))   # header byte (MERGED) + body
    shared = bytearray(b"xx" + payload + b"yy")    # send_raw's const shared buffer
    before = bytes(shared)
    wire = layer.process_outbound(shared, 2, len(payload))
    assert bytes(shared) == before                 # source untouched
    assert wire[:-4] == payload and len(wire) == len(payload) + 4
    assert int.from_bytes(wire[-4:], "little") == oracle.crc(payload, "bitwise")
    assert layer.process_inbound(wire) == payload
    bad = bytearray(wire)
    bad[7] ^= 0x40
    assert layer.process_inbound(bytes(bad)) is None
    assert layer.process_inbound(wire[:4]) is None   # < header + CRC
    assert layer.process_inbound(pkg.Crc32cLayer().process_outbound(b"\x01")) == b"\x01"
    assert layer.dropped == 2
    assert pkg.mtu_with_layer(1432) == 1428


def test_batch_entry_points_refuse_without_gpu(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; covered by the gpu suite")
    L = pkg.lib()
    buf = (ctypes.c_uint8 * 64)()
    out = (ctypes.c_uint32 * 4)()
    rc = L.lnl_crc32c_batch_fixed_dev(ctypes.addressof(buf), 16, 16, 4, ctypes.addressof(out), None)
    assert rc == -19, rc            # -ENODEV, never a CPU answer
    assert L.lnl_crc32c_last_error()
    assert list(out) == [0, 0, 0, 0]
    # n == 0 is valid and touches nothing
    assert L.lnl_crc32c_batch_fixed_dev(None, 0, 0, 0, None, None) == 0
    # the multi-device host form: every range fails the same way, nothing computed
    off = (ctypes.c_uint64 * 5)(0, 16, 32, 48, 64)
    devs = (ctypes.c_int * 2)(0, 0)
    rc = L.lnl_crc32c_batch_host_multi(ctypes.addressof(buf), ctypes.addressof(off), 4, ctypes.addressof(out),
                                       ctypes.addressof(devs), 2)
    assert rc == -19, rc
    assert b"range" in L.lnl_crc32c_last_error()
    assert list(out) == [0, 0, 0, 0]
    assert L.lnl_crc32c_batch_host_multi(ctypes.addressof(buf), ctypes.addressof(off), 4, ctypes.addressof(out),
                                         None, 0) == -22
    # the fused filter + dispatch: n == 0 needs the device for its total only
    # after the argument checks; a missing total is refused first
    tot = (ctypes.c_uint32 * 1)(7)
    st = (ctypes.c_uint8 * 4)()
    assert L.lnl_inbound_filter_dispatch_csr_dev(ctypes.addressof(buf), ctypes.addressof(off), 4,
                                                 ctypes.addressof(st), None, None, None, 0, None, None) == -22
    rc = L.lnl_inbound_filter_dispatch_csr_dev(ctypes.addressof(buf), ctypes.addressof(off), 4, ctypes.addressof(st),
                                               None, None, None, 0, ctypes.addressof(tot), None)
    assert rc == -19, rc
    assert list(st) == [0, 0, 0, 0] and tot[0] == 7
    # the host outbound layer: no device, no wire bytes
    wire = (ctypes.c_uint8 * 80)()
    rc = L.lnl_crc32c_append_host(ctypes.addressof(buf), ctypes.addressof(off), 4, ctypes.addressof(wire), None, 0)
    assert rc == -19, rc
    assert bytes(wire) == bytes(80)


def test_product_library_has_no_experiment_knobs(pkg):
    """The product .so has one kernel path per layout: no run-time path
    selection and no LNL_* environment knobs (those live in the experiments
    build, tools/kvariants.py -> build/variants/*.so)."""
    import subprocess
    from litenetlibpp_amd._lib import LIB_PATH
    blob = open(LIB_PATH, "rb").read()
    for knob in (b"LNL_CSR_PATH", b"LNL_BUCKET_WINDOW", b"LNL_BUCKET_SPREAD", b"LNL_BUCKET_XCD",
                 b"LNL_DISPATCH_ONEPASS", b"LNL_DISPATCH_NT", b"LNL_XOR_FLAT"):
        assert knob not in blob, knob
    exported = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True,
                              check=True).stdout
    assert "lnl_crc32c_set_csr_path" not in exported


def test_host_batch_offsets_checked_before_the_call(pkg):
    """The host entry points never see the buffer's size, so the wrappers check
    the offsets first: out of range, decreasing or negative offsets raise
    before any copy (a negative int64 wrapped to a huge uint64)."""
    import numpy as np
    import pytest
    data = np.zeros(100, np.uint8)
    for off in (np.array([0, 50, 101], np.uint64), np.array([0, 60, 50], np.int64),
                np.array([-8, 10], np.int64)):
        for fn in (lambda o: pkg.batch_host(data, o, 0), lambda o: pkg.inbound_filter_host(data, o, 0),
                   lambda o: pkg.batch_host_multi(data, o, [0]), lambda o: pkg.append_host(data, o, 0),
                   lambda o: pkg.egress_send_batch(0, data, o)):
            with pytest.raises(ValueError):
                fn(off)


def test_host_opts_checked_without_gpu(pkg):
    """lnl_host_opts (include/lnl_crc32c.h) is validated before anything else:
    a bad size, a nonzero reserved field or more than LNL_HOST_MAX_STREAMS
    streams give -EINVAL even for an empty batch; good options on a machine
    without a GPU give -ENODEV, never a CPU answer."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; covered by the gpu suite")
    L = pkg.lib()
    assert ctypes.sizeof(pkg.HostOpts) == 24
    buf = (ctypes.c_uint8 * 64)()
    off = (ctypes.c_uint64 * 3)(0, 16, 64)
    out = (ctypes.c_uint32 * 2)()
    bad = [pkg.HostOpts.make(streams=9), pkg.HostOpts(8, 2, 0, 0, 0), pkg.HostOpts(24, 2, 0, 1, 0)]
    for o in bad:
        for n in (0, 2):
            assert L.lnl_crc32c_batch_host_ex(ctypes.addressof(buf), ctypes.addressof(off), n, ctypes.addressof(out),
                                              0, ctypes.pointer(o)) == -22
            assert L.lnl_inbound_filter_host_ex(ctypes.addressof(buf), ctypes.addressof(off), n,
                                                ctypes.addressof(out), 0, ctypes.pointer(o)) == -22
            assert L.lnl_crc32c_append_host_ex(ctypes.addressof(buf), ctypes.addressof(off), n,
                                               ctypes.addressof(buf), None, 0, ctypes.pointer(o)) == -22
    good = pkg.HostOpts.make(streams=2, chunk_datagrams=1)
    assert L.lnl_crc32c_batch_host_ex(ctypes.addressof(buf), ctypes.addressof(off), 0, ctypes.addressof(out), 0,
                                      ctypes.pointer(good)) == 0
    assert L.lnl_crc32c_batch_host_ex(ctypes.addressof(buf), ctypes.addressof(off), 2, ctypes.addressof(out), 0,
                                      ctypes.pointer(good)) == -19
    assert L.lnl_crc32c_batch_host_ex(ctypes.addressof(buf), ctypes.addressof(off), 2, ctypes.addressof(out), 0,
                                      None) == -19
    assert list(out) == [0, 0]
    with pytest.raises(ValueError):
        pkg.batch_host(np.zeros(64, np.uint8), np.array([0, 64], np.uint64), 0, streams=9)


def test_dispatch_opts_rejected_before_device_work(pkg):
    """lnl_dispatch_csr_dev_ex / lnl_inbound_filter_dispatch_csr_dev_ex check
    their lnl_dispatch_opts first: -EINVAL for a short struct, an unknown tail
    rule or a nonzero reserved word, without touching a device (no GPU here)."""
    import ctypes
    from litenetlibpp_amd._lib import DispatchOpts
    L = pkg.lib()
    total = ctypes.c_uint32(0)
    bad = [DispatchOpts(4, 1), DispatchOpts(ctypes.sizeof(DispatchOpts), 3),
           DispatchOpts(ctypes.sizeof(DispatchOpts), 1, (ctypes.c_uint32 * 2)(0, 1))]
    for o in bad:
        for f in (L.lnl_dispatch_csr_dev_ex, L.lnl_inbound_filter_dispatch_csr_dev_ex):
            rc = f(None, None, 0, None, None, None, None, None, 0, ctypes.addressof(total), ctypes.byref(o), None)
            assert rc == -22, (f.__name__, rc)
    assert pkg.DISPATCH_TAIL_DATAGRAM == 0 and pkg.DISPATCH_TAIL_ZERO == 1 and pkg.DISPATCH_TAIL_LAYER == 2
