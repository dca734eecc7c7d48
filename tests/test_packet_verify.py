"""The packet acceptance test after the CRC layer (net_packet::verify,
/root/reference/include/lnl/net_packet.h:120-131, applied by
net_manager::on_message_received at src/lnl/net_manager.cpp:343) -- CPU.

Pinned to the REFERENCE: tests/golden/packet_verify.bin holds verify() of the
reference's own header-only net_packet, compiled where it lies by
`make -C oracle ref` (tests/golden/make_packet_golden.py).  Checked here: the
restatement in tests/oracle.py, the product's C ABI (lnl_packet_verify,
lnl_inbound_status) and, where oracle/_ref was built, the reference itself on
random packets."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def golden():
    return np.fromfile(os.path.join(GOLD, "packet_verify.bin"), dtype=np.uint8).reshape(256, 48)


@pytest.fixture(scope="module")
def pkg():
    import litenetlibpp_amd as P
    P.lib()
    return P


def test_header_sizes_match_reference():
    g = json.load(open(os.path.join(GOLD, "packet_header_sizes.json")))
    # 17 initialisers for 18 properties: EMPTY (17) reads 0 (net_packet.h:20-38 vs net_enums.h:47-68)
    assert g["header_sizes"] == oracle.HEADER_SIZES
    assert g["header_sizes"][17] == 0


def test_restatement_matches_reference_golden(golden):
    for b in range(256):
        for s in range(48):
            assert bool(golden[b, s]) == oracle.packet_verify(b, s), (b, s)


def test_product_cpu_verify_matches_reference_golden(pkg, golden):
    buf = np.zeros(64, dtype=np.uint8)
    for b in range(256):
        buf[0] = b
        for s in range(48):
            assert pkg.packet_verify(buf[:s]) == bool(golden[b, s]), (b, s)


def test_reference_itself_on_random_packets(pkg):
    L = oracle.load_ref_packet()
    if L is None:
        pytest.skip("oracle/_ref not built (no /root/reference here); golden fixture covers it")
    rng = np.random.default_rng(5)
    for _ in range(3000):
        s = int(rng.integers(0, 1433))
        p = rng.integers(0, 256, max(s, 1), dtype=np.uint8)
        ref = bool(L.ref_packet_verify(p.ctypes.data, s))
        assert ref == oracle.packet_verify(int(p[0]), s)
        assert ref == pkg.packet_verify(p[:s])


def test_inbound_status_cpu(pkg):
    rng = np.random.default_rng(6)
    layer = pkg.Crc32cLayer()
    for _ in range(2000):
        s = int(rng.integers(0, 40))
        body = rng.integers(0, 256, s, dtype=np.uint8)
        wire = np.frombuffer(layer.process_outbound(body.tobytes()), dtype=np.uint8).copy()
        if rng.random() < 0.3 and wire.size:
            wire[int(rng.integers(0, wire.size))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        exp = oracle.inbound_status(wire)
        assert pkg.inbound_status(wire) == exp
    # every status is reachable
    ok = np.frombuffer(layer.process_outbound(bytes([0x01, 0, 0, 0])), dtype=np.uint8)   # CHANNELED, 4 B
    bad = np.frombuffer(layer.process_outbound(bytes([0x01, 0, 0])), dtype=np.uint8)      # CHANNELED, 3 B
    assert pkg.inbound_status(ok) == pkg.INBOUND_ACCEPT
    assert pkg.inbound_status(bad) == pkg.INBOUND_MALFORMED
    assert pkg.inbound_status(ok[:4]) == pkg.INBOUND_DROP_CRC
