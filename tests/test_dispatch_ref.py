"""The MERGED cut pinned to the REFERENCE's own net_peer::process_packet
(/root/reference/src/lnl/net_peer.cpp:164-187).

tests/golden/dispatch_ref.* hold crafted containers and what the reference --
compiled where it lies and run as a connected net_manager pair
(oracle/refnet, tests/golden/make_dispatch_ref.py) -- delivered for each one.
Here the restatement (oracle.dispatch, then oracle.deliver as the caller's
process_packet for each dispatched packet) must give exactly those deliveries,
except where the reference reads past the datagram (its walk is bounded by the
2048-byte pooled buffer, whose zero-filled tail it then cuts): there the product
stops at the datagram's end, so it must give exactly the deliveries that
precede that read ("agree").  The GPU entry points are held to the same
fixture in tests/test_gpu_parity.py::test_dispatch_reference_fixture."""
import json
import os
import struct

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(variant="plain"):
    """(containers, connection number, per-container records) of the plain
    reference (dispatch_ref.json) or of the reference with INTEGRATION.md's
    layer compiled in (variant "layer": dispatch_ref_layer.json)."""
    blob = open(os.path.join(GOLD, "dispatch_ref.bin"), "rb").read()
    assert blob[:4] == b"LNLM"
    count, conn = struct.unpack_from("<II", blob, 4)
    pos, cont = 12, []
    for _ in range(count):
        (n,) = struct.unpack_from("<I", blob, pos)
        cont.append(blob[pos + 4:pos + 4 + n])
        pos += 4 + n
    assert pos == len(blob)
    name = {"plain": "dispatch_ref.json", "layer": "dispatch_ref_layer.json"}[variant]
    meta = json.load(open(os.path.join(GOLD, name)))
    assert meta["connection_number"] == conn and len(meta["containers"]) == count
    return cont, conn, meta["containers"]


def with_crc(c):
    return c + struct.pack("<I", oracle.crc(np.frombuffer(c, np.uint8)))


def expected(rec):
    """The deliveries the product must give for one container."""
    ref = [bytes.fromhex(p) for p in rec["delivered"]]
    return ref[: rec["agree"]] if rec["reads_past_datagram"] else ref


def reference_deliveries(rec):
    """Every delivery the reference made for one container (the tail modes
    must give all of them)."""
    return [bytes.fromhex(p) for p in rec["delivered"]]


def packet_bytes(wire, start, length, avail):
    """A dispatched packet as the caller builds it: its in-burst bytes, then
    the zero fill (include/lnl_crc32c.h, d_pkt_avail)."""
    return bytes(wire[start:start + avail]) + bytes(length - avail)


def product_deliveries(wires, packets, conn):
    """Per datagram: the user-visible deliveries of the dispatched packets
    (datagram index, start within the datagram, length)."""
    out = [[] for _ in wires]
    for i, o, L in packets:
        out[i] += oracle.deliver(wires[i][o:o + L], conn)
    return out


def test_fixture_covers_the_cases():
    cont, conn, recs = load_fixture()
    assert len(cont) >= 100 and conn == 0
    assert sum(len(r["delivered"]) for r in recs) > 300
    n_past = sum(r["reads_past_datagram"] for r in recs)
    assert 10 <= n_past < len(recs) // 4          # truncated / dangling entries, the minority
    assert any(r["agree"] < len(r["delivered"]) for r in recs)  # the reference delivers zero-padded packets
    assert any(len(c) == 1 for c in cont)          # header-only container
    assert any(len(c) >= 1400 for c in cont)       # near the MTU


def test_restatement_matches_the_reference():
    cont, conn, recs = load_fixture()
    wires = [with_crc(c) for c in cont]
    status = [oracle.inbound_status(np.frombuffer(w, np.uint8)) for w in wires]
    assert all(s == oracle.INBOUND_ACCEPT for s in status)
    got = product_deliveries(wires, oracle.dispatch(wires, status), conn)
    bad = [i for i, (g, r) in enumerate(zip(got, recs)) if g != expected(r)]
    assert not bad, bad[:10]


TAILS = [("plain", oracle.DISPATCH_TAIL_ZERO), ("layer", oracle.DISPATCH_TAIL_LAYER)]


def test_layer_fixture_differs_only_past_the_datagram():
    """The two reference variants cut every container alike up to the first
    read past the datagram; past it the layer variant reads the CRC field."""
    cont, _, plain = load_fixture("plain")
    _, _, layer = load_fixture("layer")
    assert sum(len(r["delivered"]) for r in layer) > 300
    diff = 0
    for c, p, q in zip(cont, plain, layer):
        assert p["reads_past_datagram"] == q["reads_past_datagram"]
        assert p["delivered"][:p["agree"]] == q["delivered"][:q["agree"]]
        if not p["reads_past_datagram"]:
            assert p["delivered"] == q["delivered"]
        diff += p["delivered"] != q["delivered"]
    assert diff >= 10


@pytest.mark.parametrize("variant,tail", TAILS)
def test_restatement_tail_matches_the_reference_exactly(variant, tail):
    """Under the reference's own tail rule (walk bounded by the zero-filled
    2048-byte buffer, net_peer.cpp:167-183) the restatement gives EVERY
    delivery the reference made, the zero-padded ones included."""
    cont, conn, recs = load_fixture(variant)
    wires = [with_crc(c) for c in cont]
    status = [oracle.inbound_status(np.frombuffer(w, np.uint8)) for w in wires]
    got = [[] for _ in wires]
    for i, o, L, av in oracle.dispatch_ex(wires, status, tail):
        assert 0 <= av <= L
        got[i] += oracle.deliver(packet_bytes(wires[i], o, L, av), conn, ref_tail=True)
    bad = [i for i, (g, r) in enumerate(zip(got, recs)) if g != reference_deliveries(r)]
    assert not bad, bad[:10]
    # and the padded packets really occur
    assert any(av < L for _, _, L, av in oracle.dispatch_ex(wires, status, tail))


def test_tail_rules_agree_on_well_formed_containers():
    cont, conn, recs = load_fixture()
    wires = [with_crc(c) for c, r in zip(cont, recs) if not r["reads_past_datagram"]]
    status = [oracle.INBOUND_ACCEPT] * len(wires)
    base = oracle.dispatch_ex(wires, status, oracle.DISPATCH_TAIL_DATAGRAM)
    for tail in (oracle.DISPATCH_TAIL_ZERO, oracle.DISPATCH_TAIL_LAYER):
        assert oracle.dispatch_ex(wires, status, tail) == base
