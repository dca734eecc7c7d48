#!/usr/bin/env python3
"""Fixture generator: the MERGED-container cut as the REFERENCE itself performs
it.

Crafted MERGED containers -- well-formed, nested, with a sub-header verify()
rejects, with zero-length, truncated and dangling entries, with sub-packets of
another connection number -- are sent one by one from a connected client's own
endpoint into the reference's net_manager (oracle/_ref/net/plain/refnet_driver
merged: the reference compiled where it lies, oracle/refnet/build.py), whose
net_peer::process_packet cuts them (/root/reference/src/lnl/net_peer.cpp:164-187)
and delivers every UNRELIABLE sub-packet to the listener (:240-243).  What it
delivered, per container, is the fixture:

  tests/golden/dispatch_ref.bin   the containers ("LNLM", u32 count, u32
                                  connection number, then u32 length + bytes each;
                                  no CRC field)
  tests/golden/dispatch_ref.json  per container: the reference's deliveries
                                  (hex payloads after the 1-byte header), and
                                  "agree" -- how many of them precede the first
                                  read past the datagram

The reference bounds its walk by the pooled buffer's capacity (:171,
buffer_size() = 2048), not the datagram: an entry that runs past the datagram,
or a size field in its last byte, is read from the buffer's zero-filled tail
(every pooled packet is a fresh zeroed 2048-byte buffer: pool_recycle deletes
any packet whose buffer exceeds MAX_PACKET_SIZE, net_manager.cpp:290, and
ensure() zero-fills).  The product stops at the datagram's end instead, so for
those containers only the first "agree" deliveries are common; ref_cut() below
restates the reference's rules INCLUDING the zero tail, and this script checks it
against what the reference actually delivered before writing anything.

The same containers also go through the reference with the layer compiled in
as INTEGRATION.md 2 writes it (variant crc_src: the injected datagram carries
its CRC, receive_logic strips it by shrinking the packet).  The 4 CRC bytes
then stay in the buffer right after the datagram, and the reference cuts them
before the zeros:

  tests/golden/dispatch_ref_layer.json   the same records for that variant

ref_cut(..., tail=LE32(crc)) restates that and is checked the same way.

Run in the build container (needs /root/reference and g++):
    python3 oracle/refnet/build.py plain crc_src && python3 tests/golden/make_dispatch_ref.py
"""
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "net", "plain", "refnet_driver")
DRIVER_LAYER = os.path.join(ROOT, "oracle", "_ref", "net", "crc_src", "refnet_driver")

MERGED, UNRELIABLE = 0x0C, 0x00
CAP = 2048  # buffer_size() of every pooled packet (net_packet(): ensure(1432) -> 2048)
HEADER_SIZES = [1, 4, 4, 3, 11, 18, 15, 9, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0]  # net_packet.h:20-38


def verify(b0, size):
    p = b0 & 0x1F
    if p >= 18:
        return False
    hs = HEADER_SIZES[p]
    return size >= hs and (not (b0 & 0x80) or size >= hs + 6)


def ref_cut(pkt, conn, past=False, tail=b""):
    """process_packet (net_peer.cpp:138-243) on pkt for the cases crafted here:
    the connection-number check (:156), MERGED (:164-187, walk bounded by the
    zero-filled 2048-byte buffer, whose bytes after pkt are `tail` and then
    zeros), UNRELIABLE (:240, deliver pkt[1:]).  Returns [(payload, past)]:
    past = produced after a read beyond pkt's own bytes."""
    buf = bytes(pkt) + bytes(tail) + bytes(CAP - len(pkt) - len(tail))
    if ((buf[0] & 0x60) >> 5) != conn:
        return []
    prop = buf[0] & 0x1F
    if prop == UNRELIABLE:
        return [(bytes(pkt[1:]), past)]
    if prop != MERGED:
        return []
    out, pos = [], 1
    while pos < len(pkt):
        size = buf[pos] | (buf[pos + 1] << 8)
        past_here = past or pos + 2 > len(pkt)
        pos += 2
        if CAP - pos < size:
            break
        sub = buf[pos:pos + size]
        past_here = past_here or pos + size > len(pkt)
        if not (size and verify(sub[0], size)):  # a size-0 packet's byte 0 is 0: verify() fails
            break
        pos += size
        out += ref_cut(sub, conn, past_here)
    return out


def build_containers(conn, seed=2024):
    rng = np.random.default_rng(seed)
    h = conn << 5

    def unrel(n):
        return bytes([UNRELIABLE | h]) + rng.integers(0, 256, n, dtype=np.uint8).tobytes()

    def entry(p):
        return len(p).to_bytes(2, "little") + p

    def merged(parts):
        return bytes([MERGED | h]) + b"".join(entry(p) for p in parts)

    out = []
    out.append(bytes([MERGED | h]))                                      # header only
    for _ in range(60):                                                  # well-formed
        out.append(merged([unrel(int(rng.integers(0, 300))) for _ in range(int(rng.integers(1, 7)))]))
    out.append(merged([unrel(0)] * 5))                                   # header-only sub-packets
    out.append(merged([unrel(250)] * 5))                                 # config-1 shape
    for bad in (0x1F | h, 0x01 | h, 0x81 | h, 0x80 | h, 0x11 | h):      # sub-header verify() rejects
        for k in range(3):
            parts = [unrel(int(rng.integers(1, 80))) for _ in range(4)]
            n = {0x1F: 5, 0x01: 2, 0x81: 8, 0x80: 5, 0x11: 0}[bad & 0x9F]
            parts[k] = bytes([bad]) + bytes(n)
            if bad & 0x1F == 0x11:   # property 17 (EMPTY) has header size 0: verify() accepts it
                parts[k] = bytes([bad])
            out.append(merged(parts))
    for k in range(4):                                                   # zero-length entry
        parts = [entry(unrel(int(rng.integers(1, 60)))) for _ in range(4)]
        parts.insert(k, (0).to_bytes(2, "little"))
        out.append(bytes([MERGED | h]) + b"".join(parts))
    for _ in range(12):                                                  # nested containers
        inner = merged([unrel(int(rng.integers(0, 50))) for _ in range(int(rng.integers(1, 4)))])
        parts = [unrel(int(rng.integers(0, 40))), inner, unrel(int(rng.integers(0, 40)))]
        if rng.integers(0, 2):
            parts.append(merged([inner, unrel(3)]))                      # two levels
        out.append(merged(parts))
    for other in (1, 2, 3):                                              # another connection number
        parts = [unrel(10), bytes([UNRELIABLE | (((conn + other) & 3) << 5)]) + b"xyz", unrel(20)]
        out.append(merged(parts))
    for _ in range(10):                                                  # truncated last entry
        parts = [unrel(int(rng.integers(1, 60))) for _ in range(3)]
        c = merged(parts)
        cut = int(rng.integers(1, len(parts[-1])))
        out.append(c[:-cut])
    for _ in range(4):                                                   # size field in the last byte
        out.append(merged([unrel(int(rng.integers(1, 60))) for _ in range(2)]) + bytes([int(rng.integers(1, 40))]))
    out.append(merged([unrel(5)]) + (7).to_bytes(2, "little"))           # size field, nothing after it
    out.append(merged([unrel(5)]) + (0).to_bytes(2, "little"))           # zero size field at the end
    out.append(merged([unrel(5)]) + (3000).to_bytes(2, "little") + b"\x00ab")  # past the buffer: stops
    big = merged([unrel(n) for n in (282, 282, 282, 283, 283)])         # exactly the MTU with the layer
    assert len(big) == 1428
    out.append(big)
    return out


def run_driver(driver, blob):
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.json")
        with open(fin, "wb") as f:
            f.write(blob)
        r = subprocess.run([driver, "merged", fin, fout], capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            sys.exit(f"driver failed: {r.stdout}\n{r.stderr}")
        with open(fout) as f:
            return json.load(f)


def records_for(cont, conn, res, tails):
    assert res["containers"] == len(cont) and len(res["delivered"]) == len(cont)
    records, divergent = [], 0
    for i, (c, got, tail) in enumerate(zip(cont, res["delivered"], tails)):
        assert all(m == 4 for m, _ in got), (i, got)  # DELIVERY_METHOD::UNRELIABLE (net_enums.h)
        observed = [bytes.fromhex(p) for _, p in got]
        model = ref_cut(c, conn, tail=tail)
        assert observed == [p for p, _ in model], (i, c.hex(), observed, model)
        agree = next((k for k, (_, past) in enumerate(model) if past), len(model))
        reads_past = any(past for _, past in model) or _reads_past(c, conn)
        divergent += reads_past
        records.append({"delivered": [p.hex() for p in observed], "agree": agree, "reads_past_datagram": reads_past})
    return records, divergent


def main():
    for d, v in ((DRIVER, "plain"), (DRIVER_LAYER, "crc_src")):
        if not os.path.exists(d):
            sys.exit(f"{d} missing: python3 oracle/refnet/build.py {v}")
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle  # the CPU CRC-32C (test infrastructure): the layer's field
    conn = 0  # a manager's first connection (net_manager.cpp:984 counts up from there)
    cont = build_containers(conn)
    blob = b"LNLM" + struct.pack("<II", len(cont), conn) + b"".join(struct.pack("<I", len(c)) + c for c in cont)
    src = ("oracle/_ref/net/{}/refnet_driver merged (the reference's net_peer::process_packet, "
           "net_peer.cpp:164-187), tests/golden/make_dispatch_ref.py")
    for name, driver, variant, tails in (
            ("dispatch_ref.json", DRIVER, "plain", [b""] * len(cont)),
            ("dispatch_ref_layer.json", DRIVER_LAYER, "crc_src",
             [struct.pack("<I", oracle.crc(np.frombuffer(c, np.uint8))) for c in cont])):
        records, divergent = records_for(cont, conn, run_driver(driver, blob), tails)
        with open(os.path.join(HERE, name), "w") as f:
            json.dump({"source": src.format(variant), "connection_number": conn, "containers": records}, f, indent=0)
        print(f"{name}: {len(cont)} containers, {sum(len(r['delivered']) for r in records)} deliveries, "
              f"{divergent} reading past the datagram")
    with open(os.path.join(HERE, "dispatch_ref.bin"), "wb") as f:
        f.write(blob)


def _reads_past(c, conn):
    """True when the reference's walk of c (top level) reads a byte beyond it
    even if nothing it delivers depends on that (e.g. a trailing zero size)."""
    if ((c[0] & 0x60) >> 5) != conn or (c[0] & 0x1F) != MERGED:
        return False
    buf = bytes(c) + bytes(CAP - len(c))
    pos = 1
    while pos < len(c):
        size = buf[pos] | (buf[pos + 1] << 8)
        if pos + 2 > len(c):
            return True
        pos += 2
        if CAP - pos < size:
            return False
        if pos + size > len(c):
            return True
        if not (size and verify(buf[pos], size)):
            return False
        pos += size
    return False


if __name__ == "__main__":
    main()
