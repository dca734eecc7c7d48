#!/usr/bin/env python3
"""Generate tests/golden/packet_verify.bin from the REFERENCE's own
lnl::net_packet::verify(), compiled where it lies by `make -C oracle ref`
(oracle/ref_packet_verify.cpp -> oracle/_ref/libref_packet.so).

packet_verify.bin: uint8[256][48], entry [b][s] = verify() of a packet of
size s whose byte 0 is b (remaining bytes zero).  Sizes 0..47 cover every
threshold (largest header 18, + 6 fragment bytes).
packet_header_sizes.json: get_header_size() for property bytes 0..17.

Run (in the container that has /root/reference): python tests/golden/make_packet_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    L = oracle.load_ref_packet()
    assert L is not None, "oracle/_ref/libref_packet.so was not built"
    out = np.zeros((256, 48), dtype=np.uint8)
    buf = np.zeros(64, dtype=np.uint8)
    for b in range(256):
        buf[0] = b
        for s in range(48):
            out[b, s] = L.ref_packet_verify(buf.ctypes.data, s)
    out.tofile(os.path.join(HERE, "packet_verify.bin"))
    sizes = [L.ref_packet_header_size(p) for p in range(18)]
    with open(os.path.join(HERE, "packet_header_sizes.json"), "w") as f:
        json.dump({"header_sizes": sizes, "source": "reference net_packet::get_header_size(), "
                   "oracle/ref_packet_verify.cpp"}, f, indent=1)
    print("header sizes", sizes, "accepting entries", int(out.sum()))


if __name__ == "__main__":
    main()
