#!/usr/bin/env python3
"""Generate the committed golden fixtures for the CRC-32C path.

Why generated: the reference has no CRC code and no checksum test vectors
(/root/reference/README.MD:35), so parity is pinned by
the CRC-32C standard.  The fixtures below are computed with the oracle's
BITWISE restatement (one LFSR step per bit, oracle/crc32c_oracle.c), which the
CPU suite pins against the RFC 3720 B.4 known answers (kat.json) and
cross-checks against the slicing-by-8 and SSE4.2 restatements.

Files (all little-endian):
  kat.json          known-answer vectors (standard, not generated)
  csr_bytes.bin     concatenated datagrams
  csr_offsets.u64   n+1 offsets into csr_bytes.bin (start alignment mod 16 covers 0..15)
  csr_crc.u32       expected CRC-32C per datagram
  fixed_bytes.bin   64 x 1400-byte datagrams at stride 1400 (config 2 shape)
  fixed_crc.u32
Run from anywhere: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402

# lengths named in SURVEY.md 8(c): edge sizes around words, rows and MTUs
EDGE_LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129,
                130, 131, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 1399, 1400, 1401,
                1427, 1428, 1431, 1432]

KAT = [
    {"hex": b"123456789".hex(), "crc": 0xE3069283, "what": "CRC-32C check value"},
    {"hex": (b"\x00" * 32).hex(), "crc": 0x8A9136AA, "what": "RFC 3720 B.4: 32 bytes of zeros"},
    {"hex": (b"\xff" * 32).hex(), "crc": 0x62A8AB43, "what": "RFC 3720 B.4: 32 bytes of 0xFF"},
    {"hex": bytes(range(32)).hex(), "crc": 0x46DD794E, "what": "RFC 3720 B.4: 32 incrementing bytes"},
    {"hex": bytes(range(31, -1, -1)).hex(), "crc": 0x113FDB5C, "what": "RFC 3720 B.4: 32 decrementing bytes"},
    {"hex": "", "crc": 0x00000000, "what": "empty input"},
]


def main():
    rng = np.random.default_rng(20261015)
    path = os.path.join(HERE, "kat.json")
    keep = []
    if os.path.exists(path):  # recipe pins are written by make_recipe_pins.py
        with open(path) as f:
            keep = [k for k in json.load(f) if "recipe" in k]
    with open(path, "w") as f:
        json.dump(KAT + keep, f, indent=1)

    # CSR fixture: contiguous datagrams of the edge lengths x {zeros, 0xFF,
    # random} plus random lengths; starts therefore fall on every alignment.
    # The first datagram begins at offset 0 (the kernel's "window starts
    # before d_base" path).
    pats = []
    for L in EDGE_LENGTHS:
        pats += [np.zeros(L, np.uint8), np.full(L, 0xFF, np.uint8), rng.integers(0, 256, L, dtype=np.uint8)]
    for L in rng.integers(0, 1433, 380):
        pats.append(rng.integers(0, 256, int(L), dtype=np.uint8))
    pats.append(rng.integers(0, 256, 9000, dtype=np.uint8))
    pats.append(rng.integers(0, 256, 65507, dtype=np.uint8))
    order = rng.permutation(len(pats))
    data = np.concatenate([pats[i] for i in order])
    lens = np.array([pats[i].size for i in order], dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    crc = oracle.batch_csr(data, offs, bitwise=True)
    data.tofile(os.path.join(HERE, "csr_bytes.bin"))
    offs.tofile(os.path.join(HERE, "csr_offsets.u64"))
    crc.tofile(os.path.join(HERE, "csr_crc.u32"))

    fixed = rng.integers(0, 256, 64 * 1400, dtype=np.uint8)
    fcrc = oracle.batch_csr(fixed, np.arange(0, 64 * 1400 + 1, 1400, dtype=np.uint64), bitwise=True)
    fixed.tofile(os.path.join(HERE, "fixed_bytes.bin"))
    fcrc.tofile(os.path.join(HERE, "fixed_crc.u32"))
    print(f"csr: {len(order)} datagrams, {data.size} bytes; fixed: 64 x 1400")


if __name__ == "__main__":
    main()
