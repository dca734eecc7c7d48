#!/usr/bin/env python3
"""Pins of SURVEY.md 8(d)'s synthetic-input recipes, appended to kat.json.

  config 2: 2^20 x 1400 B at stride 1400, bytes = mt19937_64(42) outputs
            stored little-endian
  config 3: 2^20 datagrams, L_i = 64 + (u_i mod 1337), u = mt19937_64(43);
            bytes = mt19937_64(44) outputs, packed CSR with u64 offsets

For each: out[0] by the oracle's BITWISE restatement, and the XOR of all
2^20 CRCs (a size-independent checksum of checksums) by the SSE4.2 and
slicing-by-8 restatements, which must agree.  The reference has no CRC
(README.MD:35), so these pin the recipe, not the reference.
Run: python tests/golden/make_recipe_pins.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402

N = 1 << 20


def config3_recipe():
    u = np.empty(N, np.uint64)
    L = oracle.load()
    L.oracle_fill_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_fill_mt19937_64.restype = None
    L.oracle_fill_mt19937_64(43, u.ctypes.data, N)
    lens = (np.uint64(64) + u % np.uint64(1337)).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return oracle.mt19937_64_bytes(44, int(off[-1])), off


def xor_all(crcs) -> int:
    return int(np.bitwise_xor.reduce(crcs))


def main():
    pins = []
    d2 = oracle.mt19937_64_bytes(42, N * 1400)
    off2 = np.arange(0, (N + 1) * 1400, 1400, dtype=np.uint64)
    hw = oracle.batch_fixed(d2, 1400, 1400, N)
    sl = np.array([oracle.crc(d2[i * 1400:(i + 1) * 1400], "sliced") for i in range(0, N, 997)], np.uint32)
    assert np.array_equal(sl, hw[::997])
    pins.append({"recipe": "config2", "n": N, "bytes": int(off2[-1]),
                 "out0": oracle.crc(d2[:1400], "bitwise"), "xor_all": xor_all(hw),
                 "what": "SURVEY 8(d) config 2: mt19937_64(42) bytes, 2^20 x 1400 B"})
    d3, off3 = config3_recipe()
    hw3 = oracle.batch_csr(d3, off3)
    sl3 = np.array([oracle.crc(d3[int(off3[i]):int(off3[i + 1])], "sliced") for i in range(0, N, 997)], np.uint32)
    assert np.array_equal(sl3, hw3[::997])
    pins.append({"recipe": "config3", "n": N, "bytes": int(off3[-1]),
                 "out0": oracle.crc(d3[:int(off3[1])], "bitwise"), "xor_all": xor_all(hw3),
                 "what": "SURVEY 8(d) config 3: L = 64 + (mt19937_64(43) mod 1337), mt19937_64(44) bytes"})
    path = os.path.join(HERE, "kat.json")
    with open(path) as f:
        kat = [k for k in json.load(f) if "recipe" not in k]
    with open(path, "w") as f:
        json.dump(kat + pins, f, indent=1)
    for p in pins:
        print(p["recipe"], hex(p["out0"]), hex(p["xor_all"]), p["bytes"])


if __name__ == "__main__":
    main()
