"""The oracle is pinned before anything is checked against it.

Three independent restatements (bitwise LFSR, slicing-by-8 tables, SSE4.2
crc32 instruction) must agree with the CRC-32C standard's known answers and
with each other, and the committed golden fixtures must match the bitwise one.
"""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KINDS = ["bitwise", "sliced", "hw"]


def kats():
    with open(os.path.join(GOLD, "kat.json")) as f:
        return [k for k in json.load(f) if "hex" in k]


def recipe_pins():
    with open(os.path.join(GOLD, "kat.json")) as f:
        return {k["recipe"]: k for k in json.load(f) if "recipe" in k}


@pytest.mark.parametrize("kind", KINDS)
def test_known_answers(kind):
    for k in kats():
        assert oracle.crc(bytes.fromhex(k["hex"]), kind) == k["crc"], k["what"]


def test_three_restatements_agree_on_random_lengths():
    rng = np.random.default_rng(1)
    for L in list(range(0, 300)) + [1399, 1400, 1401, 4096, 65507]:
        d = rng.integers(0, 256, L, dtype=np.uint8)
        vals = {oracle.crc(d, k) for k in KINDS}
        assert len(vals) == 1, L


def test_pure_python_reference_agrees():
    # a fourth, dependency-free restatement straight from the definition
    def crc_py(b):
        c = 0xFFFFFFFF
        for x in b:
            c ^= x
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        return c ^ 0xFFFFFFFF
    rng = np.random.default_rng(2)
    for L in (0, 1, 3, 4, 5, 31, 128, 129, 1400):
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert crc_py(d) == oracle.crc(d, "bitwise")


def test_extend_is_concatenation():
    L = oracle.load()
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, 777, dtype=np.uint8)
    b = rng.integers(0, 256, 1234, dtype=np.uint8)
    full = oracle.crc(np.concatenate([a, b]))
    for f in ("oracle_crc32c_bitwise_extend", "oracle_crc32c_sliced_extend", "oracle_crc32c_hw_extend"):
        ca = getattr(L, f)(0, a.ctypes.data, a.nbytes)
        assert getattr(L, f)(ca, b.ctypes.data, b.nbytes) == full


def test_golden_csr_matches_bitwise_and_batch():
    data = np.fromfile(os.path.join(GOLD, "csr_bytes.bin"), dtype=np.uint8)
    off = np.fromfile(os.path.join(GOLD, "csr_offsets.u64"), dtype=np.uint64)
    exp = np.fromfile(os.path.join(GOLD, "csr_crc.u32"), dtype=np.uint32)
    assert off.size == exp.size + 1 and off[-1] == data.size
    assert np.array_equal(oracle.batch_csr(data, off, bitwise=True), exp)
    assert np.array_equal(oracle.batch_csr(data, off, threads=4), exp)
    # the fixture covers every start alignment mod 16 and the edge lengths
    assert set((off[:-1] % 16).tolist()) == set(range(16))
    lens = np.diff(off.astype(np.int64))
    for L in (0, 1, 3, 4, 5, 127, 128, 129, 1400, 1432, 65507):
        assert L in lens


def test_golden_fixed():
    data = np.fromfile(os.path.join(GOLD, "fixed_bytes.bin"), dtype=np.uint8)
    exp = np.fromfile(os.path.join(GOLD, "fixed_crc.u32"), dtype=np.uint32)
    assert np.array_equal(oracle.batch_fixed(data, 1400, 1400, 64), exp)


def test_survey_config2_pin():
    """config 2's synthetic bytes are mt19937_64(42) outputs
    stored little-endian, and the first 1400-byte datagram's CRC-32C is
    0xD26C5CFE (computed there with an independent C++ implementation)."""
    b = oracle.mt19937_64_bytes(42, 3 * 1400)
    assert oracle.crc(b[:1400]) == 0xD26C5CFE
    assert oracle.crc(b[:1400], "bitwise") == 0xD26C5CFE
    assert oracle.crc(b[:1400], "sliced") == 0xD26C5CFE



def test_survey_config3_recipe_pin():
    """L_0 = 64 + (mt19937_64(43)[0] mod 1337) and the
    first datagram is the first L_0 bytes of mt19937_64(44); its CRC is the
    pin tests/golden/make_recipe_pins.py recorded (full batch: -m gpu)."""
    import ctypes
    pin = recipe_pins()["config3"]
    L = oracle.load()
    L.oracle_fill_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    u = np.empty(1, np.uint64)
    L.oracle_fill_mt19937_64(43, u.ctypes.data, 1)
    l0 = 64 + int(u[0]) % 1337
    b = oracle.mt19937_64_bytes(44, l0)
    for kind in KINDS:
        assert oracle.crc(b, kind) == pin["out0"]
    assert recipe_pins()["config2"]["out0"] == 0xD26C5CFE


def test_crc32c_residue():
    """CRC-32C over m || LE32(CRC-32C(m)) is the residue 0x48674BC7 for every
    m (the span kernel's verify test, crc32c_span.h kCrc32cResidue), and any
    other trailing value misses it."""
    import struct
    rng = np.random.default_rng(31)
    for n in list(range(0, 40)) + [127, 128, 129, 1400, 1432]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        c = oracle.crc(m)
        assert oracle.crc(m + struct.pack("<I", c)) == 0x48674BC7
        assert oracle.crc(m + struct.pack("<I", c ^ (1 << int(rng.integers(0, 32))))) != 0x48674BC7
