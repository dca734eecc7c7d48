"""GF(2) linear algebra for the reflected CRC-32C register.

Register convention (reflected, LSB-first, the same as the SSE4.2 ``crc32``
instruction and every table-driven CRC-32C): processing one input bit is
``c = (c >> 1) ^ (POLY & -(c & 1))`` with POLY = 0x82F63B78.  ``advance(c, n)``
is the register after n zero BYTES; it is linear in c, so it has a 32x32
matrix over GF(2) whose column k is ``advance(1 << k, n)``.

Used at build time only (code generation for the HIP kernels); no runtime
code imports this module.
"""
from __future__ import annotations

POLY = 0x82F63B78
MASK32 = 0xFFFFFFFF


def step_bits(c: int, nbits: int) -> int:
    for _ in range(nbits):
        c = (c >> 1) ^ (POLY if (c & 1) else 0)
    return c & MASK32


def advance(c: int, nbytes: int) -> int:
    """Register after ``nbytes`` zero bytes (the operator M_n)."""
    return step_bits(c, 8 * nbytes)


def matrix(nbytes: int) -> list[int]:
    """Columns: col[k] = M_n(1 << k).  Output bit i of M_n(v) is parity of
    (row_i & v) where row_i bit k = col[k] bit i."""
    return [advance(1 << k, nbytes) for k in range(32)]


def rows_of(cols: list[int]) -> list[int]:
    return [sum(((cols[k] >> i) & 1) << k for k in range(32)) for i in range(32)]


def apply(cols: list[int], v: int) -> int:
    out = 0
    for k in range(32):
        if (v >> k) & 1:
            out ^= cols[k]
    return out


def step_bits_inverse(c: int, nbits: int) -> int:
    """Inverse of step_bits: POLY has bit 31 set, so the top bit of the
    stepped register says whether POLY was xored in."""
    for _ in range(nbits):
        top = (c >> 31) & 1
        if top:
            c ^= POLY
        c = ((c << 1) | top) & MASK32
    return c
