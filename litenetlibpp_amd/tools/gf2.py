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


# ---- transpose-free stream basis ------------------------------------------
# Stream j of a 128-byte row = bit j of each of its 32 little-endian words.
# Its 32 bits sit 32 message bits apart, so its contribution to the CRC
# register is L_j(W) = step^(31-j) L(W) with L(e_k) = step^(992-32k)(POLY)
# (the register after a single 1 bit at row position 32k+31 and the rest of
# the row).  L is invertible because x^32 generates GF(2^32).  In the basis
# V = L^-1(.) the per-row Horner step is V <- A V ^ W with A = L^-1 step^1024 L
# and the fold over streams uses B^d = L^-1 step^d L.

def step_signed(c: int, nbits: int) -> int:
    return step_bits(c, nbits) if nbits >= 0 else step_bits_inverse(c, -nbits)


def cols_inverse(cols: list[int]) -> list[int]:
    """Inverse of the 32x32 GF(2) matrix given by its columns."""
    rows = []
    for i in range(32):
        r = 0
        for k in range(32):
            if (cols[k] >> i) & 1:
                r |= 1 << k
        rows.append([r, 1 << i])
    for c in range(32):
        piv = next(i for i in range(c, 32) if (rows[i][0] >> c) & 1)
        rows[c], rows[piv] = rows[piv], rows[c]
        for i in range(32):
            if i != c and (rows[i][0] >> c) & 1:
                rows[i][0] ^= rows[c][0]
                rows[i][1] ^= rows[c][1]
    inv_rows = [rows[i][1] for i in range(32)]
    return [sum(((inv_rows[i] >> k) & 1) << i for i in range(32)) for k in range(32)]


def L_cols() -> list[int]:
    return [step_signed(POLY, 992 - 32 * k) for k in range(32)]


def stream_basis_matrix(nbits: int) -> list[int]:
    """Columns of L^-1 step^nbits L."""
    Lc = L_cols()
    Li = cols_inverse(Lc)
    return [apply(Li, step_signed(apply(Lc, 1 << k), nbits)) for k in range(32)]
