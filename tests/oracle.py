"""ctypes loader for the CPU oracle (oracle/build/libcrc32c_oracle.so).

Test infrastructure: used only by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  Builds the oracle with make if
the shared object is missing (gcc only; no GPU needed).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libcrc32c_oracle.so")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    L = ctypes.CDLL(ORACLE_SO)
    for f in ("oracle_crc32c_bitwise", "oracle_crc32c_sliced", "oracle_crc32c_hw"):
        getattr(L, f).restype = ctypes.c_uint32
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for f in ("oracle_crc32c_bitwise_extend", "oracle_crc32c_sliced_extend", "oracle_crc32c_hw_extend"):
        getattr(L, f).restype = ctypes.c_uint32
        getattr(L, f).argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_has_sse42.restype = ctypes.c_int
    L.oracle_batch_fixed.restype = ctypes.c_int
    L.oracle_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    L.oracle_batch_csr.restype = ctypes.c_int
    L.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_int]
    L.oracle_batch_csr_bitwise.restype = None
    L.oracle_batch_csr_bitwise.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p]
    _lib = L
    return L


def mt19937_64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """SURVEY.md 8(d) synthetic input: mt19937_64(seed) outputs, little-endian."""
    words = np.empty((nbytes + 7) // 8, dtype=np.uint64)
    L = load()
    L.oracle_fill_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_fill_mt19937_64.restype = None
    L.oracle_fill_mt19937_64(seed, words.ctypes.data, words.size)
    return words.view(np.uint8)[:nbytes]


def _buf(b):
    arr = np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)
    return arr


def crc(data, kind: str = "hw") -> int:
    a = _buf(data)
    return int(getattr(load(), f"oracle_crc32c_{kind}")(a.ctypes.data, a.nbytes))


def batch_fixed(data: np.ndarray, stride: int, length: int, n: int, threads: int = 0) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint32)
    load().oracle_batch_fixed(data.ctypes.data, stride, length, n, out.ctypes.data, threads)
    return out


def batch_csr(data: np.ndarray, offsets: np.ndarray, threads: int = 0, bitwise: bool = False) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets).astype(np.uint64, copy=False)
    n = off.size - 1
    out = np.empty(n, dtype=np.uint32)
    if bitwise:
        load().oracle_batch_csr_bitwise(data.ctypes.data, off.ctypes.data, n, out.ctypes.data)
    else:
        load().oracle_batch_csr(data.ctypes.data, off.ctypes.data, n, out.ctypes.data, threads)
    return out
