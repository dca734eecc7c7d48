"""The kernel's algebra, checked on the CPU (no GPU needed).

* The generated XOR networks equal their GF(2) matrices (re-derived here).
* The committed crc32c_networks.inc is what the generator produces.
* tests/emu: the exact per-lane code of the kernel (crc32c_bitslice.h compiled
  with g++) reproduces the oracle for every length 0..1500 at several buffer
  positions, including windows that start before the buffer.
"""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "litenetlibpp_amd", "tools")
sys.path.insert(0, TOOLS)

import oracle  # noqa: E402
from gf2 import advance, apply, matrix, step_bits, step_bits_inverse  # noqa: E402


def test_advance_matches_crc_definition():
    # raw CRC of "123456789" via the register model == standard check value
    c = 0xFFFFFFFF
    for b in b"123456789":
        c = step_bits(c ^ b, 8)
    assert c ^ 0xFFFFFFFF == 0xE3069283


def test_operators_compose():
    rng = random.Random(5)
    m4, m8, m124 = matrix(4), matrix(8), matrix(124)
    for _ in range(50):
        v = rng.getrandbits(32)
        assert apply(m4, apply(m4, v)) == apply(m8, v) == advance(v, 8)
        assert apply(m4, apply(m124, v)) == advance(v, 128)
        assert step_bits_inverse(step_bits(v, 37), 37) == v


def test_networks_file_is_current():
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "gen_networks.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_kernel_lane_emulation(tmp_path):
    oracle.load()
    exe = tmp_path / "emu_lane"
    src = os.path.join(ROOT, "tests", "emu", "emu_lane.cpp")
    so_dir = os.path.dirname(oracle.ORACLE_SO)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src, f"-L{so_dir}",
                    "-lcrc32c_oracle", f"-Wl,-rpath,{so_dir}"], check=True)
    r = subprocess.run([str(exe), "1500"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout


def test_span_fold_tables(tmp_path):
    """tests/emu/emu_span_fold.cpp: the span kernel's table-Horner fold and
    register-basis final map equal the bit-sliced fold tree and the batch
    kernels' final map for random states and every e; its row powers are
    step^(1024 m); single-row datagrams match the oracle."""
    oracle.load()
    exe = tmp_path / "emu_span_fold"
    src = os.path.join(ROOT, "tests", "emu", "emu_span_fold.cpp")
    so_dir = os.path.dirname(oracle.ORACLE_SO)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src, f"-L{so_dir}",
                    "-lcrc32c_oracle", f"-Wl,-rpath,{so_dir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bad=0" in r.stdout
