"""The product kernels are free of scratch (CPU test, reads the built library).

The CRC kernels wait for their own row loads with counted `s_waitcnt vmcnt(N)`
(DESIGN 4.4): the compiler does not see those inline-asm loads, so a register
spill would put scratch loads and stores -- and the compiler's own vmcnt waits
for them -- into the middle of that accounting.  Every kernel in
liblnl_crc32c.so must therefore have no private segment and no VGPR spills
(SGPR spills go to VGPR lanes and touch no memory).  Read from the gfx950 code
objects' metadata notes, extracted from a copy of the library with
llvm-objdump --offloading.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "litenetlibpp_amd", "liblnl_crc32c.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def kernel_notes(tmp_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf) and os.path.exists(LIB)):
        pytest.skip("ROCm llvm tools or the built library not present")
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([objdump, "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    kernels = {}
    for f in sorted(os.listdir(tmp_path)):
        if not f.endswith("gfx950"):
            continue
        notes = subprocess.run([readelf, "--notes", str(tmp_path / f)], check=True, capture_output=True,
                               text=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
                kernels.setdefault(name, {})
                continue
            m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|vgpr_count):\s+(\d+)", line)
            if m and name:
                kernels[name][m.group(1)] = int(m.group(2))
    return kernels


def test_product_kernels_have_no_scratch(tmp_path):
    kernels = kernel_notes(tmp_path)
    ours = {k: v for k, v in kernels.items() if "lnl" in k and "private_segment_fixed_size" in v}
    assert any("crc32c_span_kernel" in k for k in ours), sorted(kernels)[:10]
    assert any("crc32c_run_kernel" in k for k in ours)
    bad = {k: v for k, v in ours.items() if v["private_segment_fixed_size"] or v.get("vgpr_spill_count", 0)}
    assert not bad, bad
