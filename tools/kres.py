#!/usr/bin/env python3
"""Kernel resources of a built library (development tool): VGPRs, spills and
scratch per kernel from the gfx950 code object's notes, for the product .so or
an experiment variant (tools/kvariants.py).

    python tools/kres.py [path/to/lib.so] [name-substring]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def notes(lib):
    out = {}
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, os.path.join(d, "lib.so"))
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", "lib.so"], cwd=d, check=True,
                       capture_output=True)
        for f in sorted(os.listdir(d)):
            if not f.endswith("gfx950"):
                continue
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(d, f)], check=True,
                                 capture_output=True, text=True).stdout
            name = None
            for line in txt.splitlines():
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m:
                    name = m.group(1)
                    out.setdefault(name, {})
                    continue
                m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|vgpr_count|sgpr_spill_count|"
                             r"agpr_count):\s+(\d+)", line)
                if m and name:
                    out[name][m.group(1)] = int(m.group(2))
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "litenetlibpp_amd", "liblnl_crc32c.so")
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, v in sorted(notes(lib).items()):
        if sub in k:
            print(f"{k[:90]:90s} vgpr {v.get('vgpr_count')} agpr {v.get('agpr_count')} "
                  f"spill {v.get('vgpr_spill_count')} scratch {v.get('private_segment_fixed_size')}")
