#!/usr/bin/env python3
"""Development tool: repeat the golden fixed-stride case N times per variant
in one process and report mismatching launches (GPU box)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
VDIR = os.path.join(ROOT, "litenetlibpp_amd", "build", "variants")

data = np.fromfile(os.path.join(ROOT, "tests", "golden", "fixed_bytes.bin"), dtype=np.uint8)
exp = np.fromfile(os.path.join(ROOT, "tests", "golden", "fixed_crc.u32"), dtype=np.uint32)
for name in sys.argv[1].split(","):
    L = ctypes.CDLL(os.path.join(VDIR, name + ".so"))
    L.lnl_crc32c_batch_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    fails = []
    for it in range(int(sys.argv[2])):
        d = torch.from_numpy(data.copy()).cuda()
        out = torch.empty(64, dtype=torch.int32, device="cuda")
        L.lnl_crc32c_batch_fixed_dev(d.data_ptr(), 1400, 1400, 64, out.data_ptr(), None)
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != exp)[0]
        if bad.size:
            fails.append((it, bad.size, bad[:8].tolist(), hex(d.data_ptr() & 0xFFF)))
    print(name, "iterations", sys.argv[2], "failing", len(fails), fails[:6], flush=True)
