#!/usr/bin/env python3
"""Development tool (GPU box): the wire burst of lnl_crc32c_append_csr_dev from
experiments-build variants (build/variants/<name>.so) against the product
library's, on a config-3-shaped burst.  usage: app_parity.py name[,name...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(9)
n = 1 << 20
lens = torch.randint(64, 1401, (n,), device=dev, generator=g, dtype=torch.int64)
off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
off[1:] = torch.cumsum(lens, 0)
d = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device=dev, generator=g)
size = int(off[-1]) + 4 * n


def burst(path):
    L = ctypes.CDLL(path)
    L.lnl_crc32c_append_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]
    w = torch.zeros(size, dtype=torch.uint8, device=dev)
    rc = L.lnl_crc32c_append_csr_dev(d.data_ptr(), off.data_ptr(), n, w.data_ptr(), None,
                                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return rc, w


_, ref = burst(os.path.join(ROOT, "litenetlibpp_amd", "liblnl_crc32c.so"))
for name in sys.argv[1].split(","):
    rc, w = burst(os.path.join(ROOT, "litenetlibpp_amd", "build", "variants", name + ".so"))
    bad = int((w != ref).sum())
    print(f"{name}: rc={rc} wire bytes differing from the product library's: {bad}", flush=True)
