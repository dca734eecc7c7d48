#!/usr/bin/env python3
"""Parity of an experiments-build variant (build/variants/<name>.so) on the
config-2 and config-3 shapes against the oracle -- kvariants times variants but
does not check them.  GPU box only.  usage: variant_parity.py name[,name...]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402

oracle.load()
dev = torch.device("cuda", 0)
for name in sys.argv[1].split(","):
    L = ctypes.CDLL(os.path.join(ROOT, "litenetlibpp_amd", "build", "variants", name + ".so"))
    L.lnl_crc32c_batch_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_void_p, ctypes.c_void_p]
    L.lnl_crc32c_batch_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p]
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    n = 1 << 20
    d = torch.randint(0, 256, (n * 1400,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    rc = L.lnl_crc32c_batch_fixed_dev(d.data_ptr(), 1400, 1400, n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    exp = oracle.batch_fixed(d.cpu().numpy(), 1400, 1400, n)
    bad = int((got != exp).sum())
    lens = torch.randint(64, 1401, (n,), device=dev, generator=g, dtype=torch.int64)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(lens, 0)
    dc = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device=dev, generator=g)
    rc2 = L.lnl_crc32c_batch_csr_dev(dc.data_ptr(), off.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got2 = out.cpu().numpy().view(np.uint32)
    exp2 = oracle.batch_csr(dc.cpu().numpy(), off.cpu().numpy().astype(np.uint64))
    bad2 = int((got2 != exp2).sum())
    print(f"{name}: fixed rc={rc} mismatches={bad}; csr rc={rc2} mismatches={bad2}", flush=True)
