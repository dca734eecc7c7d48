#!/usr/bin/env python3
"""Development tool (GPU box): the box's device-to-device copy rates beside the
outbound layer's own passes, per config-3-sized burst (2^20 datagrams of
64..1400 B), median of 10 timed batches of 5 calls after a settle period.

  torch copy   dst.copy_(src) over the payload bytes (the runtime's blit)
  csr          lnl_crc32c_batch_csr_dev (the append's CRC pass)
  append       lnl_crc32c_append_csr_dev (CRC pass + copy kernel)

append - csr is the copy kernel's share; the torch copy bounds what a copy of
the same bytes costs on this box (read + write, aligned)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from litenetlibpp_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(3)
n = 1 << 20
lens = torch.randint(64, 1401, (n,), device=dev, generator=g, dtype=torch.int64)
off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
off[1:] = torch.cumsum(lens, 0)
total = int(off[-1])
src = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
dst = torch.empty(total + 4 * n, dtype=torch.uint8, device=dev)
crc = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
L = lib()


def t_copy():
    dst[:total].copy_(src)


def t_csr():
    L.lnl_crc32c_batch_csr_dev(src.data_ptr(), off.data_ptr(), n, crc.data_ptr(), s.cuda_stream)


def t_append():
    L.lnl_crc32c_append_csr_dev(src.data_ptr(), off.data_ptr(), n, dst.data_ptr(), crc.data_ptr(), s.cuda_stream)


res = {"payload_bytes": total}
for name, fn in (("torch_copy", t_copy), ("csr", t_csr), ("append", t_append)):
    t_end = time.perf_counter() + 0.15
    while time.perf_counter() < t_end:
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5 * 1e3)
    us = float(np.median(ts))
    res[name] = {"us": round(us, 2)}
    print(name, round(us, 2), "us", flush=True)
res["copy_kernel_us"] = round(res["append"]["us"] - res["csr"]["us"], 2)
res["torch_copy_rw_gbps"] = round(2 * total / (res["torch_copy"]["us"] * 1e-6) / 1e9, 1)
res["copy_kernel_rw_gbps"] = round((2 * total + 8 * n) / (res["copy_kernel_us"] * 1e-6) / 1e9, 1)
print(json.dumps(res))
