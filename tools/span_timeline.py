#!/usr/bin/env python3
"""Per-wave timeline of the CSR span kernel (variant span_timeline,
-DLNL_SPAN_DIAG=16: each wave writes 7 s_memrealtime stamps into out[8 w ..]
instead of CRCs) on the config-3 batch: kernel entry, tables in LDS, first
wave-batch set up, rows done, stash flushed, in-wave heads combined, wave done.  GPU box only."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "litenetlibpp_amd", "build", "variants",
                             (sys.argv[1] if len(sys.argv) > 1 else "span_timeline") + ".so"))
L.lnl_crc32c_batch_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_void_p]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(42)
n = 1 << 20
lens = torch.randint(64, 1401, (n,), device=dev, generator=g, dtype=torch.int64)
off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
off[1:] = torch.cumsum(lens, 0)
data = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device=dev, generator=g)
out = torch.zeros(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for _ in range(3):
    out.zero_()
    L.lnl_crc32c_batch_csr_dev(data.data_ptr(), off.data_ptr(), n, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
t = out.cpu().numpy().view(np.uint32).astype(np.int64)[: 8 * 2048].reshape(-1, 8)[:, :7]
gw = np.arange(len(t))
# (stamps are the low 32 bits: work modulo 2^32 around the median entry; the
# heads' CRC stores land in out[] too: keep the waves whose 5 stamps are
# ordered and within 10 ms of the median entry)
med = int(np.median(t[:, 0]))
t = (t - med + (1 << 31)) % (1 << 32) - (1 << 31)
ok = np.all(np.diff(t, axis=1) >= 0, axis=1) & (np.abs(t[:, 0]) < 1_000_000) & (t[:, -1] - t[:, 0] < 1_000_000)
t = t[ok]
gw = gw[ok]
t = (t - t[:, :1].min()) * 10 / 1000.0  # 100 MHz ticks -> us from the first wave's entry
names = ["entry", "tables", "setup", "rows", "flushed", "heads", "done"]
print(f"{len(t)} waves; us from the first entry")
for i, nm in enumerate(names):
    c = t[:, i]
    print(f"  {nm:7s} min {c.min():7.1f}  p10 {np.percentile(c, 10):7.1f}  med {np.median(c):7.1f}  "
          f"p90 {np.percentile(c, 90):7.1f}  max {c.max():7.1f}")
for i in range(1, len(names)):
    d = t[:, i] - t[:, i - 1]
    print(f"  {names[i - 1]}->{names[i]:7s} med {np.median(d):7.1f}  p90 {np.percentile(d, 90):7.1f}  max {d.max():7.1f}")
rows = t[:, 3] - t[:, 2]
for nm, key in (("xcd (block % 8)", (gw // 8) % 8), ("wave in block", gw % 8), ("block // 32", (gw // 8) // 32)):
    print(f"  rows phase by {nm}: " + "  ".join(f"{k}:{np.median(rows[key == k]):.0f}" for k in np.unique(key)))
order = np.argsort(t[:, -1])
print("  slowest 8 waves (gw, rows us):", [(int(gw[i]), round(float(rows[i]), 1)) for i in order[-8:]])
sys.stdout.flush()
