#!/usr/bin/env python3
"""Development tool (GPU box): where the config-5 host path loses time against
the box's pinned H2D rate.  The config-2 batch in pinned host memory through
lnl_crc32c_batch_host_ex on 2 streams, with its offsets and output arrays
pageable (as bench.py passes them) or pinned, and the H2D of the same bytes
alone in 64 MiB copies."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import litenetlibpp_amd as P  # noqa: E402

n, L = 1 << 20, 1400
dev = torch.device("cuda", 0)
data = torch.randint(0, 256, (n * L,), dtype=torch.uint8).pin_memory()
off_pg = np.arange(0, (n + 1) * L, L, dtype=np.uint64)
off_pin = torch.from_numpy(off_pg.view(np.int64)).pin_memory().numpy().view(np.uint64)
out_pg = np.empty(n, np.uint32)
out_pin = torch.empty(n, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
opts = P.HostOpts.make(streams=2)
lib = P.lib()


def call(off, out):
    rc = lib.lnl_crc32c_batch_host_ex(data.numpy().ctypes.data, off.ctypes.data, n, out.ctypes.data, 0,
                                      ctypes.pointer(opts))
    assert rc == 0, rc


def timed(fn, reps=5):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


res = {}
for name, (o, u) in {"pageable_off_out": (off_pg, out_pg), "pinned_off_out": (off_pin, out_pin),
                     "pinned_off_pageable_out": (off_pin, out_pg), "pageable_off_pinned_out": (off_pg, out_pin)}.items():
    dt = timed(lambda: call(o, u))
    res[name] = round(n * L / dt / 1e9, 2)
    print(name, res[name], flush=True)
assert np.array_equal(out_pg, out_pin)
d = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()


def h2d():
    with torch.cuda.stream(s):
        for o in range(0, n * L - (64 << 20) + 1, 64 << 20):
            d.copy_(data[o:o + (64 << 20)], non_blocking=True)
    s.synchronize()


nb = (n * L) // (64 << 20) * (64 << 20)
res["h2d_only_64MiB"] = round(nb / timed(h2d) / 1e9, 2)
print("h2d_only_64MiB", res["h2d_only_64MiB"], flush=True)
t = time.perf_counter()
for _ in range(5):
    bad = bool((off_pg[1:] < off_pg[:-1]).any())
res["numpy_monotonic_check_ms"] = round((time.perf_counter() - t) / 5 * 1e3, 3)
print(json.dumps(res))
