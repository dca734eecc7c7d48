#!/usr/bin/env python3
"""Development tool (GPU box): where does a bench step's time go?

Times the config-2 launch (2^20 x 1400 B, fixed stride) and the read-only
streaming probe on the same device-resident data:
  isolated   one launch between HIP events, synchronize, repeat (median, min)
  b2b K      K back-to-back launches between one event pair (K = 3, 20, 100, 400),
             plus the host wall clock of the same K launches
  enqueue    host time to enqueue one launch (no GPU wait)
and prints one JSON object.  Not part of the product path.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import litenetlibpp_amd as P  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, L = 1 << 20, 1400
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    h = s.cuda_stream
    lib = P.lib()

    if len(sys.argv) > 1 and sys.argv[1] == "csr":  # config 3 instead: 64..1400 B, CSR
        lens = torch.randint(64, 1401, (n,), dtype=torch.int64, device=dev, generator=g)
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(lens, 0)

        def crc():
            lib.lnl_crc32c_batch_csr_dev(data.data_ptr(), off.data_ptr(), n, out.data_ptr(), h)
    else:
        def crc():
            lib.lnl_crc32c_batch_fixed_dev(data.data_ptr(), L, L, n, out.data_ptr(), h)

    pl = ctypes.CDLL(os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so"))
    pl.lnl_probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    def probe():
        pl.lnl_probe_stream_read(data.data_ptr(), n * L, sink.data_ptr(), h)

    res = {"bytes": n * L}
    for name, fn in (("crc", crc), ("probe", probe)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        iso = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            iso.append(e0.elapsed_time(e1) * 1e3)
        res[f"{name}_isolated_us_median"] = round(float(np.median(iso)), 2)
        res[f"{name}_isolated_us_min"] = round(float(np.min(iso)), 2)
        for K in (3, 20, 100, 400):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(s)
            for _ in range(K):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            res[f"{name}_b2b{K}_event_us"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
            res[f"{name}_b2b{K}_wall_us"] = round((time.perf_counter() - t0) / K * 1e6, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        res[f"{name}_enqueue_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 2)
        torch.cuda.synchronize()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
