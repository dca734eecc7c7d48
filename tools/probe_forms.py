#!/usr/bin/env python3
"""Development tool (GPU box): read-only streaming rates of every probe form
(litenetlibpp_amd/csrc/hbm_probe.hip) over a config-2-sized buffer, median of
10 timed batches of 10 launches after a settle period.  Forms 8-10 are the
config-2 lane-run kernel's access shape with 2 / 4 / 4 rows in flight."""
import ctypes
import json
import os
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so"))
L.lnl_probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
L.lnl_probe_stream_read.restype = ctypes.c_int
dev = torch.device("cuda", 0)
nbytes = (1 << 20) * 1400
data = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
res = {}
for form in range(11):
    nb = nbytes // 8192 * 8192
    if L.lnl_probe_stream_read(data.data_ptr(), nb, sink.data_ptr(), s.cuda_stream, form) != 0:
        continue
    t_end = time.perf_counter() + 0.1
    while time.perf_counter() < t_end:
        for _ in range(10):
            L.lnl_probe_stream_read(data.data_ptr(), nb, sink.data_ptr(), s.cuda_stream, form)
        torch.cuda.synchronize()
    times = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            L.lnl_probe_stream_read(data.data_ptr(), nb, sink.data_ptr(), s.cuda_stream, form)
        e1.record(s)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 10)
    # bytes actually read: forms 2-7 read whole 48-line segments, 8-10 whole runs
    per = {2: 48 * 128, 3: 48 * 128, 4: 48 * 128, 5: 48 * 128, 6: 48 * 128, 7: 48 * 128,
           8: 8 * 1400, 9: 8 * 1400, 10: 8 * 1400}.get(form, 1)
    eff = nb // per * per
    res[form] = round(eff / (float(np.median(times)) * 1e-3) / 1e9, 1)
    print(form, res[form], flush=True)
print(json.dumps(res))
