#!/usr/bin/env python3
"""Development tool (GPU box): pinned-host copy rates on this box -- H2D alone,
D2H alone, and both directions at once on two streams -- the bounds of the
host paths (lnl_crc32c_batch_host: H2D; lnl_crc32c_append_host: H2D + D2H)."""
import json
import time

import torch

dev = torch.device("cuda", 0)
nb = 64 << 20
reps = 24
h_src = torch.empty(nb * reps // 4, dtype=torch.uint8).pin_memory()
h_dst = torch.empty(nb * reps // 4, dtype=torch.uint8).pin_memory()
d_a = torch.empty(nb, dtype=torch.uint8, device=dev)
d_b = torch.empty(nb, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for r in range(reps):
        o = (r % (reps // 4)) * nb
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_src[o:o + nb], non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_dst[o:o + nb].copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    return nb * reps / (time.perf_counter() - t) / 1e9


run(True, True)
res = {"h2d_gbs": round(run(True, False), 1), "d2h_gbs": round(run(False, True), 1)}
both = run(True, True)
res["both_each_direction_gbs"] = round(both, 1)
print(json.dumps(res))
