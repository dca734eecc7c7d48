#!/usr/bin/env python3
"""Does the outbound copy run faster when its payload is still in the
Infinity Cache (MALL)?  (development probe; run on the GPU box under
rocprofv3 --kernel-trace --stats and read the per-kernel averages.)

A config-3-shaped burst (2^20 datagrams, lengths U[64, 1400], ~768 MB) goes
through lnl_crc32c_append_csr_dev twice: once whole (the copy kernel reads a
payload the CRC pass read ~150 us earlier, 768 MB ago: from HBM), and once in
S slices of 2^20 / S datagrams (each slice's copy reads bytes its own CRC pass
has just read: ~768/S MB ago).  The copy kernel's average duration per slice
against its whole-burst duration / S is the Infinity Cache's effect on it.

    python tools/mall_probe.py whole|sliced [slices] [rounds]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import litenetlibpp_amd as P  # noqa: E402
from litenetlibpp_amd._lib import check  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "sliced"
    slices = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n = 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(43)
    lens = torch.randint(64, 1401, (n,), generator=g, device="cuda", dtype=torch.int64)
    off = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    off[1:] = torch.cumsum(lens, 0)
    total = int(off[-1].item())
    data = torch.randint(0, 256, (total + 64,), generator=g, device="cuda", dtype=torch.uint8)
    wire = torch.empty(total + 4 * n, dtype=torch.uint8, device="cuda")
    per = n // slices
    cuts = [(k * per, (k + 1) * per if k + 1 < slices else n) for k in range(slices)]
    offs = [off[a:b + 1].contiguous() for a, b in cuts]
    L = P.lib()
    s = torch.cuda.current_stream().cuda_stream

    def whole():
        check(L.lnl_crc32c_append_csr_dev(data.data_ptr(), off.data_ptr(), n, wire.data_ptr(), None, s),
                "append")

    base = [int(off[a].item()) + 4 * a for a, _ in cuts]  # (host values, read once)

    def sliced():
        for (a, b), o, w in zip(cuts, offs, base):
            check(L.lnl_crc32c_append_csr_dev(data.data_ptr(), o.data_ptr(), b - a, wire.data_ptr() + w, None, s),
                    "append")

    for name, fn in ((mode, whole if mode == "whole" else sliced),):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(rounds):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / rounds
        print(f"{name}: {dt * 1e3:.3f} ms per burst (host clock, {slices} slices)" if name == "sliced"
              else f"{name}: {dt * 1e3:.3f} ms per burst (host clock)", flush=True)
    if mode == "whole":
        return
    # parity of the sliced wire against the whole call's
    ref = wire.clone()
    whole()
    torch.cuda.synchronize()
    w2 = wire.clone()
    wire.zero_()
    sliced()
    torch.cuda.synchronize()
    print("sliced == whole:", bool(torch.equal(wire, w2)), "and == previous:", bool(torch.equal(ref, w2)))


if __name__ == "__main__":
    main()
