#!/usr/bin/env python3
"""Config 2 through the CSR span kernel (development
probe, GPU box): the 2^20 x 1400 B batch as a CSR batch (off[i] = 1400 i)
through lnl_crc32c_batch_csr_dev, timed against lnl_crc32c_batch_fixed_dev
(the lane-run kernel) on the same bytes, interleaved rounds of K back-to-back
calls between HIP events on the launch stream.  Both outputs are compared.

    python tools/fixed_as_csr.py [rounds] [calls]
"""
import sys

import torch

sys.path.insert(0, ".")
import litenetlibpp_amd as P  # noqa: E402
from litenetlibpp_amd._lib import check  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    n, S = 1 << 20, 1400
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    data = torch.randint(0, 256, (n * S,), generator=g, device="cuda", dtype=torch.uint8)
    off = torch.arange(0, (n + 1) * S, S, dtype=torch.int64, device="cuda")
    out_f = torch.empty(n, dtype=torch.int32, device="cuda")
    out_c = torch.empty(n, dtype=torch.int32, device="cuda")
    L = P.lib()
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    fixed = lambda: check(L.lnl_crc32c_batch_fixed_dev(data.data_ptr(), S, S, n, out_f.data_ptr(), s), "fixed")
    csr = lambda: check(L.lnl_crc32c_batch_csr_dev(data.data_ptr(), off.data_ptr(), n, out_c.data_ptr(), s), "csr")
    for f in (fixed, csr):
        for _ in range(20):
            f()
    torch.cuda.synchronize()
    res = {"fixed": [], "csr": []}
    for _ in range(rounds):
        for name, f in (("fixed", fixed), ("csr", csr)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(calls):
                f()
            e1.record(st)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / calls)
    for name, v in res.items():
        v = sorted(v)
        print(f"{name}: median {v[len(v) // 2]:.1f} us per call (min {v[0]:.1f}, max {v[-1]:.1f}); "
              f"frac {n * (S + 4) / (v[len(v) // 2] * 1e-6) / 8e12:.3f}", flush=True)
    print("outputs equal:", bool(torch.equal(out_f, out_c)))


if __name__ == "__main__":
    main()
