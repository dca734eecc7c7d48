#!/usr/bin/env python3
"""Development tool: run variant libraries on small fixed/CSR batches and
print where they differ from the oracle (GPU box)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402

VDIR = os.path.join(ROOT, "litenetlibpp_amd", "build", "variants")


def load(path):
    L = ctypes.CDLL(path)
    L.lnl_crc32c_batch_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    return L


def main():
    names = sys.argv[1].split(",")
    rng = np.random.default_rng(1)
    for name in names:
        L = load(os.path.join(VDIR, name + ".so") if name != "product" else
                 os.path.join(ROOT, "litenetlibpp_amd", "liblnl_crc32c.so"))
        for (n, ln, stride) in ((64, 1400, 1400), (64, 100, 128), (64, 128, 128), (64, 200, 256), (64, 1, 128)):
            data = rng.integers(0, 256, n * stride + 256, dtype=np.uint8)
            d = torch.from_numpy(data).cuda()
            out = torch.zeros(n, dtype=torch.int32, device="cuda")
            rc = L.lnl_crc32c_batch_fixed_dev(d.data_ptr(), stride, ln, n, out.data_ptr(), None)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            exp = oracle.batch_fixed(data, stride, ln, n)
            bad = np.nonzero(got != exp)[0]
            print(name, (n, ln, stride), "rc", rc, "bad", bad.size, bad[:12].tolist(), flush=True)


if __name__ == "__main__":
    main()
