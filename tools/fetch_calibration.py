#!/usr/bin/env python3
"""FETCH_SIZE calibration for the dispatch walk's access shape (VERDICT r04
item 6; GPU box, under rocprofv3 --pmc FETCH_SIZE): dword reads at random
64-byte sectors, each sector read once (litenetlibpp_amd/csrc/hbm_probe.hip
sector_read), 1 or 2 adjacent dwords per sector.  The per-dispatch
FETCH_SIZE against the known sector count gives the counter's bytes per
random sector for this shape; tools/write_profiles.py applies it to the
dispatch workload's walk kernels.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d DIR -o f -- python3 tools/fetch_calibration.py
    python3 tools/fetch_calibration.py summarize DIR/f_counter_collection.csv [out.json]
        -> profiles/fetch_calibration.json: bytes per FETCH_SIZE byte per shape
           (the first, cold, dispatch of each kind; the rest are printed)
"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so"))
L.lnl_probe_sector_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_void_p, ctypes.c_void_p]
L.lnl_probe_sector_read.restype = ctypes.c_int64
L.lnl_probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
L.lnl_probe_stream_read.restype = ctypes.c_int
L.lnl_probe_dword_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
L.lnl_probe_dword_stream.restype = ctypes.c_int


def main():
    dev = torch.device("cuda", 0)
    nbytes = 2 << 30  # 2 GiB: 2^25 sectors, far past the Infinity Cache
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    buf.random_(0, 256)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    plan = [(1 << 22, 1), (1 << 22, 2), (1 << 24, 1), (1 << 24, 2)]
    out = {"dispatches": []}
    for n, words in plan:
        for _ in range(3):  # each dispatch shows up separately in the PMC trace
            r = L.lnl_probe_sector_read(buf.data_ptr(), nbytes, n, words, sink.data_ptr(), s.cuda_stream)
            assert r > 0, r
            torch.cuda.synchronize()
        out["dispatches"].append({"sectors": n, "words": words, "repeat": 3, "bytes_sector_floor": 64 * n})
        print(json.dumps(out["dispatches"][-1]), flush=True)
    # reference: a wide streaming read of 1 GiB (form 0: dwordx4 per lane), the
    # shape the guide's x2 rule is calibrated on
    for _ in range(3):
        assert L.lnl_probe_stream_read(buf.data_ptr(), 1 << 30, sink.data_ptr(), s.cuda_stream, 0) == 0
        torch.cuda.synchronize()
    out["dispatches"].append({"stream_read_bytes": 1 << 30, "repeat": 3})
    # one dword per lane, consecutive: 1 GiB
    for _ in range(3):
        assert L.lnl_probe_dword_stream(buf.data_ptr(), 1 << 30, sink.data_ptr(), s.cuda_stream) == 0
        torch.cuda.synchronize()
    out["dispatches"].append({"dword_stream_bytes": 1 << 30, "repeat": 3})
    print(json.dumps(out))


def summarize(csv_path, out_path):
    import csv
    rows = [r for r in csv.DictReader(open(csv_path)) if r["Counter_Name"] == "FETCH_SIZE"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    kinds = []  # (shape, known bytes per dispatch) in launch order, 3 dispatches each
    for n, words in [(1 << 22, 1), (1 << 22, 2), (1 << 24, 1), (1 << 24, 2)]:
        kinds += [(f"random_dword_sector/{n}/{words}", 64 * n)] * 3
    kinds += [("wide_stream_16B", 1 << 30)] * 3 + [("dword_stream", 1 << 30)] * 3
    probe = [r for r in rows if any(k in r["Kernel_Name"] for k in ("sector_read", "stream_read", "dword_stream"))]
    assert len(probe) == len(kinds), (len(probe), len(kinds))
    per = {}
    for (shape, known), r in zip(kinds, probe):
        fetched = float(r["Counter_Value"]) * 1024
        per.setdefault(shape, []).append(round(known / fetched, 4))
    shapes = {}
    for shape, vals in per.items():
        base = shape.split("/")[0]
        shapes.setdefault(base, []).extend(vals)
    res = {"bytes_per_fetch_byte": {k: round(sum(v) / len(v), 3) for k, v in shapes.items()},
           "per_dispatch": per,
           "what": "known bytes / (FETCH_SIZE KiB x 1024) per probe dispatch (litenetlibpp_amd/csrc/hbm_probe.hip: "
                   "sector_read = one or two dwords at each of n distinct random 64-B sectors, known bytes 64 n; "
                   "stream_read = 16 B per lane over 1 GiB; dword_stream = 4 B per lane over 1 GiB)",
           "source": "tools/fetch_calibration.py under rocprofv3 --pmc FETCH_SIZE"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["bytes_per_fetch_byte"]))


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 2 and sys.argv[1] == "summarize":
        summarize(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles",
                                                                                   "fetch_calibration.json"))
    else:
        main()
