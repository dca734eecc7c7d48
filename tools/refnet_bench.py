#!/usr/bin/env python3
"""Config 1 timing: 1000 x 256 B loopback echoes through the
REFERENCE's net_manager, UNRELIABLE and RELIABLE_ORDERED, with the CRC-32C
layer on (variant crc) and off (plain), from oracle/refnet (build it first:
python3 oracle/refnet/build.py).  Build container only (needs the reference's
objects).  Writes profiles/<tag>_config1_echo.json.

usage: python3 tools/refnet_bench.py [tag]   (default tag r02)"""
import json
import os
import platform
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NET = os.path.join(ROOT, "oracle", "_ref", "net")


def run(variant):
    r = subprocess.run([os.path.join(NET, variant, "refnet_driver"), "bench"], capture_output=True, text=True,
                       timeout=300)
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    res = {"what": "1000 x 256 B echoes over loopback through the reference net_manager "
                   "(oracle/refnet: reference sources compiled in place, layer spliced at sendto/recvfrom); "
                   "time from the first send to the 1000th echo; median and min of 5 bursts per run, 3 runs "
                   "per variant interleaved",
           "host": {"cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count()},
           "runs": {"plain": [], "crc": []}}
    for _ in range(3):
        for v in ("plain", "crc"):
            res["runs"][v].append(run(v))
    for v in ("plain", "crc"):
        for k in ("unreliable", "reliable_ordered"):
            med = sorted(r[f"{k}_s_median"] for r in res["runs"][v])[1]
            res[f"{v}_{k}_s"] = med
    out = os.path.join(ROOT, "profiles", f"{tag}_config1_echo.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k.endswith("_s")}))


if __name__ == "__main__":
    main()
