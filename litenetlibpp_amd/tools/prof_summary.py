#!/usr/bin/env python3
"""Summarise a rocprofv3 run for profiles/: per-kernel dispatch statistics
(kernel-trace), and, when the run collected PMC counters, per-kernel counter
means.  Reads either the rocpd SQLite output (*.db) or the CSV output
(*_kernel_stats.csv / *_counter_collection.csv).

    python prof_summary.py gpurun_out/prof/r01_results.db > profiles/r01_kernel_stats.md
"""
from __future__ import annotations

import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    if "crc32c_run_kernel" in name:
        return "crc32c_run_kernel"
    if "crc32c_batch_kernel" in name:
        return name.replace("void ", "").replace("lnl::(anonymous namespace)::", "").split("(")[0]
    if name.startswith("stream_read"):
        return "stream_read (HBM probe)"
    return name[:60]


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count, "
                     "scratch_size from kernels").fetchall()
    stats = defaultdict(list)
    meta = {}
    for name, dur, gx, wx, lds, vgpr, sgpr, scr in rows:
        stats[name].append(dur)
        meta[name] = (gx, wx, lds, vgpr, sgpr, scr)
    pmc = defaultdict(lambda: defaultdict(list))
    try:
        for name, counter, value in c.execute(
                "select kernel_name, counter_name, value from counters_collection"):
            pmc[name][counter].append(value)
    except sqlite3.Error:
        pass
    return stats, meta, pmc


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "*.db"))
        path = dbs[0]
    stats, meta, pmc = from_db(path)
    print(f"# rocprofv3 kernel summary: {os.path.basename(path)}\n")
    print("| kernel | calls | avg us | min us | max us | total us | grid | wg | LDS B | VGPR | SGPR | scratch |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, d in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        us = [x / 1000.0 for x in d]
        gx, wx, lds, vgpr, sgpr, scr = meta[name]
        print(f"| {short(name)} | {len(us)} | {sum(us)/len(us):.2f} | {min(us):.2f} | {max(us):.2f} | "
              f"{sum(us):.1f} | {gx} | {wx} | {lds} | {vgpr} | {sgpr} | {scr} |")
    if pmc:
        print("\n## PMC counters (mean per dispatch)\n")
        print("| kernel | counter | mean | dispatches |")
        print("|---|---|---|---|")
        for name, cs in pmc.items():
            for cn, vals in sorted(cs.items()):
                print(f"| {short(name)} | {cn} | {sum(vals)/len(vals):.6g} | {len(vals)} |")


if __name__ == "__main__":
    main()
