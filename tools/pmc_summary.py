#!/usr/bin/env python3
"""Mean PMC counter value per dispatch for every kernel of a tools/pmc_csr.sh
run (CSV output of rocprofv3 --pmc): python3 tools/pmc_summary.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                cn = row.get("Counter_Name") or row.get("Counter-Name")
                v = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id") or ""
                vals[name][cn].append(v)
    for name in sorted(vals):
        if not any(k in name for k in ("crc32c", "span", "bucket", "dispatch", "xor")):
            continue
        short = name.replace("lnl::(anonymous namespace)::", "").split("(")[0][:48]
        for cn in sorted(vals[name]):
            v = vals[name][cn]
            print(f"{short:50s} {cn:24s} {sum(v) / len(v):16.1f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
