#!/usr/bin/env python3
"""Turn a tools/profile_round.sh run into the committed profiles/ files:

    python tools/write_profiles.py r01 fixed     (reads gpurun_out/prof_r01_fixed/)

writes profiles/<tag>_<wl>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<tag>_<wl>_summary.md (kernel trace + every PMC pass) and
profiles/traffic_<wl>.json (HBM bytes per launch of the CRC kernel, from the
PMC passes: FETCH_SIZE x 2 -- gfx950 reports half of wide streaming reads,
MI355X_MICROARCH.md HBM section -- plus WRITE_SIZE; both in KiB), which
bench.py reports as roofline.traffic.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "litenetlibpp_amd", "tools"))
from prof_summary import from_db, short  # noqa: E402

# kernels of liblnl_crc32c.so (rocprofv3 names contain these)
PRODUCT_KERNELS = ("crc32c_", "bucket_count", "bucket_scatter", "bucket_hist", "bucket_scan", "bucket_place",
                   "pair_count", "pair_scatter", "seg_prep", "seg_fixup", "verify_from_wire", "csr_plan",
                   "dispatch_", "xor_layer", "xor_flat", "xor_csr_flat", "xor_csr_stream", "xor_csr_grid",
                   "xor_chunk_map", "span_prep", "append_")


# FETCH_SIZE's bytes per byte read, by access shape (MI355X_MICROARCH.md HBM
# section: gfx950 counts half of a wide coalesced streaming read; the other
# shapes calibrated by tools/fetch_calibration.py on known byte counts,
# profiles/fetch_calibration.json).  Kernels not listed read in wide streams.
FETCH_SHAPE = {
    "dispatch_count_kernel": "random_dword_sector",   # the MERGED walk: dword pairs at random 64-B sectors
    "dispatch_emit_kernel": "dword_stream",           # records and counts, one dword per lane
}


def fetch_factor(kernel):
    cal = os.path.join(ROOT, "profiles", "fetch_calibration.json")
    shape = next((v for k, v in FETCH_SHAPE.items() if k in kernel), "wide_stream_16B")
    if shape == "wide_stream_16B" or not os.path.exists(cal):
        return 2.0, shape
    return float(json.load(open(cal))["bytes_per_fetch_byte"][shape]), shape


def main():
    tag, wl = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{wl}")
    dst = os.environ.get("PROFILES_DIR", os.path.join(ROOT, "profiles"))
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "t_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))
    md = [f"# {tag} {wl}: rocprofv3 summaries of `python3 bench.py --workload {wl} --steps 20 --warmup 5 "
          f"--no-cpu-baseline --no-host-path`\n",
          "Produced by `tools/profile_round.sh` on one MI355X; each section is a separate rocprofv3 run "
          "(kernel trace; then one PMC pass per counter group).\n"]
    # HBM bytes per API call: every product kernel the call launches (the CRC
    # kernel plus, for CSR, its bucket pre-pass), counter totals divided by the
    # dispatch count of the dominant product kernel (the one with the most time)
    pmc_tot = {}
    fetch_bytes = 0.0   # FETCH_SIZE x its shape's factor, per kernel
    shapes = {}
    kernels = set()
    trace_stats = None
    for part in ("trace", "fetch", "write", "clk", "sq"):
        d = os.path.join(src, part)
        db = [f for f in os.listdir(d) if f.endswith(".db")][0]
        out = subprocess.run([sys.executable, os.path.join(ROOT, "litenetlibpp_amd", "tools", "prof_summary.py"),
                              os.path.join(d, db)], capture_output=True, text=True, check=True).stdout
        md.append(f"## {part}\n\n" + out.split("\n", 2)[2])
        stats, _, pmc = from_db(os.path.join(d, db))
        if part == "trace":
            trace_stats = stats
        if part == "trace":
            crc = {n: d for n, d in trace_stats.items() if any(k in n for k in PRODUCT_KERNELS)}
            dom = max(crc, key=lambda n: sum(crc[n]))
            crc_kernel = short(dom)
            calls = len(crc[dom])
        # the bench's settle phase is time-based, so each pass has its own
        # dispatch count: per pass, the product kernels launched as often as the
        # dominant one (once per API call; setup launches building the workload
        # are not the call's), summed as means per dispatch
        pass_calls = None
        for name, cs in pmc.items():
            if short(name) == crc_kernel:
                pass_calls = max(len(v) for v in cs.values())
        for name, cs in pmc.items():
            if pass_calls and any(k in name for k in PRODUCT_KERNELS) and all(len(v) == pass_calls for v in cs.values()):
                kernels.add(short(name))
                for cn, vals in cs.items():
                    pmc_tot[cn] = pmc_tot.get(cn, 0.0) + sum(vals) / pass_calls
                    if cn == "FETCH_SIZE":
                        f, shape = fetch_factor(name)
                        shapes[short(name)] = [shape, f]
                        fetch_bytes += sum(vals) / pass_calls * 1024 * f
    pmc_means = dict(pmc_tot)
    with open(os.path.join(dst, f"{tag}_{wl}_summary.md"), "w") as f:
        f.write("\n".join(md))
    fetch = fetch_bytes
    write = pmc_means["WRITE_SIZE"] * 1024
    tr = {"kernel": crc_kernel, "kernels_per_call": sorted(kernels), "workload": wl, "hbm_bytes_per_launch": round(fetch + write),
          "fetch_bytes": round(fetch), "fetch_size_raw_bytes": round(pmc_means["FETCH_SIZE"] * 1024),
          "write_bytes": round(write), "fetch_shapes": shapes,
          "how": "rocprofv3 PMC passes (tools/profile_round.sh): per product kernel FETCH_SIZE (KiB) x 1024 x its "
                 "access shape's factor (x 2 for wide streaming reads, MI355X_MICROARCH.md; the others from "
                 "profiles/fetch_calibration.json, tools/fetch_calibration.py) + WRITE_SIZE (KiB) x 1024, summed over "
                 "the product kernels of one API call",
          "source": f"profiles/{tag}_{wl}_summary.md"}
    with open(os.path.join(dst, f"traffic_{wl}.json"), "w") as f:
        json.dump(tr, f, indent=1)
    print(json.dumps(tr))


if __name__ == "__main__":
    main()
