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


def main():
    tag, wl = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{wl}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "t_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))
    md = [f"# {tag} {wl}: rocprofv3 summaries of `python3 bench.py --workload {wl} --steps 20 --warmup 5 "
          f"--no-cpu-baseline`\n",
          "Produced by `tools/profile_round.sh` on one MI355X; each section is a separate rocprofv3 run "
          "(kernel trace; then one PMC pass per counter group).\n"]
    pmc_means = {}
    crc_kernel = None
    for part in ("trace", "fetch", "write", "clk", "sq"):
        d = os.path.join(src, part)
        db = [f for f in os.listdir(d) if f.endswith(".db")][0]
        out = subprocess.run([sys.executable, os.path.join(ROOT, "litenetlibpp_amd", "tools", "prof_summary.py"),
                              os.path.join(d, db)], capture_output=True, text=True, check=True).stdout
        md.append(f"## {part}\n\n" + out.split("\n", 2)[2])
        _, _, pmc = from_db(os.path.join(d, db))
        for name, cs in pmc.items():
            if "crc32c" in name:
                crc_kernel = short(name)
                for cn, vals in cs.items():
                    pmc_means[cn] = sum(vals) / len(vals)
    with open(os.path.join(dst, f"{tag}_{wl}_summary.md"), "w") as f:
        f.write("\n".join(md))
    fetch = pmc_means["FETCH_SIZE"] * 1024 * 2
    write = pmc_means["WRITE_SIZE"] * 1024
    tr = {"kernel": crc_kernel, "workload": wl, "hbm_bytes_per_launch": round(fetch + write),
          "fetch_bytes": round(fetch), "write_bytes": round(write),
          "how": "rocprofv3 PMC passes (tools/profile_round.sh): FETCH_SIZE (KiB) x 1024 x 2 "
                 "(gfx950 counts half of wide streaming reads) + WRITE_SIZE (KiB) x 1024, mean per dispatch",
          "source": f"profiles/{tag}_{wl}_summary.md"}
    with open(os.path.join(dst, f"traffic_{wl}.json"), "w") as f:
        json.dump(tr, f, indent=1)
    print(json.dumps(tr))


if __name__ == "__main__":
    main()
