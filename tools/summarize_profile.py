"""Summarise a tools/profile.sh run: per-kernel stats and the intersect kernel's HBM traffic.

    python3 tools/summarize_profile.py gpurun_out/prof_r01 profiles/r01 cornell dragon_5 800x800

Writes <dst>_kernel_stats.csv (rocprofv3 --stats, copied), <dst>_summary.json, and
profiles/traffic_<scene>_<mesh>_<res>.json (bytes per k_trace launch from FETCH_SIZE x 2 --
the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md -- plus WRITE_SIZE, both in KB).
"""
import csv
import json
import os
import shutil
import sys


def per_dispatch(path, counter, match):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and match in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    src, dst, scene, mesh, res = sys.argv[1:6]
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, dst + "_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    out = {"kernels": {}}
    for r in rows:
        out["kernels"][r["Name"][:90]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                          "pct": float(r["Percentage"])}
    fpath = os.path.join(src, "pmc_fetch", "run_counter_collection.csv")
    wpath = os.path.join(src, "pmc_write", "run_counter_collection.csv")
    fetch, write = per_dispatch(fpath, "FETCH_SIZE", "k_trace"), per_dispatch(wpath, "WRITE_SIZE", "k_trace")
    if fetch and write:
        f = 2.0 * 1024 * sum(fetch) / len(fetch)  # KB -> B, x2 gfx950 FETCH_SIZE correction
        w = 1024 * sum(write) / len(write)
        out["k_trace_hbm_bytes_per_launch"] = {"fetch": f, "write": w, "total": f + w, "launches": len(fetch)}
        tfile = os.path.join(os.path.dirname(dst), f"traffic_{scene}_{mesh}_{res}.json")
        json.dump({"kernel": "k_trace", "hbm_bytes_per_launch": round(f + w),
                   "fetch_bytes": round(f), "write_bytes": round(w), "launches": len(fetch),
                   "source": os.path.basename(dst) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"},
                  open(tfile, "w"), indent=1)
    json.dump(out, open(dst + "_summary.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
