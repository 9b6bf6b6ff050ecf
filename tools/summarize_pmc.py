"""Summarise a tools/pmc_profile.sh run into a committed profile (profiles/) that bench.py reads.

    python3 tools/summarize_pmc.py gpurun_out/TAG profiles/TAG [--workload cornell_dragon_5_800x800]

Writes
  profiles/TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the bench command (concurrent launches)
  profiles/TAG_pmc.json           per kernel family: dispatches, summed counters of every PMC pass,
                                  exclusive durations, and the derived per-ray / per-path figures
  profiles/pmc_<workload>.json    the same, as bench.py's roofline source (with the kernel-source hash)

Counting rules (MI355X_MICROARCH.md, "HBM" and "rocprofv3 PMC slots"): FETCH_SIZE and WRITE_SIZE are in KB;
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950, so it is doubled; GRBM_GUI_ACTIVE sums
the 8 XCDs, so /8 gives the dispatch's clock cycles; SQ_INSTS_VALU counts wave64 instructions, each of which
holds a SIMD-32 for 2 clocks.  rocprofv3 serialises dispatches while counting, so every PMC-pass launch ran
alone on the GPU (on the CUs of its own grid).
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PASSES = ["pmc_sq_a", "pmc_sq_b", "pmc_fetch", "pmc_write"]


def family(name):
    if "k_trace<" in name:
        return "k_trace" if ", false," in name else "k_trace_count"
    for k in ("k_shade_fused", "k_shade<", "k_gen_geoms", "k_geoms", "k_gen_rays", "k_accumulate_batch", "k_scan",
              "k_scatter"):
        if k in name:
            return k.rstrip("<")
    return "other"


def bench_line(log):
    for line in open(log):
        if line.startswith('{"metric"'):
            return json.loads(line)
    return None


def load_pass(d):
    fam = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        f = family(r["Kernel_Name"])
        e = fam.setdefault(f, {"dispatches": set(), "counters": {}, "dur_ns": {}, "grid": {}})
        did = r["Dispatch_Id"]
        e["dispatches"].add(did)
        e["counters"][r["Counter_Name"]] = e["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["dur_ns"][did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e["grid"][did] = (int(r["Grid_Size"]), int(r["Workgroup_Size"]))
    return fam


def main():
    src, dst = sys.argv[1], sys.argv[2]
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "cornell_dragon_5_800x800"
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), dst + "_kernel_stats.csv")
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        f = family(r["Name"])
        s = stats.setdefault(f, {"calls": 0, "total_ms": 0.0})
        s["calls"] += int(r["Calls"])
        s["total_ms"] += float(r["TotalDurationNs"]) / 1e6
    trace_bench = bench_line(os.path.join(src, "trace.log"))
    out = {"source_run": os.path.basename(src), "bench_under_trace": trace_bench, "kernel_stats_concurrent": stats,
           "passes": {}, "kernels": {}}
    b = None
    for p in PASSES:
        d = os.path.join(src, p)
        if not os.path.isdir(d):
            continue
        fam = load_pass(d)
        b = bench_line(os.path.join(src, p + ".log")) or b
        out["passes"][p] = {f: {"dispatches": len(e["dispatches"]), "counters": e["counters"],
                                "exclusive_ms": sum(e["dur_ns"].values()) / 1e6,
                                "cus": sum(g // wg if wg == 1024 else g // wg for g, wg in e["grid"].values())}
                            for f, e in fam.items()}
    out["bench_under_pmc"] = b
    iters = b["config"].get("spp_per_frame", b["config"].get("spp_per_step")) * b["steps"]
    rays = b["roofline"]["rays_per_launch"] * b["roofline"]["launches"]  # k_trace rays of the timed iterations
    segs = b["segments_per_iteration"] * (iters + 1)  # shading also ran the counting iteration
    P = out["passes"]

    def c(p, f, name):
        return P.get(p, {}).get(f, {}).get("counters", {}).get(name)

    for f, units, per in (("k_trace", "ray", rays), ("k_shade_fused", "path", segs)):
        a = P.get("pmc_sq_a", {}).get(f)
        if not a:
            continue
        k = {"dispatches": a["dispatches"], "exclusive_ms_per_dispatch": a["exclusive_ms"] / a["dispatches"],
             "units": units, "units_counted": per}
        valu = c("pmc_sq_a", f, "SQ_INSTS_VALU")
        k["valu_per_" + units] = valu / per
        if f == "k_trace":
            k["valu_per_ray"] = valu / per
        grbm = c("pmc_sq_a", f, "GRBM_GUI_ACTIVE")
        if grbm:
            cycles = grbm / 8.0
            # SIMD-clocks the dispatches had: cycles x 4 SIMDs x CUs of the grid (one 1024-thread WG per CU for
            # k_trace; k_shade_fused's 256-thread WGs spread over every CU: 256 CUs)
            cus = 256 if f != "k_trace" else None
            if f == "k_trace":
                # grid WGs (one per CU) of each dispatch, averaged
                d = P["pmc_sq_a"][f]
                cus = d["cus"] / d["dispatches"]
            k["clock_ghz"] = cycles / (a["exclusive_ms"] * 1e6) * 1.0
            k["valu_busy_frac"] = valu * 2.0 / (cycles * 4 * cus)
            k["cus"] = cus
        for name in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_WAVES"):
            v = c("pmc_sq_a", f, name)
            if v is not None:
                k[name.lower().replace("sq_", "") + "_per_" + units] = v / per
        wc = c("pmc_sq_a", f, "SQ_WAVE_CYCLES")
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                         "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VMEM", "SQ_ACTIVE_INST_SCA"):
                v = c("pmc_sq_b", f, name)
                if v is not None:
                    k[name.lower() + "_share_of_wave_cycles"] = v / wc
            av = c("pmc_sq_a", f, "SQ_ACTIVE_INST_VALU")
            if av is not None:
                k["sq_active_inst_valu_share_of_wave_cycles"] = av / wc
        bc = c("pmc_sq_b", f, "SQ_LDS_BANK_CONFLICT")
        if bc is not None:
            k["lds_bank_conflict_cycles_per_" + units] = bc / per
        fetch, write = c("pmc_fetch", f, "FETCH_SIZE"), c("pmc_write", f, "WRITE_SIZE")
        if fetch is not None and write is not None:
            fb, wb = 2.0 * 1024 * fetch, 1024 * write
            k["fetch_bytes_per_" + units] = fb / per
            k["write_bytes_per_" + units] = wb / per
            k["hbm_bytes_per_" + units] = (fb + wb) / per
            if f == "k_trace":
                k["hbm_bytes_per_ray"] = (fb + wb) / per
            ms = P["pmc_fetch"][f]["exclusive_ms"]
            k["hbm_GBps_exclusive"] = (fb / 1e9) / (ms * 1e-3) + (wb / 1e9) / (P["pmc_write"][f]["exclusive_ms"] * 1e-3)
            k["hbm_frac_exclusive"] = k["hbm_GBps_exclusive"] / 8000.0
        out["kernels"][f] = k
    # every kernel family, per dispatch (each ran alone under PMC): time, VALU issue, waits, HBM bytes
    out["per_dispatch"] = {}
    for f, a in P.get("pmc_sq_a", {}).items():
        n = a["dispatches"]
        r = {"dispatches": n, "exclusive_ms": a["exclusive_ms"] / n}
        valu, wc = c("pmc_sq_a", f, "SQ_INSTS_VALU"), c("pmc_sq_a", f, "SQ_WAVE_CYCLES")
        grbm = c("pmc_sq_a", f, "GRBM_GUI_ACTIVE")
        if valu is not None:
            r["valu_wave_insts"] = valu / n
        if valu and grbm:
            cus = a["cus"] / n if f == "k_trace" else 256
            r["valu_busy_frac"] = valu * 2.0 / (grbm / 8.0 * 4 * cus)
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                v = c("pmc_sq_b", f, name)
                if v is not None:
                    r[name.lower() + "_share"] = v / wc
        fetch, write = c("pmc_fetch", f, "FETCH_SIZE"), c("pmc_write", f, "WRITE_SIZE")
        if fetch is not None and write is not None:
            fb, wb = 2.0 * 1024 * fetch / n, 1024 * write / n
            r["hbm_bytes"] = fb + wb
            fms = P["pmc_fetch"][f]["exclusive_ms"] / n
            wms = P["pmc_write"][f]["exclusive_ms"] / n
            r["hbm_GBps"] = fb / 1e9 / (fms * 1e-3) + wb / 1e9 / (wms * 1e-3)
            r["hbm_frac"] = r["hbm_GBps"] / 8000.0
        out["per_dispatch"][f] = r
    # provenance: the bench run under PMC printed the build recipe hash and the code-object hash of the
    # library it loaded, so the profile names the exact machine code it measured
    roof = (b or {}).get("roofline", {})
    out["kernel_source_sha"] = roof.get("kernel_source_sha")
    out["code_object_sha"] = roof.get("code_object_sha")
    try:
        out["git_head"] = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                         cwd=ROOT).stdout.strip()
    except OSError:
        pass
    json.dump(out, open(dst + "_pmc.json", "w"), indent=1)
    json.dump({"kernel_source_sha": out["kernel_source_sha"], "code_object_sha": out["code_object_sha"],
               "git_head": out.get("git_head"), "source": os.path.basename(dst) + "_pmc.json",
               "kernels": out["kernels"], "per_dispatch": out["per_dispatch"]}, open(os.path.join(ROOT, "profiles", f"pmc_{workload}.json"), "w"), indent=1)
    print(json.dumps({"kernels": out["kernels"], "per_dispatch": out["per_dispatch"]}, indent=1))


if __name__ == "__main__":
    main()
