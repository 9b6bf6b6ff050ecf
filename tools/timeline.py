"""Concurrency timeline of a rocprofv3 --kernel-trace csv (the bench's pipelined iterations).

    python tools/timeline.py kernel_trace.csv [--last-ms 30]

Over the window (the last --last-ms of the trace, i.e. the timed steps): the average number of
k_trace launches in flight (and the CU-equivalents they hold: workgroups x 1 CU each), shading
launches in flight, the share of time with nothing running, and per-kernel busy time."""
import argparse
import csv
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-ms", type=float, default=30.0)
    ap.add_argument("--shares", type=int, default=4, help="k_trace launches that fill the chip (1 / grid share)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        wg = int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 0)) or 1)
        ev.append((s, e, short(r["Kernel_Name"]), grid // max(1, wg)))
    t_end = max(e for _, e, _, _ in ev)
    t0 = t_end - int(a.last_ms * 1e6)
    pts = []
    for s, e, n, nwg in ev:
        s, e = max(s, t0), min(e, t_end)
        if e <= s:
            continue
        pts.append((s, 1, n, nwg))
        pts.append((e, -1, n, nwg))
    pts.sort()
    cur = defaultdict(int)
    cur_wg = defaultdict(int)
    acc = defaultdict(float)
    acc_wg = defaultdict(float)
    idle = 0.0
    starved = 0.0   # fewer k_trace launches in flight than fill the chip, while shading runs
    exposed = 0.0   # no k_trace at all in flight, while shading runs
    hist = defaultdict(float)
    last = t0
    for t, d, n, nwg in pts:
        dt = t - last
        if dt > 0:
            tot = sum(cur.values())
            if tot == 0:
                idle += dt
            for k, v in cur.items():
                acc[k] += v * dt
            for k, v in cur_wg.items():
                acc_wg[k] += v * dt
            hist[cur.get("k_trace", 0)] += dt
            shading = cur.get("k_shade_fused_b", 0) + cur.get("k_shade_fused", 0) + cur.get("k_shade", 0)
            if shading > 0 and cur.get("k_trace", 0) < a.shares:
                starved += dt
            if shading > 0 and cur.get("k_trace", 0) == 0:
                exposed += dt
            last = t
        cur[n] += d
        cur_wg[n] += d * nwg
    span = float(t_end - t0)
    print(f"window {span / 1e6:.2f} ms, idle {idle / span:.3f}")
    for k in sorted(acc, key=lambda k: -acc[k]):
        print(f"{k:24s} avg in flight {acc[k] / span:6.2f}   avg workgroups {acc_wg[k] / span:9.1f}")
    print("k_trace launches in flight: " + ", ".join(f"{k}: {v / span:.3f}" for k, v in sorted(hist.items())))
    # shading on the critical path: time in which a batch's shading runs while k_trace does not fill the chip
    # (fewer than --shares launches in flight), and while no k_trace runs at all
    print(f"shading with k_trace under {a.shares} launches: {starved / span:.4f}; with no k_trace: {exposed / span:.4f}")


if __name__ == "__main__":
    main()
