"""The reference's own benchmark table on MI355X: per-iteration intersect-kernel time for the four
intersect kernels (presentation/benchmarks.py:482 columns) on the meshes of presentation/resultformat*.py
that exist in the reference tree.

  bruteforce  = pathTraceOneBounce, usebbox off        (enable_kd 0, use_bbox 0)
  bbox        = pathTraceOneBounce, usebbox on         (enable_kd 0, use_bbox 1)
  kd          = pathTraceOneBounceKDbare + traverseKDbare          (short_stack 0)
  short-stack = pathTraceOneBounceKDbare + traverseKDbareShortHybrid (short_stack 1)

Measured like the reference's TESTINGMODE (src/pathtrace.cu:2478-2481,2565-2574,2612-2616): one
iteration at a time, HIP events around each bounce's intersect launch(es), summed over the bounces of the
iteration, mean over --iters iterations.  Scene cornell.txt, 800x800, depth 8 (the
reference's setting is unrecorded; this is the likely one).  The GTX 980M numbers are BASELINE.md's.

  python tools/reference_columns.py [--meshes dragon_1 ...] [--iters 10] [--out profiles/x.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# BASELINE.md section 1 (GTX 980M): brute, bbox, kd, short-stack ms per iteration
GTX980M = {
    "dragon_1": (53.5, 49.3, 51.7, 40.8), "dragon_2": (79.0, 72.9, 56.6, 44.0),
    "dragon_3": (156.0, 143.9, 69.1, 49.7), "dragon_4": (315.4, 294.5, 94.2, 59.0),
    "dragon_5": (642.2, 593.0, 136.4, 79.4), "sphere_low_1": (5.1, 5.2, 25.0, 25.4),
    "sphere_low_2": (7.3, 7.1, 26.9, 27.1), "sphere_low_3": (13.1, 13.1, 27.9, 28.3),
    "sphere_low_4": (19.1, 19.0, 28.7, 28.9), "sphere_low_5": (26.8, 26.6, 30.1, 29.7),
    "sphere_low_6": (37.7, 36.8, 30.9, 30.4), "sphere_low_7": (49.8, 48.2, 31.6, 30.8),
    "sphere_low_8": (62.0, 60.3, 32.4, 31.3),
}
# presentation/resultformat_low.py:10-376 test1..test8 = sphere_low_1..8 (means of its 10 runs per column)
MODES = {"bruteforce": dict(enable_kd=0, use_bbox=0), "bbox": dict(enable_kd=0, use_bbox=1),
         "kd": dict(enable_kd=1, short_stack=0), "short-stack": dict(enable_kd=1, short_stack=1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--meshes", nargs="+", default=list(GTX980M))
    ap.add_argument("--modes", nargs="+", default=list(MODES))
    ap.add_argument("--res", type=int, nargs=2, default=(800, 800))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime in the process, shared with libkdpt)
    from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene

    rows = []
    for mesh in args.meshes:
        sd = SceneData.from_description(load_fixture_scene("cornell", mesh, res=tuple(args.res), depth=8))
        row = {"mesh": mesh, "tris": int(sd.view.polyidxcount // 3), "kd_nodes": int(sd.view.num_nodes)}
        for mode in args.modes:
            with PathTracer(sd, default_options(testing_mode=1, **MODES[mode])) as pt:
                pt.trace_iteration(1)  # warm-up (module load, first-touch)
                ms, seg = 0.0, 0
                for it in range(3, 3 + args.iters):
                    pt.trace_iteration(it)
                    st = pt.stats()
                    ms += st.ms_intersect
                    seg += st.segments
            k = list(MODES).index(mode)
            ref = GTX980M.get(mesh, (None,) * 4)[k]
            row[mode] = {"intersect_ms_per_iter": round(ms / args.iters, 4),
                         "Msegments_per_s": round(seg / (ms * 1e-3) / 1e6, 2),
                         "segments_per_iter": seg // args.iters,
                         "gtx980m_ms": ref, "speedup_vs_980m": round(ref / (ms / args.iters), 1) if ref else None}
            print(json.dumps({"mesh": mesh, "mode": mode, **row[mode]}), flush=True)
        rows.append(row)
    out = {"what": "per-iteration intersect-kernel ms (sum over bounces, HIP events), cornell.txt "
                   f"{args.res[0]}x{args.res[1]} depth 8, mean of {args.iters} iterations (3..{2 + args.iters}), "
                   "1x MI355X; gtx980m_ms from BASELINE.md 1", "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    hdr = f"{'mesh':<14}" + "".join(f"{m:>26}" for m in args.modes)
    print(hdr)
    for r in rows:
        cells = "".join(f"{r[m]['intersect_ms_per_iter']:>12.3f} ms ({r[m]['gtx980m_ms'] or '-':>6})  " for m in args.modes)
        print(f"{r['mesh']:<14}{cells}")


if __name__ == "__main__":
    main()
