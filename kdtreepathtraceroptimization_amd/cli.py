"""Headless command line of the path tracer: the reference's `main(argc, argv)` (src/main.cpp:1013-1038)
without the GLFW window.

    python -m kdtreepathtraceroptimization_amd SCENE.txt [MESH.obj] [options]

The reference loads the scene (and the OBJ with its KD tree), renders ITERATIONS samples per pixel with
the flag state of src/main.cpp:35-60 (changed interactively by the keys of src/main.cpp:1187-1306), then
saveImage()s a PNG (src/main.cpp:1087-1108) and exits (runCuda, src/main.cpp:1110-1185).  Here the flags
are options, the iterations run on the GPU through the C-ABI (kdpt_trace_iterations keeps several in
flight; bit-identical to one pathtrace() call per iteration), and the output is the same PNG (and
optionally the Radiance HDR image::saveHDR writes).  Flag -> reference variable:

    --dof-angle A      dofAngle (0; keys -/=)          --focal F        dofDistance (6; keys [ ])
    --softness S       softness (0; keys 1/2)          --sss            SSS (false)
    --cacherays        rayCaching (false; key C)       --no-aa          antialias = false (key A)
    --no-compaction    COMPACTION = false              --bare           SHORTSTACK = false
    --brute            ENABLEKD = false                --bbox           USEBBOX = true (with --brute)
    --viz-kd           VIZKD = true                    --testing        TESTINGMODE (per-bounce timing)
    --iterations N     the scene's ITERATIONS          --res W H / --depth D   scene overrides
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def scene_header(path: str) -> dict:
    """ITERATIONS and FILE of the scene's CAMERA block (Scene::loadCamera, src/scene.cpp:190-223)."""
    out = {"iterations": None, "file": None}
    with open(path) as f:
        for line in f:
            tok = line.split()
            if len(tok) >= 2 and tok[0] == "ITERATIONS":
                out["iterations"] = int(float(tok[1]))
            elif len(tok) >= 2 and tok[0] == "FILE":
                out["file"] = tok[1]
    return out


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="python -m kdtreepathtraceroptimization_amd",
                                 description="Headless KD-tree path tracer on MI355X (reference: src/main.cpp).")
    ap.add_argument("scene", help="scene text file (scenes/*.txt)")
    ap.add_argument("mesh", nargs="?", default=None, help="optional OBJ mesh (KD tree built on the host)")
    ap.add_argument("--iterations", "--spp", type=int, default=None, help="samples per pixel (default: ITERATIONS)")
    ap.add_argument("--res", type=int, nargs=2, default=None, metavar=("W", "H"))
    ap.add_argument("--depth", type=int, default=None, help="traceDepth override")
    ap.add_argument("--bounce-cap", type=int, default=8, help="bounces per iteration (reference: 8)")
    ap.add_argument("--dof-angle", type=float, default=0.0)
    ap.add_argument("--focal", type=float, default=6.0)
    ap.add_argument("--softness", type=float, default=0.0)
    ap.add_argument("--sss", action="store_true")
    ap.add_argument("--cacherays", action="store_true")
    ap.add_argument("--no-aa", action="store_true")
    ap.add_argument("--no-compaction", action="store_true")
    ap.add_argument("--bare", action="store_true", help="traverseKDbare instead of the short-stack hybrid")
    ap.add_argument("--brute", action="store_true", help="no KD tree: every OBJ triangle (pathTraceOneBounce)")
    ap.add_argument("--bbox", action="store_true", help="brute force: each shape's bbox test first")
    ap.add_argument("--viz-kd", action="store_true", help="draw the KD node boxes")
    ap.add_argument("--testing", action="store_true", help="TESTINGMODE: time the intersect kernel per bounce")
    ap.add_argument("--first-iteration", type=int, default=1, help="first (1-based) iteration number")
    ap.add_argument("--out", default=None, help="output base name (default: the scene's FILE + samples)")
    ap.add_argument("--no-png", action="store_true")
    ap.add_argument("--hdr", action="store_true", help="also write BASE.hdr (image::saveHDR)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=8, help="batches in flight (throughput only)")
    ap.add_argument("--batch", type=int, default=16,
                    help="iterations sharing an intersect launch (<= 16, MAXB); 8 x 16 is bench.py's shape")
    ap.add_argument("--kd-build", choices=["gpu", "host"], default="gpu",
                    help="build the KD tree on the GPU (default; byte-identical) or with the host recursion")
    ap.add_argument("--dry-run", action="store_true", help="load and build the scene, print it, render nothing")
    return ap.parse_args(argv)


def options_from_args(a: argparse.Namespace):
    from .runtime import default_options
    return default_options(focal_length=a.focal, dof_angle=a.dof_angle, softness=a.softness,
                           cacherays=int(a.cacherays), antialias=0 if a.no_aa else 1, enable_sss=int(a.sss),
                           testing_mode=int(a.testing), compaction=0 if a.no_compaction else 1,
                           enable_kd=0 if a.brute else 1, viz_kd=int(a.viz_kd), use_bbox=int(a.bbox),
                           short_stack=0 if a.bare else 1, bounce_cap=a.bounce_cap)


def main(argv=None) -> int:
    a = parse_args(argv)
    from .runtime import PathTracer, SceneData
    hdr = scene_header(a.scene)
    iterations = a.iterations if a.iterations is not None else (hdr["iterations"] or 1)
    if iterations < 1:
        raise SystemExit("--iterations must be >= 1")
    kd_dev = a.device if (a.kd_build == "gpu" and not a.dry_run) else None  # --dry-run needs no GPU
    sd = SceneData.from_files(a.scene, a.mesh, res=tuple(a.res) if a.res else None, depth=a.depth, kd_device=kd_dev)
    W, H = sd.resolution
    info = {"scene": a.scene, "mesh": a.mesh, "resolution": [W, H], "iterations": iterations,
            "geoms": sd.view.num_geoms, "materials": sd.view.num_materials, "kd_nodes": sd.view.num_nodes,
            "kd_tri_refs": sd.view.num_tris, "kd_build": a.kd_build if kd_dev is not None else "host",
            "kd_build_ms": round(sd.kd_build_ms(), 3) if kd_dev is not None else None}
    if a.dry_run:
        print(json.dumps(info), flush=True)
        sd.close()
        return 0
    opt = options_from_args(a)
    with PathTracer(sd, opt, device=a.device) as pt:
        t0 = time.perf_counter()
        if a.testing:  # one synchronous pathtrace() per iteration, like TESTINGMODE
            for it in range(a.first_iteration, a.first_iteration + iterations):
                pt.trace_iteration(it)
        else:
            pt.trace_iterations(a.first_iteration, iterations, pipeline=a.pipeline, batch=a.batch)
            pt.synchronize()
        dt = time.perf_counter() - t0
        st = pt.stats()
        base = a.out or f"{hdr['file'] or os.path.splitext(os.path.basename(a.scene))[0]}.{iterations}samp"
        written = []
        if not a.no_png:
            pt.save_png(base + ".png", float(iterations))
            written.append(base + ".png")
        if a.hdr:
            pt.save_hdr(base + ".hdr", float(iterations))
            written.append(base + ".hdr")
    info.update({"segments": int(st.total_segments), "seconds": round(dt, 4),
                 "mrays_per_s": round(st.total_segments / dt / 1e6, 2) if dt > 0 else None,
                 "ms_per_iteration": round(dt * 1e3 / iterations, 4), "written": written})
    if a.testing:
        info["intersect_ms_total"] = round(st.intersect_ms_total, 4)
    print(json.dumps(info), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
