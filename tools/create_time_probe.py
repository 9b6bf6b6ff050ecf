"""kdpt_create's wall time on C3 (cornell + dragon_5, 800x800, depth 8) for the process's first context and later
ones, and the masked cull's share of it (kdpt_stats.create_ms / mask_build_ms).

    python tools/create_time_probe.py [--contexts 4]
"""
import argparse
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--contexts", type=int, default=4)
a = ap.parse_args()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime, torch's)
from kdtreepathtraceroptimization_amd import runtime as kdpt  # noqa: E402
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene  # noqa: E402

sd = kdpt.SceneData.from_description(load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8))
for i in range(a.contexts):
    t = time.perf_counter()
    with kdpt.PathTracer(sd, kdpt.default_options()) as pt:
        st = pt.stats()
        n = pt.trace_config()["cull_mask_n"]
        print({"context": i, "create_ms": round(st.create_ms, 2), "mask_build_ms": round(st.mask_build_ms, 2),
               "cull_mask_n": n, "wall_ms_incl_destroy": round(1e3 * (time.perf_counter() - t), 1)}, flush=True)
