"""Shading phase times from a -DKDPT_SHADE_PROF variant (tools/build_variant.sh shprof -DKDPT_SHADE_PROF):
per tile, shade_one (+ the tile barrier) / look-back / survivor writes, in s_memrealtime ticks (100 MHz).

    KDPT_LIBRARY=ab/shprof.so python tools/shade_prof.py [PIPELINExBATCH ...]
"""
import ctypes as C
import json
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene  # noqa: E402

sd = SceneData.from_description(load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8))
for cfg in sys.argv[1:] or ["8x4", "1x1"]:
    p, b = (int(v) for v in cfg.split("x"))
    pt = PathTracer(sd, default_options(testing_mode=1))
    fn = pt.lib.kdpt_debug_shade_prof
    out = (C.c_ulonglong * 8)()
    pt.trace_iterations(1, 4 * p * b, pipeline=p, batch=b)
    pt.synchronize()
    fn(out)  # warm-up counts dropped
    t0 = time.perf_counter()
    pt.trace_iterations(1 + 4 * p * b, 8 * p * b, pipeline=p, batch=b)
    pt.synchronize()
    wall = time.perf_counter() - t0
    fn(out)
    tiles = max(1, out[3])
    print(json.dumps({"cfg": cfg, "iterations": 8 * p * b, "wall_ms": round(wall * 1e3, 2), "tiles": int(out[3]),
                      "paths": int(out[4]),
                      "us_per_tile": {"ticket_stage": round(out[5] / tiles / 100, 2),
                                      "loads": round(out[6] / tiles / 100, 2),
                                      "publish_barrier": round(out[7] / tiles / 100, 2),
                                      "shade_compute": round((out[0] - out[6] - out[7]) / tiles / 100, 2),
                                      "lookback": round(out[1] / tiles / 100, 2),
                                      "writes": round(out[2] / tiles / 100, 2)},
                      "tile_us_sum_per_iteration": round((out[0] + out[1] + out[2]) / 100 / (8 * p * b), 1)}),
          flush=True)
    pt.close()
