"""Intersect-workgroup tail share from a -DKDPT_TAIL_PROF variant (tools/build_variant.sh tailprof -DKDPT_TAIL_PROF):
the part of each k_trace workgroup's life after its first wave found the launch's ray queue empty.

    KDPT_LIBRARY=ab/tailprof.so python tools/tail_prof.py [PIPELINExBATCH ...]
"""
import ctypes as C
import json
import os
import sys

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene  # noqa: E402

sd = SceneData.from_description(load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8))
for cfg in sys.argv[1:] or ["8x4", "1x4"]:
    p, b = (int(v) for v in cfg.split("x"))
    pt = PathTracer(sd, default_options())
    out = (C.c_ulonglong * 4)()
    pt.trace_iterations(1, 4 * p * b, pipeline=p, batch=b)
    pt.synchronize()
    pt.lib.kdpt_debug_tail_prof(out)
    pt.trace_iterations(1 + 4 * p * b, 8 * p * b, pipeline=p, batch=b)
    pt.synchronize()
    pt.lib.kdpt_debug_tail_prof(out)
    life, tail, wgs = out[0], out[1], max(1, out[2])
    print(json.dumps({"cfg": cfg, "workgroups": int(out[2]), "wg_life_us": round(life / wgs / 100, 1),
                      "wg_tail_us": round(tail / wgs / 100, 1), "tail_share": round(tail / max(1, life), 3)}),
          flush=True)
    pt.close()
