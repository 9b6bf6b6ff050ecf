"""Wave profile of the intersect kernel under kdpt_trace_iterations (tuning knob "profile_batches")."""
import json
import os
import sys

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene

# KDPT_PROF_RES=1600x1600 KDPT_PROF_DEPTH=16 KDPT_PROF_CAP=16 for C5 (icosphere_8)
_res = tuple(int(v) for v in os.environ.get("KDPT_PROF_RES", "800x800").split("x"))
_depth = int(os.environ.get("KDPT_PROF_DEPTH", "8"))
_cap = int(os.environ.get("KDPT_PROF_CAP", "8"))
sd = SceneData.from_description(load_fixture_scene("cornell", sys.argv[1] if len(sys.argv) > 1 else "dragon_5",
                                                   res=_res, depth=_depth))
for cfg in (sys.argv[2] if len(sys.argv) > 2 else "1x1,2x2,1x4").split(","):
    p, b = (int(v) for v in cfg.split("x"))
    pt = PathTracer(sd, default_options(testing_mode=1, bounce_cap=_cap))
    pt.set_tuning("profile_batches", 2 if os.environ.get("KDPT_PROFILE_STEPS") else 1)
    for kv in os.environ.get("KDPT_TUNE", "").split(","):  # e.g. KDPT_TUNE=cluster_slab=0
        if kv:
            pt.set_tuning(kv.split("=")[0], float(kv.split("=")[1]))
    pt.trace_iterations(1, 4 * p * b, pipeline=p, batch=b)
    pt.synchronize()
    prof = pt.wave_profile()
    prof.pop("wave_life_10us", None)
    hist = prof.pop("ray_steps_hist4", None)
    cs, cn = prof.pop("chord_steps", None), prof.pop("chord_rays", None)
    if hist:
        print(json.dumps({"cfg": cfg, "ray_steps_hist4": hist,
                          "steps_by_chord8": [round(a / max(1, b), 1) for a, b in zip(cs, cn)], "rays_by_chord8": cn}),
              flush=True)
    rays = max(1, pt.stats().total_trace_rays)
    print(json.dumps({"cfg": cfg, "rays": rays, "per_ray": {k: round(v / rays, 3) for k, v in prof.items()}}),
          flush=True)
    w = max(1, prof["chunks"])
    eff = prof["node_lane_steps"] / max(1, prof["node_trips"]) / 64
    print(json.dumps({"cfg": cfg, "waves": w, "node_trips_per_wave": round(prof["node_trips"] / w, 1),
                      "node_simd_eff": round(eff, 3), "small_phases_per_wave": round(prof["small_phases"] / w, 1),
                      "cyc_frac": {k: round(prof[k] / max(1, prof["chunk_cycles"]), 3)
                                   for k in prof if k.endswith("_cycles") and k != "chunk_cycles"}}), flush=True)
    pt.close()
