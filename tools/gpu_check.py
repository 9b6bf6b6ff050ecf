"""Quick GPU parity + timing check (cornell scenes vs the oracle), for development runs."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
from kdtreepathtraceroptimization_amd import PathTracer, SceneData, imgsum, load_fixture_scene  # noqa: E402

an = json.load(open(os.path.join(ROOT, "tests/golden/anchors.json")))
for a in an["survey_anchor_table"]:
    desc = load_fixture_scene(a["scene"], a["mesh"], res=a["res"], depth=a["depth"])
    sd = SceneData.from_description(desc)
    with PathTracer(sd) as pt:
        seg = 0
        t0 = time.time()
        for it in range(a["iters"][0], a["iters"][1] + 1):
            pt.trace_iteration(it)
            seg += pt.stats().segments
        img = pt.image()
        dt = time.time() - t0
        ms = pt.stats().ms_last_iteration
    print(json.dumps({"mesh": a["mesh"], "res": a["res"], "segments": seg, "expect_segments": a["segments"],
                      "imgsum": round(imgsum(img), 6), "expect_imgsum": a["imgsum"], "wall_s": round(dt, 3),
                      "ms_last_iter": round(ms, 3)}), flush=True)
    if a["res"][0] <= 200:
        ref, st = oracle_lib.OracleScene.from_description(desc).render(a["iters"][0], a["iters"][1] - a["iters"][0] + 1)
        diff = img != ref
        print("  bit-exact vs oracle:", not diff.any(), "ndiff", int(diff.sum()), "maxabs", float(np.abs(img - ref).max()))
# timing: dragon_5 800x800, 10 iterations
desc = load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8)
with PathTracer(SceneData.from_description(desc)) as pt:
    pt.trace_iteration(1)
    ts, segs = [], []
    for it in range(3, 13):
        pt.trace_iteration(it)
        st = pt.stats()
        ts.append(st.ms_last_iteration)
        segs.append(st.segments)
    print(json.dumps({"dragon5_ms_per_iter": [round(t, 3) for t in ts], "mean_ms": float(np.mean(ts)),
                      "Mseg_per_s": float(np.sum(segs) / np.sum(ts) / 1e3)}))
    print("counters", pt.count_iteration(3))
