"""Per-frame time of C4's 32-spp frames (cornell8 + dragon_5, 800x800, 8 x 16 in flight) for the first context
of a process and for later ones: A (first), A again with B created, B (second), A again, A after B is closed,
C (created after A and B are closed).  Measured (profiles/r05_ab_log.md): the first context 6.7-7.5 ms a frame,
every later one 12.2-14.1, whether or not the others are alive, with the margin-only cull too, after a 20 GB
allocation made and freed before A, and with every stream pooled: what a later context does differently is
not found yet.

    python tools/context_order_probe.py [NAME=VALUE ...] [--dummy-first]
"""
import json, os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from kdtreepathtraceroptimization_amd import runtime as kdpt
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene
sd = kdpt.SceneData.from_description(load_fixture_scene("cornell8", "dragon_5", res=(800, 800), depth=8))
opt = kdpt.default_options()
TUNE = [kv.split("=") for kv in sys.argv[1:] if "=" in kv]
if "--dummy-first" in sys.argv:  # a large device allocation made and freed before the first context
    x = torch.empty(20 << 30, dtype=torch.uint8, device="cuda"); del x; torch.cuda.empty_cache()
def make():
    pt = kdpt.PathTracer(sd, opt, device=0)
    for k, v in TUNE:
        pt.set_tuning(k, float(v))
    return pt
def per_frame(pt, n0=8, n1=88):
    ts = []
    for n in (n0, n1):
        pt.reset(); pt.synchronize()
        t = time.perf_counter(); pt.render_frames(0, n, 32, pipeline=8, batch=16); pt.synchronize()
        ts.append(time.perf_counter() - t)
    st = pt.stats()
    dl = st.intersect_device_ms_total / max(1, st.intersect_device_launches_total)
    return [round(1e3 * (ts[1] - ts[0]) / (n1 - n0), 3), round(dl, 4), st.intersect_device_launches_total]
out = {}
A = make()
per_frame(A, 2, 4)
out["A_alone"] = per_frame(A)
B = make()
out["A_with_B_created"] = per_frame(A)
per_frame(B, 2, 4)
out["B_second"] = per_frame(B)
out["A_again"] = per_frame(A)
B.close()
out["A_after_B_closed"] = per_frame(A)
A.close()
C = make()
per_frame(C, 2, 4)
out["C_after_A_B_closed"] = per_frame(C)
print(json.dumps(out), flush=True)
