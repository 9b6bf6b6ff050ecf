"""C4's per-GPU frame through the two C-ABI multi-GPU entry points on one GPU:
kdpt_render_sharded(devices=[0], RCCL reduce) against a context's kdpt_render_frames, 32-spp frames of
cornell8 + dragon_5 at 800x800, depth 8, pipeline 8 x 16.

kdpt_render_sharded creates and destroys its contexts inside the call, so each form is timed at two frame
counts and the per-frame time taken from the difference (setup cancels).

    python tools/sharded_vs_frames.py [--spp 32] [--frames 8 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kdtreepathtraceroptimization_amd import runtime as kdpt  # noqa: E402
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--frames", type=int, nargs=2, default=(8, 40))
    ap.add_argument("--repeats", type=int, default=2)
    a = ap.parse_args()
    sd = kdpt.SceneData.from_description(load_fixture_scene("cornell8", "dragon_5", res=(800, 800), depth=8))
    opt = kdpt.default_options()
    res = {}

    def sharded(n):
        t = time.perf_counter()
        kdpt.render_sharded(sd, [0], 0, n, a.spp, options=opt, pipeline=8, batch=16, reduce=kdpt.REDUCE_RCCL)
        return time.perf_counter() - t

    pt = kdpt.PathTracer(sd, opt, device=0)
    segs = {}

    def frames(n):
        pt.reset()
        pt.synchronize()
        t = time.perf_counter()
        pt.render_frames(0, n, a.spp, pipeline=8, batch=16)
        pt.synchronize()
        dt = time.perf_counter() - t
        segs[n] = pt.stats().total_segments
        return dt

    for name, fn in (("render_frames", frames), ("render_sharded_rccl", sharded)):
        fn(a.frames[0])  # warm-up (code objects, masks, RCCL init)
        per = []
        for _ in range(a.repeats):
            t0, t1 = fn(a.frames[0]), fn(a.frames[1])
            per.append((t1 - t0) / (a.frames[1] - a.frames[0]))
        res[name] = {"ms_per_frame": 1e3 * min(per), "all_ms": [round(1e3 * p, 3) for p in per]}
    seg_frame = (segs[a.frames[1]] - segs[a.frames[0]]) / (a.frames[1] - a.frames[0])
    for v in res.values():
        v["Mrays_per_s"] = seg_frame / (v["ms_per_frame"] * 1e-3) / 1e6
    res["sharded_over_frames"] = res["render_sharded_rccl"]["Mrays_per_s"] / res["render_frames"]["Mrays_per_s"]
    res["spp"] = a.spp
    pt.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
