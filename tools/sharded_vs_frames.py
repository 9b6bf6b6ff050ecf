"""C4's per-GPU frame through the C-ABI multi-GPU entry points on one GPU:
kdpt_render_sharded(devices=[0]) with the RCCL and the copy reduce, against a context's kdpt_render_frames
without and with a one-rank RCCL communicator; 32-spp frames of cornell8 + dragon_5 at 800x800, depth 8,
pipeline 8 x 16, every frame copied out to pinned host memory.

Each form runs in a context of its own, created and destroyed around the run, and is timed at two frame counts;
the per-frame time is the difference (setup cancels). Only one context is alive at a time: HIP maps a process's
streams onto its few hardware queues in creation order, and another context's idle streams change where a
context's batch streams land (with two contexts alive, render_frames measured 13.7 instead of 7.4 ms a frame).

    python tools/sharded_vs_frames.py [--spp 32] [--frames 8 168]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402  (pinned host memory)
from kdtreepathtraceroptimization_amd import runtime as kdpt  # noqa: E402
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--frames", type=int, nargs=2, default=(8, 168))
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--warm", action="store_true", help="also: render_frames in one context kept across runs")
    a = ap.parse_args()
    sd = kdpt.SceneData.from_description(load_fixture_scene("cornell8", "dragon_5", res=(800, 800), depth=8))
    opt = kdpt.default_options()
    lib = kdpt.load_library()
    w, h = sd.resolution
    # (a pageable `out` would be registered by the call itself, a cost that grows with the frame count)
    host = torch.empty((a.frames[1], h, w, 3), dtype=torch.float32, pin_memory=True)
    hptr = host.data_ptr()
    segs = {}

    def frames_with(rccl1):
        def run(n):
            with kdpt.PathTracer(sd, opt, device=0) as pt:
                if rccl1:  # a one-rank communicator: the library's ncclReduce per frame (a fresh id each)
                    uid = (C.c_ubyte * 128)()
                    assert lib.kdpt_comm_unique_id(uid) == 0
                    assert lib.kdpt_comm_init(pt._ctx, 1, 0, uid) == 0, lib.kdpt_last_error()
                pt.synchronize()
                t = time.perf_counter()
                pt.render_frames(0, n, a.spp, pipeline=8, batch=16, out=hptr)
                pt.synchronize()
                dt = time.perf_counter() - t
                segs[n] = pt.stats().total_segments
            return dt
        return run

    def sharded_with(reduce):
        def run(n):
            devs = (C.c_int * 1)(0)
            t = time.perf_counter()
            rc = lib.kdpt_render_sharded(C.byref(sd.view), C.byref(opt), 1, devs, 0, int(n), int(a.spp), 8, 16,
                                         int(reduce), C.c_void_p(hptr))
            assert rc == 0, lib.kdpt_last_error()
            return time.perf_counter() - t
        return run

    warm = {}

    def frames_warm(n):  # one context for every run (created at the first)
        if "pt" not in warm:
            warm["pt"] = kdpt.PathTracer(sd, opt, device=0)
        pt = warm["pt"]
        pt.reset()
        pt.synchronize()
        t = time.perf_counter()
        pt.render_frames(0, n, a.spp, pipeline=8, batch=16, out=hptr)
        pt.synchronize()
        return time.perf_counter() - t

    res = {}
    for name, fn in (("render_frames", frames_with(False)), ("render_frames_rccl1", frames_with(True)),
                     ("render_sharded_rccl", sharded_with(kdpt.REDUCE_RCCL)),
                     ("render_sharded_copy", sharded_with(kdpt.REDUCE_COPY))):
        fn(a.frames[0])  # warm-up (code objects, masks, RCCL init)
        per = []
        for _ in range(a.repeats):
            t0, t1 = fn(a.frames[0]), fn(a.frames[1])
            per.append((t1 - t0) / (a.frames[1] - a.frames[0]))
        res[name] = {"ms_per_frame": 1e3 * min(per), "all_ms": [round(1e3 * p, 3) for p in per]}
    if a.warm:
        fn = frames_warm
        fn(a.frames[0])
        per = []
        for _ in range(a.repeats):
            t0, t1 = fn(a.frames[0]), fn(a.frames[1])
            per.append((t1 - t0) / (a.frames[1] - a.frames[0]))
        res["render_frames_warm_context"] = {"ms_per_frame": 1e3 * min(per), "all_ms": [round(1e3 * p, 3) for p in per]}
        warm["pt"].close()
    seg_frame = (segs[a.frames[1]] - segs[a.frames[0]]) / (a.frames[1] - a.frames[0])
    for v in res.values():
        v["Mrays_per_s"] = seg_frame / (v["ms_per_frame"] * 1e-3) / 1e6
    res["sharded_rccl_over_frames"] = res["render_sharded_rccl"]["Mrays_per_s"] / res["render_frames"]["Mrays_per_s"]
    res["spp"] = a.spp
    print(json.dumps(res))


if __name__ == "__main__":
    main()
