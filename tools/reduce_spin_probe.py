"""Is the frame pipeline immune to a slow reduce?  

At N > 1 GPUs a frame's ncclReduce waits for the slowest peer.  The knob "reduce_spin_us" puts a device spin of
that length on the reduce stream before every frame's reduce, so one GPU sees what a waiting reduce does to its
queues.  This probe renders C4's per-GPU frame shape (cornell8 + dragon_5, 800x800, depth 8, 32-spp frames,
8 x 16 iterations in flight) and reports ms per frame, with and without a spin, for

- A: the process's first context, render_frames;
- B: a second context created after A (still alive), render_frames;
- S: kdpt_render_sharded(devices=[0, 0], COPY): two contexts on the GPU, the peer-copy reduce (the spin is set as
  the process default, kdpt_set_tuning(NULL, ...), for the contexts the call creates);

each timed at two frame counts (setup cancels).  The GPU's hardware queue count is the process's
GPU_MAX_HW_QUEUES (bench.py asks for 24; HIP's default is 4): pass --queues to set it before HIP starts.

    python tools/reduce_spin_probe.py [--queues 24] [--spin 5000] [--frames 8 88]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument("--queues", type=int, default=None)
ap.add_argument("--spin", type=float, default=5000.0)
ap.add_argument("--frames", type=int, nargs=2, default=(8, 88))
ap.add_argument("--spp", type=int, default=32)
ap.add_argument("--cu-mask", action="store_true", help="contexts' batch / reduce streams with an all-CU mask")
a = ap.parse_args()
if a.queues:
    os.environ["GPU_MAX_HW_QUEUES"] = str(a.queues)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime, torch's)
from kdtreepathtraceroptimization_amd import runtime as kdpt  # noqa: E402
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene  # noqa: E402

sd = kdpt.SceneData.from_description(load_fixture_scene("cornell8", "dragon_5", res=(800, 800), depth=8))
opt = kdpt.default_options()
lib = kdpt.load_library()
n0, n1 = a.frames


def per_frame_ctx(pt, spin):
    pt.set_tuning("reduce_spin_us", spin)
    ts = []
    for n in (n0, n1):
        pt.reset()
        pt.synchronize()
        t = time.perf_counter()
        pt.render_frames(0, n, a.spp, pipeline=8, batch=16)
        pt.synchronize()
        ts.append(time.perf_counter() - t)
    return round(1e3 * (ts[1] - ts[0]) / (n1 - n0), 3)


def per_frame_sharded(spin, repeats=3):
    # each call creates and destroys its two contexts: the per-frame time is the difference of two frame counts,
    # the median of a few repeats (the creation's cost varies from call to call)
    assert lib.kdpt_set_tuning(None, b"reduce_spin_us", C.c_double(spin)) == 0, lib.kdpt_last_error()
    per = []
    for _ in range(repeats):
        ts = []
        for n in (n0, 2 * n1):
            t = time.perf_counter()
            kdpt.render_sharded(sd, [0, 0], 0, n, a.spp, options=opt, pipeline=8, batch=16, reduce=kdpt.REDUCE_COPY)
            ts.append(time.perf_counter() - t)
        per.append(1e3 * (ts[1] - ts[0]) / (2 * n1 - n0))
    assert lib.kdpt_set_tuning(None, b"reduce_spin_us", C.c_double(0.0)) == 0
    return round(sorted(per)[len(per) // 2], 3)


lib.kdpt_set_tuning.argtypes = [C.c_void_p, C.c_char_p, C.c_double]
if a.cu_mask:
    kdpt.set_process_tuning("cu_mask_streams", 1)
out = {"queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"), "spin_us": a.spin, "spp": a.spp,
       "cu_mask_streams": a.cu_mask}
A = kdpt.PathTracer(sd, opt, device=0)
per_frame_ctx(A, 0)  # warm
out["A_first"] = {"spin0": per_frame_ctx(A, 0), "spin": per_frame_ctx(A, a.spin)}
B = kdpt.PathTracer(sd, opt, device=0)
per_frame_ctx(B, 0)
out["B_second"] = {"spin0": per_frame_ctx(B, 0), "spin": per_frame_ctx(B, a.spin)}
out["A_again"] = {"spin0": per_frame_ctx(A, 0), "spin": per_frame_ctx(A, a.spin)}
B.close()
A.close()
out["S_sharded_copy_00"] = {"spin0": per_frame_sharded(0), "spin": per_frame_sharded(a.spin)}
for k, v in out.items():
    if isinstance(v, dict):
        v["ratio"] = round(v["spin0"] / v["spin"], 4)
print(json.dumps(out), flush=True)
