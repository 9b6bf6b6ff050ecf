"""The product's spp-sharded multi-rank path on the GPU (SURVEY.md 8(e), config C4's workload).

Two fresh processes (spawned before either touches the GPU; both on cuda:0 of this one-GPU box) each
create their own PathTracer whose accumulation image is an external device buffer (a torch tensor, as
bench.py gives it an RCCL buffer), render their shard of global iterations 1 + k*2 + r with
kdpt_trace_iterations(stride = 2) -- the bench's pipelined form -- and sum the shard images on rank 0
with a gloo reduce of host copies (RCCL needs one GPU per rank).  The reduced image must equal, bit for
bit, the oracle's renders of the same iterations summed in the same grouping: each shard in iteration
order, then the two shard sums.  Iteration 2 (the material sort) lands on rank 1.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kdtreepathtraceroptimization_amd.distributed import shard_iterations
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene

pytestmark = pytest.mark.gpu

SCENE, MESH, RES, DEPTH = "cornell8", "dragon_5", (800, 800), 8  # C4's workload
STEPS = 4  # per rank: global iterations 1..8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options
    from kdtreepathtraceroptimization_amd.distributed import global_iteration, reduce_image
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        W, H = RES
        accum = torch.zeros(3 * W * H, dtype=torch.float32, device="cuda:0")
        sd = SceneData.from_description(load_fixture_scene(SCENE, MESH, res=RES, depth=DEPTH))
        pt = PathTracer(sd, default_options(external_image=accum.data_ptr()), device=0)
        pt.trace_iterations(global_iteration(0, world, rank), STEPS, stride=world, pipeline=2, batch=2)
        pt.synchronize()
        seg = torch.tensor([pt.stats().total_segments], dtype=torch.int64)
        reduce_image(accum, dist)  # gloo: host round trip inside reduce_image
        dist.reduce(seg, dst=0)
        if rank == 0:
            np.save(out, accum.cpu().numpy())
            np.save(out + ".seg.npy", seg.numpy())
        pt.close()
    finally:
        dist.destroy_process_group()


def test_spp_sharded_world2_equals_oracle_grouping(tmp_path, oracle):
    world = 2
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    seg = int(np.load(out + ".seg.npy")[0])
    s = oracle.OracleScene.from_description(load_fixture_scene(SCENE, MESH, res=RES, depth=DEPTH))
    parts, oseg = [], 0
    for r in range(world):
        acc = None
        for it in shard_iterations(0, STEPS, world, r):
            im, st = s.render(it, 1)
            oseg += st.segments
            acc = im.copy() if acc is None else acc + im
        parts.append(acc.reshape(-1))
    expect = parts[0] + parts[1]
    assert seg == oseg
    assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), \
        f"{int(np.sum(got != expect))} values differ"


def test_bench_main_world2_gloo(tmp_path):
    """bench.py's own N > 1 main(): two ranks launched by torch.distributed.run (sharing this box's one GPU,
    so the framebuffer reduce goes through gloo; the driver's 8-GPU run takes the RCCL branch of the same
    code), the stats all-reduces and the in-timed-region reduce.  The reduced image rank 0 dumps must equal
    the two shards rendered here by the product one after the other and added (a + b is exact in either
    order), and the segment count must be the shards' sum."""
    import json
    import subprocess
    import sys

    from conftest import ROOT
    from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options
    from kdtreepathtraceroptimization_amd.distributed import global_iteration

    res, steps, warmup, spp, world = (160, 120), 2, 1, 4, 2
    out = str(tmp_path / "bench_img.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--dist-backend", "gloo", "--steps", str(steps), "--warmup", str(warmup),
           "--spp-per-step", str(spp), "--res", *map(str, res), "--no-cpu-baseline", "--dump-image", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric"')][-1])
    assert line["n_gpus"] == world and line["steps"] == steps and line["value"] > 0
    got = np.load(out)
    sd = SceneData.from_description(load_fixture_scene("cornell", "dragon_5", res=res, depth=8))
    parts, seg = [], 0
    for rank in range(world):
        with PathTracer(sd, default_options(testing_mode=1, short_stack=1, bounce_cap=8), device=0) as pt:
            pt.trace_iterations(global_iteration(warmup * spp, world, rank), steps * spp, stride=world)
            pt.synchronize()
            parts.append(pt.image().reshape(-1))
            seg += pt.stats().total_segments
    assert line["segments_per_iteration"] * steps * spp * world == pytest.approx(seg, abs=1)
    expect = parts[0] + parts[1]
    assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), f"{int(np.sum(got != expect))} differ"
