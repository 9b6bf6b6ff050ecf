"""bench.py -- the reference's headline metric on MI355X.

Metric (BASELINE.json): Mrays/s at 800x800, depth 8, cornell + dragon (dragon_5.obj: the
only dragon mesh present -- cornell9.txt does not exist).
A step = one iteration = one sample per pixel through the whole hot path
(camera rays -> up to 8 x [intersect + KD traversal + scatter + shade + gather +
stable compaction]).  Mrays/s = path segments launched into the intersect kernel,
summed over all ranks, / the max-over-ranks wall time of the K timed steps.

Multi-GPU (one process per GPU, `torch.distributed.run`): samples per pixel shard
across ranks (rank r renders global iterations r+1, r+1+N, ...: weak scaling) and the
float3 accumulation images are summed on rank 0 with one RCCL reduce over xGMI inside
the timed region.

Roofline: the dominant kernel is k_trace, the KD traversal of the rays that meet the KD root box (the
analytic geoms and the root-box test of every ray run before it: in k_geoms for camera rays, fused into the
previous bounce's shading/compaction otherwise; a ray that misses the root box ends there).  HBM-bound
framing with SURVEY.md 8(d)'s per-segment bytes B = 352 + 52*N_aabb + 36*N_tri + 40*N_hit restricted to the
traversal k_trace performs: per counting iteration 76*n_k + 52*(N_aabb - N_root_miss) + 36*N_tri + 40*N_hit
(n_k = segments handed to k_trace, 76 = PathSegment read 56 + ShadeableIntersection write 20), scaled to the
timed segments; achieved = bytes per launch / the average k_trace launch time on the device clock inside the
kernel (first workgroup start to last workgroup end; agrees with rocprofv3's kernel-trace durations).  HIP
events around the intersect stage are reported beside it: with several iterations in flight they also
count the time a launch waits behind the other iterations' kernels.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# kdpt_trace_iterations keeps `--pipeline` iterations in flight on their own HIP streams plus one
# accumulation stream; HIP's default of 4 hardware queues per process would make some of them share
# a queue (and serialise), so ask for 16 before the runtime initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=192)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--mesh", default="dragon_5")
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--res", type=int, nargs=2, default=(800, 800))
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--bare", action="store_true", help="traverseKDbare instead of the short-stack hybrid")
    ap.add_argument("--bounce-cap", type=int, default=8,
                    help="bounces per iteration (8 = the reference's `depth > 7`; 16 for the C5 stress config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--pipeline", type=int, default=8,
                    help="batches in flight (kdpt_trace_iterations; bit-identical to one at a time)")
    ap.add_argument("--batch", type=int, default=4, help="iterations sharing each intersect launch (<= 4)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = host-side reduce, for rehearsing the "
                         "N > 1 path with several ranks sharing one GPU")
    return ap.parse_args()


def cpu_baseline(args, threads=None, seconds=None):
    """The oracle (plain-C port of the reference path) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    seconds = args.cpu_seconds if seconds is None else seconds
    s = oracle_lib.OracleScene.from_description(
        load_fixture_scene(args.scene, args.mesh, res=tuple(args.res), depth=args.depth))
    seg, t, it = 0, 0.0, 3
    while t < seconds and it < 3 + 64:
        t0 = time.perf_counter()
        _, st = s.render(it, 1, nthreads=threads, shortstack=0 if args.bare else 1, bounce_cap=args.bounce_cap)
        t += time.perf_counter() - t0
        seg += st.segments
        it += 1
    return {"value": round(seg / t / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle (plain-C restatement of the reference's host-side kernels), {it - 3} iteration(s) "
                      f"3..{it - 1} of the same workload, {t:.1f} s, OpenMP over paths"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev if args.dist_backend == "gloo" else local  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene

    desc = load_fixture_scene(args.scene, args.mesh, res=tuple(args.res), depth=args.depth)
    sd = SceneData.from_description(desc)
    W, H = sd.resolution
    accum = torch.zeros(3 * W * H, dtype=torch.float32, device=f"cuda:{local}")
    opt = default_options(testing_mode=1, short_stack=0 if args.bare else 1, external_image=accum.data_ptr(),
                          bounce_cap=args.bounce_cap)
    pt = PathTracer(sd, opt, device=local)

    from kdtreepathtraceroptimization_amd.distributed import global_iteration, reduce_image

    def global_iter(step):  # 1-based, distinct across ranks and steps (spp sharding)
        return global_iteration(step, world, rank)

    # warmup (iterations disjoint from the timed ones); iteration 2's extra sort lands here
    if args.warmup:
        pt.trace_iterations(global_iter(0), args.warmup, stride=world, pipeline=args.pipeline, batch=args.batch)
        pt.synchronize()
    # roofline counters from one untimed counting iteration of the timed range
    aabb, tri, hit = pt.count_iteration(global_iter(args.warmup))
    try:
        aabb_prep, cand = pt.count_split()
    except AttributeError:  # an older libkdpt (A/B runs): no split, the whole stage
        aabb_prep, cand = 0, None
    cnt_stats = pt.stats()
    accum.zero_()
    torch.cuda.synchronize()
    st0 = pt.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pt.trace_iterations(global_iter(args.warmup), args.steps, stride=world, pipeline=args.pipeline,
                        batch=args.batch)
    pt.synchronize()
    reduce_image(accum, dist)  # spp shards -> one framebuffer (the only exchange step)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st1 = pt.stats()
    seg = st1.total_segments - st0.total_segments
    ev_ms = st1.intersect_ms_total - st0.intersect_ms_total  # HIP events around each intersect launch
    ev_launches = st1.intersect_launches_total - st0.intersect_launches_total
    kernel_ms = st1.intersect_device_ms_total - st0.intersect_device_ms_total  # device clock, per launch
    launches = st1.intersect_device_launches_total - st0.intersect_device_launches_total
    if dist:
        t = torch.tensor([dt, float(seg), kernel_ms, float(launches), ev_ms, float(ev_launches)], dtype=torch.float64,
                         device=f"cuda:{local}" if args.dist_backend == "nccl" else "cpu")
        tmax = t[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt, seg, kernel_ms, launches = float(tmax[0]), int(tsum[0]), float(tsum[1]), int(tsum[2])
        ev_ms, ev_launches = float(tsum[3]), int(tsum[4])
    if rank != 0:
        pt.close()
        if dist:
            dist.destroy_process_group()
        return
    # roofline of the dominant kernel, k_trace (the KD traversal of the rays that meet the root box), per
    # launch: algorithmic bytes of the counting iteration's k_trace work, scaled to the timed segments
    count_seg = max(1, sum(cnt_stats.seg_per_bounce[d] for d in range(32)) or seg // max(1, args.steps * world))
    cand = count_seg if cand is None else cand
    aabb_k = aabb - aabb_prep  # the root-box tests of rays that end before k_trace are not its work
    iter_bytes = 76 * cand + 52 * aabb_k + 36 * tri + 40 * hit
    per_seg_bytes = iter_bytes / count_seg
    avg_launch_ms = kernel_ms / max(1, launches)
    bytes_per_launch = per_seg_bytes * seg / max(1, launches)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    traffic = None
    tfile = os.path.join(ROOT, "profiles", f"traffic_{args.scene}_{args.mesh}_{W}x{H}.json")
    if os.path.exists(tfile):
        traffic = json.load(open(tfile)).get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC,
        "value": round(seg / dt / 1e6, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic camera rays over the reference's own scene assets (cornell.txt + dragon_5.obj, "
                "parsed fixtures under tests/golden); deterministic RNG seeded by iteration",
        "config": {"workload": f"{args.scene}.txt + {args.mesh}.obj, {W}x{H}, depth {args.depth}, "
                               f"bounce cap {args.bounce_cap}, 1 spp per step "
                               f"per GPU ({args.pipeline} x {args.batch} iterations in flight), "
                               + ("short-stack hybrid KD traversal" if not args.bare else "bare traversal"),
                   "scene": args.scene, "mesh": args.mesh, "resolution": [W, H], "depth": args.depth,
                   "bounce_cap": args.bounce_cap,
                   "kd_nodes": sd.view.num_nodes, "kd_tri_refs": sd.view.num_tris,
                   "parallelism": (f"spp-sharded x{world} + " + ("RCCL reduce" if args.dist_backend == "nccl" else
                                                                 "gloo host reduce (ranks sharing GPUs)"))
                   if world > 1 else "single GPU"},
        "segments_per_step": seg / (args.steps * world),
        "primary_rays_per_s": round(W * H * args.steps * world / dt, 1),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "k_trace (KD traversal of the rays that meet the KD root box)",
                     "k_trace_segments_per_launch": round(cand / count_seg * seg / max(1, launches), 1),
                     "launch_grid_share": round(pt.trace_grid_share(), 4),
                     "avg_launch_ms": round(avg_launch_ms, 5), "launches": launches,
                     "avg_launch_ms_events": round(ev_ms / max(1, ev_launches), 5),
                     "aggregate_GBps": round(per_seg_bytes * seg / dt / 1e9, 2),
                     "bytes_per_segment": round(per_seg_bytes, 2),
                     "per_segment_counts": {"aabb": round(aabb / count_seg, 4), "tri": round(tri / count_seg, 4),
                                            "hit": round(hit / count_seg, 5),
                                            "aabb_before_k_trace": round(aabb_prep / count_seg, 4),
                                            "k_trace_share": round(cand / count_seg, 4)}},
        "reference_980m_intersect_ms_per_iter": 79.4,
        "intersect_ms_per_iter": round(kernel_ms / (args.steps * world), 4),
        "roofline_note": "achieved = algorithmic bytes per k_trace launch / its average duration, as the contract "
                         "defines it; with `pipeline` batches in flight each launch runs on launch_grid_share of the "
                         "CUs concurrently with the others, so the chip-level algorithmic rate is aggregate_GBps "
                         "(bytes of all segments / wall time of the timed region)",
        "timing_note": "avg_launch_ms: k_trace launches on the device clock (s_memrealtime, first block start to "
                       "last block end), comparable with rocprofv3 kernel-trace durations; avg_launch_ms_events: HIP "
                       "events on the launching stream around the intersect stage (k_geoms when it runs + k_trace), "
                       "which also count queueing behind the other in-flight iterations' kernels",
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
        # SURVEY 8(d) / BASELINE.md 3: the same oracle on one core as well (at least one whole iteration)
        out["cpu_baseline_1core"] = cpu_baseline(args, threads=1, seconds=args.cpu_seconds / 2)
    pt.close()
    if dist:
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
