"""bench.py -- the reference's headline metric on MI355X.

Metric (BASELINE.json): Mrays/s at 800x800, depth 8, cornell + dragon (dragon_5.obj: the only dragon mesh
present -- cornell9.txt does not exist), plus ms per iteration.

A step is one frame (kdpt_render_frames): `--spp-per-step` samples per pixel per GPU (default 1024, weak
scaling) or a fixed `--total-spp` split over the GPUs (strong scaling, C4's "256 spp sharded 32/GPU").  A
sample is one iteration of the whole hot path (camera rays -> up to 8 x [intersect + KD traversal + scatter +
shade + gather + stable compaction]) with its own global iteration number (RNG seed).  Frames stay in flight
back to back (frame f + 1 renders while frame f is reduced), so the GPU stays at steady state.  Mrays/s =
path segments launched into the intersect stage, summed over all ranks, / the max-over-ranks wall time of
the K timed frames; `ms_per_iteration` is reported beside `ms_per_step`.  The driver's `--steps 20 --warmup 5`
times 20 480 iterations (about 8.5 s of GPU work for C3).

Multi-GPU (one process per GPU, `torch.distributed.run`): rank r renders the frame's global iterations
f*F + 1 + r, stride N, and each frame's float3 image is summed on rank 0 by one RCCL ncclReduce issued inside
libkdpt (kdpt_comm_init / kdpt_render_frames; the communicator's unique id goes out over the process group).
The gloo backend (ranks sharing a GPU, CPU rehearsals) hands each rank's frame shares out and reduces them here.

Roofline: the dominant kernel is k_trace (the KD traversal of the rays that meet the KD root box).  It is
bound by VALU issue and latency, not HBM (its tree lives in LDS, its triangles in L2), so the
roofline is VALU issue: peak = 256 CUs x 4 SIMDs x 1/2 wave64 VALU instruction per clock x 2.4 GHz.
achieved = k_trace's VALU wave-instructions per launch / (launch duration x the grid share the launch ran
on): the instructions per k_trace ray come from rocprofv3 SQ_INSTS_VALU of the same kernel sources
(profiles/pmc_<workload>.json, matched by the hash of the library's gfx950 code objects (.hip_fatbin),
i.e. the exact machine code -- null when it differs; the hash of the kernel sources + compile flags is
recorded beside it), the rays per
launch and the launch duration are measured live (device counters, s_memrealtime).  traffic = HBM bytes
per launch from the same profile (FETCH_SIZE x 2, the gfx950 correction of MI355X_MICROARCH.md, +
WRITE_SIZE), scaled to the live rays per launch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# kdpt_trace_iterations keeps `--pipeline` batches in flight on their own HIP streams plus one accumulation
# stream; HIP's default of 4 hardware queues per process would make some of them share a queue (and
# serialise), so ask for 24 (<= 32) before the runtime initialises: the batch streams, the context's, the
# accumulation and torch's, and the queues an RCCL communicator takes (multi-GPU runs) all get their own
# (16 queues under RCCL at 12 batches: 4687 against 5695 Mrays/s, profiles/r03_ab_log.md).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# VALU issue: 256 CUs x 4 SIMD-32 x one wave64 instruction per 2 clocks x 2.4 GHz (MI355X_MICROARCH.md)
VALU_PEAK_GINST = 256 * 4 * 0.5 * 2.4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--spp-per-step", type=int, default=1024,
                    help="weak scaling (default): samples per pixel per GPU in each step's frame")
    ap.add_argument("--total-spp", type=int, default=None,
                    help="strong scaling: samples per pixel of each step's frame, split over the GPUs "
                         "(C4: 256, 32 per GPU on 8)")
    ap.add_argument("--mesh", default="dragon_5")
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--res", type=int, nargs=2, default=(800, 800))
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--bare", action="store_true", help="traverseKDbare instead of the short-stack hybrid")
    ap.add_argument("--bounce-cap", type=int, default=8,
                    help="bounces per iteration (8 = the reference's `depth > 7`; 16 for the C5 stress config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-repeats", type=int, default=3, help="CPU-baseline repeats (median and spread)")
    ap.add_argument("--cpu-iters", type=int, default=8, help="iterations per repeat of the multi-thread CPU leg")
    ap.add_argument("--pipeline", type=int, default=8,
                    help="batches in flight (kdpt_trace_iterations; bit-identical to one at a time)")
    ap.add_argument("--batch", type=int, default=16, help="iterations sharing each intersect launch (<= MAXB = 16)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the process-group path (barriers, the in-timed-region reduce, stat all-reduces) even "
                         "with one rank, e.g. to exercise RCCL on a one-GPU box")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = host-side reduce, for rehearsing the "
                         "N > 1 path with several ranks sharing one GPU")
    ap.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                    help="kdpt_set_tuning knob for A/B runs (not for reported numbers)")
    ap.add_argument("--dump-image", default=None, help="rank 0 saves the sum of the timed frames' reduced float3 "
                    "images here (.npy; tests/test_gpu_sharded.py checks the N > 1 path with it)")
    ap.add_argument("--pmc-profile", default=None, help="profile JSON for the VALU roofline (default: "
                    "profiles/pmc_<scene>_<mesh>_<W>x<H>.json)")
    return ap.parse_args()


def kernel_source_hash() -> str:
    """Kernel sources + device compile flags (the build recipe of the code object)."""
    from kdtreepathtraceroptimization_amd import _build
    return _build.kernel_source_sha()


def code_object_hash() -> str | None:
    """The gfx950 code objects of the library this process loads (KDPT_LIBRARY or the in-tree build)."""
    from kdtreepathtraceroptimization_amd import _build, runtime
    return _build.code_object_sha(runtime.LIB_PATH)


def host_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": omp}


def cpu_baseline(args, threads=None, iters=None):
    """The oracle (plain-C port of the reference path, OpenMP over paths) on this host's cores, on a
    bounded sample of the same workload: `repeats` runs of `iters` consecutive iterations each, median and
    spread reported.  Threads: the CPUs this process may run on, capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box allots 16 host CPUs per GPU and sets it to 16).  `cpu_util` = process
    CPU time / (wall x threads): below 1 the host was shared or the threads stalled, which is how a run-to-run
    drift shows itself."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene
    info = host_info()
    if threads is None:
        threads = info["affinity_cpus"]
        if info["omp_num_threads"]:
            threads = max(1, min(threads, int(info["omp_num_threads"])))
    iters = args.cpu_iters if iters is None else iters
    s = oracle_lib.OracleScene.from_description(
        load_fixture_scene(args.scene, args.mesh, res=tuple(args.res), depth=args.depth))
    runs, utils = [], []
    it = 3
    for _ in range(max(1, args.cpu_repeats)):
        seg, t, c = 0, 0.0, 0.0
        for _ in range(iters):
            t0, c0 = time.perf_counter(), time.process_time()
            _, st = s.render(it, 1, nthreads=threads, shortstack=0 if args.bare else 1, bounce_cap=args.bounce_cap)
            t += time.perf_counter() - t0
            c += time.process_time() - c0
            seg += st.segments
            it += 1
        runs.append(seg / t / 1e6)
        utils.append(c / (t * threads))
    runs_sorted = sorted(runs)
    med = runs_sorted[len(runs) // 2]
    return {"value": round(med, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "repeats": [round(r, 4) for r in runs], "spread": round((max(runs) - min(runs)) / med, 4),
            "cpu_util": [round(u, 3) for u in utils],
            "sample": f"oracle (plain-C restatement of the reference's host-side kernels), median of {len(runs)} "
                      f"repeats of {iters} iteration(s) each (iterations 3..{it - 1}) of the same workload, "
                      f"OpenMP over paths, {threads} thread(s)",
            "host": info}


def valu_roofline(args, W, H, rays_per_launch, launch_ms, share):
    """VALU-issue roofline of one k_trace launch from the committed PMC profile (see module docstring)."""
    path = args.pmc_profile or os.path.join(ROOT, "profiles", f"pmc_{args.scene}_{args.mesh}_{W}x{H}.json")
    out = {"bound": "valu-issue", "unit": "G VALU wave-instructions/s", "peak": VALU_PEAK_GINST,
           "achieved": None, "frac": None, "traffic": None, "kernel": "k_trace",
           "pmc_source": os.path.relpath(path, ROOT)}
    src, cos = kernel_source_hash(), code_object_hash()
    out["kernel_source_sha"], out["code_object_sha"] = src, cos
    if not os.path.exists(path):
        out["note"] = "no PMC profile for this workload"
        return out
    prof = json.load(open(path))
    k = prof.get("kernels", {}).get("k_trace")
    # the profile must have measured this exact machine code: the code objects' hash decides (the
    # source + flags hash is recorded beside it; a comment-only source edit leaves the code objects equal)
    if prof.get("code_object_sha") != cos or not k:
        out["note"] = (f"PMC profile is for code object {prof.get('code_object_sha')} (kernel build "
                       f"{prof.get('kernel_source_sha')}), not {cos} ({src}): stale")
        return out
    out["pmc_kernel_source_sha"] = prof.get("kernel_source_sha")
    inst = k["valu_per_ray"] * rays_per_launch
    eff_s = launch_ms * 1e-3 * share  # the launch ran on `share` of the chip's CUs
    out["achieved"] = round(inst / eff_s / 1e9, 2) if eff_s > 0 else None
    out["frac"] = round(out["achieved"] / VALU_PEAK_GINST, 4) if out["achieved"] else None
    if k.get("hbm_bytes_per_ray") is not None:
        out["traffic"] = round(k["hbm_bytes_per_ray"] * rays_per_launch)
        out["traffic_GBps"] = round(out["traffic"] / (launch_ms * 1e-3) / 1e9, 2) if launch_ms > 0 else None
        out["traffic_hbm_frac"] = round(out["traffic_GBps"] / HBM_PEAK_GBS, 4) if out["traffic_GBps"] else None
    out["valu_inst_per_launch"] = round(inst)
    out["valu_per_ray"] = k["valu_per_ray"]
    out["pmc_exclusive_valu_frac"] = k.get("valu_busy_frac")
    out["pmc_git_head"] = prof.get("git_head")
    return out


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
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene
    from kdtreepathtraceroptimization_amd.distributed import frame_share
    from kdtreepathtraceroptimization_amd.runtime import comm_library, comm_unique_id

    # a step is one frame: weak scaling renders spp-per-step samples per GPU per frame, strong scaling a fixed
    # --total-spp per frame split over the GPUs
    strong = args.total_spp is not None
    F = max(1, args.total_spp if strong else args.spp_per_step * world)  # global iterations per frame
    desc = load_fixture_scene(args.scene, args.mesh, res=tuple(args.res), depth=args.depth)
    sd = SceneData.from_description(desc)
    W, H = sd.resolution
    opt = default_options(testing_mode=1, short_stack=0 if args.bare else 1, bounce_cap=args.bounce_cap)
    from kdtreepathtraceroptimization_amd.runtime import set_process_tuning
    for kv in args.tune:  # "process.NAME": a knob contexts start with (kdpt_set_tuning(NULL, ...))
        name, val = kv.split("=", 1)
        if name.startswith("process."):
            set_process_tuning(name[len("process."):], float(val))
    pt = PathTracer(sd, opt, device=local)
    for kv in args.tune:
        name, val = kv.split("=", 1)
        if not name.startswith("process."):
            pt.set_tuning(name, float(val))
    # the framebuffer reduce: RCCL inside the library (kdpt_comm_init: rank 0's unique id handed out through
    # the process group), or -- gloo rehearsals, ranks sharing a GPU -- each rank's frame shares handed out
    # and reduced here over gloo
    gloo = dist is not None and args.dist_backend == "gloo"
    rccl_lib = None
    if dist is not None:
        if gloo:
            pt.comm_init(world, rank, None)
        else:
            ids = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(ids, src=0)
            pt.comm_init(world, rank, ids[0])
            rccl_lib = comm_library()  # the librccl the library's reduces actually go through

    # warmup: frames disjoint from the timed ones (iteration 2's extra sort lands here)
    shares = torch.empty((args.steps, 3 * W * H), dtype=torch.float32, device=f"cuda:{local}") if gloo else None
    if args.warmup:
        pt.render_frames(0, args.warmup, F, pipeline=args.pipeline, batch=args.batch)
        pt.synchronize()
    # per-segment work counters from one untimed counting iteration of the timed range (informational)
    first_timed, _ = frame_share(args.warmup, F, world, rank)
    aabb, tri, hit = pt.count_iteration(first_timed)
    aabb_prep, cand = pt.count_split()
    cnt_stats = pt.stats()
    pt.reset()  # zero image and totals: the timed frames alone
    st0 = pt.stats()
    image = torch.zeros(3 * W * H, dtype=torch.float32) if gloo and rank == 0 else None
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pt.render_frames(args.warmup, args.steps, F, pipeline=args.pipeline, batch=args.batch,
                     out=shares.data_ptr() if gloo else None)
    pt.synchronize()  # (RCCL: every frame's reduce included)
    if gloo:  # the same per-frame reduce over gloo, rank 0 adding the frames in order
        for k in range(args.steps):
            host = shares[k].cpu()
            dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                image += host
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st1 = pt.stats()
    seg = st1.total_segments - st0.total_segments
    rays = st1.total_trace_rays - st0.total_trace_rays  # handed to k_trace
    kernel_ms = st1.intersect_device_ms_total - st0.intersect_device_ms_total  # device clock, per launch
    launches = st1.intersect_device_launches_total - st0.intersect_device_launches_total
    # the same launches timed by the HIP events the library records around each one on its own stream
    # (testing_mode): dispatch to end, as rocprofv3's kernel trace times them
    ev_ms = st1.intersect_ms_total - st0.intersect_ms_total
    ev_n = st1.intersect_launches_total - st0.intersect_launches_total
    if dist:
        dev = f"cuda:{local}" if args.dist_backend == "nccl" else "cpu"
        t = torch.tensor([dt, float(seg), float(rays), kernel_ms, float(launches), ev_ms, float(ev_n)],
                         dtype=torch.float64, device=dev)
        tmax = t[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt = float(tmax[0])
        seg, rays, kernel_ms, launches = int(tsum[0]), int(tsum[1]), float(tsum[2]), int(tsum[3])
        ev_ms, ev_n = float(tsum[4]), int(tsum[5])
    if rank == 0 and args.dump_image:
        import numpy as np
        np.save(args.dump_image, image.numpy() if gloo else pt.image().reshape(-1))
    if rank != 0:
        pt.close()
        if dist:
            dist.destroy_process_group()
        return
    iters = args.steps * F
    avg_launch_ms = kernel_ms / max(1, launches)
    rays_per_launch = rays / max(1, launches)
    share = pt.trace_grid_share()
    roof = valu_roofline(args, W, H, rays_per_launch, avg_launch_ms, share)
    count_seg = max(1, sum(cnt_stats.seg_per_bounce[d] for d in range(32)))
    alg_bytes = 76 * cand + 52 * (aabb - aabb_prep) + 36 * tri + 40 * hit  # SURVEY 8(d) model, k_trace's part
    roof.update({
        "launch_grid_share": round(share, 4), "avg_launch_ms": round(avg_launch_ms, 5), "launches": launches,
        "avg_launch_ms_hip_events": round(ev_ms / ev_n, 5) if ev_n else None,
        "rays_per_launch": round(rays_per_launch, 1),
        "k_trace_ms_per_step": round(kernel_ms / max(1, args.steps * world), 4),
        "k_trace_busy_share": round(kernel_ms * share / (dt * 1e3 * world), 4),
        # every k_trace instruction of the timed region over its wall time and the whole chip: a lower bound on
        # the kernel's issue rate that does not depend on launch spans (with more launches in flight than grid
        # shares, busy share > 1, a launch's span includes waiting for CUs the other launches hold)
        "chip_wide_achieved": (round(roof["valu_per_ray"] * rays / (dt * world) / 1e9, 2)
                               if roof.get("valu_per_ray") else None),
        "chip_wide_frac": (round(roof["valu_per_ray"] * rays / (dt * world) / 1e9 / VALU_PEAK_GINST, 4)
                           if roof.get("valu_per_ray") else None),
        "algorithmic": {"bytes_per_ray": round(alg_bytes / max(1, cand), 1),
                        "GBps_per_launch": round(alg_bytes / max(1, cand) * rays_per_launch / (avg_launch_ms * 1e-3)
                                                 / 1e9, 1) if avg_launch_ms > 0 else None,
                        "note": "SURVEY 8(d) byte model of k_trace's work; most of these bytes are LDS/L2 hits, "
                                "so it is not an HBM rate"},
        "per_segment_counts": {"aabb": round(aabb / count_seg, 4), "tri": round(tri / count_seg, 4),
                               "hit": round(hit / count_seg, 5), "aabb_before_k_trace": round(aabb_prep / count_seg, 4),
                               "k_trace_share": round(cand / count_seg, 4)},
    })
    per_gpu = F / world
    out = {
        "metric": METRIC,
        "value": round(seg / dt / 1e6, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic camera rays over the reference's own scene assets ({args.scene}.txt + {args.mesh}.obj, "
                "parsed fixtures under tests/golden); deterministic RNG seeded by global iteration",
        "config": {"workload": f"{args.scene}.txt + {args.mesh}.obj, {W}x{H}, depth {args.depth}, "
                               f"bounce cap {args.bounce_cap}, one {F}-spp frame per step"
                               + (f" ({per_gpu:g} spp per GPU)" if world > 1 else "")
                               + f", {args.pipeline} x {args.batch} iterations in flight, "
                               + ("short-stack hybrid KD traversal" if not args.bare else "bare traversal"),
                   "scene": args.scene, "mesh": args.mesh, "resolution": [W, H], "depth": args.depth,
                   "bounce_cap": args.bounce_cap, "spp_per_frame": F, "spp_per_gpu_per_frame": per_gpu,
                   "kd_nodes": sd.view.num_nodes, "kd_tri_refs": sd.view.num_tris,
                   "intersect": {**pt.trace_config(), "create_ms": round(pt.stats().create_ms, 2),
                                 "mask_build_ms": round(pt.stats().mask_build_ms, 2)},
                   **({"tuning": args.tune} if args.tune else {}),
                   "parallelism": (f"spp-sharded x{world}, one framebuffer reduce per frame: "
                                   + ("RCCL ncclReduce inside libkdpt (kdpt_render_frames)"
                                      if args.dist_backend == "nccl" else "gloo host reduce (ranks sharing GPUs)"))
                   if world > 1 else ("single GPU, one-rank RCCL communicator: ncclReduce per frame inside libkdpt"
                                      if dist is not None and not gloo else "single GPU"),
                   **({"rccl_library": rccl_lib} if rccl_lib else {})},
        "ms_per_iteration": round(dt * 1e3 * world / iters, 4),
        "segments_per_iteration": round(seg / iters, 1),
        "primary_rays_per_s": round(W * H * iters / dt, 1),
        "roofline": roof,
        "reference_980m_intersect_ms_per_iter": 79.4,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
        # SURVEY 8(d) / BASELINE.md 3: the same oracle on one core as well
        out["cpu_baseline_1core"] = cpu_baseline(args, threads=1, iters=1)
    pt.close()
    if dist:
        dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
