"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Bar: bit-exact images (the path is float32 throughout and every op is restated in
reference order), exact segment counts, and at the 800x800 configs the survey's own
anchors plus size-independent properties.  The soft-lobe and fake-SSS branches call glibc
acosf / double cos / double sin; those are restated for gfx950 (kdpt_math.h) and proved equal
to glibc on every argument the reference can pass (digests below), so they are bit-exact too.
"""
import json
import os

import numpy as np
import pytest

from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene
from kdtreepathtraceroptimization_amd.runtime import imgsum

pytestmark = pytest.mark.gpu


def _pt(kdpt, desc, **opts):
    return kdpt.PathTracer(kdpt.SceneData.from_description(desc), kdpt.default_options(**opts), device=0)


def _gpu_render(kdpt, desc, iters, **opts):
    with _pt(kdpt, desc, **opts) as pt:
        segs = []
        for it in iters:
            pt.trace_iteration(it)
            segs.append(pt.stats().segments)
        return pt.image(), segs


_ORC_KEYS = {"short_stack": "shortstack", "compaction": "compaction", "antialias": "antialias",
             "dof_angle": "dofAngle", "focal_length": "focalLength", "softness": "softness",
             "enable_sss": "enableSss", "bounce_cap": "bounce_cap", "cacherays": "cacherays"}


def test_device_sincos_equals_glibc(kdpt, oracle):
    rs = np.random.RandomState(1)
    x = np.concatenate([rs.uniform(0, 2 * np.pi, 1 << 20), rs.uniform(-130, 130, 1 << 18),
                        rs.uniform(-1e6, 1e6, 1 << 16), np.array([0, -0.0, 1e-30, 3.1415927, 120.0, 1e30])]
                       ).astype(np.float32)
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib = kdpt.load_library()
    fp = lambda a: a.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_float))  # noqa: E731
    assert lib.kdpt_selftest_math(fp(x), len(x), fp(s), fp(c)) == 0
    rs_, rc_ = oracle.sincos(x)
    assert np.array_equal(s.view(np.uint32), rs_.view(np.uint32))
    assert np.array_equal(c.view(np.uint32), rc_.view(np.uint32))


@pytest.mark.parametrize("fn,first,count", [
    (0, 0, 1 << 32),                       # acosf: every float bit pattern
    (1, 0, 0x41000000), (1, 0x80000000, 0x41000000),  # sin((double)x), every float with |x| < 8
    (2, 0, 0x41000000), (2, 0x80000000, 0x41000000),  # cos((double)x)
], ids=["acosf_all", "sin_pos", "sin_neg", "cos_pos", "cos_neg"])
def test_device_libm_digest_equals_glibc(kdpt, oracle, fn, first, count):
    """gfx950 restatements of glibc acosf / sin / cos vs the host's libm.so.6, as order-independent
    digests over every argument of the set (src/interactions.h:67-83: theta < 2 pi, phi <= pi)."""
    d = kdpt.C.c_ulonglong(0)
    assert kdpt.load_library().kdpt_selftest_libm_digest(fn, first, count, kdpt.C.byref(d)) == 0
    assert d.value == oracle.libm_digest(fn, first, count)


def test_device_libm_samples_equal_glibc(kdpt, oracle):
    """Element-wise on the arguments the scatter actually forms (2 pi u, acosf(pi u angle - 1) and
    dot products in [-1, 1]), including |x| > 1 and NaN for acosf."""
    rs = np.random.RandomState(4)
    u = rs.uniform(0, 1, 1 << 18).astype(np.float32)
    pi = np.float32(np.pi)
    theta = (np.float32(2) * pi * u).astype(np.float32)
    acos_in = np.concatenate([(np.float32(0.02) * pi * u - np.float32(1)).astype(np.float32),
                              rs.uniform(-1, 1, 1 << 18).astype(np.float32),
                              np.array([1, -1, 1.0000001, -1.0000001, np.nan, 0, -0.0, 0.5, -0.5], np.float32)])
    lib = kdpt.load_library()
    fp = lambda a: a.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_float))  # noqa: E731
    for fn, x in ((0, acos_in), (1, theta), (2, theta)):
        out = np.empty(len(x), np.float64)
        assert lib.kdpt_selftest_libm(fn, fp(x), len(x), out.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_double))) == 0
        assert np.array_equal(out.view(np.uint64), oracle.libm(fn, x).view(np.uint64)), fn


def test_device_rng_equals_oracle(kdpt, oracle):
    rs = np.random.RandomState(2)
    iid = np.stack([rs.randint(1, 10000, 50000), rs.randint(0, 2 ** 22, 50000), rs.randint(0, 16, 50000)], 1)
    iid = np.ascontiguousarray(iid.astype(np.int32))
    lib = kdpt.load_library()
    for k in (0, 1, 7):
        u = np.empty(len(iid), np.float32)
        assert lib.kdpt_selftest_rng(iid.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_int)), len(iid), k,
                                     u.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_float))) == 0
        assert np.array_equal(u, oracle.u01(iid, k))


@pytest.mark.parametrize("ior", [1.52, 1.5, 1.0 / 1.52])
def test_device_fresnel_equals_glibc_pow(kdpt, oracle, ior):
    c = np.random.RandomState(3).uniform(-1, 1, 1 << 20).astype(np.float32)
    f = np.empty_like(c)
    lib = kdpt.load_library()
    fp = lambda a: a.ctypes.data_as(kdpt.C.POINTER(kdpt.C.c_float))  # noqa: E731
    assert lib.kdpt_selftest_fresnel(fp(c), len(c), float(np.float32(ior)), fp(f)) == 0
    assert np.array_equal(f, oracle.fresnel(c, ior))


@pytest.mark.parametrize("row", range(4))
def test_survey_anchor_rows_on_gpu(kdpt, anchors, row):
    a = anchors["survey_anchor_table"][row]
    desc = load_fixture_scene(a["scene"], a["mesh"], res=a["res"], depth=a["depth"])
    img, segs = _gpu_render(kdpt, desc, range(a["iters"][0], a["iters"][1] + 1))
    assert sum(segs) == a["segments"]
    assert round(imgsum(img), 6) == a["imgsum"]


CASES = [
    # (id, scene, mesh, res, depth, iters, opts)
    ("c1_64_d2", "cornell", None, (64, 64), 2, [1], {}),
    ("sphere_128_it1-4", "cornell", "sphere_low_1", (128, 128), 8, [1, 2, 3, 4], {}),
    ("dragon_128_it1-3", "cornell", "dragon_5", (128, 128), 8, [1, 2, 3], {}),
    ("dragon_96_bare", "cornell", "dragon_5", (96, 96), 8, [1, 2], {"short_stack": 0}),
    ("dragon_96_noaa", "cornell", "dragon_5", (96, 80), 8, [5], {"antialias": 0}),
    ("dragon_64_nocompact", "cornell", "dragon_5", (64, 64), 8, [1, 3], {"compaction": 0}),
    ("dragon_64_dof", "cornell", "dragon_5", (64, 64), 8, [4], {"dof_angle": 0.03}),
    ("sphere_64_cacherays", "cornell", "sphere_low_1", (64, 64), 8, [1, 3], {"cacherays": 1}),
    ("cornell8_dragon_128", "cornell8", "dragon_5", (128, 128), 8, [1, 2], {}),
    ("sphere_64_depth16_cap16", "cornell", "sphere_low_1", (64, 64), 16, [1, 2], {"bounce_cap": 16}),
    ("ragged_1x1", "cornell", "dragon_5", (1, 1), 8, [1, 2, 3], {}),
    ("ragged_257x3", "cornell", "sphere_low_1", (257, 3), 8, [1, 2], {}),
    # fake-SSS scatter (transmittance > 0, src/interactions.h:195-230) with DEFAULT flags: the reference's
    # own SSS scene and mesh (scenes/cornellout_bunny.txt, stanford_bunny.obj/.mtl Tf 1.0 0.7 0.7)
    ("bunny_sss_scatter_128", "cornellout_bunny", "stanford_bunny", (128, 128), 8, [1, 2, 3], {}),
    # ... with the SSS shading term on (enable_sss, src/pathtrace.cu:2334-2345)
    ("bunny_enable_sss_128", "cornellout_bunny", "stanford_bunny", (128, 128), 8, [1, 2], {"enable_sss": 1}),
    # two materials: the SSS bunny inside the cornell box with its mirror (REFL 1) material, soft lobes on
    ("cornell_bunny_soft_sss_96", "cornell", "stanford_bunny", (96, 96), 8, [1, 2], {"softness": 0.5,
                                                                                    "enable_sss": 1}),
    # soft reflection / refraction lobes (softness > 0): glass sphere, dragon
    ("sphere_soft_128", "cornell", "sphere_low_1", (128, 128), 8, [1, 2], {"softness": 0.5}),
    ("dragon_soft_96", "cornell", "dragon_5", (96, 96), 8, [1, 3], {"softness": 0.5}),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_bit_exact_vs_oracle(kdpt, oracle, case):
    _, scene, mesh, res, depth, iters, opts = case
    desc = load_fixture_scene(scene, mesh, res=res, depth=depth)
    g_img, g_segs = _gpu_render(kdpt, desc, iters, **opts)
    s = oracle.OracleScene.from_description(desc)
    o = {_ORC_KEYS[k]: v for k, v in opts.items()}
    o_img, o_segs = None, []
    for it in iters:  # one image add per pixel per iteration, so float32 accumulation here is exact
        im, st = s.render(it, 1, **o)
        o_segs.append(st.segments)
        o_img = im if o_img is None else (o_img + im)
    assert g_segs == o_segs
    assert np.array_equal(g_img.view(np.uint32), o_img.view(np.uint32)), \
        f"{int(np.sum(g_img != o_img))} values differ, max |d| = {float(np.abs(g_img - o_img).max())}"


@pytest.mark.parametrize("stop_depth", [0, 1, 4])
def test_path_state_after_each_bounce(kdpt, oracle, stop_depth):
    """PathSegment arrays (reference layout) after bounce d: same order (stable compaction), same bits."""
    desc = load_fixture_scene("cornell", "dragon_5", res=(96, 96), depth=8)
    with _pt(kdpt, desc) as pt:
        g = pt.debug_paths(3, stop_depth)
    o = oracle.OracleScene.from_description(desc).paths_after(3, stop_depth)
    assert len(g) == len(o)
    for f in ("origin", "direction", "color", "pixelIndex", "remainingBounces", "materialIdHit", "isinside"):
        assert np.array_equal(g[f], o[f]), f


@pytest.mark.parametrize("res", [(96, 96), (800, 800)])
def test_fused_shading_equals_scan_scatter(kdpt, oracle, res):
    """k_shade_fused (single-pass decoupled look-back compaction) and k_shade + k_scan + k_scatter
    (kdpt_set_tuning "shade_fused" = 0) give the same images and path arrays; the small size also against the oracle.
    800x800 has 2500 tiles per bounce, so most tiles find their offset through other tiles' counts."""
    desc = load_fixture_scene("cornell", "dragon_5", res=res, depth=8)
    out = {}
    for fused in ("1", "0"):
        with _pt(kdpt, desc) as pt:
            pt.set_tuning("shade_fused", int(fused))
            paths = pt.debug_paths(3, 2)
            pt.reset()
            for it in (1, 3, 4):
                pt.trace_iteration(it)
            out[fused] = (paths, pt.image().copy())
    for f in ("origin", "direction", "color", "pixelIndex", "remainingBounces", "materialIdHit", "isinside"):
        assert np.array_equal(out["1"][0][f], out["0"][0][f]), f
    assert np.array_equal(out["1"][1].view(np.uint32), out["0"][1].view(np.uint32))
    if res == (96, 96):
        o = oracle.OracleScene.from_description(desc).paths_after(3, 2)
        assert np.array_equal(out["1"][0]["pixelIndex"], o["pixelIndex"])


def test_iteration2_sort_order(kdpt, oracle):
    """Iteration 2 stable-sorts the live paths by materialIdHit after compaction (src/pathtrace.cu:2600-2606)."""
    desc = load_fixture_scene("cornell", "sphere_low_1", res=(80, 80), depth=8)
    with _pt(kdpt, desc) as pt:
        g = pt.debug_paths(2, 0)
    o = oracle.OracleScene.from_description(desc).paths_after(2, 0)
    assert np.all(np.diff(g["materialIdHit"]) >= 0)
    assert np.array_equal(g["pixelIndex"], o["pixelIndex"])


def test_full_size_properties_dragon(kdpt):
    """800x800 (the benchmark config): determinism, accumulation linearity, monotone live counts."""
    desc = load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8)
    with _pt(kdpt, desc) as pt:
        pt.trace_iteration(7)
        a = pt.image().copy()
        st = pt.stats()
        pb = [st.seg_per_bounce[d] for d in range(st.bounces)]
        assert all(x >= y for x, y in zip(pb, pb[1:])) and pb[0] == 640000
        pt.trace_iteration(8)
        ab = pt.image().copy()
        pt.reset()
        pt.trace_iteration(8)
        b = pt.image().copy()
        pt.reset()
        pt.trace_iteration(7)
        assert np.array_equal(pt.image(), a)
    assert np.isfinite(ab).all() and (ab >= 0).all()
    assert np.array_equal(ab, (a + b).astype(np.float32))


def test_counters_match_oracle(kdpt, oracle):
    desc = load_fixture_scene("cornell", "dragon_5", res=(128, 128), depth=8)
    with _pt(kdpt, desc) as pt:
        aabb, tri, hit = pt.count_iteration(1)
    _, st = oracle.OracleScene.from_description(desc).render(1, 1)
    assert (aabb, tri, hit) == (st.aabb_tests, st.tri_tests, st.tri_hits)


def test_pbo_matches_send_image_to_pbo(kdpt):
    desc = load_fixture_scene("cornell", "sphere_low_1", res=(32, 24), depth=8)
    with _pt(kdpt, desc) as pt:
        for it in (1, 2, 3):
            pt.trace_iteration(it)
        img, pbo = pt.image(), pt.pbo(3)
    exp = np.clip(((img / np.float32(3)).astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    assert np.array_equal(pbo[..., :3], exp.astype(np.uint8)) and (pbo[..., 3] == 0).all()


def test_pbo_into_device_memory(kdpt):
    """The reference's pbo is the GL-mapped device buffer: kdpt_write_pbo writes device memory directly (the
    drop-in shim passes it through) and gives the same bytes as the host-memory form."""
    import ctypes as C
    import torch
    desc = load_fixture_scene("cornell", "sphere_low_1", res=(32, 24), depth=8)
    with _pt(kdpt, desc) as pt:
        for it in (1, 2):
            pt.trace_iteration(it)
        host = pt.pbo(2)
        dev = torch.full((24, 32, 4), 7, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        rc = pt.lib.kdpt_write_pbo(pt._ctx, 2, C.cast(C.c_void_p(dev.data_ptr()), C.POINTER(C.c_uint8)))
        assert rc == 0
        assert np.array_equal(dev.cpu().numpy(), host)


@pytest.mark.parametrize("pipeline,batch", [(1, 1), (3, 1), (2, 3), (1, 4), (8, 4), (5, 2), (12, 4), (3, 8), (8, 8), (2, 5),
                                            (2, 16), (8, 16), (3, 13)])
def test_pipelined_iterations_bit_exact(kdpt, pipeline, batch):
    """kdpt_trace_iterations (batches sharing intersect launches, several batches in flight, partial
    images added in order) gives the same image bits and segment counts as one kdpt_trace_iteration
    after another."""
    desc = load_fixture_scene("cornell", "dragon_5", res=(96, 80), depth=8)
    sd = kdpt.SceneData.from_description(desc)
    seq = kdpt.PathTracer(sd, kdpt.default_options())
    n_it = max(7, pipeline * batch + 3)  # enough to wrap around every slot group
    for it in range(1, n_it + 1):
        seq.trace_iteration(it)
    img_seq = seq.image()
    tot_seq = seq.stats().total_segments
    seq.close()
    pip = kdpt.PathTracer(sd, kdpt.default_options())
    pip.trace_iterations(1, n_it, pipeline=pipeline, batch=batch)
    pip.synchronize()
    img_pip = pip.image()
    tot_pip = pip.stats().total_segments
    pip.close()
    assert tot_pip == tot_seq
    assert np.array_equal(img_pip.view(np.uint32), img_seq.view(np.uint32))


@pytest.mark.gpu
def test_entry_points_order_after_pipelined_accumulation(kdpt):
    """kdpt_trace_iterations returns with partial images still being added on its accumulation stream;
    a following kdpt_trace_iteration (gather into the image on the context's stream) and kdpt_write_pbo
    must see every earlier addition without an explicit kdpt_synchronize in between."""
    desc = load_fixture_scene("cornell", "dragon_5", res=(96, 80), depth=8)
    sd = kdpt.SceneData.from_description(desc)
    with kdpt.PathTracer(sd, kdpt.default_options()) as seq:
        for it in range(1, 18):
            seq.trace_iteration(it)
        img_seq, pbo_seq = seq.image(), seq.pbo(17)
    with kdpt.PathTracer(sd, kdpt.default_options()) as pip:
        pip.trace_iterations(1, 16, pipeline=4, batch=4)
        pip.trace_iteration(17)  # no synchronize before it
        pbo = pip.pbo(17)
        img = pip.image()
    assert np.array_equal(img.view(np.uint32), img_seq.view(np.uint32))
    assert np.array_equal(pbo, pbo_seq)


@pytest.mark.gpu
def test_tuning_knobs_keep_parity(kdpt):
    """Every kdpt_set_tuning route gives the default route's bits (the knobs change scheduling only);
    unknown names are refused."""
    desc = load_fixture_scene("cornell", "dragon_5", res=(96, 80), depth=8)
    sd = kdpt.SceneData.from_description(desc)
    with kdpt.PathTracer(sd, kdpt.default_options()) as pt:
        pt.trace_iterations(1, 8, pipeline=2, batch=4)
        pt.synchronize()
        ref = pt.image().copy()
        with pytest.raises(kdpt.KdptError):
            pt.set_tuning("no_such_knob", 1)
    for name, val in (("tree_global", 1), ("tree_format", 32), ("tree_format", 16), ("early_walk", 0), ("early_leaf", 65), ("chunk_width0", 64),
                      ("chunk_width1", 8), ("trace_grid_frac", 0.1), ("shade_fused", 0), ("shade_batch", 0),
                      ("gen_geoms", 0), ("cluster_cull", 0), ("cull_margin", 1e-3), ("cluster_obb", 0),
                      ("super_slab", 0), ("flat_obb", 0), ("cull_exact", 0), ("cull_mask_n", 8),
                      ("cull_mask_n", 2), ("cull_mask_n", 32), ("cull_fast_k", 1e-4), ("cull_fast_k", 1e-2)):
        with kdpt.PathTracer(sd, kdpt.default_options()) as pt:
            pt.set_tuning(name, val)
            pt.trace_iterations(1, 8, pipeline=2, batch=4)
            pt.synchronize()
            assert np.array_equal(pt.image().view(np.uint32), ref.view(np.uint32)), name


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,res,depth,cap,iters,knobs", [("dragon_5", (800, 800), 8, 8, 16, {}),
                                                            ("dragon_5", (800, 800), 8, 8, 8,
                                                             {"cull_mask_n": 32, "cull_fast_k": 1e-4}),
                                                            ("icosphere_8", (1600, 1600), 16, 16, 2, {})],
                         ids=["c3", "c3-masks32-k1e-4", "c5"])
def test_cluster_cull_equals_no_cull_at_scale(kdpt, mesh, res, depth, cap, iters, knobs):
    """The cluster cull (default margin) against no cull at all (tuning cluster_cull = 0: every cluster of
    every visited big leaf swept, the reference's semantics by construction) on the headline workloads at
    full size: C3 (dragon_5, 800^2, 16 iterations, ~40 M segments) and C5 (the 1.31 M-triangle icosphere,
    1600^2, cap 16, 2 iterations, ~24 M segments).  Every ray of these renders is a differential case of the
    cull: the images and segment counts must be bit-equal.  Both culls are exact by construction: C5's by its
    rigorous margin, dragon_5's -- whose triangles are too large for a rigorous margin that still culls -- by
    the masked one-level cull (kdpt_clusters.h build_dir_masks)."""
    desc = load_fixture_scene("cornell", mesh, res=res, depth=depth)
    sd = kdpt.SceneData.from_description(desc)
    imgs, segs, info = [], [], None
    for cull in (1, 0):
        with kdpt.PathTracer(sd, kdpt.default_options(bounce_cap=cap)) as pt:
            for k, v in knobs.items():  # (the masked cull at round 5's first resolution and box coefficient)
                pt.set_tuning(k, v)
            if info is None:
                info = pt.cull_margin()
            pt.set_tuning("cluster_cull", cull)
            pt.trace_iterations(1, iters, pipeline=2, batch=2)
            pt.synchronize()
            imgs.append(pt.image())
            segs.append(pt.stats().total_segments)
    # exact for both: C5 by its rigorous margin, dragon_5 by the direction masks (kdpt_clusters.h build_dir_masks)
    assert info["cull_exact"], info
    assert segs[0] == segs[1]
    assert np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))


@pytest.mark.parametrize("mesh,level,knobs,want", [("dragon_5", None, {"tree_format": 16}, "lds-16B-derived"),
                                                   (None, 6, {}, "lds-16B-derived"),
                                                   (None, 7, {}, "lds-16B-derived+hbm-clusters"),
                                                   (None, 7, {"cull_exact": 0}, "lds-16B-derived+supers"),
                                                   (None, 7, {"cull_exact": 0, "cluster_slab": 0},
                                                    "lds-16B-derived+supers"),
                                                   (None, 7, {"super_cull": 0}, "lds-16B-derived+hbm-clusters")])
def test_derived_box_tree_in_lds(kdpt, oracle, mesh, level, knobs, want):
    """The 16-byte NodesDerived records (boxes derived on the walk): the default LDS route for trees whose
    32-byte copy does not fit (the icosphere's big leaves: its cluster boxes then stay in HBM, culled in one
    level -- the masked exact cull, level 7's triangles being too large for a rigorous margin -- or, with
    cull_exact 0, in two levels under super-cluster boxes kept in LDS, with or without the clusters' normal
    slabs), and on request
    (tree_format 16) for the reference's meshes.  Images equal the oracle's and the 32-byte / HBM route's bit
    for bit."""
    from kdtreepathtraceroptimization_amd.meshes import attach_icosphere
    desc = load_fixture_scene("cornell", mesh, res=(64, 48), depth=8)
    if level is not None:
        desc = attach_icosphere(desc, level)
    sd = kdpt.SceneData.from_description(desc)
    imgs = {}
    for f in ("knobs", 32):
        with kdpt.PathTracer(sd, kdpt.default_options()) as pt:
            for k, v in (knobs.items() if f == "knobs" else (("tree_format", 32),)):
                pt.set_tuning(k, v)
            cfg = pt.trace_config()
            if f == "knobs":
                assert cfg["tree"] == want, cfg
            for it in (1, 2, 3):
                pt.trace_iteration(it)
            imgs[f] = pt.image()
    ref, _ = oracle.OracleScene.from_description(desc).render(1, 3)
    for f, im in imgs.items():
        assert np.array_equal(im.view(np.uint32), ref.view(np.uint32)), f


def test_process_knobs_keep_parity(kdpt):
    """The process-wide knobs (kdpt_set_tuning(NULL, ...): defaults of contexts created afterwards) change the
    cluster layout and the stream kind only: plain streams instead of CU-masked ones, Morton-run clusters or
    normal cones of another chord give the default route's bits -- on the C5 mesh family (icosphere_8, whose
    margin is rigorous, so its default is normal cones) and on dragon_5 with pipelined iterations."""
    from kdtreepathtraceroptimization_amd.runtime import set_process_tuning
    cases = [("icosphere_8", (48, 40), 16, 16), ("dragon_5", (96, 80), 8, 8)]
    try:
        for mesh, res, depth, cap in cases:
            sd = kdpt.SceneData.from_description(load_fixture_scene("cornell", mesh, res=res, depth=depth))
            imgs = []
            for knobs in ({}, {"cu_mask_streams": 0}, {"cluster_chord": 0}, {"cluster_chord": 0.1}):
                for k, v in knobs.items():
                    set_process_tuning(k, v)
                with kdpt.PathTracer(sd, kdpt.default_options(bounce_cap=cap)) as pt:
                    pt.trace_iterations(1, 8, pipeline=2, batch=4)
                    pt.synchronize()
                    imgs.append(pt.image().copy())
                set_process_tuning("cu_mask_streams", 1)
                set_process_tuning("cluster_chord", -1)
            for k in range(1, len(imgs)):
                assert np.array_equal(imgs[k].view(np.uint32), imgs[0].view(np.uint32)), (mesh, k)
    finally:
        set_process_tuning("cu_mask_streams", 1)
        set_process_tuning("cluster_chord", -1)
