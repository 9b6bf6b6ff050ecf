"""Parity of the work bench.py actually times.

The driver's command (`bench.py --steps 20 --warmup 5`, C3: cornell + dragon_5, 800x800, depth 8) renders frames
of 1 024 global iterations with 8 batches of 16 in flight; its timed frames start at frame 5 = iterations
5 121 - 6 144.  Here:

- that whole frame, rendered through kdpt_render_frames with the bench's pipeline shape, is bit-equal with the
  default (masked, exact) cluster cull and with no cull at all (cluster_cull = 0, the reference's
  semantics by construction);
- four of its iterations, traced alone, are bit-equal to the oracle run live on this host;
- C3 seen from four other eye positions around the orbit camera's look-at point (the zoom / phi / theta
  camera runCuda recomputes, src/main.cpp:1111-1129, which the mouse moves, :1317-1324), iterations 1-3 at
  256x256, is bit-equal to the oracle: the cull's exactness must not depend on which lines the camera makes.
"""
import numpy as np
import pytest

from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene

pytestmark = pytest.mark.gpu

FRAME, SPP = 5, 1024  # bench.py's first timed frame at --warmup 5
TIMED = (FRAME * SPP + 1, FRAME * SPP + 300, FRAME * SPP + 777, (FRAME + 1) * SPP)


def test_timed_frame_equals_no_cull(kdpt):
    desc = load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8)
    sd = kdpt.SceneData.from_description(desc)
    imgs, segs = [], []
    for cull in (1, 0):
        with kdpt.PathTracer(sd, kdpt.default_options(testing_mode=1), device=0) as pt:
            if cull:
                assert pt.cull_margin()["cull_exact"], pt.cull_margin()
            pt.set_tuning("cluster_cull", cull)
            pt.render_frames(FRAME, 1, SPP, pipeline=8, batch=16)
            pt.synchronize()
            imgs.append(pt.image())
            segs.append(pt.stats().total_segments)
    assert segs[0] == segs[1] and segs[0] > 1000 * 2_400_000, segs
    assert np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32)), \
        f"{int(np.sum(imgs[0] != imgs[1]))} values differ"


def test_timed_iterations_equal_oracle(kdpt, oracle):
    desc = load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8)
    sd = kdpt.SceneData.from_description(desc)
    o = oracle.OracleScene.from_description(desc)
    with kdpt.PathTracer(sd, kdpt.default_options(), device=0) as pt:
        for it in TIMED:
            pt.reset()
            pt.trace_iteration(it)
            got, seg = pt.image(), pt.stats().segments
            ref, st = o.render(it, 1)
            assert seg == st.segments, (it, seg, st.segments)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
                (it, int(np.sum(got != ref)))


# eye positions inside the box, around scenes/cornell.txt's LOOKAT (0, 5, 0): the dragon seen from the
# front left, below, above and behind
EYES = [(3.5, 6.5, 3.5), (-3.0, 2.0, 4.0), (4.0, 8.5, -1.0), (-4.2, 4.0, -3.5)]


@pytest.mark.parametrize("eye", EYES, ids=[f"eye{i}" for i in range(len(EYES))])
def test_orbit_cameras_equal_oracle(kdpt, oracle, eye):
    desc = load_fixture_scene("cornell", "dragon_5", res=(256, 256), depth=8)
    desc.eye = np.array(eye, np.float32)
    sd = kdpt.SceneData.from_description(desc)
    with kdpt.PathTracer(sd, kdpt.default_options(), device=0) as pt:
        assert pt.cull_margin()["cull_exact"]
        for it in (1, 2, 3):
            pt.trace_iteration(it)
        got, seg = pt.image(), pt.stats().total_segments
    ref, st = oracle.OracleScene.from_description(desc).render(1, 3)
    assert seg == st.segments, (seg, st.segments)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), int(np.sum(got != ref))
