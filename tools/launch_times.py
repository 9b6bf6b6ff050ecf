"""A few iterations one at a time (for rocprofv3 --kernel-trace): per-bounce intersect launch durations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from kdtreepathtraceroptimization_amd import PathTracer, SceneData, default_options, load_fixture_scene  # noqa: E402

mesh = sys.argv[1] if len(sys.argv) > 1 else "dragon_5"
sd = SceneData.from_description(load_fixture_scene("cornell", mesh, res=(800, 800), depth=8))
with PathTracer(sd, default_options(testing_mode=1)) as pt:
    for it in range(1, 6):
        pt.trace_iteration(it)
        st = pt.stats()
        print(it, round(st.ms_intersect, 3), [st.seg_per_bounce[d] for d in range(st.bounces)], flush=True)
