"""Record the oracle's full-size per-iteration results as committed pins (tests/golden/oracle_anchors.json).

For each BASELINE config that fits one GPU (C1, C2, C3 and C4's workload at 800x800) the oracle renders
iterations 1..3 one at a time; each single-iteration float32 image is pinned by sha256, segment count and
imgsum, and the in-order float32 sum of the three by its sha256.  The GPU tests render the same
iterations through the C-ABI and compare with these values and with the oracle run live on the GPU box's
host, so a drift of either side (or of the box's libm) shows up as a mismatch against the committed pin.

Run here:  python tests/golden/make_oracle_anchors.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib  # noqa: E402
from kdtreepathtraceroptimization_amd.fixtures import load_fixture_scene  # noqa: E402
from kdtreepathtraceroptimization_amd.runtime import imgsum  # noqa: E402

# (id, scene, mesh, res, depth, options) -- SURVEY.md 8(d) configs as substituted in BASELINE.md
CONFIGS = [
    ("C1", "cornell", None, (64, 64), 2, {}),
    ("C2", "cornell", "sphere_low_1", (800, 800), 8, {}),
    ("C3", "cornell", "dragon_5", (800, 800), 8, {}),
    ("C4w", "cornell8", "dragon_5", (800, 800), 8, {}),
    ("C3_bare", "cornell", "dragon_5", (800, 800), 8, {"shortstack": 0}),
    ("sss_800", "cornellout_bunny", "stanford_bunny", (800, 800), 8, {}),
]
ITERS = [1, 2, 3]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def render(cfg):
    cid, scene, mesh, res, depth, opts = cfg
    s = oracle_lib.OracleScene.from_description(load_fixture_scene(scene, mesh, res=res, depth=depth))
    per, acc = [], None
    for it in ITERS:
        im, st = s.render(it, 1, **opts)
        per.append({"iter": it, "segments": int(st.segments), "sha256": sha(im), "imgsum": round(imgsum(im), 6)})
        acc = im.copy() if acc is None else acc + im
    return {"id": cid, "scene": scene, "mesh": mesh, "res": list(res), "depth": depth, "options": opts,
            "iterations": per, "sum_sha256": sha(acc)}


def main():
    out = {"note": "oracle (oracle/kdpt_oracle.c) single-iteration float32 images, sha256 of the raw bytes "
                   "(H x W x 3, row-major); sum_sha256 = float32 in-order sum of the iterations",
           "configs": [render(c) for c in CONFIGS]}
    with open(os.path.join(HERE, "oracle_anchors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("written", len(out["configs"]), "configs")


if __name__ == "__main__":
    main()
