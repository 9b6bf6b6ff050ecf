"""The oracle (CPU restatement) against the reference's own pins.

- rnd/houdini/data -> dataout: the reference's only committed known answer (KD builder).
- SURVEY.md 8(c) anchor table: segments and image sums of the reference's kernels run host-side.
- sha256 of NodeBare[]/TriBare[] produced by oracle/_ref (the reference's own builder sources).
"""
import hashlib
import os
import tempfile

import numpy as np
import pytest

from conftest import HAS_REFERENCE, REFERENCE, needs_reference
from kdtreepathtraceroptimization_amd.fixtures import FIXTURE_DIR, load_fixture_scene
from kdtreepathtraceroptimization_amd.runtime import imgsum


def _kat_dump(oracle, maxdepth):
    tris = np.load(os.path.join(FIXTURE_DIR, "houdini_kat_triangles.npy"))
    with tempfile.TemporaryDirectory() as td:
        src, out = os.path.join(td, "data"), os.path.join(td, "out")
        with open(src, "w") as f:
            for v in tris.reshape(-1):
                f.write("%.9g\n" % float(v))
        assert oracle.lib().orc_kd_kat(src.encode(), maxdepth, out.encode()) == 0
        return open(out, "rb").read()


def test_houdini_kat_split30(oracle, anchors):
    dump = _kat_dump(oracle, 30)
    assert hashlib.sha256(dump).hexdigest() == anchors["houdini_kat"]["dataout_sha256_no_cr"]
    assert dump.count(b"\n") == anchors["houdini_kat"]["lines"] == 1071


@needs_reference
def test_houdini_kat_against_reference_file(oracle):
    dump = _kat_dump(oracle, 30)
    ref = open(os.path.join(REFERENCE, "rnd/houdini/dataout"), "rb").read().replace(b"\r", b"")
    assert dump == ref


def test_houdini_kat_split13_differs(oracle):
    # survey probe: split(13) gives 1055 lines, i.e. the KAT really pins the depth
    assert _kat_dump(oracle, 13).count(b"\n") == 1055


@pytest.mark.parametrize("mesh", ["dragon_5", "dragon_1", "dragon_2", "dragon_3", "dragon_4",
                                  *[f"sphere_low_{k}" for k in range(1, 9)]])
def test_oracle_kd_sha256(oracle, anchors, mesh):
    """KD arrays equal to the reference's own builder (oracle/_ref, sha256 in anchors.json)."""
    s = oracle.OracleScene.from_description(load_fixture_scene("cornell", mesh))
    exp = anchors["kd_sha256"][mesh]
    assert s.s.num_nodes == exp["num_nodes"] and s.s.num_tris == exp["num_tris"]
    assert hashlib.sha256(s.nodes_bytes()).hexdigest() == exp["nodes"]
    assert hashlib.sha256(s.tris_bytes()).hexdigest() == exp["tris"]
    if mesh not in anchors["survey_kd_sha256_prefix_suffix"]:
        return
    pre = anchors["survey_kd_sha256_prefix_suffix"][mesh]
    assert exp["nodes"].startswith(pre["nodes"][0]) and exp["nodes"].endswith(pre["nodes"][1])
    assert exp["tris"].startswith(pre["tris"][0]) and exp["tris"].endswith(pre["tris"][1])


@pytest.mark.parametrize("row", range(4))
def test_oracle_reproduces_survey_anchor(oracle, anchors, row):
    a = anchors["survey_anchor_table"][row]
    s = oracle.OracleScene.from_description(load_fixture_scene(a["scene"], a["mesh"], res=a["res"], depth=a["depth"]))
    img, st = s.render(a["iters"][0], a["iters"][1] - a["iters"][0] + 1)
    assert st.segments == a["segments"]
    assert round(imgsum(img), 6) == a["imgsum"]


def test_oracle_survey_counters_dragon(oracle):
    # hybrid 11.74 AABB / 96.64 tri / 0.080 hits per segment on dragon_5 @ 800^2
    s = oracle.OracleScene.from_description(load_fixture_scene("cornell", "dragon_5", res=(800, 800), depth=8))
    _, st = s.render(1, 1)
    assert round(st.aabb_tests / st.segments, 2) == 11.74
    assert round(st.tri_tests / st.segments, 2) == 96.64
    assert round(st.tri_hits / st.segments, 3) == 0.080


def _py_utilhash(a):
    M = 0xFFFFFFFF
    a = ((a + 0x7ed55d16) + (a << 12)) & M
    a = ((a ^ 0xc761c23c) ^ (a >> 19)) & M
    a = ((a + 0x165667b1) + (a << 5)) & M
    a = ((a + 0xd3a2646c) ^ (a << 9)) & M
    a = ((a + 0xfd7046c5) + (a << 3)) & M
    a = ((a ^ 0xb55a4f09) ^ (a >> 16)) & M
    return a


def _py_u01(iter_, index, depth, k):
    h = _py_utilhash((0x80000000 | (depth << 22) | iter_) & 0xFFFFFFFF) ^ _py_utilhash(index & 0xFFFFFFFF)
    x = h % 2147483647 or 1
    for _ in range(k + 1):
        x = (x * 48271) % 2147483647
    return np.float32(np.float32(x - 1) / np.float32(2147483648.0))


def test_rng_known_answers(oracle):
    rs = np.random.RandomState(0)
    for _ in range(300):
        it, idx, d, k = int(rs.randint(1, 5000)), int(rs.randint(0, 2 ** 21)), int(rs.randint(0, 16)), int(rs.randint(0, 8))
        assert np.float32(oracle.lib().orc_u01_sequence(it, idx, d, k)) == _py_u01(it, idx, d, k)
    for a in [0, 1, 2, 12345, 0xFFFFFFFF, 0x80000000]:
        assert oracle.lib().orc_utilhash(a) == _py_utilhash(a)


@needs_reference
@pytest.mark.parametrize("mesh", ["sphere_low_1", "dragon_5"])
def test_oracle_files_equal_fixture(oracle, mesh):
    a = oracle.OracleScene.from_files(os.path.join(REFERENCE, "scenes/cornell.txt"),
                                      os.path.join(REFERENCE, f"scenes/{mesh}.obj"))
    b = oracle.OracleScene.from_description(load_fixture_scene("cornell", mesh))
    for m in ("nodes_bytes", "tris_bytes", "geoms_bytes", "materials_bytes", "camera_bytes"):
        assert getattr(a, m)() == getattr(b, m)(), m


def test_oracle_reproduces_committed_fullsize_pins(oracle):
    """The oracle here reproduces tests/golden/oracle_anchors.json (first iteration of every config), the
    pins the GPU full-size tests compare against (tests/test_gpu_fullsize.py)."""
    import json
    with open(os.path.join(FIXTURE_DIR, "oracle_anchors.json")) as f:
        cfgs = json.load(f)["configs"]
    for c in cfgs:
        s = oracle.OracleScene.from_description(load_fixture_scene(c["scene"], c["mesh"], res=c["res"],
                                                                   depth=c["depth"]))
        rec = c["iterations"][0]
        im, st = s.render(rec["iter"], 1, **c["options"])
        assert st.segments == rec["segments"], c["id"]
        assert hashlib.sha256(im.tobytes()).hexdigest() == rec["sha256"], c["id"]
