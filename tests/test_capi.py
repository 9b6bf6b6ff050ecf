"""The C-ABI library loads and exports exactly what include/kdpt.h declares (no GPU needed)."""
import ctypes
import os
import re
import subprocess

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "kdpt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kdpt_[a-z_0-9]+)\s*\(", src)))


def test_every_declared_symbol_is_exported(kdpt):
    names = _declared()
    assert len(names) >= 20
    lib = kdpt.load_library()
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", kdpt.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n
    assert set(names) == set(kdpt.EXPORTS)


def test_struct_layouts(kdpt):
    C = ctypes
    assert C.sizeof(kdpt.Geom) == 236 and C.sizeof(kdpt.Material) == 56 and C.sizeof(kdpt.Camera) == 84
    assert C.sizeof(kdpt.NodeBare) == 64 and C.sizeof(kdpt.TriBare) == 76 and C.sizeof(kdpt.PathSegment) == 56
    assert kdpt.PathSegment.materialIdHit.offset == 52 and kdpt.PathSegment.sdepth.offset == 28
    assert kdpt.NodeBare.triIdSize.offset == 52 and kdpt.TriBare.mtlIdx.offset == 72
    assert kdpt.Geom.invTranspose.offset == 172 and kdpt.Camera.pixelLength.offset == 76


def test_default_options_match_reference_flags(kdpt):
    o = kdpt.default_options()  # src/main.cpp:35-60
    assert (o.focal_length, o.dof_angle, o.softness) == (6.0, 0.0, 0.0)
    assert (o.cacherays, o.antialias, o.enable_sss, o.testing_mode) == (0, 1, 0, 0)
    assert (o.compaction, o.enable_kd, o.viz_kd, o.use_bbox, o.short_stack) == (1, 1, 0, 0, 1)
    assert o.bounce_cap == 8


def test_gfx950_code_object_present(kdpt):
    blob = open(kdpt.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_errors_are_codes_not_exits(kdpt):
    lib = kdpt.load_library()
    h = ctypes.c_void_p()
    rc = lib.kdpt_scene_load(b"/nonexistent/scene.txt", None, 0, 0, 0, ctypes.byref(h))
    assert rc != 0
    assert lib.kdpt_create(None, None, 0, ctypes.byref(h)) != 0
    assert b"null" in lib.kdpt_last_error()
