"""ctypes binding of the C-ABI in include/kdpt.h.

Python here is plumbing (tests, bench, torch.distributed); the path tracer is
the in-tree HIP library ``libkdpt.so``.  There is no CPU fallback: if the
library is missing or cannot open a HIP device every entry point raises.

Mirrors the reference's operator interface (src/pathtrace.h:6-21):
``PathTracer(scene, options)``          ~ pathtraceInit(Scene*, enablekd)
``PathTracer.trace_iteration(iter)``    ~ pathtrace(pbo, frame, iter, ...flags)
``PathTracer.close()``                  ~ pathtraceFree(Scene*, enablekd)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KDPT_LIBRARY") or os.path.join(HERE, "libkdpt.so")

KDPT_OK = 0


class KdptError(RuntimeError):
    pass


# ---------------------------------------------------------------- structs
class Geom(C.Structure):  # struct Geom, src/sceneStructs.h:22-31
    _fields_ = [("type", C.c_int), ("materialid", C.c_int), ("translation", C.c_float * 3),
                ("rotation", C.c_float * 3), ("scale", C.c_float * 3), ("transform", C.c_float * 16),
                ("inverseTransform", C.c_float * 16), ("invTranspose", C.c_float * 16)]


class Material(C.Structure):  # struct Material, src/sceneStructs.h:33-44
    _fields_ = [("color", C.c_float * 3), ("specular_exponent", C.c_float), ("specular_color", C.c_float * 3),
                ("hasReflective", C.c_float), ("hasRefractive", C.c_float), ("indexOfRefraction", C.c_float),
                ("emittance", C.c_float), ("transmittance", C.c_float * 3)]


class Camera(C.Structure):  # struct Camera, src/sceneStructs.h:46-55
    _fields_ = [("resolution", C.c_int * 2), ("position", C.c_float * 3), ("lookAt", C.c_float * 3),
                ("view", C.c_float * 3), ("up", C.c_float * 3), ("right", C.c_float * 3), ("fov", C.c_float * 2),
                ("pixelLength", C.c_float * 2)]


class NodeBare(C.Structure):  # KDN::NodeBare, src/KDnode.h:64-82
    _fields_ = [("axis", C.c_int), ("splitPos", C.c_float), ("mins", C.c_float * 3), ("maxs", C.c_float * 3),
                ("ID", C.c_int), ("parentID", C.c_int), ("leftID", C.c_int), ("rightID", C.c_int),
                ("triIdStart", C.c_int), ("triIdSize", C.c_int), ("tmin", C.c_float), ("tmax", C.c_float)]


class TriBare(C.Structure):  # KDN::TriBare, src/KDnode.h:51-62
    _fields_ = [(n, C.c_float) for n in ("x1", "x2", "x3", "y1", "y2", "y3", "z1", "z2", "z3",
                                          "nx1", "nx2", "nx3", "ny1", "ny2", "ny3", "nz1", "nz2", "nz3")] + [
        ("mtlIdx", C.c_int)]


class PathSegment(C.Structure):  # struct PathSegment, src/sceneStructs.h:65-71
    _fields_ = [("origin", C.c_float * 3), ("direction", C.c_float * 3), ("isinside", C.c_uint8),
                ("pad_", C.c_uint8 * 3), ("sdepth", C.c_float), ("color", C.c_float * 3), ("pixelIndex", C.c_int),
                ("remainingBounces", C.c_int), ("materialIdHit", C.c_int)]


class Scene(C.Structure):
    _fields_ = [("camera", Camera), ("traceDepth", C.c_int), ("geoms", C.POINTER(Geom)), ("num_geoms", C.c_int),
                ("materials", C.POINTER(Material)), ("num_materials", C.c_int), ("has_obj", C.c_int),
                ("nodes", C.POINTER(NodeBare)), ("num_nodes", C.c_int), ("tris", C.POINTER(TriBare)),
                ("num_tris", C.c_int), ("obj_materialOffsets", C.POINTER(C.c_int)), ("num_shapes", C.c_int),
                ("obj_verts", C.POINTER(C.c_float)), ("num_obj_verts", C.c_int), ("obj_norms", C.POINTER(C.c_float)),
                ("num_obj_norms", C.c_int), ("obj_polyoffsets", C.POINTER(C.c_int)),
                ("obj_polysidxflat", C.POINTER(C.c_int)), ("polyidxcount", C.c_int),
                ("obj_bboxes", C.POINTER(C.c_float)), ("num_bbox_floats", C.c_int)]


class Options(C.Structure):
    _fields_ = [("focal_length", C.c_float), ("dof_angle", C.c_float), ("softness", C.c_float),
                ("cacherays", C.c_int), ("antialias", C.c_int), ("enable_sss", C.c_int), ("testing_mode", C.c_int),
                ("compaction", C.c_int), ("enable_kd", C.c_int), ("viz_kd", C.c_int), ("use_bbox", C.c_int),
                ("short_stack", C.c_int), ("bounce_cap", C.c_int), ("block_size", C.c_int),
                ("external_image", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("segments", C.c_longlong), ("seg_per_bounce", C.c_longlong * 32), ("bounces", C.c_int),
                ("iterations", C.c_int), ("ms_last_iteration", C.c_float), ("ms_intersect", C.c_float),
                ("total_segments", C.c_longlong), ("intersect_ms_total", C.c_double),
                ("intersect_launches_total", C.c_longlong), ("intersect_device_ms_total", C.c_double),
                ("intersect_device_launches_total", C.c_longlong), ("intersect_grid_share", C.c_float),
                ("total_trace_rays", C.c_longlong), ("create_ms", C.c_double), ("mask_build_ms", C.c_double)]


class SceneDesc(C.Structure):
    _fields_ = [("res", C.c_int * 2), ("fovy", C.c_float), ("iterations", C.c_int), ("traceDepth", C.c_int),
                ("eye", C.c_float * 3), ("lookAt", C.c_float * 3), ("up", C.c_float * 3),
                ("num_materials", C.c_int), ("materials", C.POINTER(Material)), ("num_geoms", C.c_int),
                ("geom_type", C.POINTER(C.c_int)), ("geom_material", C.POINTER(C.c_int)),
                ("geom_trs", C.POINTER(C.c_float)), ("ntri", C.c_int), ("verts9", C.POINTER(C.c_float)),
                ("norms9", C.POINTER(C.c_float)), ("shape_of_tri", C.POINTER(C.c_int)), ("num_shapes", C.c_int),
                ("shape_materials", C.POINTER(Material)), ("kd_max_depth", C.c_int)]


assert C.sizeof(Geom) == 236 and C.sizeof(Material) == 56 and C.sizeof(Camera) == 84
assert C.sizeof(NodeBare) == 64 and C.sizeof(TriBare) == 76 and C.sizeof(PathSegment) == 56

EXPORTS = [
    "kdpt_default_options", "kdpt_create", "kdpt_trace_iteration", "kdpt_trace_iteration_async", "kdpt_trace_iterations", "kdpt_synchronize",
    "kdpt_read_image", "kdpt_write_pbo", "kdpt_reset", "kdpt_get_stats", "kdpt_destroy", "kdpt_last_error",
    "kdpt_image_device_ptr", "kdpt_debug_paths", "kdpt_count_iteration", "kdpt_count_split", "kdpt_wave_profile", "kdpt_selftest_math", "kdpt_selftest_rng", "kdpt_selftest_rng_draws",
    "kdpt_selftest_fresnel", "kdpt_selftest_libm", "kdpt_selftest_libm_digest", "kdpt_scene_load", "kdpt_scene_build", "kdpt_scene_view", "kdpt_scene_free",
    "kdpt_save_rgb8", "kdpt_save_png", "kdpt_save_hdr", "kdpt_png_encode", "kdpt_write_png", "kdpt_hdr_encode",
    "kdpt_write_hdr", "kdpt_free", "kdpt_set_tuning", "kdpt_selftest_glm", "kdpt_set_options", "kdpt_scene_build_device",
    "kdpt_scene_kd_build_ms", "kdpt_build_kd_device", "kdpt_scene_load_device", "kdpt_trace_config",
    "kdpt_cull_margin", "kdpt_comm_unique_id", "kdpt_comm_init", "kdpt_render_frames", "kdpt_render_sharded",
    "kdpt_comm_library", "kdpt_cull_masks",
]

REDUCE_RCCL, REDUCE_COPY = 0, 1  # kdpt_render_sharded's reduce (KDPT_REDUCE_*)


def set_process_tuning(name: str, value: float):
    """kdpt_set_tuning(NULL, ...): a process-wide knob that contexts created afterwards start with
    ("reduce_spin_us", "cluster_chord")."""
    lib = load_library()
    _check(lib.kdpt_set_tuning(None, name.encode(), float(value)), f"kdpt_set_tuning(NULL, {name})")

_lib = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load the in-tree libkdpt.so (HIP runtime shared with torch when torch is imported)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise KdptError(f"{path} is missing: run `python -m kdtreepathtraceroptimization_amd._build` "
                        "(there is no CPU fallback)")
    try:  # one HIP runtime per process: let torch's libamdhip64 (same soname) win if present
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(path)
    P = C.POINTER
    lib.kdpt_default_options.argtypes = [P(Options)]
    lib.kdpt_default_options.restype = None
    lib.kdpt_create.argtypes = [P(Scene), P(Options), C.c_int, P(C.c_void_p)]
    lib.kdpt_trace_iteration.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.kdpt_trace_iteration_async.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.kdpt_trace_iterations.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.kdpt_synchronize.argtypes = [C.c_void_p]
    lib.kdpt_read_image.argtypes = [C.c_void_p, P(C.c_float)]
    lib.kdpt_write_pbo.argtypes = [C.c_void_p, C.c_int, P(C.c_uint8)]
    lib.kdpt_reset.argtypes = [C.c_void_p]
    lib.kdpt_get_stats.argtypes = [C.c_void_p, P(Stats)]
    lib.kdpt_destroy.argtypes = [C.c_void_p]
    lib.kdpt_last_error.restype = C.c_char_p
    lib.kdpt_image_device_ptr.argtypes = [C.c_void_p, P(C.c_void_p)]
    lib.kdpt_debug_paths.argtypes = [C.c_void_p, C.c_int, C.c_int, P(PathSegment), P(C.c_int)]
    lib.kdpt_count_iteration.argtypes = [C.c_void_p, C.c_int, P(C.c_ulonglong)]
    if hasattr(lib, "kdpt_count_split"):  # diagnostic; absent from older builds used in A/B runs
        lib.kdpt_count_split.argtypes = [C.c_void_p, P(C.c_ulonglong)]
    lib.kdpt_wave_profile.argtypes = [C.c_void_p, P(C.c_ulonglong), C.c_int]
    lib.kdpt_selftest_math.argtypes = [P(C.c_float), C.c_int, P(C.c_float), P(C.c_float)]
    lib.kdpt_selftest_rng.argtypes = [P(C.c_int), C.c_int, C.c_int, P(C.c_float)]
    lib.kdpt_selftest_fresnel.argtypes = [P(C.c_float), C.c_int, C.c_float, P(C.c_float)]
    lib.kdpt_trace_config.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int), P(C.c_longlong)]
    if hasattr(lib, "kdpt_cull_margin"):  # absent from older builds used in A/B runs
        lib.kdpt_cull_margin.argtypes = [C.c_void_p, P(C.c_float), P(C.c_double), P(C.c_int)]
    if hasattr(lib, "kdpt_cull_masks"):
        lib.kdpt_cull_masks.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), C.c_void_p]
    if hasattr(lib, "kdpt_render_frames"):
        lib.kdpt_comm_unique_id.argtypes = [C.c_void_p]
        lib.kdpt_comm_init.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        if hasattr(lib, "kdpt_comm_library"):
            lib.kdpt_comm_library.argtypes = [C.c_char_p, C.c_int]
        lib.kdpt_render_frames.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.kdpt_render_sharded.argtypes = [P(Scene), P(Options), C.c_int, P(C.c_int), C.c_int, C.c_int, C.c_int,
                                            C.c_int, C.c_int, C.c_int, C.c_void_p]
    lib.kdpt_selftest_rng_draws.argtypes = [C.c_int, P(C.c_uint32), C.c_int, C.c_int, P(C.c_float)]
    if hasattr(lib, "kdpt_selftest_libm"):  # absent from older builds used in A/B runs
        lib.kdpt_selftest_libm.argtypes = [C.c_int, P(C.c_float), C.c_int, P(C.c_double)]
        lib.kdpt_selftest_libm_digest.argtypes = [C.c_int, C.c_uint32, C.c_ulonglong, P(C.c_ulonglong)]
    lib.kdpt_scene_load.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, P(C.c_void_p)]
    lib.kdpt_scene_build.argtypes = [P(SceneDesc), P(C.c_void_p)]
    lib.kdpt_scene_view.argtypes = [C.c_void_p, P(Scene)]
    lib.kdpt_scene_free.argtypes = [C.c_void_p]
    lib.kdpt_save_rgb8.argtypes = [C.c_void_p, C.c_float, P(C.c_uint8)]
    lib.kdpt_save_png.argtypes = [C.c_void_p, C.c_char_p, C.c_float]
    lib.kdpt_save_hdr.argtypes = [C.c_void_p, C.c_char_p, C.c_float]
    lib.kdpt_png_encode.argtypes = [P(C.c_uint8), C.c_int, C.c_int, P(P(C.c_uint8)), P(C.c_size_t)]
    lib.kdpt_write_png.argtypes = [C.c_char_p, P(C.c_uint8), C.c_int, C.c_int]
    lib.kdpt_hdr_encode.argtypes = [P(C.c_float), C.c_int, C.c_int, P(P(C.c_uint8)), P(C.c_size_t)]
    lib.kdpt_write_hdr.argtypes = [C.c_char_p, P(C.c_float), C.c_int, C.c_int]
    lib.kdpt_free.argtypes = [C.c_void_p]
    lib.kdpt_free.restype = None
    if hasattr(lib, "kdpt_scene_build_device"):
        lib.kdpt_scene_build_device.argtypes = [P(SceneDesc), C.c_int, P(C.c_void_p)]
        lib.kdpt_scene_kd_build_ms.argtypes = [C.c_void_p, P(C.c_double)]
        lib.kdpt_scene_load_device.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                               P(C.c_void_p)]
        lib.kdpt_build_kd_device.argtypes = [P(C.c_float), P(C.c_float), P(C.c_int), C.c_int, C.c_int, C.c_int,
                                             P(C.c_void_p), P(C.c_int), P(C.c_void_p), P(C.c_int), P(C.c_double)]
    if hasattr(lib, "kdpt_set_options"):
        lib.kdpt_set_options.argtypes = [C.c_void_p, P(Options)]
    if hasattr(lib, "kdpt_selftest_glm"):
        lib.kdpt_selftest_glm.argtypes = [C.c_int, P(C.c_float), C.c_int, P(C.c_float)]
    if hasattr(lib, "kdpt_set_tuning"):  # absent from older builds used in A/B runs
        lib.kdpt_set_tuning.argtypes = [C.c_void_p, C.c_char_p, C.c_double]
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != KDPT_OK:
        msg = load_library().kdpt_last_error().decode(errors="replace")
        raise KdptError(f"{what} failed ({rc}): {msg}")


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _iptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int))


MATERIAL_DTYPE = np.dtype([("color", "<f4", 3), ("specular_exponent", "<f4"), ("specular_color", "<f4", 3),
                           ("hasReflective", "<f4"), ("hasRefractive", "<f4"), ("indexOfRefraction", "<f4"),
                           ("emittance", "<f4"), ("transmittance", "<f4", 3)])
assert MATERIAL_DTYPE.itemsize == 56


@dataclass
class SceneDescription:
    """What the reference's parsers produce before any matrix/camera/KD work."""
    res: tuple
    fovy: float
    iterations: int
    trace_depth: int
    eye: np.ndarray
    look_at: np.ndarray
    up: np.ndarray
    materials: np.ndarray          # MATERIAL_DTYPE[nm]
    geom_type: np.ndarray          # int32[ng]
    geom_material: np.ndarray      # int32[ng]
    geom_trs: np.ndarray           # float32[ng, 9]
    verts9: Optional[np.ndarray] = None   # float32[ntri, 9]
    norms9: Optional[np.ndarray] = None   # float32[ntri, 9]
    shape_of_tri: Optional[np.ndarray] = None  # int32[ntri]
    shape_materials: Optional[np.ndarray] = None  # MATERIAL_DTYPE[nshapes]
    kd_max_depth: int = 13                 # KDtree::split(13) in Scene::loadObj (src/scene.cpp:868-872)

    def with_overrides(self, res=None, depth=None) -> "SceneDescription":
        import dataclasses
        d = dataclasses.replace(self)
        if res is not None:
            d.res = (int(res[0]), int(res[1]))
        if depth is not None:
            d.trace_depth = int(depth)
        return d

    def to_c(self):
        """Build a SceneDesc (the numpy arrays it points into are returned to keep them alive)."""
        keep = []

        def arr(x, dt):
            a = np.ascontiguousarray(x, dtype=dt)
            keep.append(a)
            return a

        mats = arr(self.materials, MATERIAL_DTYPE)
        d = SceneDesc()
        d.res[0], d.res[1] = int(self.res[0]), int(self.res[1])
        d.fovy = float(np.float32(self.fovy))
        d.iterations = int(self.iterations)
        d.traceDepth = int(self.trace_depth)
        for i in range(3):
            d.eye[i], d.lookAt[i], d.up[i] = float(self.eye[i]), float(self.look_at[i]), float(self.up[i])
        d.num_materials = len(mats)
        d.materials = mats.ctypes.data_as(C.POINTER(Material))
        gt, gm, gtrs = arr(self.geom_type, np.int32), arr(self.geom_material, np.int32), arr(self.geom_trs, np.float32)
        d.num_geoms = len(gt)
        d.geom_type, d.geom_material, d.geom_trs = _iptr(gt), _iptr(gm), _fptr(gtrs)
        if self.verts9 is not None and len(self.verts9):
            v9, n9 = arr(self.verts9, np.float32), arr(self.norms9, np.float32)
            st, sm = arr(self.shape_of_tri, np.int32), arr(self.shape_materials, MATERIAL_DTYPE)
            d.ntri = len(st)
            d.verts9, d.norms9, d.shape_of_tri = _fptr(v9), _fptr(n9), _iptr(st)
            d.num_shapes = len(sm)
            d.shape_materials = sm.ctypes.data_as(C.POINTER(Material))
        d.kd_max_depth = int(self.kd_max_depth)
        return d, keep


class SceneData:
    """A built scene (Scene::geoms/materials/newNodesBare/newTrianglesBare + camera), owned by libkdpt."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle
        self.view = Scene()
        _check(load_library().kdpt_scene_view(self._h, C.byref(self.view)), "kdpt_scene_view")

    @classmethod
    def from_files(cls, scene_path: str, obj_path: Optional[str] = None, res=None, depth=None,
                   kd_device: Optional[int] = None) -> "SceneData":
        """kdpt_scene_load (host KD build) or kdpt_scene_load_device (KD tree built on GPU kd_device)."""
        lib = load_library()
        h = C.c_void_p()
        w, hh = (res if res is not None else (0, 0))
        if kd_device is None:
            rc = lib.kdpt_scene_load(scene_path.encode(), obj_path.encode() if obj_path else None, int(w), int(hh),
                                     int(depth or 0), C.byref(h))
        else:
            rc = lib.kdpt_scene_load_device(scene_path.encode(), obj_path.encode() if obj_path else None, int(w),
                                            int(hh), int(depth or 0), int(kd_device), C.byref(h))
        _check(rc, f"kdpt_scene_load({scene_path}, {obj_path})")
        return cls(h)

    @classmethod
    def from_description(cls, desc: SceneDescription, kd_device: Optional[int] = None) -> "SceneData":
        """kdpt_scene_build (host KD build), or kdpt_scene_build_device with the KD tree built on GPU
        `kd_device` (byte-identical)."""
        lib = load_library()
        d, keep = desc.to_c()
        h = C.c_void_p()
        if kd_device is None:
            _check(lib.kdpt_scene_build(C.byref(d), C.byref(h)), "kdpt_scene_build")
        else:
            _check(lib.kdpt_scene_build_device(C.byref(d), int(kd_device), C.byref(h)), "kdpt_scene_build_device")
        del keep
        return cls(h)

    def kd_build_ms(self) -> float:
        ms = C.c_double()
        _check(load_library().kdpt_scene_kd_build_ms(self._h, C.byref(ms)), "kdpt_scene_kd_build_ms")
        return float(ms.value)

    @property
    def resolution(self):
        return int(self.view.camera.resolution[0]), int(self.view.camera.resolution[1])

    def nodes_bytes(self) -> bytes:
        return C.string_at(self.view.nodes, C.sizeof(NodeBare) * self.view.num_nodes)

    def tris_bytes(self) -> bytes:
        return C.string_at(self.view.tris, C.sizeof(TriBare) * self.view.num_tris)

    def geoms_bytes(self) -> bytes:
        return C.string_at(self.view.geoms, C.sizeof(Geom) * self.view.num_geoms)

    def materials_bytes(self) -> bytes:
        return C.string_at(self.view.materials, C.sizeof(Material) * self.view.num_materials)

    def camera_bytes(self) -> bytes:
        return bytes(self.view.camera)

    def close(self):
        if self._h:
            load_library().kdpt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _encoded(fn, ptr, w, h, what) -> bytes:
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    _check(fn(ptr, int(w), int(h), C.byref(out), C.byref(n)), what)
    try:
        return C.string_at(out, n.value)
    finally:
        load_library().kdpt_free(out)


def png_encode(rgb: np.ndarray) -> bytes:
    """PNG bytes of an (H, W, 3) uint8 image, as stb_image_write's stbi_write_png encodes them."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w = rgb.shape[:2]
    return _encoded(load_library().kdpt_png_encode, rgb.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, "kdpt_png_encode")


def hdr_encode(rgb: np.ndarray) -> bytes:
    """Radiance .hdr bytes of an (H, W, 3) float32 image, as stb_image_write's stbi_write_hdr writes them."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    return _encoded(load_library().kdpt_hdr_encode, _fptr(rgb), w, h, "kdpt_hdr_encode")


def default_options(**overrides) -> Options:
    o = Options()
    load_library().kdpt_default_options(C.byref(o))
    for k, v in overrides.items():
        if not hasattr(o, k):
            raise KeyError(k)
        setattr(o, k, v)
    return o


class PathTracer:
    """One device context: pathtraceInit / pathtrace / pathtraceFree."""

    def __init__(self, scene: SceneData, options: Optional[Options] = None, device: int = 0):
        self.scene = scene
        self.lib = load_library()
        self.opt = options if options is not None else default_options()
        self._ctx = C.c_void_p()
        _check(self.lib.kdpt_create(C.byref(scene.view), C.byref(self.opt), int(device), C.byref(self._ctx)),
               "kdpt_create")
        self.width, self.height = scene.resolution

    def trace_iteration(self, iteration: int, frame: int = 0):
        _check(self.lib.kdpt_trace_iteration(self._ctx, int(frame), int(iteration)), "kdpt_trace_iteration")

    def trace_iteration_async(self, iteration: int, frame: int = 0):
        _check(self.lib.kdpt_trace_iteration_async(self._ctx, int(frame), int(iteration)), "kdpt_trace_iteration_async")

    def trace_iterations(self, first: int, count: int, stride: int = 1, pipeline: int = 3, batch: int = 1,
                         frame: int = 0):
        """Iterations first + k*stride (k < count): batches of `batch` sharing each intersect launch,
        `pipeline` batches in flight (kdpt_trace_iterations; async)."""
        _check(self.lib.kdpt_trace_iterations(self._ctx, int(frame), int(first), int(count), int(stride),
                                              int(pipeline), int(batch)), "kdpt_trace_iterations")

    def synchronize(self):
        _check(self.lib.kdpt_synchronize(self._ctx), "kdpt_synchronize")

    def comm_init(self, nranks: int, rank: int, comm_id: Optional[bytes]):
        """kdpt_comm_init: join an spp-sharded group (comm_id from comm_unique_id() on rank 0; None = no
        communicator, render_frames hands each rank's frame shares out for the caller to reduce)."""
        buf = None if comm_id is None else C.create_string_buffer(bytes(comm_id), COMM_ID_BYTES)
        _check(self.lib.kdpt_comm_init(self._ctx, int(nranks), int(rank), buf), "kdpt_comm_init")

    def render_frames(self, first_frame: int, frames: int, spp: int, pipeline: int = 8, batch: int = 8,
                      out=None):
        """kdpt_render_frames (async): this rank's share of frames of `spp` global iterations each, reduced
        to rank 0 and added into its image; out: None, a device pointer (int) or a float32 numpy array of
        frames * 3*W*H values (host copies complete at synchronize())."""
        ptr = None if out is None else (int(out) if isinstance(out, int) else out.ctypes.data)
        _check(self.lib.kdpt_render_frames(self._ctx, int(first_frame), int(frames), int(spp), int(pipeline),
                                           int(batch), ptr), "kdpt_render_frames")

    def image(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 3), dtype=np.float32)
        _check(self.lib.kdpt_read_image(self._ctx, _fptr(out)), "kdpt_read_image")
        return out

    def pbo(self, iteration: int) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), dtype=np.uint8)
        _check(self.lib.kdpt_write_pbo(self._ctx, int(iteration), out.ctypes.data_as(C.POINTER(C.c_uint8))),
               "kdpt_write_pbo")
        return out

    def set_options(self, options: Options):
        """kdpt_set_options: pathtrace()'s per-call flags for the next iterations (same context)."""
        _check(self.lib.kdpt_set_options(self._ctx, C.byref(options)), "kdpt_set_options")
        self.opt = options

    def set_tuning(self, name: str, value: float):
        """kdpt_set_tuning: an explicit A/B or diagnostic knob (the library reads no environment)."""
        _check(self.lib.kdpt_set_tuning(self._ctx, name.encode(), float(value)), f"kdpt_set_tuning({name})")

    def reset(self):
        _check(self.lib.kdpt_reset(self._ctx), "kdpt_reset")

    def save_rgb8(self, samples: float) -> np.ndarray:
        """saveImage's bytes (src/main.cpp:1087-1108, src/image.cpp:22-35), computed on the GPU."""
        out = np.empty((self.height, self.width, 3), dtype=np.uint8)
        _check(self.lib.kdpt_save_rgb8(self._ctx, float(samples), out.ctypes.data_as(C.POINTER(C.c_uint8))),
               "kdpt_save_rgb8")
        return out

    def save_png(self, path: str, samples: float):
        """image::savePNG of the current image: the PNG the reference writes (stb encoder, restated)."""
        _check(self.lib.kdpt_save_png(self._ctx, os.fsencode(path), float(samples)), "kdpt_save_png")

    def save_hdr(self, path: str, samples: float):
        """image::saveHDR (Radiance RGBE, stb encoder restated)."""
        _check(self.lib.kdpt_save_hdr(self._ctx, os.fsencode(path), float(samples)), "kdpt_save_hdr")

    def stats(self) -> Stats:
        s = Stats()
        _check(self.lib.kdpt_get_stats(self._ctx, C.byref(s)), "kdpt_get_stats")
        return s

    def image_device_ptr(self) -> int:
        p = C.c_void_p()
        _check(self.lib.kdpt_image_device_ptr(self._ctx, C.byref(p)), "kdpt_image_device_ptr")
        return int(p.value or 0)

    def debug_paths(self, iteration: int, stop_depth: int):
        n = self.width * self.height
        out = (PathSegment * n)()
        cnt = C.c_int()
        _check(self.lib.kdpt_debug_paths(self._ctx, int(iteration), int(stop_depth), out, C.byref(cnt)),
               "kdpt_debug_paths")
        return np.frombuffer(bytes(out), dtype=PATH_DTYPE)[: cnt.value].copy()

    def count_iteration(self, iteration: int):
        out = (C.c_ulonglong * 3)()
        _check(self.lib.kdpt_count_iteration(self._ctx, int(iteration), out), "kdpt_count_iteration")
        return int(out[0]), int(out[1]), int(out[2])

    TREE_MODES = {0: "hbm-64B", 1: "hbm-32B", 2: "lds-32B", 3: "lds-16B-derived", 4: "lds-16B-derived+hbm-clusters",
                  5: "lds-16B-derived+supers"}

    def trace_config(self) -> dict:
        """kdpt_trace_config: where the intersect kernel reads the tree, its workgroup, grid and LDS."""
        m, b, g, l = C.c_int(), C.c_int(), C.c_int(), C.c_longlong()
        _check(self.lib.kdpt_trace_config(self._ctx, C.byref(m), C.byref(b), C.byref(g), C.byref(l)),
               "kdpt_trace_config")
        out = {"tree": self.TREE_MODES.get(m.value, str(m.value)), "block": b.value, "grid": g.value,
               "lds_tree_bytes": l.value}
        if hasattr(self.lib, "kdpt_cull_margin"):
            out.update(self.cull_margin())
        if hasattr(self.lib, "kdpt_cull_masks"):
            n, ncl = C.c_int(), C.c_int()
            _check(self.lib.kdpt_cull_masks(self._ctx, C.byref(n), C.byref(ncl), None), "kdpt_cull_masks")
            out["cull_mask_n"] = n.value
        return out

    def cull_margin(self) -> dict:
        """kdpt_cull_margin: the cluster cull's margin coefficient, the scene's rigorous one, exact or not."""
        k, r, e = C.c_float(), C.c_double(), C.c_int()
        _check(self.lib.kdpt_cull_margin(self._ctx, C.byref(k), C.byref(r), C.byref(e)), "kdpt_cull_margin")
        return {"cull_margin": k.value, "cull_rigorous": r.value, "cull_exact": bool(e.value)}

    def cull_masks(self):
        """kdpt_cull_masks: (mask_n, masks) of the masked cull as the device built them, a bucket-major array of
        shape [6 mask_n^2, num_clusters]; (0, None) when the scene has none."""
        n, ncl = C.c_int(), C.c_int()
        _check(self.lib.kdpt_cull_masks(self._ctx, C.byref(n), C.byref(ncl), None), "kdpt_cull_masks")
        if n.value == 0:
            return 0, None
        masks = np.zeros((6 * n.value * n.value, ncl.value), np.uint64)
        _check(self.lib.kdpt_cull_masks(self._ctx, C.byref(n), C.byref(ncl), masks.ctypes.data), "kdpt_cull_masks")
        return n.value, masks

    def trace_grid_share(self) -> float:
        return float(self.stats().intersect_grid_share)

    def count_split(self):
        """(AABB tests made before the intersect kernel, segments handed to it) of the last count_iteration."""
        out = (C.c_ulonglong * 2)()
        _check(self.lib.kdpt_count_split(self._ctx, out), "kdpt_count_split")
        return int(out[0]), int(out[1])

    def wave_profile(self):
        """Cycle profile of the intersect kernel in the last count_iteration (kdpt_wave_profile)."""
        out = (C.c_ulonglong * 256)()
        n = self.lib.kdpt_wave_profile(self._ctx, out, 256)
        _check(0 if n > 0 else n, "kdpt_wave_profile")
        keys = ("node_trips", "node_cycles", "big_sweeps", "big_cycles", "small_phases", "small_rounds",
                "small_cycles", "final_cycles", "setup_cycles", "geom_cycles", "post_cycles", "node_lane_steps",
                "big_leaves", "big_clusters", "big_pass", "big_multi", "small_pairs", "node_leafwait_steps",
                "node_done_steps", "tail_cycles", "tail_node_done_steps", "big_supers", "big_cull_cycles",
                "chunks", "chunk_cycles", "aabb", "tri", "hit")
        prof = dict(zip(keys, (int(out[k]) for k in range(len(keys)))))
        k0 = len(keys)
        if n >= k0 + 64:
            prof["wave_life_10us"] = [int(out[k]) for k in range(k0, k0 + 64)]
        if n >= k0 + 144:
            prof["ray_steps_hist4"] = [int(out[k]) for k in range(k0 + 64, k0 + 128)]
            prof["chord_steps"] = [int(out[k]) for k in range(k0 + 128, k0 + 136)]
            prof["chord_rays"] = [int(out[k]) for k in range(k0 + 136, k0 + 144)]
        return prof

    def close(self):
        if self._ctx:
            self.lib.kdpt_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


PATH_DTYPE = np.dtype([("origin", "<f4", 3), ("direction", "<f4", 3), ("isinside", "u1"), ("pad", "u1", 3),
                       ("sdepth", "<f4"), ("color", "<f4", 3), ("pixelIndex", "<i4"), ("remainingBounces", "<i4"),
                       ("materialIdHit", "<i4")])
assert PATH_DTYPE.itemsize == 56


def imgsum(image: np.ndarray) -> float:
    """Sum as the survey's anchor table defines it: per-pixel float32 (r+g+b), accumulated in double."""
    im = np.asarray(image, dtype=np.float32).reshape(-1, 3)
    per_px = (im[:, 0] + im[:, 1]) + im[:, 2]  # float32 adds, left to right
    return float(np.sum(per_px.astype(np.float64)))


COMM_ID_BYTES = 128


def comm_library() -> str:
    """kdpt_comm_library: the RCCL library file the library's reduces go through."""
    lib = load_library()
    buf = C.create_string_buffer(4096)
    _check(lib.kdpt_comm_library(buf, 4096), "kdpt_comm_library")
    return buf.value.decode(errors="replace")


def comm_unique_id() -> bytes:
    """kdpt_comm_unique_id: the RCCL unique id rank 0 hands to every rank."""
    lib = load_library()
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib.kdpt_comm_unique_id(buf), "kdpt_comm_unique_id")
    return buf.raw


def render_sharded(scene: "SceneData", devices, first_frame: int, frames: int, spp: int,
                   options: Optional[Options] = None, pipeline: int = 8, batch: int = 8,
                   reduce: int = REDUCE_RCCL) -> np.ndarray:
    """kdpt_render_sharded: one process, one context per device; returns the reduced frames
    (frames, H, W, 3)."""
    lib = load_library()
    opt = options if options is not None else default_options()
    devs = (C.c_int * len(devices))(*devices)
    w, h = scene.resolution
    out = np.zeros((frames, h, w, 3), dtype=np.float32)
    _check(lib.kdpt_render_sharded(C.byref(scene.view), C.byref(opt), len(devices), devs, int(first_frame),
                                   int(frames), int(spp), int(pipeline), int(batch), int(reduce),
                                   out.ctypes.data), "kdpt_render_sharded")
    return out


def build_kd_device(verts9: np.ndarray, norms9: np.ndarray, mtl: np.ndarray, maxdepth: int = 13, device: int = 0):
    """kdpt_build_kd_device over a triangle soup: (NodeBare bytes, TriBare bytes, build ms)."""
    lib = load_library()
    v = np.ascontiguousarray(verts9, np.float32).reshape(-1, 9)
    n = np.ascontiguousarray(norms9, np.float32).reshape(-1, 9)
    m = np.ascontiguousarray(mtl, np.int32).reshape(-1)
    nodes, tris = C.c_void_p(), C.c_void_p()
    nn, nt, ms = C.c_int(), C.c_int(), C.c_double()
    _check(lib.kdpt_build_kd_device(_fptr(v), _fptr(n), _iptr(m), len(v), int(maxdepth), int(device), C.byref(nodes),
                                    C.byref(nn), C.byref(tris), C.byref(nt), C.byref(ms)), "kdpt_build_kd_device")
    try:
        nb = C.string_at(nodes.value, 64 * nn.value) if nn.value else b""
        tb = C.string_at(tris.value, 76 * nt.value) if nt.value else b""
    finally:
        lib.kdpt_free(nodes)
        lib.kdpt_free(tris)
    return nb, tb, float(ms.value)
