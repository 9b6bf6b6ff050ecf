"""MI355X-native (gfx950) rebuild of the reddeupenn/kdtreePathTracerOptimization hot path.

The per-sample KD-tree bounce (short-stack hybrid traversal + triangle test,
scatterRay/shadeMaterial, stable stream compaction) runs in hand-written HIP
kernels behind the C-ABI in include/kdpt.h (``libkdpt.so``, built in-tree by
``_build.py``).  This package holds only the host plumbing around it.
"""
from .runtime import (KdptError, PathTracer, SceneData, SceneDescription, default_options, imgsum,  # noqa: F401
                      load_library)
from .fixtures import load_fixture_scene, FIXTURE_DIR  # noqa: F401

__all__ = ["KdptError", "PathTracer", "SceneData", "SceneDescription", "default_options", "imgsum",
           "load_library", "load_fixture_scene", "FIXTURE_DIR"]
