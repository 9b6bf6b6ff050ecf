"""Synthetic meshes for the configurations whose assets are missing from the reference tree.

BASELINE.md C5 names `dragon_8.obj` (~1M triangles, 1600x1600, depth 16): it is a missing blob
(`.MISSING_LARGE_BLOBS:10`) and `scenes/dragon.obj` has no normals.  The substitute
is a subdivided icosahedron with per-vertex normals: level L has 20 * 4^L triangles (level 8:
1,310,720).  Fully determined by L (no random numbers): float64 midpoints projected to the sphere with
IEEE +, *, / and sqrt only, then rounded to float32, so every machine builds the same bits.

The mesh is handed to the host builder as the same per-triangle soup the OBJ loader produces
(vertices, vertex-index normals, one shape with the dragon's material from dragon.mtl), and
`write_obj` writes it as an OBJ file for the reference's own KD builder (oracle/_ref) to pin the tree.
"""
from __future__ import annotations

import numpy as np

from .runtime import MATERIAL_DTYPE

CENTER = (0.0, 2.0, 0.0)  # inside scenes/cornell.txt's box, where the dragon sits
RADIUS = 2.0


def _unit(p: np.ndarray) -> np.ndarray:
    n = np.sqrt(p[..., 0] * p[..., 0] + p[..., 1] * p[..., 1] + p[..., 2] * p[..., 2])
    return p / n[..., None]


def icosphere_unit(level: int) -> np.ndarray:
    """(20 * 4^level, 3, 3) float64 triangles on the unit sphere, counter-clockwise seen from outside."""
    t = (1.0 + np.sqrt(5.0)) / 2.0
    v = _unit(np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t],
                        [0, 1, -t], [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], np.float64))
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]])
    tri = v[f]
    for _ in range(level):
        a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
        ab, bc, ca = _unit(a + b), _unit(b + c), _unit(c + a)
        tri = np.stack([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1), np.stack([c, ca, bc], 1),
                        np.stack([ab, bc, ca], 1)], 1).reshape(-1, 3, 3)
    return tri


def icosphere_soup(level: int, center=CENTER, radius: float = RADIUS):
    """verts9, norms9 (float32, (T, 9)) as Scene::getTrianglesFromScene_ lists them."""
    u = icosphere_unit(level)
    verts = (u * radius + np.asarray(center, np.float64)).astype(np.float32)
    norms = u.astype(np.float32)
    return verts.reshape(-1, 9), norms.reshape(-1, 9)


def dragon_material() -> np.ndarray:
    """scenes/dragon.mtl through Scene::loadObj's illum > 3 branch (src/scene.cpp:748-760)."""
    m = np.zeros(1, MATERIAL_DTYPE)
    m["color"] = (0.3, 0.3, 0.05)
    m["specular_exponent"] = 1.0
    m["specular_color"] = (0.35, 0.35, 0.35)
    m["hasReflective"] = 1.0
    m["hasRefractive"] = 1.0
    m["indexOfRefraction"] = 1.5
    return m


def attach_icosphere(desc, level: int):
    """Give a SceneDescription the level-L icosphere as its OBJ (one shape)."""
    v9, n9 = icosphere_soup(level)
    desc.verts9, desc.norms9 = v9, n9
    desc.shape_of_tri = np.zeros(len(v9), np.int32)
    desc.shape_materials = dragon_material()
    return desc


def write_obj(path: str, level: int):
    """The icosphere as an OBJ file (vertex i = soup vertex i, normal i likewise): %.9g round-trips float32."""
    v9, n9 = icosphere_soup(level)
    v, n = v9.reshape(-1, 3), n9.reshape(-1, 3)
    with open(path, "w") as f:
        f.write(f"# icosphere level {level}: {len(v9)} triangles\n")
        f.writelines(f"v {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in v.tolist())
        f.writelines(f"vn {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in n.tolist())
        f.writelines(f"f {3 * t + 1}//{3 * t + 1} {3 * t + 2}//{3 * t + 2} {3 * t + 3}//{3 * t + 3}\n"
                     for t in range(len(v9)))
