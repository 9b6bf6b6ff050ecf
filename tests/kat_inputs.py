"""TEST INFRASTRUCTURE: deterministic inputs of the reference-pinned known-answer tests.

The same seeded generators feed tests/golden/make_ref_pins.py (which runs the reference's own code,
compiled by oracle/ref, and commits digests of its outputs) and the CPU/GPU tests (which run the
oracle, the host-compiled device code and the gfx950 code on them).  numpy's PCG64 stream for a fixed
seed is stable across numpy versions.
"""
import hashlib

import numpy as np

GLM_FNS = {0: "intersectRayTriangle", 1: "normalize", 2: "reflect", 3: "refract", 4: "rotate_quat_vec3"}
GLM_IN = {0: 15, 1: 3, 2: 6, 3: 7, 4: 7}
GLM_OUT = {0: 4, 1: 3, 2: 3, 3: 3, 4: 3}
GLM_N = 1 << 20
# bary slots glm leaves unwritten keep this quiet-NaN payload (no arithmetic produces it)
SENTINEL_BITS = np.uint32(0x7FC0DEAD)


def _unit(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def glm_inputs(fn: int, n: int = GLM_N, seed: int = 20261016) -> np.ndarray:
    rng = np.random.default_rng(seed + 97 * fn)
    if fn == 0:  # rays at triangles: every exit of glm's test (det < eps, u/v out of range, t < 0, hit)
        v0 = rng.uniform(-1, 1, (n, 3))
        v1 = v0 + rng.uniform(-1, 1, (n, 3))
        v2 = v0 + rng.uniform(-1, 1, (n, 3))
        deg = rng.random(n) < 0.03  # degenerate (collinear) triangles
        v2[deg] = v0[deg] + (v1[deg] - v0[deg]) * rng.uniform(-2, 2, (deg.sum(), 1))
        b = rng.uniform(-0.3, 1.3, (n, 2))
        target = v0 + (v1 - v0) * b[:, :1] + (v2 - v0) * b[:, 1:]
        orig = rng.uniform(-3, 3, (n, 3))
        d = target - orig
        d[rng.random(n) < 0.1] *= -1.0  # triangle behind the ray
        rnd = rng.random(n) < 0.1
        d[rnd] = rng.normal(size=(rnd.sum(), 3))
        d = d / np.linalg.norm(d, axis=1, keepdims=True)
        axis0 = rng.random(n) < 0.02  # axis-aligned directions (zero components)
        d[axis0] = np.eye(3)[rng.integers(0, 3, axis0.sum())] * rng.choice([-1, 1], (axis0.sum(), 1))
        x = np.concatenate([orig, d, v0, v1, v2], axis=1)
    elif fn == 1:  # magnitudes from 1e-30 to 1e30, zeros, axis vectors
        v = rng.normal(size=(n, 3)) * (10.0 ** rng.uniform(-30, 30, (n, 1)))
        v[rng.random(n) < 0.01] = 0.0
        x = v
    elif fn == 2:
        x = np.concatenate([_unit(rng, n), _unit(rng, n) * rng.uniform(0.5, 1.5, (n, 1))], axis=1)
    elif fn == 3:  # eta around the reference's 1 / ior and ior (incl. total internal reflection)
        eta = rng.uniform(0.3, 2.5, (n, 1))
        x = np.concatenate([_unit(rng, n), _unit(rng, n), eta], axis=1)
    elif fn == 4:  # unit quaternions (w = cos a/2, xyz = axis sin a/2) as generateRayFromCamera builds
        a = rng.uniform(0, np.pi, (n, 1)).astype(np.float32)
        ax = _unit(rng, n)
        x = np.concatenate([np.cos(a / 2), ax * np.sin(a / 2), _unit(rng, n)], axis=1)
    else:
        raise ValueError(fn)
    return np.ascontiguousarray(x, np.float32)


def glm_sentinels(fn: int, n: int) -> np.ndarray:
    out = np.zeros((n, GLM_OUT[fn]), np.float32)
    out.view(np.uint32)[:] = SENTINEL_BITS
    return out


def geom_trs(seed: int = 7, n: int = 20000) -> np.ndarray:
    """translation / rotation (degrees) / scale triples: the scene files' kinds of values and random ones,
    incl. rotations about several axes, negative and tiny scales."""
    rng = np.random.default_rng(seed)
    t = rng.uniform(-20, 20, (n, 3))
    r = rng.uniform(-360, 360, (n, 3))
    r[: n // 4] = np.round(r[: n // 4] / 15.0) * 15.0  # the scene files' multiples of 15/45/90
    s = rng.uniform(0.01, 10, (n, 3)) * rng.choice([-1, 1], (n, 3), p=[0.05, 0.95])
    return np.ascontiguousarray(np.concatenate([t, r, s], axis=1), np.float32)


def images(seed: int = 3):
    """(name, float image HxWx3) inputs of the PNG/HDR writers: ragged sizes, values below 0, above 1,
    tiny and huge (RGBE exponent range), exact multiples of 1/255."""
    rng = np.random.default_rng(seed)
    out = []
    for (h, w) in ((1, 1), (3, 7), (64, 64), (5, 257), (96, 80)):
        im = rng.uniform(-0.2, 1.3, (h, w, 3))
        k = rng.random((h, w)) < 0.1
        im[k] = rng.integers(0, 256, (k.sum(), 3)) / 255.0
        big = rng.random((h, w)) < 0.05
        im[big] = 10.0 ** rng.uniform(-30, 30, (big.sum(), 3))
        out.append((f"rand_{h}x{w}", np.ascontiguousarray(im, np.float32)))
    return out


RNG_K = 8  # draws per engine: scatterRay's deepest branch (fake SSS + soft lobe) draws fewer


def rng_inputs(mode: str, seed: int = 62) -> np.ndarray:
    """Inputs of the RNG pin (tests/golden/make_ref_pins.py, oracle/ref/thrust_rng_driver.cpp):
    "seeded" (iter, index, depth) int32 rows for makeSeededRandomEngine (src/pathtrace.cu:62-66): the
    grid of small iterations x every depth 0..16 x the first/last pixels of 800^2 and 1600^2, plus random
    rows; "camera" iterations for engine(utilhash(iter)) (src/pathtrace.cu:334); "raw" uint32 seeds,
    incl. the seeding edge cases (0, multiples of m = 2^31 - 1, m +- 1, 2^32 - 1)."""
    rng = np.random.default_rng(seed)
    if mode == "seeded":
        it = np.arange(0, 33)
        idx = np.array([0, 1, 2, 63, 64, 799, 800, 639999, 640000 - 1, 2559999, 2 ** 21, 2 ** 22 - 1])
        d = np.arange(0, 17)
        grid = np.stack(np.meshgrid(it, idx, d, indexing="ij"), -1).reshape(-1, 3)
        n = 1 << 18
        rnd = np.stack([rng.integers(1, 1 << 22, n), rng.integers(0, 1 << 22, n), rng.integers(0, 17, n)], 1)
        return np.ascontiguousarray(np.concatenate([grid, rnd]), np.int32)
    if mode == "camera":
        return np.ascontiguousarray(np.concatenate([np.arange(0, 1 << 16), rng.integers(0, 1 << 31, 1 << 14)]),
                                    np.int32)
    if mode == "raw":
        m = 2 ** 31 - 1
        edge = [0, 1, 2, m - 1, m, m + 1, 2 * m - 1, 2 * m, 2 * m + 1, 2 ** 31, 2 ** 32 - 1, 48271, 16807]
        return np.ascontiguousarray(np.concatenate([edge, rng.integers(0, 1 << 32, 1 << 16, dtype=np.uint64)]),
                                    np.uint32)
    raise ValueError(mode)


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def sha256_nan_canonical(a: np.ndarray) -> str:
    """sha256 with every NaN replaced by one bit pattern: IEEE 754 leaves a generated NaN's sign and
    payload open (x86 SSE makes 0xffc00000, gfx950 0x7fc00000); NaN positions still count."""
    b = np.ascontiguousarray(a, np.float32).copy()
    b.view(np.uint32)[np.isnan(b)] = np.uint32(0x7FC00000)
    return sha256(b)
