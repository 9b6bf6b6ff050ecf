"""The scatter's glibc calls, restated in kdpt_math.h for gfx950, against the system glibc (CPU).

The reference's soft lobes and fake-SSS branch (src/interactions.h:67-83,195-230) call glibc acosf,
double cos and double sin; the diffuse lobe and rotateVector call sinf/cosf.  kdpt_math.h restates
each from glibc 2.35 (flt-32 e_acosf.c; dbl-64 s_sin.c as the x86_64 FMA ifunc variant evaluates it;
flt-32 s_sinf.c/s_cosf.c).  The same source is compiled here for the host with the device's
numerics flags (-ffp-contract=off, explicit fma) and compared bit for bit with libm.so.6:
  - acosf: every one of the 2^32 float bit patterns;
  - sin/cos: every float argument with |x| < 8 (the reference's arguments are theta = 2 pi u < 2 pi
    and phi = acosf(...) <= pi, both floats widened to double), plus random doubles up to 1.05e8;
  - sinf/cosf: every third float bit pattern (NaNs skipped).
The GPU side runs the same functions on gfx950 (tests/test_gpu_parity.py, digests over the same sets).
"""
import json
import os
import subprocess

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def libm_diff():
    exe = os.path.join(ROOT, "build", "libm_diff")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-fno-fast-math",
                    "-fno-builtin-sin", "-fno-builtin-cos", "-fno-builtin-sinf", "-fno-builtin-cosf",
                    "-include", "omp.h", os.path.join(ROOT, "tests", "native", "libm_diff.cpp"), "-o", exe + f".{os.getpid()}", "-lm"],
                   check=True)
    os.replace(exe + f".{os.getpid()}", exe)  # parallel workers may be running the old one
    return exe


def _run(exe, *args):
    out = subprocess.run([exe, *map(str, args)], check=True, capture_output=True, text=True, timeout=600).stdout
    return json.loads(out.strip().splitlines()[-1])


def test_acosf_every_float(libm_diff):
    r = _run(libm_diff, "acosf", 1)
    assert r["checked"] == 1 << 32
    assert r["mismatches"] == 0, r["first"]


def test_sin_cos_every_float_below_8(libm_diff):
    r = _run(libm_diff, "sincos", 8.0, 1)
    assert r["checked"] == 4 * 0x41000000
    assert r["mismatches"] == 0, r["first"]


def test_sin_cos_random_doubles(libm_diff):
    r = _run(libm_diff, "sincos_random", 4_000_000, 5)
    assert r["checked"] > 7_000_000
    assert r["mismatches"] == 0, r["first"]


def test_sinf_cosf_every_float(libm_diff):
    r = _run(libm_diff, "sincosf", 3)  # every third bit pattern: ~1.4e9 floats x 2 functions
    assert r["checked"] > 2_800_000_000
    assert r["mismatches"] == 0, r["first"]
