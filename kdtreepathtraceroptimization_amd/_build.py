"""Build the gfx950 shared library ``libkdpt.so`` in-tree (hipcc + g++).

The product is one C-ABI library (include/kdpt.h): HIP kernels + runtime
(csrc/kdpt_runtime.hip) and the host scene builder (csrc/scene_host.cpp).
Numerics flags are part of the contract: ``-ffp-contract=off`` and no
fast-math on both the device and the host side, so that every float/double
operation is the one the reference spells ("Hard parts").
"""
from __future__ import annotations

import hashlib
import os
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libkdpt.so")
BUILD = os.path.join(ROOT, "build")
RESOURCE_LOG = os.path.join(BUILD, "kdpt_runtime.build.log")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KDPT_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(ROOT, "include")]
# the runtime kernels' code-generation flags beyond COMMON: the max-ILP machine scheduler (A/B +1.2 %,
# k_trace launch -1 %, profiles/r02_ab_log.md; it reorders instructions only, so the results stay
# bit-identical).  tools/build_variant.sh takes them from here, so A/B variants build like the product.
DEVICE_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
# the sources whose device code the runtime's kernels are compiled from
KERNEL_SOURCES = ["kdpt_device.h", "kdpt_math.h", "kdpt_runtime.hip", "glibc_sincostab.h"]


def _run(cmd, log=None):
    print("+", " ".join(cmd), flush=True)
    if log is None:
        subprocess.run(cmd, check=True)
        return
    with open(log, "w") as f:  # long remark output goes to a file, never through a pipe that may close
        r = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        sys.stderr.write(open(log).read()[-4000:])
        raise subprocess.CalledProcessError(r.returncode, cmd)


def _sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))] + [os.path.join(ROOT, "include", "kdpt.h")]


def kernel_source_sha() -> str:
    """Hash of the runtime kernels' sources AND their compile flags (bench.py's roofline provenance)."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(" ".join([ARCH, *COMMON[:5], *DEVICE_FLAGS]).encode())
    return h.hexdigest()[:16]


def code_object_sha(lib: str = LIB) -> str | None:
    """sha256 (16 hex) of the library's .hip_fatbin section: the gfx950 code objects themselves, so a
    profile identifies the exact machine code it measured (independent of host-side code)."""
    try:
        with open(lib, "rb") as f:
            elf = f.read()
    except OSError:
        return None
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return None
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    sec = [struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = sec[shstrndx][4]
    for name, _t, _f, _a, off, size in sec:
        end = elf.index(b"\0", stroff + name)
        if elf[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(elf[off:off + size]).hexdigest()[:16]
    return None


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(s) <= t for s in _sources())


def build(force: bool = False) -> str:
    if not force and up_to_date() and os.path.exists(RESOURCE_LOG):
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    host_obj = os.path.join(BUILD, "scene_host.o")
    io_obj = os.path.join(BUILD, "image_io.o")
    dev_obj = os.path.join(BUILD, "kdpt_runtime.o")
    kd_obj = os.path.join(BUILD, "kd_build.o")
    _run(["g++", *COMMON, "-c", os.path.join(CSRC, "scene_host.cpp"), "-o", host_obj])
    _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-c", os.path.join(CSRC, "kd_build.hip"), "-o", kd_obj])
    _run(["g++", *COMMON, "-c", os.path.join(CSRC, "image_io.cpp"), "-o", io_obj])
    # the per-kernel resource report (VGPRs, scratch, occupancy) goes to the build log, which
    # tests/test_build_resources.py checks: a hot kernel that starts spilling or calling out-of-line
    # functions (scratch > 0) fails the CPU suite instead of silently losing half its occupancy
    _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, *DEVICE_FLAGS, "-Rpass-analysis=kernel-resource-usage", "-c",
          os.path.join(CSRC, "kdpt_runtime.hip"), "-o", dev_obj], log=RESOURCE_LOG)
    tmp = LIB + ".tmp"
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, dev_obj, kd_obj, host_obj, io_obj])
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    if "--device-flags" in sys.argv:  # for tools/build_variant.sh
        print(" ".join(DEVICE_FLAGS))
    else:
        build(force="--force" in sys.argv)
        print(LIB)
