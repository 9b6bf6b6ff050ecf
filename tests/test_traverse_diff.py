"""Host differential test: the product's compact visited-state KD traversal
(kdpt_device.h traverseKD, compiled for the host) against the oracle's literal
visited-bitmap restatement of traverseKDbareShortHybrid / traverseKDbare
(src/pathtrace.cu) on random rays: every hit field bit-exact."""
import json
import os
import subprocess

import pytest

from conftest import ROOT as REPO, needs_reference

REF_SCENES = "/root/reference/scenes"


@pytest.fixture(scope="module")
def traverse_diff(oracle):
    exe = os.path.join(REPO, "build", "traverse_diff")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "native", "traverse_diff.cpp"), "-L", os.path.join(REPO, "oracle"),
                    "-loracle", "-Wl,-rpath," + os.path.join(REPO, "oracle"), "-o", exe + f".{os.getpid()}"], check=True)
    os.replace(exe + f".{os.getpid()}", exe)  # parallel workers may be running the old one
    return exe


@needs_reference
@pytest.mark.parametrize("mesh", ["dragon_5", "sphere_low_1"])
@pytest.mark.parametrize("hybrid", [1, 0])
def test_compact_traversal_matches_bitmap(traverse_diff, mesh, hybrid):
    out = subprocess.run([traverse_diff, f"{REF_SCENES}/cornell.txt", f"{REF_SCENES}/{mesh}.obj", "40000", "11",
                          str(hybrid)], check=True, capture_output=True, text=True, timeout=300).stdout
    r = json.loads(out.strip().splitlines()[-1])
    assert r["mismatches"] == 0
    assert r["obj_hits"] > 0
