"""The gfx950 build's per-kernel resource report (hipcc -Rpass-analysis=kernel-resource-usage, written to
build/kdpt_runtime.build.log by kdtreepathtraceroptimization_amd/_build.py): the hot kernels keep their
occupancy, and their scratch (register spills or out-of-line calls) stays within the per-kernel budget below:
zero for most, a few bytes where a measured A/B accepted a small, loop-external spill."""
import os
import re

import pytest

from kdtreepathtraceroptimization_amd import _build


def _report():
    if not os.path.exists(_build.RESOURCE_LOG):
        _build.build(force=True)
    out, cur = {}, None
    for line in open(_build.RESOURCE_LOG):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split()[0]] = int(m.group(2))
    return out


# kernel name fragment -> minimum waves per SIMD
HOT = {"k_traceILb1ELb0ELi2E": 4, "k_traceILb0ELb0ELi2E": 4, "k_traceILb1ELb0ELi3E": 4, "k_traceILb0ELb0ELi3E": 4,
       "k_traceILb1ELb0ELi4E": 4, "k_traceILb0ELb0ELi4E": 4,
       "k_traceILb1ELb0ELi5E": 4, "k_traceILb0ELb0ELi5E": 4, "k_shade_fused": 6, "k_geoms": 4, "k_gen_rays": 4}


# k_trace is compiled for 5 waves per SIMD (96 VGPRs) so that a shading wave of another batch fits beside its
# 4 waves: the few values that no longer fit are spilled once at the start and reloaded once per round (a node
# phase + a leaf phase), outside the node and leaf loops; measured +2.8 % overall (profiles/r02_ab_log.md)
# The max-ILP machine scheduler (the runtime's build flags) spills up to 20 B of the fused shading at its
# 80-VGPR cap; the build with it measured +1.2 % over the default scheduler's spill-free one (profiles/r02_ab_log.md).
# Writing the candidates' rays in queue order (round 4) takes the per-iteration form (knob shade_batch = 0) to 28 B;
# the batched k_shade_fused_b the pipeline runs stays at 12 B.
# The derived-box route (NodesDerived, the C5 icosphere's tree in LDS) keeps the current node's box in 6 more
# registers at the same 96-VGPR cap; its spills are the price of the tree in LDS (+10.6 % on C5, and a 4-wave
# cap without spills measured 8 % slower; profiles/r03_ab_log.md)
# The two-level cull route (TREE_LDS16S, the C5 icosphere) adds the super pass's survivor bookkeeping on top,
# and the oriented-box second level (three slabs) 16 B more: measured +3.9 % on C5 all the same (r04_ab_log.md).
# Batches of up to 16 iterations per intersect launch (MAXB) cost the derived-box routes a few more bytes.
# TREE_LDS16 (mode 3: derived records with the cluster boxes in LDS, e.g. the level-6 icosphere) measured
# 60 / 44 B with MAXB 16.
# The masked exact cull (round 5: a missed pair's danger mask is requested with the box test and walked after the
# pass's sweeps, two normal records per trip) keeps the mask live across the sweep: +4 B on the LDS-tree route C3
# runs (mode 2), +30-40 B on the derived-record routes (modes 3 / 4) that carry the masked cull for larger trees;
# the C5 route (mode 5, no masks) is unchanged.  Measured with the spills: profiles/r05_ab_log.md.
SCRATCH_OK = {"k_traceILb1ELb0ELi2E": 40, "k_traceILb0ELb0ELi2E": 40, "k_traceILb1ELb0ELi3E": 104,
              "k_traceILb0ELb0ELi3E": 104, "k_traceILb1ELb0ELi4E": 92,
              "k_traceILb0ELb0ELi4E": 92, "k_traceILb1ELb0ELi5E": 116, "k_traceILb0ELb0ELi5E": 116,
              "k_shade_fused": 28}


@pytest.mark.parametrize("frag", sorted(HOT))
def test_hot_kernels_scratch_and_occupancy_within_budget(kdpt, frag):
    rep = _report()
    ks = [k for k in rep if frag in k]
    assert ks, frag
    for k in ks:
        assert rep[k].get("ScratchSize", 0) <= SCRATCH_OK.get(frag, 0), (k, rep[k])
        assert rep[k].get("Occupancy", 0) >= HOT[frag], (k, rep[k])
