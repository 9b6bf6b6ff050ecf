// kd_build.h -- the KD-tree builds of Scene::loadObj (src/scene.cpp:866-968), shared by the C-ABI.
#pragma once
#include <vector>

#include "kdpt.h"

namespace kdpt_host {
// Host restatement (csrc/scene_host.cpp), the reference's depth-first recursion.
void build_kd(const float* v9, const float* n9, const int* mtl, int ntri, int maxdepth,
              std::vector<kdpt_node_bare>& nodes_out, std::vector<kdpt_tri_bare>& tris_out);
// The same tree built level by level on the GPU (csrc/kd_build.hip), byte-identical; ms = wall time
// including uploads and read-back.
int build_kd_device(const float* v9, const float* n9, const int* mtl, int ntri, int maxdepth, int device,
                    std::vector<kdpt_node_bare>& nodes_out, std::vector<kdpt_tri_bare>& tris_out, double* ms);
}  // namespace kdpt_host
