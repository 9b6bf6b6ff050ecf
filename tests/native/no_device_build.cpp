// TEST INFRASTRUCTURE: host-only builds of csrc/scene_host.cpp (the sanitizer suite) link this instead of
// the GPU KD build (csrc/kd_build.hip).
#include "../../kdtreepathtraceroptimization_amd/csrc/kd_build.h"

namespace kdpt_host {
int build_kd_device(const float*, const float*, const int*, int, int, int, std::vector<kdpt_node_bare>&,
                    std::vector<kdpt_tri_bare>&, double*) {
  return KDPT_ERR_UNSUPPORTED;
}
}  // namespace kdpt_host
