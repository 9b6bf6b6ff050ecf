// TEST INFRASTRUCTURE: drives integration/pathtrace_kdpt.cpp the way the reference's main.cpp drives
// pathtrace.cu (pathtraceInit, pathtrace per iteration with the flags of src/main.cpp:1152-1166,
// pathtraceFree), with a Scene filled from the product's own scene builder.  Writes scene->state.image
// after the last iteration (3*W*H floats).
//   shim_driver SCENE.txt OBJ|- W H ITERS OUT.f32 [softness dof sss shortstack compaction enablekd [reinits]]
// reinits: that many more times, pathtraceFree + pathtraceInit and the iterations again from 1 (what runCuda does
// after a camera move, src/main.cpp:1134-1137); the image written is the last run's, and the JSON line carries
// every pathtraceInit's wall time.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kdpt.h"
#include "pathtrace.h"

int main(int argc, char** argv) {
  if (argc < 7) return 2;
  kdpt_scene_data* sd = nullptr;
  if (kdpt_scene_load(argv[1], strcmp(argv[2], "-") ? argv[2] : nullptr, atoi(argv[3]), atoi(argv[4]), 0, &sd))
    return 3;
  kdpt_scene v;
  kdpt_scene_view(sd, &v);
  const int iters = atoi(argv[5]);
  const float softness = argc > 7 ? (float)atof(argv[7]) : 0.0f, dof = argc > 8 ? (float)atof(argv[8]) : 0.0f;
  const bool sss = argc > 9 && atoi(argv[9]), shortstack = argc > 10 ? atoi(argv[10]) != 0 : true;
  const bool compaction = argc > 11 ? atoi(argv[11]) != 0 : true, enablekd = argc > 12 ? atoi(argv[12]) != 0 : true;
  Scene s;
  s.geoms.assign(reinterpret_cast<const Geom*>(v.geoms), reinterpret_cast<const Geom*>(v.geoms) + v.num_geoms);
  s.materials.assign(reinterpret_cast<const Material*>(v.materials),
                     reinterpret_cast<const Material*>(v.materials) + v.num_materials);
  memcpy(&s.state.camera, &v.camera, sizeof v.camera);
  s.state.traceDepth = v.traceDepth;
  const int W = v.camera.resolution[0], H = v.camera.resolution[1];
  s.state.image.assign((size_t)W * H, glm::vec3{0, 0, 0});
  s.hasObj = v.has_obj != 0;
  s.numNodes = v.num_nodes;
  s.numTriangles = v.num_tris;
  s.newNodesBare = reinterpret_cast<KDN::NodeBare*>(const_cast<kdpt_node_bare*>(v.nodes));
  s.newTrianglesBare = reinterpret_cast<KDN::TriBare*>(const_cast<kdpt_tri_bare*>(v.tris));
  s.obj_materialOffsets = const_cast<int*>(v.obj_materialOffsets);
  s.obj_numshapes = v.num_shapes;
  ObjMesh mesh;
  mesh.attrib.vertices.assign(v.obj_verts, v.obj_verts + v.num_obj_verts);
  mesh.attrib.normals.assign(v.obj_norms, v.obj_norms + v.num_obj_norms);
  s.objmesh = &mesh;
  s.obj_verts = const_cast<float*>(v.obj_verts);
  s.obj_norms = const_cast<float*>(v.obj_norms);
  s.obj_polyoffsets = const_cast<int*>(v.obj_polyoffsets);
  s.obj_polysidxflat = const_cast<int*>(v.obj_polysidxflat);
  s.polyidxcount = v.polyidxcount;
  s.obj_bboxes = const_cast<float*>(v.obj_bboxes);
  std::vector<uchar4> pbo((size_t)W * H);
  const int reinits = argc > 13 ? atoi(argv[13]) : 0;
  std::vector<double> init_ms;
  for (int run = 0; run <= reinits; run++) {
    if (run > 0) pathtraceFree(&s, enablekd);
    const auto t0 = std::chrono::steady_clock::now();
    pathtraceInit(&s, enablekd);
    init_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    for (int it = 1; it <= iters; it++)
      pathtrace(pbo.data(), 0, it, 6.0f, dof, false, true, softness, sss, false, compaction, enablekd, false, false,
                shortstack);
  }
  FILE* f = fopen(argv[6], "wb");
  fwrite(s.state.image.data(), sizeof(float), 3 * (size_t)W * H, f);
  fclose(f);
  pathtraceFree(&s, enablekd);
  kdpt_scene_free(sd);
  printf("{\"W\": %d, \"H\": %d, \"iterations\": %d, \"init_ms\": [", W, H, iters);
  for (size_t k = 0; k < init_ms.size(); k++) printf("%s%.3f", k ? ", " : "", init_ms[k]);
  printf("]}\n");
  return 0;
}
