// pathtrace_kdpt.cpp -- the reference's pathtrace.h API (src/pathtrace.h:6-21) on top of libkdpt.so.
//
// A maintainer replaces src/pathtrace.cu with this file and links libkdpt.so; nothing
// else in the reference changes: Scene still parses the scene text, builds the KD tree on the host
// (src/scene.cpp:866-968) and owns the arrays, which pass through as pointers (the layouts are the
// reference's, include/kdpt.h).  tests/test_integration_shim.py compiles this file against include/kdpt.h
// and a layout-identical stand-in of the reference's pathtrace.h / Scene (tests/native/shim/pathtrace.h)
// and, on the GPU, runs it against the C-ABI directly.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kdpt.h"
#include "pathtrace.h"

namespace {

kdpt_ctx* g_ctx = nullptr;
Scene* g_scene = nullptr;
kdpt_options g_opt;

void check(int rc, const char* what) {
  if (rc != KDPT_OK) {  // the reference exits on any CUDA error (src/pathtrace.cu:42-60); keep that here
    fprintf(stderr, "%s: %s\n", what, kdpt_last_error());
    exit(EXIT_FAILURE);
  }
}

kdpt_scene view_of(Scene* s) {
  static_assert(sizeof(Camera) == sizeof(kdpt_camera), "Camera layout");
  static_assert(sizeof(Geom) == sizeof(kdpt_geom), "Geom layout");
  static_assert(sizeof(Material) == sizeof(kdpt_material), "Material layout");
  static_assert(sizeof(KDN::NodeBare) == sizeof(kdpt_node_bare), "NodeBare layout");
  static_assert(sizeof(KDN::TriBare) == sizeof(kdpt_tri_bare), "TriBare layout");
  kdpt_scene v = {};
  memcpy(&v.camera, &s->state.camera, sizeof v.camera);
  v.traceDepth = s->state.traceDepth;
  v.geoms = reinterpret_cast<const kdpt_geom*>(s->geoms.data());
  v.num_geoms = (int)s->geoms.size();
  v.materials = reinterpret_cast<const kdpt_material*>(s->materials.data());
  v.num_materials = (int)s->materials.size();
  v.has_obj = s->hasObj ? 1 : 0;
  v.nodes = reinterpret_cast<const kdpt_node_bare*>(s->newNodesBare);
  v.num_nodes = s->numNodes;
  v.tris = reinterpret_cast<const kdpt_tri_bare*>(s->newTrianglesBare);
  v.num_tris = s->numTriangles;
  v.obj_materialOffsets = s->obj_materialOffsets;
  v.num_shapes = s->obj_numshapes;
  if (s->hasObj) {  // the raw OBJ arrays pathTraceOneBounce reads when enablekd == false (src/pathtrace.cu:225-257)
    v.obj_verts = s->obj_verts;
    v.num_obj_verts = (int)s->objmesh->attrib.vertices.size();
    v.obj_norms = s->obj_norms;
    v.num_obj_norms = (int)s->objmesh->attrib.normals.size();
    v.obj_polyoffsets = s->obj_polyoffsets;
    v.obj_polysidxflat = s->obj_polysidxflat;
    v.polyidxcount = s->polyidxcount;
    v.obj_bboxes = s->obj_bboxes;
    v.num_bbox_floats = 6 * s->obj_numshapes;
  }
  return v;
}

void create(Scene* scene) {
  const kdpt_scene v = view_of(scene);
  check(kdpt_create(&v, &g_opt, /*device=*/0, &g_ctx), "pathtraceInit");
}

}  // namespace

// src/pathtrace.cu:201-272: caches the scene and uploads it
void pathtraceInit(Scene* scene, bool enablekd) {
  g_scene = scene;
  kdpt_default_options(&g_opt);
  g_opt.enable_kd = enablekd ? 1 : 0;
  create(scene);
}

// src/pathtrace.cu:274-305
void pathtraceFree(Scene*, bool) {
  if (g_ctx) kdpt_destroy(g_ctx);
  g_ctx = nullptr;
}

// src/pathtrace.cu:2405-2635: one iteration (1 sample per pixel), synchronous; the accumulated image lands in
// scene->state.image like the reference's cudaMemcpy at :2631-2632
void pathtrace(uchar4* pbo, int frame, int iteration, float focalLength, float dofAngle, bool cacherays,
               bool antialias, float softness, bool enableSss, bool testingmode, bool compaction,
               bool enablekd, bool vizkd, bool USEBBOX, bool SHORTSTACK) {
  kdpt_options o = g_opt;  // the per-call flags, as the reference passes them
  o.focal_length = focalLength;
  o.dof_angle = dofAngle;
  o.cacherays = cacherays;
  o.antialias = antialias;
  o.softness = softness;
  o.enable_sss = enableSss;
  o.testing_mode = testingmode;
  o.compaction = compaction;
  o.enable_kd = enablekd;
  o.viz_kd = vizkd;
  o.use_bbox = USEBBOX;
  o.short_stack = SHORTSTACK;
  const bool structural = o.enable_kd != g_opt.enable_kd || o.viz_kd != g_opt.viz_kd || o.use_bbox != g_opt.use_bbox;
  g_opt = o;
  if (structural) {  // a different intersect kernel and upload: a new context (the image restarts, like the
    pathtraceFree(g_scene, enablekd);  // reference's re-init after a change)
    create(g_scene);
  } else {
    check(kdpt_set_options(g_ctx, &g_opt), "pathtrace options");
  }
  check(kdpt_trace_iteration(g_ctx, frame, iteration), "pathtrace");
  check(kdpt_read_image(g_ctx, reinterpret_cast<float*>(g_scene->state.image.data())), "pathtrace image");
  if (pbo) {  // sendImageToPBO (src/pathtrace.cu:69-89): under GL interop the PBO is the mapped device buffer,
    // which kdpt_write_pbo writes directly; a headless caller may pass host memory instead
    check(kdpt_write_pbo(g_ctx, iteration, reinterpret_cast<uint8_t*>(pbo)), "pathtrace pbo");
  }
}
