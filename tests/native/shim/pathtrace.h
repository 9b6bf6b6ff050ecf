// TEST INFRASTRUCTURE: a layout-identical stand-in for the reference's pathtrace.h + Scene, so that
// integration/pathtrace_kdpt.cpp compiles (and, on the GPU, runs) without the reference's CUDA headers.
// Field names, types and order follow src/scene.h:38-79, src/sceneStructs.h:15-63 and src/KDnode.h:51-82;
// tests/test_integration_shim.py checks the sizes against include/kdpt.h.
#pragma once
#include <string>
#include <vector>

struct uchar4 { unsigned char x, y, z, w; };
namespace glm {
struct vec2 { float x, y; };
struct vec3 { float x, y, z; };
struct mat4 { float m[16]; };
}  // namespace glm

enum GeomType { SPHERE, CUBE };
struct Geom {
  enum GeomType type;
  int materialid;
  glm::vec3 translation, rotation, scale;
  glm::mat4 transform, inverseTransform, invTranspose;
};
struct Material {
  glm::vec3 color;
  struct { float exponent; glm::vec3 color; } specular;
  float hasReflective, hasRefractive, indexOfRefraction, emittance;
  glm::vec3 transmittance;
};
struct Camera {
  glm::vec2 resolution_i;  // glm::ivec2 in the reference: two 32-bit ints
  glm::vec3 position, lookAt, view, up, right;
  glm::vec2 fov, pixelLength;
};
struct RenderState {
  Camera camera;
  unsigned int iterations;
  int traceDepth;
  std::vector<glm::vec3> image;
  std::string imageName;
};
namespace KDN {
struct NodeBare {
  int axis;
  float splitPos;
  float mins[3], maxs[3];
  int ID, parentID, leftID, rightID, triIdStart, triIdSize;
  float tmin, tmax;
};
struct TriBare {
  float x1, x2, x3, y1, y2, y3, z1, z2, z3;
  float nx1, nx2, nx3, ny1, ny2, ny3, nz1, nz2, nz3;
  int mtlIdx;
};
}  // namespace KDN
struct ObjMesh {
  struct { std::vector<float> vertices, normals; } attrib;
};
struct Scene {
  std::vector<Geom> geoms;
  std::vector<Material> materials;
  RenderState state;
  ObjMesh* objmesh = nullptr;
  int obj_numshapes = 0;
  float* obj_verts = nullptr;
  float* obj_norms = nullptr;
  float* obj_bboxes = nullptr;
  int* obj_materialOffsets = nullptr;
  bool hasObj = false;
  int* obj_polyoffsets = nullptr;
  int* obj_polysidxflat = nullptr;
  int polyidxcount = 0;
  int numNodes = 0;
  int numTriangles = 0;
  KDN::NodeBare* newNodesBare = nullptr;
  KDN::TriBare* newTrianglesBare = nullptr;
};

void pathtraceInit(Scene* scene, bool enablekd);
void pathtraceFree(Scene* scene, bool enablekd);
void pathtrace(uchar4* pbo, int frame, int iteration, float focalLength, float dofAngle, bool cacherays,
               bool antialias, float softness, bool enableSss, bool testingmode, bool compaction, bool enablekd,
               bool vizkd, bool USEBBOX, bool SHORTSTACK);
