// scene_host.cpp -- host side of the drop-in: the reference's Scene / ObjMesh /
// KDtree code path restated in C++ so the flattened NodeBare[] / TriBare[] /
// Geom[] / Material[] / Camera bytes equal what the reference's host code hands
// to pathtraceInit (checked against oracle/_ref, the reference's own
// KDnode.cpp/KDtree.cpp/tiny_obj_loader.cpp, and the survey's sha256 pins).
//
//   scene text      src/scene.cpp:7-271, src/utilities.cpp:265-303
//   OBJ + MTL       src/tiny_obj_loader.cpp:160-276 (number parsing),
//                   :425-486 (fan triangulation), :488-799 (LoadMtl),
//                   :872-1156 (LoadObj), src/scene.cpp:531-822 (shape glue)
//   KD build        src/KDnode.cpp:112-249, src/KDtree.cpp, src/scene.cpp:866-968
//   geom matrices   src/utilities.cpp:256-263 + glm inverse / inverseTranspose
//   camera          src/scene.cpp:215-225, src/main.cpp:1059-1073,1111-1129
//
// Float semantics: compiled with -ffp-contract=off, no fast-math; every float
// and double operation is the one the reference spells (incl. its float ->
// double promotions), libm calls go to the same glibc the reference links.
//
// The OBJ/MTL parsing restates tinyobjloader (MIT, Copyright (c) 2012-2016 Syoyo Fujita and many
// contributors); its notice is in THIRD_PARTY_NOTICES.md at the repository root.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include "kd_build.h"
#include <string>
#include <vector>

#include "../../include/kdpt.h"
#include "kdpt_math.h"

using namespace kdpt;

struct kdpt_scene_data {
  kdpt_camera camera{};
  int traceDepth = 0;
  int iterations = 0;
  std::vector<kdpt_geom> geoms;
  std::vector<kdpt_material> materials;
  std::vector<kdpt_node_bare> nodes;
  std::vector<kdpt_tri_bare> tris;
  std::vector<int> obj_materialOffsets;
  bool has_obj = false;
  // the raw OBJ arrays of the brute-force mode (src/scene.cpp:603-712), in triangle-soup form
  std::vector<float> obj_verts, obj_norms, obj_bboxes;
  std::vector<int> obj_polyoffsets, obj_polysidxflat;
  double kd_build_ms = 0.0;  // kdpt_scene_build_device: the GPU KD build's wall time
};

namespace {

thread_local std::string g_err;

// ------------------------------------------------------------------ mat4
struct Mat {
  f4 c[4];
  float at(int col, int row) const { return (&c[col].x)[row]; }
  void set(int col, int row, float v) { (&c[col].x)[row] = v; }
};
Mat identity() {
  Mat m;
  m.c[0] = f4{1, 0, 0, 0};
  m.c[1] = f4{0, 1, 0, 0};
  m.c[2] = f4{0, 0, 1, 0};
  m.c[3] = f4{0, 0, 0, 1};
  return m;
}
Mat matmul(const Mat& a, const Mat& b) {  // glm type_mat4x4.inl:686-703
  Mat r;
  for (int i = 0; i < 4; i++)
    r.c[i] = add4(add4(add4(scl4(a.c[0], b.c[i].x), scl4(a.c[1], b.c[i].y)), scl4(a.c[2], b.c[i].z)),
                  scl4(a.c[3], b.c[i].w));
  return r;
}
Mat translate(const Mat& m, f3 v) {  // gtc/matrix_transform.inl
  Mat r = m;
  r.c[3] = add4(add4(add4(scl4(m.c[0], v.x), scl4(m.c[1], v.y)), scl4(m.c[2], v.z)), m.c[3]);
  return r;
}
Mat rotate(const Mat& m, float angle, f3 v) {  // gtc/matrix_transform.inl (std::cos(float) == cosf)
  const float c = std::cos(angle), s = std::sin(angle);
  const f3 axis = normalize(v);
  const f3 temp = scl(axis, 1.0f - c);
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = 0.0f + temp.x * axis.y + s * axis.z;
  R[0][2] = 0.0f + temp.x * axis.z - s * axis.y;
  R[1][0] = 0.0f + temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = 0.0f + temp.y * axis.z + s * axis.x;
  R[2][0] = 0.0f + temp.z * axis.x + s * axis.y;
  R[2][1] = 0.0f + temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  Mat r;
  for (int i = 0; i < 3; i++)
    r.c[i] = add4(add4(scl4(m.c[0], R[i][0]), scl4(m.c[1], R[i][1])), scl4(m.c[2], R[i][2]));
  r.c[3] = m.c[3];
  return r;
}
Mat scale(const Mat& m, f3 v) {
  Mat r;
  r.c[0] = scl4(m.c[0], v.x);
  r.c[1] = scl4(m.c[1], v.y);
  r.c[2] = scl4(m.c[2], v.z);
  r.c[3] = m.c[3];
  return r;
}
Mat inverse(const Mat& mm) {  // glm type_mat4x4.inl:37-92
  auto M = [&](int c, int r) { return mm.at(c, r); };
  const float Coef00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
  const float Coef02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
  const float Coef03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
  const float Coef04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
  const float Coef06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
  const float Coef07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
  const float Coef08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
  const float Coef10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
  const float Coef11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
  const float Coef12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
  const float Coef14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
  const float Coef15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
  const float Coef16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
  const float Coef18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
  const float Coef19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
  const float Coef20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
  const float Coef22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
  const float Coef23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
  const f4 Fac0{Coef00, Coef00, Coef02, Coef03}, Fac1{Coef04, Coef04, Coef06, Coef07};
  const f4 Fac2{Coef08, Coef08, Coef10, Coef11}, Fac3{Coef12, Coef12, Coef14, Coef15};
  const f4 Fac4{Coef16, Coef16, Coef18, Coef19}, Fac5{Coef20, Coef20, Coef22, Coef23};
  const f4 Vec0{M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, Vec1{M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
  const f4 Vec2{M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, Vec3{M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
  const f4 Inv0 = add4(sub4(mul4(Vec1, Fac0), mul4(Vec2, Fac1)), mul4(Vec3, Fac2));
  const f4 Inv1 = add4(sub4(mul4(Vec0, Fac0), mul4(Vec2, Fac3)), mul4(Vec3, Fac4));
  const f4 Inv2 = add4(sub4(mul4(Vec0, Fac1), mul4(Vec1, Fac3)), mul4(Vec3, Fac5));
  const f4 Inv3 = add4(sub4(mul4(Vec0, Fac2), mul4(Vec1, Fac4)), mul4(Vec2, Fac5));
  const f4 SignA{+1, -1, +1, -1}, SignB{-1, +1, -1, +1};
  Mat I;
  I.c[0] = mul4(Inv0, SignA);
  I.c[1] = mul4(Inv1, SignB);
  I.c[2] = mul4(Inv2, SignA);
  I.c[3] = mul4(Inv3, SignB);
  const f4 Row0{I.c[0].x, I.c[1].x, I.c[2].x, I.c[3].x};
  const f4 Dot0 = mul4(mm.c[0], Row0);
  const float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
  const float OneOverDeterminant = 1.0f / Dot1;
  Mat r;
  for (int i = 0; i < 4; i++) r.c[i] = scl4(I.c[i], OneOverDeterminant);
  return r;
}
Mat inverseTranspose(const Mat& mm) {  // glm gtc/matrix_inverse.inl:95-147
  auto M = [&](int c, int r) { return mm.at(c, r); };
  const float S00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
  const float S01 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
  const float S02 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
  const float S03 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
  const float S04 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
  const float S05 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
  const float S06 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
  const float S07 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
  const float S08 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
  const float S09 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
  const float S10 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
  const float S11 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
  const float S12 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
  const float S13 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
  const float S14 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
  const float S15 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
  const float S16 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
  const float S17 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
  const float S18 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
  Mat I;
  I.set(0, 0, +(M(1, 1) * S00 - M(1, 2) * S01 + M(1, 3) * S02));
  I.set(0, 1, -(M(1, 0) * S00 - M(1, 2) * S03 + M(1, 3) * S04));
  I.set(0, 2, +(M(1, 0) * S01 - M(1, 1) * S03 + M(1, 3) * S05));
  I.set(0, 3, -(M(1, 0) * S02 - M(1, 1) * S04 + M(1, 2) * S05));
  I.set(1, 0, -(M(0, 1) * S00 - M(0, 2) * S01 + M(0, 3) * S02));
  I.set(1, 1, +(M(0, 0) * S00 - M(0, 2) * S03 + M(0, 3) * S04));
  I.set(1, 2, -(M(0, 0) * S01 - M(0, 1) * S03 + M(0, 3) * S05));
  I.set(1, 3, +(M(0, 0) * S02 - M(0, 1) * S04 + M(0, 2) * S05));
  I.set(2, 0, +(M(0, 1) * S06 - M(0, 2) * S07 + M(0, 3) * S08));
  I.set(2, 1, -(M(0, 0) * S06 - M(0, 2) * S09 + M(0, 3) * S10));
  I.set(2, 2, +(M(0, 0) * S11 - M(0, 1) * S09 + M(0, 3) * S12));
  I.set(2, 3, -(M(0, 0) * S08 - M(0, 1) * S10 + M(0, 2) * S12));
  I.set(3, 0, -(M(0, 1) * S13 - M(0, 2) * S14 + M(0, 3) * S15));
  I.set(3, 1, +(M(0, 0) * S13 - M(0, 2) * S16 + M(0, 3) * S17));
  I.set(3, 2, -(M(0, 0) * S14 - M(0, 1) * S16 + M(0, 3) * S18));
  I.set(3, 3, +(M(0, 0) * S15 - M(0, 1) * S17 + M(0, 2) * S18));
  const float det = +M(0, 0) * I.at(0, 0) + M(0, 1) * I.at(0, 1) + M(0, 2) * I.at(0, 2) + M(0, 3) * I.at(0, 3);
  for (int i = 0; i < 4; i++) I.c[i] = f4{I.c[i].x / det, I.c[i].y / det, I.c[i].z / det, I.c[i].w / det};
  return I;
}
Mat buildTransformationMatrix(f3 t, f3 r, f3 s) {  // src/utilities.cpp:256-263
  const Mat id = identity();
  const Mat T = translate(id, t);
  Mat R = rotate(id, r.x * (float)PI_F / 180, mk3(1, 0, 0));
  R = matmul(R, rotate(id, r.y * (float)PI_F / 180, mk3(0, 1, 0)));
  R = matmul(R, rotate(id, r.z * (float)PI_F / 180, mk3(0, 0, 1)));
  const Mat S = scale(id, s);
  return matmul(matmul(T, R), S);
}

// ------------------------------------------------------------------ KD tree
struct Tri {
  float x1, x2, x3, y1, y2, y3, z1, z2, z3;
  float nx1, nx2, nx3, ny1, ny2, ny3, nz1, nz2, nz3;
  float mins[3], maxs[3];
  int mtlIdx;
};
struct BBox {  // KDnode.h:229-305 (size is never read on the build path)
  float mins[3], maxs[3], center[3];
  void updateCentroid() {
    for (int i = 0; i < 3; i++) center[i] = (float)((double)(mins[i] + maxs[i]) / 2.0);
  }
};
struct Node {
  int axis = 0;
  float splitPos = 0.0f;
  Node* parent = nullptr;
  std::unique_ptr<Node> left, right;
  BBox bbox{};
  std::vector<const Tri*> tris;
  int ID = 0, parentID = -1, leftID = -1, rightID = -1, triIdStart = -1, triIdSize = -1;
};
void computeBounds(Tri& t) {  // KDnode.h:216-225
  t.mins[0] = t.x1 < t.x2 ? (t.x1 < t.x3 ? t.x1 : t.x3) : (t.x2 < t.x3 ? t.x2 : t.x3);
  t.mins[1] = t.y1 < t.y2 ? (t.y1 < t.y3 ? t.y1 : t.y3) : (t.y2 < t.y3 ? t.y2 : t.y3);
  t.mins[2] = t.z1 < t.z2 ? (t.z1 < t.z3 ? t.z1 : t.z3) : (t.z2 < t.z3 ? t.z2 : t.z3);
  t.maxs[0] = t.x1 > t.x2 ? (t.x1 > t.x3 ? t.x1 : t.x3) : (t.x2 > t.x3 ? t.x2 : t.x3);
  t.maxs[1] = t.y1 > t.y2 ? (t.y1 > t.y3 ? t.y1 : t.y3) : (t.y2 > t.y3 ? t.y2 : t.y3);
  t.maxs[2] = t.z1 > t.z2 ? (t.z1 > t.z3 ? t.z1 : t.z3) : (t.z2 > t.z3 ? t.z2 : t.z3);
}
void merge(BBox& a, const float* mn, const float* mx) {  // KDnode::mergeBbox :99-110
  for (int i = 0; i < 3; i++) {
    a.mins[i] = a.mins[i] > mn[i] ? mn[i] : a.mins[i];
    a.maxs[i] = a.maxs[i] < mx[i] ? mx[i] : a.maxs[i];
  }
  a.updateCentroid();
}
// KDnode::updateBbox (:112-149): bounds of the node's own triangles (children are
// merged too, but the builder only calls it on fresh, childless nodes), then a
// 0.001 pad that does NOT refresh the centroid.
void updateBbox(Node& n) {
  if (!n.tris.empty()) {
    for (int i = 0; i < 3; i++) { n.bbox.mins[i] = n.tris[0]->mins[i]; n.bbox.maxs[i] = n.tris[0]->maxs[i]; }
    n.bbox.updateCentroid();
  }
  for (size_t i = 1; i < n.tris.size(); i++) merge(n.bbox, n.tris[i]->mins, n.tris[i]->maxs);
  const float pad = (float)0.001;
  for (int i = 0; i < 3; i++) { n.bbox.mins[i] -= pad; n.bbox.maxs[i] += pad; }
}
struct Builder {
  int currentID = 0;  // the reference's file-static counter (KDnode.cpp:2), per build here
  std::unique_ptr<Node> child(std::vector<const Tri*>&& side, int axis) {
    std::unique_ptr<Node> c(new Node());
    c->tris = std::move(side);
    c->axis = axis;
    updateBbox(*c);  // KDnode(Triangle**, size, axis) constructor
    return c;
  }
  void split(Node* self, int level, int maxdepth) {  // KDnode::split (:151-249)
    const size_t num = self->tris.size();
    if (num == 0) {
      if (self->left) split(self->left.get(), level + 1, maxdepth);
      if (self->right) split(self->right.get(), level + 1, maxdepth);
      return;
    }
    if (num <= 2 || level > maxdepth) return;
    const int ax = level % 3;
    std::vector<const Tri*> L, R;
    const double c = (double)self->bbox.center[ax];
    for (const Tri* t : self->tris) {
      if ((double)t->mins[ax] < c + 0.0001) L.push_back(t);
      if ((double)t->maxs[ax] >= c - 0.0001) R.push_back(t);
    }
    if (L.size() == num || R.size() == num) return;
    const BBox pb = self->bbox;
    if (!L.empty()) {
      self->left = child(std::move(L), (ax + 1) % 3);
      self->left->ID = ++currentID;
      self->left->parentID = self->ID;
      self->leftID = self->left->ID;
      self->left->parent = self;
      BBox& b = self->left->bbox;  // setBounds(parent) then maxs[axis] = parent centre
      for (int i = 0; i < 3; i++) { b.mins[i] = pb.mins[i]; b.maxs[i] = pb.maxs[i]; }
      b.maxs[ax] = pb.center[ax];
      b.updateCentroid();
      self->left->splitPos = pb.maxs[ax];
      split(self->left.get(), level + 1, maxdepth);
    }
    if (!R.empty()) {
      self->right = child(std::move(R), (ax + 1) % 3);
      self->right->ID = ++currentID;
      self->right->parentID = self->ID;
      self->rightID = self->right->ID;
      self->right->parent = self;
      BBox& b = self->right->bbox;
      for (int i = 0; i < 3; i++) { b.mins[i] = pb.mins[i]; b.maxs[i] = pb.maxs[i]; }
      b.mins[ax] = pb.center[ax];
      b.updateCentroid();
      self->right->splitPos = pb.mins[ax];
      split(self->right.get(), level + 1, maxdepth);
    }
    self->tris.clear();  // triangles.erase(begin, end)
  }
};
void preorder(Node* n, std::vector<Node*>& out) {
  if (!n) return;
  out.push_back(n);
  preorder(n->left.get(), out);
  preorder(n->right.get(), out);
}

// Scene::loadObj KD section (src/scene.cpp:866-968): IDs are assigned in pre-order,
// so the ID-sorted node list is the pre-order walk; leaves' triangles are listed in
// that order (duplicates included).
void build_kd_impl(const float* v9, const float* n9, const int* mtl, int ntri, int maxdepth,
                   std::vector<kdpt_node_bare>& nodes_out, std::vector<kdpt_tri_bare>& tris_out) {
  std::vector<Tri> T(ntri);
  for (int i = 0; i < ntri; i++) {
    const float* v = v9 + 9 * (size_t)i;
    const float* n = n9 + 9 * (size_t)i;
    Tri& t = T[i];
    t.x1 = v[0]; t.y1 = v[1]; t.z1 = v[2];
    t.x2 = v[3]; t.y2 = v[4]; t.z2 = v[5];
    t.x3 = v[6]; t.y3 = v[7]; t.z3 = v[8];
    t.nx1 = n[0]; t.ny1 = n[1]; t.nz1 = n[2];
    t.nx2 = n[3]; t.ny2 = n[4]; t.nz2 = n[5];
    t.nx3 = n[6]; t.ny3 = n[7]; t.nz3 = n[8];
    t.mtlIdx = mtl[i];
    computeBounds(t);
  }
  Node root;
  root.tris.reserve(ntri);
  for (int i = 0; i < ntri; i++) root.tris.push_back(&T[i]);
  updateBbox(root);  // KDT->rootNode->updateBbox()
  Builder b;
  b.split(&root, 0, maxdepth);
  std::vector<Node*> order;
  preorder(&root, order);
  nodes_out.assign(order.size(), kdpt_node_bare{});
  tris_out.clear();
  int tc = 0;
  for (Node* n : order) {  // cacheTriangles_ (:409-459)
    if (!n->tris.empty()) {
      n->triIdStart = tc;
      n->triIdSize = (int)n->tris.size();
      tc += n->triIdSize;
      for (const Tri* t : n->tris) {
        kdpt_tri_bare o;
        o.x1 = t->x1; o.x2 = t->x2; o.x3 = t->x3;
        o.y1 = t->y1; o.y2 = t->y2; o.y3 = t->y3;
        o.z1 = t->z1; o.z2 = t->z2; o.z3 = t->z3;
        o.nx1 = t->nx1; o.nx2 = t->nx2; o.nx3 = t->nx3;
        o.ny1 = t->ny1; o.ny2 = t->ny2; o.ny3 = t->ny3;
        o.nz1 = t->nz1; o.nz2 = t->nz2; o.nz3 = t->nz3;
        o.mtlIdx = t->mtlIdx;
        tris_out.push_back(o);
      }
    }
  }
  for (Node* n : order) {  // cacheNodesBare (:905-932)
    kdpt_node_bare& o = nodes_out[n->ID];
    memset(&o, 0, sizeof o);
    o.axis = n->axis;
    o.splitPos = n->splitPos;
    for (int a = 0; a < 3; a++) { o.mins[a] = n->bbox.mins[a]; o.maxs[a] = n->bbox.maxs[a]; }
    o.ID = n->ID;
    o.parentID = n->parentID;
    o.leftID = n->leftID;
    o.rightID = n->rightID;
    o.triIdStart = n->triIdStart;
    o.triIdSize = n->triIdSize;
    o.tmin = 0.0f;
    o.tmax = 0.0f;
  }
}

// ------------------------------------------------------------------ text input
// utilityCore::safeGetline (src/utilities.cpp:273-303) over an in-memory file
struct LineReader {
  std::string buf;
  size_t pos = 0;
  bool eof = false;
  bool open(const char* path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    buf = ss.str();
    return true;
  }
  bool more() const { return pos < buf.size(); }
  std::string getline() {
    std::string t;
    for (;;) {
      if (pos >= buf.size()) {
        if (t.empty()) eof = true;
        return t;
      }
      char c = buf[pos++];
      if (c == '\n') return t;
      if (c == '\r') {
        if (pos < buf.size() && buf[pos] == '\n') pos++;
        return t;
      }
      t += c;
    }
  }
};
std::vector<std::string> tokenize(const std::string& s) {  // istream_iterator<string>
  std::stringstream ss(s);
  std::vector<std::string> out;
  std::string w;
  while (ss >> w) out.push_back(w);
  return out;
}

// tinyobjloader tryParseDouble (src/tiny_obj_loader.cpp:160-266)
bool tryParseDouble(const char* s, const char* s_end, double* result) {
  if (s >= s_end) return false;
  double mantissa = 0.0;
  int exponent = 0;
  char sign = '+', exp_sign = '+';
  const char* curr = s;
  int read = 0;
  bool end_not_reached = false;
  auto isdig = [](char x) { return (unsigned int)(x - '0') < 10u; };
  if (*curr == '+' || *curr == '-') {
    sign = *curr;
    curr++;
  } else if (!isdig(*curr)) {
    return false;
  }
  end_not_reached = (curr != s_end);
  while (end_not_reached && isdig(*curr)) {
    mantissa *= 10;
    mantissa += static_cast<int>(*curr - 0x30);
    curr++;
    read++;
    end_not_reached = (curr != s_end);
  }
  if (read == 0) return false;
  if (end_not_reached) {
    bool exp_part = false;
    if (*curr == '.') {
      curr++;
      read = 1;
      end_not_reached = (curr != s_end);
      while (end_not_reached && isdig(*curr)) {
        mantissa += static_cast<int>(*curr - 0x30) * std::pow(10.0, -read);
        read++;
        curr++;
        end_not_reached = (curr != s_end);
      }
      exp_part = end_not_reached;
    } else if (*curr == 'e' || *curr == 'E') {
      exp_part = true;
    }
    if (exp_part && (*curr == 'e' || *curr == 'E')) {
      curr++;
      end_not_reached = (curr != s_end);
      if (end_not_reached && (*curr == '+' || *curr == '-')) {
        exp_sign = *curr;
        curr++;
      } else if (!isdig(*curr)) {
        return false;
      }
      read = 0;
      end_not_reached = (curr != s_end);
      while (end_not_reached && isdig(*curr)) {
        exponent *= 10;
        exponent += static_cast<int>(*curr - 0x30);
        curr++;
        read++;
        end_not_reached = (curr != s_end);
      }
      exponent *= (exp_sign == '+' ? 1 : -1);
      if (read == 0) return false;
    }
  }
  *result = (sign == '+' ? 1 : -1) * std::ldexp(mantissa * std::pow(5.0, exponent), exponent);
  return true;
}
float parseFloat(const char** token, double def = 0.0) {  // :268-276
  (*token) += strspn(*token, " \t");
  const char* end = (*token) + strcspn(*token, " \t\r");
  double val = def;
  tryParseDouble(*token, end, &val);
  *token = end;
  return static_cast<float>(val);
}

struct MtlRec {
  std::string name;
  float ambient[3]{}, diffuse[3]{}, specular[3]{}, transmittance[3]{};
  float ior = 1.f;
  int illum = 0;
};

// LoadMtl (src/tiny_obj_loader.cpp:488-799): pushes on newmtl and always at the end.
void load_mtl(const std::string& path, std::vector<MtlRec>& mats, std::map<std::string, int>& map) {
  LineReader r;
  bool ok = r.open(path.c_str());
  MtlRec m;
  auto issp = [](char ch) { return ch == ' ' || ch == '\t'; };
  while (ok && r.more()) {
    std::string line = r.getline();
    if (!line.empty()) line = line.substr(0, line.find_last_not_of(" \t") + 1);
    if (!line.empty() && line.back() == '\n') line.pop_back();
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    const char* token = line.c_str();
    token += strspn(token, " \t");
    if (token[0] == '\0' || token[0] == '#') continue;
    if (strncmp(token, "newmtl", 6) == 0 && issp(token[6])) {
      if (!m.name.empty()) {
        map.insert(std::make_pair(m.name, (int)mats.size()));
        mats.push_back(m);
      }
      m = MtlRec();
      char nb[4096] = {0};
      sscanf(token + 7, "%4095s", nb);
      m.name = nb;
      continue;
    }
    auto three = [&](float* dst) {
      token += 2;
      for (int k = 0; k < 3; k++) dst[k] = parseFloat(&token);
    };
    if (token[0] == 'K' && token[1] == 'a' && issp(token[2])) { three(m.ambient); continue; }
    if (token[0] == 'K' && token[1] == 'd' && issp(token[2])) { three(m.diffuse); continue; }
    if (token[0] == 'K' && token[1] == 's' && issp(token[2])) { three(m.specular); continue; }
    if ((token[0] == 'K' && token[1] == 't' && issp(token[2])) || (token[0] == 'T' && token[1] == 'f' && issp(token[2]))) {
      three(m.transmittance);
      continue;
    }
    if (token[0] == 'N' && token[1] == 'i' && issp(token[2])) {
      token += 2;
      m.ior = parseFloat(&token);
      continue;
    }
    if (strncmp(token, "illum", 5) == 0 && issp(token[5])) {
      token += 6;
      token += strspn(token, " \t");
      m.illum = atoi(token);
      continue;
    }
  }
  map.insert(std::make_pair(m.name, (int)mats.size()));
  mats.push_back(m);
}

struct ObjSoup {
  std::vector<float> v9, n9;
  std::vector<int> shape;
  std::vector<kdpt_material> shape_mats;
};

int load_obj(const char* path, ObjSoup& out) {
  LineReader r;
  if (!r.open(path)) return KDPT_ERR_IO;
  std::string p(path);
  const std::string base = p.substr(0, p.find_last_of("/\\") + 1);
  std::vector<float> v, vn;
  int vtn = 0;
  std::vector<MtlRec> mats;
  std::map<std::string, int> mat_map;
  int material = -1;
  std::vector<std::vector<int>> faceGroup;
  std::vector<int> shape_idx;               // current shape's triangulated vertex indices
  std::vector<std::vector<int>> shapes;     // finished shapes
  auto issp = [](char ch) { return ch == ' ' || ch == '\t'; };
  auto isnl = [](char ch) { return ch == '\r' || ch == '\n' || ch == '\0'; };
  auto fixIndex = [](int idx, int n) { return idx > 0 ? idx - 1 : (idx == 0 ? 0 : n + idx); };
  auto flush = [&]() {  // exportFaceGroupToShape: fan triangulation
    if (faceGroup.empty()) return false;
    for (const auto& face : faceGroup) {
      int i0 = face[0], i1 = -1, i2 = face.size() > 1 ? face[1] : -1;
      for (size_t k = 2; k < face.size(); k++) {
        i1 = i2;
        i2 = face[k];
        shape_idx.push_back(i0);
        shape_idx.push_back(i1);
        shape_idx.push_back(i2);
      }
    }
    return true;
  };
  while (r.more()) {
    std::string line = r.getline();
    if (!line.empty() && line.back() == '\n') line.pop_back();
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    const char* token = line.c_str();
    token += strspn(token, " \t");
    if (token[0] == '\0' || token[0] == '#') continue;
    if (token[0] == 'v' && issp(token[1])) {
      token += 2;
      for (int k = 0; k < 3; k++) v.push_back(parseFloat(&token));
      continue;
    }
    if (token[0] == 'v' && token[1] == 'n' && issp(token[2])) {
      token += 3;
      for (int k = 0; k < 3; k++) vn.push_back(parseFloat(&token));
      continue;
    }
    if (token[0] == 'v' && token[1] == 't' && issp(token[2])) {
      vtn++;
      continue;
    }
    if (token[0] == 'f' && issp(token[1])) {
      token += 2;
      token += strspn(token, " \t");
      std::vector<int> face;
      while (!isnl(token[0])) {
        // parseTriple (:322-353): only the vertex index is used downstream
        const int vi = fixIndex(atoi(token), (int)(v.size() / 3));
        token += strcspn(token, "/ \t\r");
        if (token[0] == '/') {
          token++;
          if (token[0] == '/') {
            token++;
            token += strcspn(token, "/ \t\r");
          } else {
            token += strcspn(token, "/ \t\r");
            if (token[0] == '/') {
              token++;
              token += strcspn(token, "/ \t\r");
            }
          }
        }
        face.push_back(vi);
        token += strspn(token, " \t\r");
      }
      faceGroup.push_back(std::move(face));
      continue;
    }
    if (strncmp(token, "usemtl", 6) == 0 && issp(token[6])) {
      char nb[4096] = {0};
      sscanf(token + 7, "%4095s", nb);
      auto it = mat_map.find(nb);
      const int nid = it == mat_map.end() ? -1 : it->second;
      if (nid != material) {
        flush();
        faceGroup.clear();
        material = nid;
      }
      continue;
    }
    if (strncmp(token, "mtllib", 6) == 0 && issp(token[6])) {
      char nb[4096] = {0};
      if (sscanf(token + 7, "%4095s", nb) == 1) load_mtl(base + nb, mats, mat_map);
      continue;
    }
    if ((token[0] == 'g' || token[0] == 'o') && issp(token[1])) {
      if (flush()) shapes.push_back(shape_idx);
      shape_idx.clear();
      faceGroup.clear();
      continue;
    }
  }
  if (flush()) shapes.push_back(shape_idx);
  (void)vtn;
  // Scene::getTrianglesFromScene_ (src/scene.cpp:531-577): normals by VERTEX index
  for (size_t si = 0; si < shapes.size(); si++) {
    const std::vector<int>& ix = shapes[si];
    for (size_t j = 0; j + 2 < ix.size(); j += 3) {
      for (int c = 0; c < 3; c++) {
        const size_t pi = 3 * (size_t)ix[j + c];
        for (int a = 0; a < 3; a++) {
          out.v9.push_back(pi + a < v.size() ? v[pi + a] : 0.0f);
          out.n9.push_back(pi + a < vn.size() ? vn[pi + a] : 0.0f);
        }
      }
      out.shape.push_back((int)si);
    }
  }
  // per-shape materials (src/scene.cpp:716-822)
  for (size_t i = 0; i < shapes.size(); i++) {
    kdpt_material om{};
    if (mats.size() > i) {
      const MtlRec& t = mats[i];
      for (int c = 0; c < 3; c++) om.color[c] = t.ambient[c] > t.diffuse[c] ? t.ambient[c] : t.diffuse[c];
      if (t.illum <= 2) {
        om.specular_exponent = 0.0f;
      } else if (t.illum == 3) {
        om.specular_exponent = 1.0f;
        for (int c = 0; c < 3; c++) om.specular_color[c] = t.specular[c];
        om.hasReflective = 1.0f;
      } else {
        om.specular_exponent = 1.0f;
        for (int c = 0; c < 3; c++) om.specular_color[c] = t.specular[c];
        om.hasReflective = 1.0f;
        om.hasRefractive = 1.0f;
        om.indexOfRefraction = t.ior;
      }
      for (int c = 0; c < 3; c++) om.transmittance[c] = t.transmittance[c];
    } else {
      for (int c = 0; c < 3; c++) om.color[c] = 1.0f;
    }
    om.emittance = 0.0f;
    out.shape_mats.push_back(om);
  }
  return KDPT_OK;
}

struct ParsedScene {
  int res[2] = {0, 0};
  float fovy = 0;
  int iterations = 0, depth = 0;
  float eye[3] = {0, 0, 0}, look[3] = {0, 0, 0}, up[3] = {0, 0, 0};
  std::vector<kdpt_material> mats;
  std::vector<int> gtype, gmat;
  std::vector<float> gtrs;
};

int parse_scene_text(const char* path, ParsedScene& ps) {
  LineReader r;
  if (!r.open(path)) return KDPT_ERR_IO;
  while (!r.eof) {
    std::string line = r.getline();
    if (line.empty()) continue;
    std::vector<std::string> tok = tokenize(line);
    if (tok.empty()) continue;
    if (tok[0] == "MATERIAL" && tok.size() > 1) {  // Scene::loadMaterial
      if (atoi(tok[1].c_str()) != (int)ps.mats.size()) continue;
      kdpt_material m{};
      for (int i = 0; i < 7; i++) {
        std::vector<std::string> t = tokenize(r.getline());
        if (t.empty()) continue;
        auto f = [&](int k) { return (float)atof(t[k].c_str()); };
        if (t[0] == "RGB" && t.size() >= 4) { m.color[0] = f(1); m.color[1] = f(2); m.color[2] = f(3); }
        else if (t[0] == "SPECEX" && t.size() >= 2) m.specular_exponent = f(1);
        else if (t[0] == "SPECRGB" && t.size() >= 4) { m.specular_color[0] = f(1); m.specular_color[1] = f(2); m.specular_color[2] = f(3); }
        else if (t[0] == "REFL" && t.size() >= 2) m.hasReflective = f(1);
        else if (t[0] == "REFR" && t.size() >= 2) m.hasRefractive = f(1);
        else if (t[0] == "REFRIOR" && t.size() >= 2) m.indexOfRefraction = f(1);
        else if (t[0] == "EMITTANCE" && t.size() >= 2) m.emittance = f(1);
      }
      ps.mats.push_back(m);
    } else if (tok[0] == "OBJECT" && tok.size() > 1) {  // Scene::loadGeom
      if (atoi(tok[1].c_str()) != (int)ps.gtype.size()) continue;
      int type = -1, mat = 0;
      std::string l = r.getline();
      if (!l.empty() && !r.eof) type = l == "sphere" ? 0 : (l == "cube" ? 1 : -1);
      l = r.getline();
      if (!l.empty() && !r.eof) {
        std::vector<std::string> t = tokenize(l);
        if (t.size() > 1) mat = atoi(t[1].c_str());
      }
      float trs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      l = r.getline();
      while (!l.empty() && !r.eof) {
        std::vector<std::string> t = tokenize(l);
        if (t.size() >= 4) {
          float vv[3] = {(float)atof(t[1].c_str()), (float)atof(t[2].c_str()), (float)atof(t[3].c_str())};
          if (t[0] == "TRANS") memcpy(trs, vv, 12);
          else if (t[0] == "ROTAT") memcpy(trs + 3, vv, 12);
          else if (t[0] == "SCALE") memcpy(trs + 6, vv, 12);
        }
        l = r.getline();
      }
      ps.gtype.push_back(type);
      ps.gmat.push_back(mat);
      ps.gtrs.insert(ps.gtrs.end(), trs, trs + 9);
    } else if (tok[0] == "CAMERA") {  // Scene::loadCamera
      for (int i = 0; i < 5; i++) {
        std::vector<std::string> t = tokenize(r.getline());
        if (t.empty()) continue;
        if (t[0] == "RES" && t.size() >= 3) { ps.res[0] = atoi(t[1].c_str()); ps.res[1] = atoi(t[2].c_str()); }
        else if (t[0] == "FOVY" && t.size() >= 2) ps.fovy = (float)atof(t[1].c_str());
        else if (t[0] == "ITERATIONS" && t.size() >= 2) ps.iterations = atoi(t[1].c_str());
        else if (t[0] == "DEPTH" && t.size() >= 2) ps.depth = atoi(t[1].c_str());
      }
      std::string l = r.getline();
      while (!l.empty() && !r.eof) {
        std::vector<std::string> t = tokenize(l);
        if (t.size() >= 4) {
          float vv[3] = {(float)atof(t[1].c_str()), (float)atof(t[2].c_str()), (float)atof(t[3].c_str())};
          if (t[0] == "EYE") memcpy(ps.eye, vv, 12);
          else if (t[0] == "LOOKAT") memcpy(ps.look, vv, 12);
          else if (t[0] == "UP") memcpy(ps.up, vv, 12);
        }
        l = r.getline();
      }
    }
  }
  return KDPT_OK;
}

// loadCamera (src/scene.cpp:215-225) + main()/runCuda camera (src/main.cpp:1059-1073,1111-1129)
void build_camera(const kdpt_scene_desc& d, kdpt_camera& cam) {
  memset(&cam, 0, sizeof cam);
  cam.resolution[0] = d.res[0];
  cam.resolution[1] = d.res[1];
  memcpy(cam.position, d.eye, 12);
  memcpy(cam.lookAt, d.lookAt, 12);
  memcpy(cam.up, d.up, 12);
  const float fovy = d.fovy;
  const float yscaled = std::tan(fovy * (PI_F / 180));
  const float xscaled = (yscaled * cam.resolution[0]) / cam.resolution[1];
  const float fovx = (std::atan(xscaled) * 180) / PI_F;
  cam.fov[0] = fovx;
  cam.fov[1] = fovy;
  cam.pixelLength[0] = 2 * xscaled / (float)cam.resolution[0];
  cam.pixelLength[1] = 2 * yscaled / (float)cam.resolution[1];
  const f3 pos = mk3(d.eye[0], d.eye[1], d.eye[2]);
  const f3 look = mk3(d.lookAt[0], d.lookAt[1], d.lookAt[2]);
  const f3 view = normalize(sub(look, pos));
  const f3 viewXZ = mk3(view.x, 0.0f, view.z), viewZY = mk3(0.0f, view.y, view.z);
  const float phi = std::acos(dot(normalize(viewXZ), mk3(0, 0, -1)));
  const float theta = std::acos(dot(normalize(viewZY), mk3(0, 1, 0)));
  const float zoom = length(sub(pos, look));
  const f3 camoffset = mk3(0, 0, 0);
  f3 cp;
  cp.x = zoom * std::sin(phi) * std::sin(theta) + camoffset.x;
  cp.y = zoom * std::cos(theta) + camoffset.y;
  cp.z = zoom * std::cos(phi) * std::sin(theta) + camoffset.z;
  const f3 v = neg(normalize(cp));
  const f3 rr = cross(v, mk3(0, 1, 0));
  const f3 nu = cross(rr, v);
  memcpy(cam.view, &v, 12);
  memcpy(cam.up, &nu, 12);
  memcpy(cam.right, &rr, 12);
  cp = add(cp, add(look, camoffset));
  memcpy(cam.position, &cp, 12);
}

// The OBJ arrays Scene::loadObj keeps for the brute-force kernel (src/scene.cpp:603-712), from the
// per-triangle soup: vertex index 3*t+k holds triangle t's k-th vertex and its vertex-index-gathered
// normal, so every value pathTraceOneBounce reads is the one the reference reads.  Shapes are the runs of
// shape_of_tri.  Bboxes as the reference's loop computes them: first vertex of each triangle only, max
// initialised to 0, stored at [iterator .. iterator+5] (the buffer is sized so that stays in bounds).
void obj_arrays(const kdpt_scene_desc& d, kdpt_scene_data& sd) {
  const int nt = d.ntri, nsh = d.num_shapes;
  sd.obj_verts.assign(d.verts9, d.verts9 + 9 * (size_t)nt);
  sd.obj_norms.assign(d.norms9, d.norms9 + 9 * (size_t)nt);
  sd.obj_polysidxflat.resize(3 * (size_t)nt);
  for (int j = 0; j < 3 * nt; j++) sd.obj_polysidxflat[j] = j;
  sd.obj_polyoffsets.assign(std::max(nsh, 0), 0);
  for (int t = 0; t < nt; t++) {
    const int sh = d.shape_of_tri[t];
    if (sh >= 0 && sh < nsh) sd.obj_polyoffsets[sh] += 3;
  }
  int nb = 6 * nsh, it = 0;
  for (int i = 0; i < nsh; i++) {
    nb = std::max(nb, it + 6);
    it += sd.obj_polyoffsets[i];
  }
  sd.obj_bboxes.assign(std::max(nb, nsh + 5), 0.0f);
  int iterator = 0;
  for (int i = 0; i < nsh; i++) {
    float minx = FLT_MAX, maxx = 0.0f, miny = FLT_MAX, maxy = 0.0f, minz = FLT_MAX, maxz = 0.0f;
    for (int j = iterator; j < iterator + sd.obj_polyoffsets[i]; j += 3) {
      const float* v = sd.obj_verts.data() + 3 * (size_t)sd.obj_polysidxflat[j];
      if (v[0] < minx) minx = v[0];
      if (v[0] > maxx) maxx = v[0];
      if (v[1] < miny) miny = v[1];
      if (v[1] > maxy) maxy = v[1];
      if (v[2] < minz) minz = v[2];
      if (v[2] > maxz) maxz = v[2];
    }
    float* b = sd.obj_bboxes.data() + iterator;
    b[0] = minx; b[1] = miny; b[2] = minz; b[3] = maxx; b[4] = maxy; b[5] = maxz;
    iterator += sd.obj_polyoffsets[i];
  }
}

}  // namespace

namespace kdpt_host {
void build_kd(const float* v9, const float* n9, const int* mtl, int ntri, int maxdepth,
              std::vector<kdpt_node_bare>& nodes_out, std::vector<kdpt_tri_bare>& tris_out) {
  build_kd_impl(v9, n9, mtl, ntri, maxdepth, nodes_out, tris_out);
}

// boxIntersectionTestBox's matrices for a KD node (src/intersections.h:51-63): the unit cube scaled by
// maxs - mins, moved to (mins + maxs) * 0.5 (double product -> float, glm::mat4's converting
// constructor), and its glm::inverse (the same restatement the analytic geoms use).
void node_box_matrices(const float* mins, const float* maxs, float* transform16, float* inverse16) {
  Mat t = identity();
  for (int a = 0; a < 3; a++) {
    t.set(a, a, maxs[a] - mins[a]);
    t.set(3, a, (float)((double)(mins[a] + maxs[a]) * 0.5));
  }
  const Mat inv = inverse(t);
  memcpy(transform16, &t, 64);
  memcpy(inverse16, &inv, 64);
}
}  // namespace kdpt_host

extern "C" {

namespace {
// Scene::Scene + Scene::loadObj from parsed values; the KD tree on the host (device < 0) or on the GPU
int scene_build(const kdpt_scene_desc* d, int device, kdpt_scene_data** out) {
  if (!d || !out) return KDPT_ERR_ARG;
  *out = nullptr;
  if (d->res[0] <= 0 || d->res[1] <= 0) return KDPT_ERR_ARG;
  std::unique_ptr<kdpt_scene_data> sd(new kdpt_scene_data());
  sd->traceDepth = d->traceDepth;
  sd->iterations = d->iterations;
  sd->materials.assign(d->materials, d->materials + d->num_materials);
  for (int i = 0; i < d->num_geoms; i++) {
    kdpt_geom g{};
    g.type = d->geom_type[i];
    g.materialid = d->geom_material[i];
    const float* trs = d->geom_trs + 9 * (size_t)i;
    memcpy(g.translation, trs, 12);
    memcpy(g.rotation, trs + 3, 12);
    memcpy(g.scale, trs + 6, 12);
    const Mat T = buildTransformationMatrix(mk3(trs[0], trs[1], trs[2]), mk3(trs[3], trs[4], trs[5]),
                                            mk3(trs[6], trs[7], trs[8]));
    const Mat I = inverse(T), IT = inverseTranspose(T);
    memcpy(g.transform, &T, 64);
    memcpy(g.inverseTransform, &I, 64);
    memcpy(g.invTranspose, &IT, 64);
    sd->geoms.push_back(g);
  }
  build_camera(*d, sd->camera);
  if (d->ntri > 0) {
    for (int i = 0; i < d->num_shapes; i++) {
      sd->obj_materialOffsets.push_back((int)sd->materials.size());
      sd->materials.push_back(d->shape_materials[i]);
    }
    const int maxdepth = d->kd_max_depth > 0 ? d->kd_max_depth : 13;
    if (device < 0) {
      kdpt_host::build_kd(d->verts9, d->norms9, d->shape_of_tri, d->ntri, maxdepth, sd->nodes, sd->tris);
    } else {
      const int rc = kdpt_host::build_kd_device(d->verts9, d->norms9, d->shape_of_tri, d->ntri, maxdepth, device,
                                                sd->nodes, sd->tris, &sd->kd_build_ms);
      if (rc) return rc;
    }
    sd->has_obj = true;
    obj_arrays(*d, *sd);
  }
  *out = sd.release();
  return KDPT_OK;
}
}  // namespace

int kdpt_scene_build(const kdpt_scene_desc* d, kdpt_scene_data** out) { return scene_build(d, -1, out); }

int kdpt_scene_build_device(const kdpt_scene_desc* d, int device, kdpt_scene_data** out) {
  if (device < 0) return KDPT_ERR_ARG;
  return scene_build(d, device, out);
}

int kdpt_scene_kd_build_ms(const kdpt_scene_data* sd, double* ms) {
  if (!sd || !ms) return KDPT_ERR_ARG;
  *ms = sd->kd_build_ms;
  return KDPT_OK;
}

int kdpt_build_kd_device(const float* verts9, const float* norms9, const int* mtl, int ntri, int maxdepth, int device,
                         kdpt_node_bare** nodes, int* nnodes, kdpt_tri_bare** tris, int* ntris, double* ms) {
  if (!verts9 || !norms9 || !mtl || ntri < 0 || !nodes || !nnodes || !tris || !ntris) return KDPT_ERR_ARG;
  std::vector<kdpt_node_bare> nv;
  std::vector<kdpt_tri_bare> tv;
  const int rc = kdpt_host::build_kd_device(verts9, norms9, mtl, ntri, maxdepth > 0 ? maxdepth : 13, device, nv, tv, ms);
  if (rc) return rc;
  *nodes = (kdpt_node_bare*)malloc(std::max<size_t>(1, nv.size()) * sizeof(kdpt_node_bare));
  *tris = (kdpt_tri_bare*)malloc(std::max<size_t>(1, tv.size()) * sizeof(kdpt_tri_bare));
  if (!*nodes || !*tris) {
    free(*nodes);
    free(*tris);
    return KDPT_ERR_ARG;
  }
  if (!nv.empty()) memcpy(*nodes, nv.data(), nv.size() * sizeof(kdpt_node_bare));
  if (!tv.empty()) memcpy(*tris, tv.data(), tv.size() * sizeof(kdpt_tri_bare));
  *nnodes = (int)nv.size();
  *ntris = (int)tv.size();
  return KDPT_OK;
}


namespace {
int scene_load(const char* scene_path, const char* obj_path, int res_w, int res_h, int depth, int device,
               kdpt_scene_data** out) {
  if (!scene_path || !out) return KDPT_ERR_ARG;
  ParsedScene ps;
  int rc = parse_scene_text(scene_path, ps);
  if (rc) return rc;
  ObjSoup soup;
  if (obj_path && obj_path[0]) {
    rc = load_obj(obj_path, soup);
    if (rc) return rc;
  }
  kdpt_scene_desc d{};
  d.res[0] = res_w > 0 && res_h > 0 ? res_w : ps.res[0];
  d.res[1] = res_w > 0 && res_h > 0 ? res_h : ps.res[1];
  d.fovy = ps.fovy;
  d.iterations = ps.iterations;
  d.traceDepth = depth > 0 ? depth : ps.depth;
  memcpy(d.eye, ps.eye, 12);
  memcpy(d.lookAt, ps.look, 12);
  memcpy(d.up, ps.up, 12);
  d.num_materials = (int)ps.mats.size();
  d.materials = ps.mats.data();
  d.num_geoms = (int)ps.gtype.size();
  d.geom_type = ps.gtype.data();
  d.geom_material = ps.gmat.data();
  d.geom_trs = ps.gtrs.data();
  d.ntri = (int)soup.shape.size();
  d.verts9 = soup.v9.data();
  d.norms9 = soup.n9.data();
  d.shape_of_tri = soup.shape.data();
  d.num_shapes = (int)soup.shape_mats.size();
  d.shape_materials = soup.shape_mats.data();
  return scene_build(&d, device, out);
}
}  // namespace

int kdpt_scene_load(const char* scene_path, const char* obj_path, int res_w, int res_h, int depth,
                    kdpt_scene_data** out) {
  return scene_load(scene_path, obj_path, res_w, res_h, depth, -1, out);
}

int kdpt_scene_load_device(const char* scene_path, const char* obj_path, int res_w, int res_h, int depth, int device,
                           kdpt_scene_data** out) {
  if (device < 0) return KDPT_ERR_ARG;
  return scene_load(scene_path, obj_path, res_w, res_h, depth, device, out);
}

int kdpt_scene_view(const kdpt_scene_data* sd, kdpt_scene* o) {
  if (!sd || !o) return KDPT_ERR_ARG;
  memset(o, 0, sizeof *o);
  o->camera = sd->camera;
  o->traceDepth = sd->traceDepth;
  o->geoms = sd->geoms.data();
  o->num_geoms = (int)sd->geoms.size();
  o->materials = sd->materials.data();
  o->num_materials = (int)sd->materials.size();
  o->has_obj = sd->has_obj ? 1 : 0;
  o->nodes = sd->nodes.data();
  o->num_nodes = (int)sd->nodes.size();
  o->tris = sd->tris.data();
  o->num_tris = (int)sd->tris.size();
  o->obj_materialOffsets = sd->obj_materialOffsets.data();
  o->num_shapes = (int)sd->obj_materialOffsets.size();
  o->obj_verts = sd->obj_verts.data();
  o->num_obj_verts = (int)sd->obj_verts.size();
  o->obj_norms = sd->obj_norms.data();
  o->num_obj_norms = (int)sd->obj_norms.size();
  o->obj_polyoffsets = sd->obj_polyoffsets.data();
  o->obj_polysidxflat = sd->obj_polysidxflat.data();
  o->polyidxcount = (int)sd->obj_polysidxflat.size();
  o->obj_bboxes = sd->obj_bboxes.data();
  o->num_bbox_floats = (int)sd->obj_bboxes.size();
  return KDPT_OK;
}

int kdpt_scene_free(kdpt_scene_data* sd) {
  delete sd;
  return KDPT_OK;
}

}  // extern "C"
