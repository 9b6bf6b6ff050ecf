// kdpt_device.h -- the per-path bounce of the reference, as __host__ __device__
// functions over the gfx950 data layout (SoA float4 nodes/triangles).
//
// Follows src/pathtrace.cu:1571-1734 (pathTraceOneBounceKDbare),
// :1023-1235 (traverseKDbareShortHybrid), :881-1020 (traverseKDbare),
// :2304-2369 (shadeMaterial), src/intersections.h and src/interactions.h.
//
// KD traversal state.  The reference keeps a per-thread `bool nodeIDs[4000]`
// visited bitmap (4 KB zeroed per ray per bounce).  Traversal only moves
// parent<->child, a node is marked before control leaves it upward, so it is
// never re-entered, and the only flags ever read belong to the current node,
// its parent and its two children.  The only writes to nodes off the current
// root-to-node path are the hybrid "skip other side" marks, which land on the
// children of nodes[0] or nodes[1] (the bug `nodes[nodeIDs[parentID]]`).
// So the bitmap is exactly representable by
//   cb    : 2 bits per level L = visited flags of the two children of the
//           path node at level L (reset when that level is (re)entered),
//   ps    : bit L = which child the path took at level L,
//   rootv : visited flag of the root,
//   g     : flags of nodes[1]'s two children while the path is outside
//           node 1's subtree (loaded into cb level 1 on entering node 1),
//   sink  : nodeIDs[-1] (written by leaf "children" marks, read by the skip
//           line when the current leaf is the root).
// Everything lives in 4 scalars per lane -- no LDS, no scratch.
#pragma once

#include "kdpt_math.h"

namespace kdpt {

// Per-material record, read by divergent lanes.
struct DevMaterial {
  float color[3];
  float spec_exponent;
  float spec_color[3];
  float hasReflective;
  float hasRefractive;
  float indexOfRefraction;
  float emittance;
  float transmittance[3];
  float fresnel_R0;  // glm::pow((1-ior)/(1+ior), 2.0f), precomputed (folds to r*r)
  float pad_[3];
};

struct DevGeom {
  int type;
  int materialid;
  int pad_[2];
  float transform[16];
  float inverseTransform[16];
  float invTranspose[16];
  // world-space bounds of the unit cube / sphere under `transform`, enlarged by a margin far above
  // float rounding: a ray that misses them cannot hit the object (used to skip the exact test)
  float wlo[4], whi[4];
};

// Conservative skip test for the analytic geoms (invdir finite).  The exact object-space test
// (boxIntersectionTest / sphereIntersectionTest) reports a hit only for rays passing within rounding
// distance of the object, ahead of the origin; the bounds carry a margin far above that.
KDPT_HD bool geom_may_hit(const DevGeom& G, f3 o, f3 invdir) {
  const float t1x = (G.wlo[0] - o.x) * invdir.x, t2x = (G.whi[0] - o.x) * invdir.x;
  const float t1y = (G.wlo[1] - o.y) * invdir.y, t2y = (G.whi[1] - o.y) * invdir.y;
  const float t1z = (G.wlo[2] - o.z) * invdir.z, t2z = (G.whi[2] - o.z) * invdir.z;
  const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  return tmax >= tmin && tmax >= 0.0f;
}

// Entry distance of the ray into the geom's enlarged world bounds: a lower bound of the exact test's t
// whenever that test hits (the bounds' margin, >= 1e-3 x extent + 1e-3, exceeds the exact test's 1e-4
// pull-back along the object-space direction, <= 1e-4 x the largest scale, plus rounding).  false: the
// exact test would miss (as geom_may_hit).
KDPT_HD bool geom_entry_bound(const DevGeom& G, f3 o, f3 invdir, float& lo) {
  const float t1x = (G.wlo[0] - o.x) * invdir.x, t2x = (G.whi[0] - o.x) * invdir.x;
  const float t1y = (G.wlo[1] - o.y) * invdir.y, t2y = (G.whi[1] - o.y) * invdir.y;
  const float t1z = (G.wlo[2] - o.z) * invdir.z, t2z = (G.whi[2] - o.z) * invdir.z;
  const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  lo = tmin;
  return tmax >= tmin && tmax >= 0.0f;
}

struct DevScene {
  const DevGeom* geoms;
  int num_geoms;
  int num_boxes;  // viz_kd: the KD node boxes, stored after the analytic geoms in `geoms`
  const DevMaterial* materials;
  int num_materials;
  int has_obj;
  int num_nodes;
  int root;
  // nodes: 64-byte records [4*i .. 4*i+3] = {minx,miny,minz,maxx}, {maxy,maxz,left,right},
  // {parent,triStart,triSize,axis}, padding; held as integer words (floats as their bits) so
  // that no float move can canonicalise the -1 links
  const int4* nodes;
  const int4* pnodes;  // the same tree as 32-byte NodesPacked records, or null when ineligible
  const int4* dnodes;  // ... and as 16-byte NodesDerived records (boxes derived on the walk), or null
  // triangles: v0 (w = mtlIdx bits), e1 = v1-v0, e2 = v2-v0 (exactly glm's e1/e2)
  const float4* tv0;
  const float4* te1;
  const float4* te2;
  const float4* tn0;
  const float4* tn1;
  const float4* tn2;
  const int* obj_material_offsets;
  // children of nodes[0] and nodes[1] for the hybrid skip line (-1 when absent)
  int n0_left, n0_right, n1_left, n1_right;
  // big leaves (>= BIG_LEAF triangles) as clusters of <= 64 triangles in Morton order, each with its
  // box: leaf_cl[node] = {first cluster, count} (count 0: not big); cl_lo/cl_hi boxes; cl_info =
  // {first triangle, size}; cluster-order copies of v0/e1/e2 with the original index in e1.w, each
  // cluster padded to CLUSTER entries (cluster c = entries [CLUSTER c, CLUSTER (c + 1)); padding: zeros, index -1)
  const int2* leaf_cl;
  int num_clusters;
  // 1 when some big leaf has more clusters than ceil(size / CLUSTER) (normal-cone grouping: balanced runs per
  // cone), so the kernels read each leaf's count from leaf_cl instead of deriving it from the leaf's size
  int cl_counts;
  const float4* cl_lo;
  const float4* cl_hi;
  const int2* cl_info;
  // super-clusters: a big leaf's clusters in runs of SUPER (consecutive in Morton order), as 16-byte records:
  // the box in half precision rounded outward (lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16) and
  // first cluster << 5 | (count - 1); snodes = the NodesDerived records with a big leaf's first super instead
  // of its first cluster (TREE_LDS16S: records and supers in LDS, the two-level cull), or null
  const int4* sup;
  int num_supers;
  // per super-cluster: the unit normal of its triangles' summed area vectors and the largest chord to their
  // unit normals (sup_n = (n, chord)), and the slab [sup_b.x, sup_b.y] of n . (q - c) holding them (c: the
  // centre of the half-precision box); the first cull level tests survivors of the box against it with the
  // direction-dependent margin when sup_slab is set (knob "super_slab")
  const float4* sup_n;
  const float4* sup_b;
  int sup_slab;
  // per cluster: the unit normal of its triangles' summed area vectors (xyz); every point q of its triangles
  // has n . (q - c) in [cl_lo.w, cl_hi.w], c = 0.5f * (lo + hi) (bounds rounded outward); n = 0: no slab.
  // The two-level cull tests the line against this slab as well as the box (knob "cluster_slab")
  const float4* cl_n;
  int cl_slab;
  // ... and the patch's extent along two unit directions u, v in its plane (u: the principal axis of its
  // vertices projected on the plane, v = n x u): cl_u = (u, min u.(q - c)), cl_v = (v, min v.(q - c)),
  // cl_w = (max u.(q - c), max v.(q - c), -, -), bounds rounded outward; with the slab an oriented box the
  // second cull level tests when cl_obb is set (knob "cluster_obb")
  const float4* cl_u;
  const float4* cl_v;
  const float4* cl_w;
  int cl_obb;
  // the one-level route (TREE_LDS / LDS16 / LDS16G...) also tests its box survivors against the cluster's
  // oriented box from HBM (knob "flat_obb")
  int flat_obb;
  // the cull's margin coefficients (kdpt_clusters.h cluster_margin): cl_margin for the box-only tests;
  // the slab level uses cull_margin_dir(): max(cl_margin_lo, min(cl_margin, cull_a / g + cull_c)),
  // g = |n . d| - cl_n.w - cull_b
  float cl_margin, cl_margin_lo, cull_a, cull_b, cull_c;
  // the exact one-level cull (kdpt_clusters.h build_dir_masks): per cluster c and direction bucket b,
  // cl_mask[b * num_clusters + c] = the danger mask over the cluster's 64 entries (bucket-major: a ray's
  // pairs, consecutive clusters of one leaf in one bucket, share cache lines); null: the fast-margin cull
  // (tuning "cull_exact" = 0) or no one-level cull at all
  const unsigned long long* cl_mask;  // [6 mask_n^2][num_clusters] danger masks
  int mask_n;                          // cube-map cells per face edge (dir_bucket)
  // per cluster entry: the triangle's unit normal (float) and 17.5 u rho (the exact cull's per-triangle
  // bound); w = -1: never passes (padding, small degenerate), w = +inf: may pass for any direction
  const float4* cl_tn;
  const int4* snodes;
  const float4* c_v0;
  const float4* c_e1;
  const float4* c_e2;
  float4 rlo, rhi;  // the KD root's box (trace-order classes only; not used for results)
  int trace_mode;   // 1 class+octant, 2 octant, 3 class (experiments)
  int early_walk, early_leaf;  // leaf phase starts when <= early_walk lanes walk and >= early_leaf wait
  int trip_limit;  // bound on node steps per ray (a valid tree needs < 4 per node)
  int* fault;      // set to 1 when a ray exceeds trip_limit (never for a validated tree)
};

struct Ray {
  f3 origin, direction;
  bool isinside;
  float sdepth;
};

KDPT_HD f3 getPointOnRay(const Ray& r, float t) {  // src/intersections.h:30-32
  return add(r.origin, scl(normalize(r.direction), t - .0001f));
}

// src/intersections.h:107-149
KDPT_HD float boxIntersectionTest(const DevGeom& box, const Ray& r, f3& ip, f3& nrm) {
  Ray q;
  q.origin = mulMV(box.inverseTransform, f4{r.origin.x, r.origin.y, r.origin.z, 1.0f});
  q.direction = normalize(mulMV(box.inverseTransform, f4{r.direction.x, r.direction.y, r.direction.z, 0.0f}));
  float tmin = -1e38f, tmax = 1e38f;
  int tmin_axis = -1, tmax_axis = -1;
  float tmin_s = 0.0f, tmax_s = 0.0f;
#pragma unroll
  for (int xyz = 0; xyz < 3; ++xyz) {
    float qd = comp(q.direction, xyz);
    float qo = comp(q.origin, xyz);
    float t1 = (-0.5f - qo) / qd;
    float t2 = (+0.5f - qo) / qd;
    float ta = glm_min(t1, t2);
    float tb = glm_max(t1, t2);
    float ns = t2 < t1 ? +1.0f : -1.0f;
    if (ta > 0 && ta > tmin) { tmin = ta; tmin_axis = xyz; tmin_s = ns; }
    if (tb < tmax) { tmax = tb; tmax_axis = xyz; tmax_s = ns; }
  }
  if (tmax >= tmin && tmax > 0) {
    if (tmin <= 0) { tmin = tmax; tmin_axis = tmax_axis; tmin_s = tmax_s; }
    f3 n = mk3(tmin_axis == 0 ? tmin_s : 0.0f, tmin_axis == 1 ? tmin_s : 0.0f, tmin_axis == 2 ? tmin_s : 0.0f);
    f3 p = getPointOnRay(q, tmin);
    ip = mulMV(box.transform, f4{p.x, p.y, p.z, 1.0f});
    nrm = normalize(mulMV(box.transform, f4{n.x, n.y, n.z, 0.0f}));
    return length(sub(r.origin, ip));
  }
  return -1;
}

// src/intersections.h:161-203
KDPT_HD float sphereIntersectionTest(const DevGeom& sphere, const Ray& r, f3& ip, f3& nrm) {
  float radius = .5f;
  f3 ro = mulMV(sphere.inverseTransform, f4{r.origin.x, r.origin.y, r.origin.z, 1.0f});
  f3 rd = normalize(mulMV(sphere.inverseTransform, f4{r.direction.x, r.direction.y, r.direction.z, 0.0f}));
  Ray rt;
  rt.origin = ro;
  rt.direction = rd;
  float vDotDirection = dot(rt.origin, rt.direction);
  float radicand = vDotDirection * vDotDirection - (dot(rt.origin, rt.origin) - radius * radius);
  if (radicand < 0) return -1;
  float squareRoot = sqrtf(radicand);
  float firstTerm = -vDotDirection;
  float t1 = firstTerm + squareRoot, t2 = firstTerm - squareRoot;
  float t = 0;
  bool outside;
  if (t1 < 0 && t2 < 0) return -1;
  else if (t1 > 0 && t2 > 0) { t = std_min(t1, t2); outside = true; }
  else { t = std_max(t1, t2); outside = false; }
  f3 os = getPointOnRay(rt, t);
  ip = mulMV(sphere.transform, f4{os.x, os.y, os.z, 1.f});
  nrm = normalize(mulMV(sphere.invTranspose, f4{os.x, os.y, os.z, 0.f}));
  if (!outside) nrm = neg(nrm);
  return length(sub(r.origin, ip));
}

// src/intersections.h:253-286 with invdir hoisted per ray (same values)
KDPT_HD bool intersectAABB(f3 o, f3 invdir, float4 b0, float4 b1, float& dist) {
  float v1 = (b0.x - o.x) * invdir.x;
  float v2 = (b0.w - o.x) * invdir.x;
  float v3 = (b0.y - o.y) * invdir.y;
  float v4 = (b1.x - o.y) * invdir.y;
  float v5 = (b0.z - o.z) * invdir.z;
  float v6 = (b1.y - o.z) * invdir.z;
  float dmin = std_max(std_max(std_min(v1, v2), std_min(v3, v4)), std_min(v5, v6));
  float dmax = std_min(std_min(std_max(v1, v2), std_max(v3, v4)), std_max(v5, v6));
  if (dmax < 0) { dist = dmax; return false; }
  if (dmin > dmax) { dist = dmax; return false; }
  dist = dmin;
  return true;
}

#if defined(__HIPCC__) || defined(__HIP__)
// intersectAABB's decision (hit, and dist when hit) with IEEE min/max (v_min3/v_max3).
// Equal to the std::min/max ternaries whenever no product is NaN -- i.e. whenever every
// invdir component is finite -- because the results only feed comparisons (+-0 alike).
__device__ inline bool intersectAABB_fast(f3 o, f3 invdir, float4 b0, float4 b1, float& dist) {
  const float v1 = (b0.x - o.x) * invdir.x, v2 = (b0.w - o.x) * invdir.x;
  const float v3 = (b0.y - o.y) * invdir.y, v4 = (b1.x - o.y) * invdir.y;
  const float v5 = (b0.z - o.z) * invdir.z, v6 = (b1.y - o.z) * invdir.z;
  // v_min/v_max straight from the products: the compiler's fminf/fmaxf would first quiet each input
  // (six v_max x, x, x per node step) although a product is never a signalling NaN
  float l1, l2, l3, h1, h2, h3, dmin, dmax;
  asm("v_min_f32 %0, %1, %2" : "=v"(l1) : "v"(v1), "v"(v2));
  asm("v_min_f32 %0, %1, %2" : "=v"(l2) : "v"(v3), "v"(v4));
  asm("v_min_f32 %0, %1, %2" : "=v"(l3) : "v"(v5), "v"(v6));
  asm("v_max_f32 %0, %1, %2" : "=v"(h1) : "v"(v1), "v"(v2));
  asm("v_max_f32 %0, %1, %2" : "=v"(h2) : "v"(v3), "v"(v4));
  asm("v_max_f32 %0, %1, %2" : "=v"(h3) : "v"(v5), "v"(v6));
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(dmin) : "v"(l1), "v"(l2), "v"(l3));
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(dmax) : "v"(h1), "v"(h2), "v"(h3));
  dist = dmin;
  return !(dmax < 0.0f) && !(dmin > dmax);
}
#endif

struct Hit {
  float t_min;
  int hit_geom_index;
  f3 ip, normal;
  bool obj_intersect;
  int objMaterialIdx;
};

struct TraverseCounters {
  uint32_t aabb, tri, hit;
};

// traverseKDbareShortHybrid (HYBRID) / traverseKDbare, with the compact visited state.  on_leaf(node) is
// called for every leaf whose triangles are tested (host tools: tests/native/cull_diff.cpp --sim).
struct NoLeafHook {
#if defined(__HIPCC__) || defined(__HIP__)
  __host__ __device__
#endif
  void operator()(int) const {}
};
template <bool HYBRID, bool COUNT, typename LeafHook = NoLeafHook>
KDPT_HD void traverseKD(const DevScene& S, const Ray& ray, Hit& h, int material_size, TraverseCounters& cnt,
                        LeafHook on_leaf = LeafHook{}) {
  if (S.num_nodes == 0) return;
  const f3 o = ray.origin, d = ray.direction;
  const f3 invdir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float hit_eps = HYBRID ? 0.0001f : 0.00001f;
  int cur = S.root;
  int L = 0;
  uint32_t cb = 0, ps = 0, g = 0;
  bool rootv = false, sink = false;
  bool hitGeom = false;
  float dist = -1.0f;
  float bz = FLT_MAXV;  // bary.z
  while (true) {
    if (cur == -1) break;
    const int4 q0 = S.nodes[4 * cur];
    const int4 q1 = S.nodes[4 * cur + 1];
    const int4 meta = S.nodes[4 * cur + 2];
    const float4 b0 = make_float4(ibits(q0.x), ibits(q0.y), ibits(q0.z), ibits(q0.w));
    const float4 b1 = make_float4(ibits(q1.x), ibits(q1.y), 0.0f, 0.0f);
    const int left = q1.z, right = q1.w, parent = meta.x;
    const int lvlbit = (L > 0) ? (2 * (L - 1) + (int)((ps >> (L - 1)) & 1u)) : 0;
    const bool curVis = (L == 0) ? rootv : (((cb >> lvlbit) & 1u) != 0u);
    if (!hitGeom && cur == S.root && curVis) break;
    hitGeom = intersectAABB(o, invdir, b0, b1, dist);
    if (COUNT) cnt.aabb++;
    bool up = false;
    if (curVis) {
      up = true;
    } else {
      if (!hitGeom && cur == S.root) break;
      if (!hitGeom || dist > bz) up = true;
    }
    if (up) {
      // nodeIDs[ID] = nodeIDs[leftID] = nodeIDs[rightID] = true; currID = parentID
      if (L == 0) rootv = true; else cb |= 1u << lvlbit;
      if (left == -1) sink = true; else cb |= 1u << (2 * L);
      if (right == -1) sink = true; else cb |= 1u << (2 * L + 1);
      cur = parent;
      L--;
      continue;
    }
    const bool leftFirst = HYBRID ? (comp(d, meta.w) > 0.0f) : true;
    const uint32_t fside = leftFirst ? 0u : 1u;
    const int first = leftFirst ? left : right, second = leftFirst ? right : left;
    int next = -1;
    uint32_t nside = 0;
    if (first != -1 && !((cb >> (2 * L + fside)) & 1u)) { next = first; nside = fside; }
    else if (second != -1 && !((cb >> (2 * L + (fside ^ 1u))) & 1u)) { next = second; nside = fside ^ 1u; }
    if (next != -1) {
      ps = (ps & ~(1u << L)) | (nside << L);
      const uint32_t lv = 2u * (uint32_t)(L + 1);
      cb &= ~(3u << lv);
      if (L == 0 && nside == 0u) cb |= g << 2;  // entering nodes[1]: its children may carry skip marks
      L++;
      cur = next;
      continue;
    }
    // nodeIDs[node->ID] == false here (the visited branch above took the true case)
    if (L == 0) rootv = true; else cb |= 1u << lvlbit;
    const int size = meta.z;
    if (size > 0) {
      on_leaf(cur);
      const int start = meta.y, end = start + size;
      for (int i = start; i < end; i++) {
        const float4 tv = S.tv0[i];
        const float4 e1v = S.te1[i];
        const float4 e2v = S.te2[i];
        const f3 v0 = mk3(tv.x, tv.y, tv.z), e1 = mk3(e1v.x, e1v.y, e1v.z), e2 = mk3(e2v.x, e2v.y, e2v.z);
        if (COUNT) cnt.tri++;
        // glm::intersectRayTriangle (gtx/intersect.inl:37-74)
        const f3 p = cross(d, e2);
        const float a = dot(e1, p);
        if (a < FLT_EPS) continue;
        const float f = 1.0f / a;
        const f3 s = sub(o, v0);
        const float bx = f * dot(s, p);
        if (bx < 0.0f) continue;
        if (bx > 1.0f) continue;
        const f3 q = cross(s, e1);
        const float by = f * dot(d, q);
        if (by < 0.0f) continue;
        if (by + bx > 1.0f) continue;
        bz = f * dot(e2, q);
        if (!(bz >= 0.0f)) continue;
        if (COUNT) cnt.hit++;
        if (HYBRID) {
          // nodeIDs[nodes[nodeIDs[node->parentID]].(right|left)ID] = true
          const bool parVis = (L == 0) ? sink
                              : (L == 1 ? rootv
                                        : (((cb >> (2 * (L - 2) + (int)((ps >> (L - 2)) & 1u))) & 1u) != 0u));
          const int b = parVis ? 1 : 0;
          int target = -1;
          if (b < S.num_nodes) target = (b == 0) ? (leftFirst ? S.n0_right : S.n0_left) : (leftFirst ? S.n1_right : S.n1_left);
          if (target == -1) {
            sink = true;
          } else if (b == 0) {
            cb |= 1u << (leftFirst ? 1 : 0);
          } else {
            const uint32_t bit = leftFirst ? 1u : 0u;
            if (L >= 1 && (ps & 1u) == 0u) cb |= 1u << (2 + bit);
            else g |= 1u << bit;
          }
        }
        const float4 n1v = S.tn0[i], n2v = S.tn1[i], n3v = S.tn2[i];
        const int mtl = fbits(tv.w);
        h.objMaterialIdx = mtl + material_size - 1;
        f3 hit = add(o, scl(d, bz));
        const float w0 = 1 - bx - by;
        const f3 norm = normalize(add(add(scl(mk3(n1v.x, n1v.y, n1v.z), w0), scl(mk3(n2v.x, n2v.y, n2v.z), bx)),
                                      scl(mk3(n3v.x, n3v.y, n3v.z), by)));
        hit = add(hit, scl(norm, hit_eps));
        const float t = distance(o, hit);
        if (t > 0.0f && h.t_min > t) {
          h.t_min = t;
          h.hit_geom_index = S.obj_material_offsets[mtl];
          h.ip = hit;
          h.normal = norm;
          h.obj_intersect = true;
        }
      }
    }
    // stay on this node: the next trip finds it visited and climbs
  }
}

// glm::intersectRayTriangle on (o, d) and triangle i; returns 0 = miss before the u/v
// tests passed, 1 = passed u/v but t < 0 (bary.z still written), 2 = intersected.
struct TriData {
  float4 v0, e1, e2;
};
KDPT_HD int tri_test_v(const TriData& T, f3 o, f3 d, float& bx, float& by, float& bz) {
  const float4 tv = T.v0, e1v = T.e1, e2v = T.e2;
  const f3 v0 = mk3(tv.x, tv.y, tv.z), e1 = mk3(e1v.x, e1v.y, e1v.z), e2 = mk3(e2v.x, e2v.y, e2v.z);
  const f3 p = cross(d, e2);
  const float a = dot(e1, p);
  if (a < FLT_EPS) return 0;
  const float f = 1.0f / a;
  const f3 s = sub(o, v0);
  bx = f * dot(s, p);
  if (bx < 0.0f) return 0;
  if (bx > 1.0f) return 0;
  const f3 q = cross(s, e1);
  by = f * dot(d, q);
  if (by < 0.0f) return 0;
  if (by + bx > 1.0f) return 0;
  bz = f * dot(e2, q);
  return (bz >= 0.0f) ? 2 : 1;
}

// ---------------------------------------------------------------------------
// Big leaves (>= BIG_LEAF triangles) are swept in clusters of 64; the C5 route groups SUPER clusters under
// one half-precision box.  The cluster cull below is host-compilable so that tests/native/cull_diff.cpp
// can check it against tri_test_v on adversarial lines ("Cluster cull").
// ---------------------------------------------------------------------------
#ifndef KDPT_CLUSTER
#define KDPT_CLUSTER 64  // tools/build_variant.sh experiments only (64 or 32)
#endif
constexpr int CLUSTER = KDPT_CLUSTER;  // triangles per cluster (a sweep tests 64 / CLUSTER clusters at once)
static_assert(CLUSTER == 64 || CLUSTER == 32, "cluster size");
#ifndef KDPT_SUPER
#define KDPT_SUPER (1024 / KDPT_CLUSTER)  // tools/build_variant.sh experiments only (a power of two <= 32)
#endif
constexpr int SUPER = KDPT_SUPER;  // clusters per super-cluster
#ifndef KDPT_BIG_LEAF
#define KDPT_BIG_LEAF 48  // tools/build_variant.sh experiments only
#endif
constexpr int BIG_LEAF = KDPT_BIG_LEAF;  // leaves this size or larger are tested cluster by cluster

// IEEE half bits -> float (exact).  The device converts in one instruction; g++ 11 has no _Float16.
KDPT_HD float half_to_float(uint32_t h) {
#if defined(__clang__)
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(h & 0xffffu));
#else
  const uint32_t s = (h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  uint32_t b;
  if (e == 0x1fu) b = s | 0x7f800000u | (m << 13);
  else if (e) b = s | ((e + 112u) << 23) | (m << 13);
  else if (!m) b = s;
  else {  // subnormal half: m x 2^-24, exact in float
    const float v = (float)m * 5.9604644775390625e-8f;
    return s ? -v : v;
  }
  float f;
  memcpy(&f, &b, 4);
  return f;
#endif
}
KDPT_HD float half_lo(uint32_t w) { return half_to_float(w & 0xffffu); }
KDPT_HD float half_hi(uint32_t w) { return half_to_float(w >> 16); }

// May the LINE through o (both directions: glm's u/v tests ignore the sign of t) cross the cluster's
// triangles?  The box is widened by 1e-4 x (distance + size), orders of magnitude above the rounding
// of the Moller-Trumbore u/v tests, so a culled cluster holds no triangle that would pass them.
KDPT_HD bool cluster_may_pass(float4 lo, float4 hi, f3 o, f3 inv, float K) {
  const float cx = 0.5f * (lo.x + hi.x), cy = 0.5f * (lo.y + hi.y), cz = 0.5f * (lo.z + hi.z);
  const float m = K * (1.0f + fabsf(o.x - cx) + fabsf(o.y - cy) + fabsf(o.z - cz) + (hi.x - lo.x) +
                           (hi.y - lo.y) + (hi.z - lo.z));
  const float t1x = (lo.x - m - o.x) * inv.x, t2x = (hi.x + m - o.x) * inv.x;
  const float t1y = (lo.y - m - o.y) * inv.y, t2y = (hi.y + m - o.y) * inv.y;
  const float t1z = (lo.z - m - o.z) * inv.z, t2z = (hi.z + m - o.z) * inv.z;
  const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  return tmin <= tmax;
}

// The margin coefficient of the slab level for a line of direction d and a cluster of normal n (n.w = the
// largest chord |N_t / |N_t| - n| over the cluster's triangles): glm's determinant of every triangle t of the
// cluster is then at least |N_t| (|n . d| - n.w - cull_b), which bounds the float u/v error and so the margin a
// u/v pass can need ("Cluster cull"); min with the direction-free rigorous cl_margin, max with
// the fast floor cl_margin_lo.  A line nearly parallel to the cluster's patch gets the direction-free one.
struct CullK {
  float hi, lo, a, b, c;  // DevScene::cl_margin, cl_margin_lo, cull_a, cull_b, cull_c
};
KDPT_HD float cull_margin_dir(float nd, float spread, const CullK& k) {
  const float g = fabsf(nd) - spread - k.b;
  const float kd = g > 0.0f ? k.a / g + k.c : k.hi;
  return fmaxf(k.lo, fminf(k.hi, kd));
}

// cluster_may_pass and the cluster's slab {q : n . (q - c) in [lo.w, hi.w]}: the line's parameter interval
// through the slab, widened by the same margin, must meet its interval through the box.  A triangle the line
// crosses has its crossing point in both (a convex combination of its vertices), so the cull stays
// conservative; a line (nearly) parallel to the slab passes it.  A curved-surface patch is thin along its
// normal, so a line that only grazes the patch's box is culled.
KDPT_HD bool cluster_may_pass_slab(float4 lo, float4 hi, float4 n, f3 o, f3 inv, f3 d, const CullK& k) {
  const float nd = n.x * d.x + n.y * d.y + n.z * d.z;
  const float K = cull_margin_dir(nd, n.w, k);
  const float cx = 0.5f * (lo.x + hi.x), cy = 0.5f * (lo.y + hi.y), cz = 0.5f * (lo.z + hi.z);
  const float m = K * (1.0f + fabsf(o.x - cx) + fabsf(o.y - cy) + fabsf(o.z - cz) + (hi.x - lo.x) +
                           (hi.y - lo.y) + (hi.z - lo.z));
  const float t1x = (lo.x - m - o.x) * inv.x, t2x = (hi.x + m - o.x) * inv.x;
  const float t1y = (lo.y - m - o.y) * inv.y, t2y = (hi.y + m - o.y) * inv.y;
  const float t1z = (lo.z - m - o.z) * inv.z, t2z = (hi.z + m - o.z) * inv.z;
  float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  const float no = n.x * (o.x - cx) + n.y * (o.y - cy) + n.z * (o.z - cz);
  if (fabsf(nd) > 1e-12f) {
    const float rn = 1.0f / nd;
    const float s1 = (lo.w - m - no) * rn, s2 = (hi.w + m - no) * rn;
    tmin = fmaxf(tmin, fminf(s1, s2));
    tmax = fminf(tmax, fmaxf(s1, s2));
  }
  return tmin <= tmax;
}

// cluster_may_pass_slab and the patch's u and v slabs: the line's interval through the cluster's oriented box
// (n, u, v) must meet its interval through the axis-aligned one, every slab widened by the same margin.  A
// point the float u/v tests accept lies within the margin of the line and inside every one of them, so the
// cull stays as conservative as the box alone.
KDPT_HD void slab_clip(float lo, float hi, float m, float sd, float so, float& tmin, float& tmax) {
  if (fabsf(sd) > 1e-12f) {
    const float rs = 1.0f / sd;
    const float s1 = (lo - m - so) * rs, s2 = (hi + m - so) * rs;
    tmin = fmaxf(tmin, fminf(s1, s2));
    tmax = fminf(tmax, fmaxf(s1, s2));
  }
}
KDPT_HD bool cluster_may_pass_obb_k(float4 lo, float4 hi, float4 n, float4 u, float4 v, float4 w, f3 o, f3 inv, f3 d,
                                    float nd, float K) {
  const float cx = 0.5f * (lo.x + hi.x), cy = 0.5f * (lo.y + hi.y), cz = 0.5f * (lo.z + hi.z);
  const float m = K * (1.0f + fabsf(o.x - cx) + fabsf(o.y - cy) + fabsf(o.z - cz) + (hi.x - lo.x) +
                           (hi.y - lo.y) + (hi.z - lo.z));
  const float t1x = (lo.x - m - o.x) * inv.x, t2x = (hi.x + m - o.x) * inv.x;
  const float t1y = (lo.y - m - o.y) * inv.y, t2y = (hi.y + m - o.y) * inv.y;
  const float t1z = (lo.z - m - o.z) * inv.z, t2z = (hi.z + m - o.z) * inv.z;
  float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  const float ox = o.x - cx, oy = o.y - cy, oz = o.z - cz;
  slab_clip(lo.w, hi.w, m, nd, n.x * ox + n.y * oy + n.z * oz, tmin, tmax);
  slab_clip(u.w, w.x, m, u.x * d.x + u.y * d.y + u.z * d.z, u.x * ox + u.y * oy + u.z * oz, tmin, tmax);
  slab_clip(v.w, w.y, m, v.x * d.x + v.y * d.y + v.z * d.z, v.x * ox + v.y * oy + v.z * oz, tmin, tmax);
  return tmin <= tmax;
}
KDPT_HD bool cluster_may_pass_obb(float4 lo, float4 hi, float4 n, float4 u, float4 v, float4 w, f3 o, f3 inv, f3 d,
                                  const CullK& k) {
  const float nd = n.x * d.x + n.y * d.y + n.z * d.z;
  return cluster_may_pass_obb_k(lo, hi, n, u, v, w, o, inv, d, nd, cull_margin_dir(nd, n.w, k));
}

// Direction buckets of the exact one-level cull (kdpt_clusters.h build_dir_masks): a cube map of n x n cells
// per face.  The face is the largest |component| (ties: x before y before z), (u, v) the other two components
// over it, cell (floor((u + 1) n / 2), floor((v + 1) n / 2)) clamped to n - 1.  The host bounds each cell's
// directions (grown by 1e-5 in u and v, far above this function's rounding), so any float d maps to a cell
// whose bound holds it.  Any finite nonzero d works (the cull only runs for lanes whose 1 / d components are
// all finite).
// 1 / x for box_miss and dir_bucket: the hardware reciprocal (1 ulp) on the device, the division on the host;
// box_miss's 1e-5 slack and the masks' 1e-5 cell growth cover either.  A float within 1 ulp of 1 / x is the
// rounded quotient or one of its two neighbours: the cull harness (tests/native/cull_diff.cpp, KDPT_RCP_ULP)
// evaluates every line with each of the three.
#if !defined(__HIP_DEVICE_COMPILE__) && defined(KDPT_RCP_ULP)
extern thread_local int kdpt_rcp_ulp;  // -1, 0, +1: the host quotient moved by that many ulps
#endif
KDPT_HD float kd_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#elif defined(KDPT_RCP_ULP)
  const float r = 1.0f / x;
  return kdpt_rcp_ulp == 0 ? r : std::nextafter(r, kdpt_rcp_ulp > 0 ? HUGE_VALF : -HUGE_VALF);
#else
  return 1.0f / x;
#endif
}
KDPT_HD int dir_bucket(f3 d, int n) {
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  int face;
  float a, b, m;
  if (ax >= ay && ax >= az) {
    face = d.x > 0.0f ? 0 : 1;
    a = d.y;
    b = d.z;
    m = ax;
  } else if (ay >= az) {
    face = d.y > 0.0f ? 2 : 3;
    a = d.x;
    b = d.z;
    m = ay;
  } else {
    face = d.z > 0.0f ? 4 : 5;
    a = d.x;
    b = d.y;
    m = az;
  }
  const float h = 0.5f * (float)n * kd_rcp(m);
  int i = (int)((a + m) * h), j = (int)((b + m) * h);
  i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
  j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
  return (face * n + j) * n + i;
}

// How far the LINE through o (direction 1 / inv, every component finite) misses the box [lo, hi], in the units
// of cluster_may_pass's margin coefficient: the smallest K for which cluster_may_pass(lo, hi, o, inv, K) holds.
// With the margin m = K W (W = 1 + |o - c|_1 + size_1), each slab's parameter interval [a_i, b_i] grows by
// m |inv_i| at both ends, so the intervals meet once m >= (a_i - b_j) / (|inv_i| + |inv_j|) for every pair of
// axes.  The line's distance from the box is at least that m (an L-infinity distance), so a point the float u/v
// tests accept lies within K_t W of the line only if K_t >= the result.  Rounded down by 1e-5 relative; 0 when
// the line meets the box.
KDPT_HD float box_miss(float4 lo, float4 hi, f3 o, f3 inv) {
  const float cx = 0.5f * (lo.x + hi.x), cy = 0.5f * (lo.y + hi.y), cz = 0.5f * (lo.z + hi.z);
  const float W = 1.0f + fabsf(o.x - cx) + fabsf(o.y - cy) + fabsf(o.z - cz) + (hi.x - lo.x) + (hi.y - lo.y) +
                  (hi.z - lo.z);
  const float tlx = (lo.x - o.x) * inv.x, thx = (hi.x - o.x) * inv.x;
  const float tly = (lo.y - o.y) * inv.y, thy = (hi.y - o.y) * inv.y;
  const float tlz = (lo.z - o.z) * inv.z, thz = (hi.z - o.z) * inv.z;
  const float ax = fminf(tlx, thx), bx = fmaxf(tlx, thx), ay = fminf(tly, thy), by = fmaxf(tly, thy);
  const float az = fminf(tlz, thz), bz = fmaxf(tlz, thz);
  const float wx = fabsf(inv.x), wy = fabsf(inv.y), wz = fabsf(inv.z);
  const float mxy = fmaxf(ax - by, ay - bx) * kd_rcp(wx + wy);
  const float mxz = fmaxf(ax - bz, az - bx) * kd_rcp(wx + wz);
  const float myz = fmaxf(ay - bz, az - by) * kd_rcp(wy + wz);
  const float m = fmaxf(0.0f, fmaxf(mxy, fmaxf(mxz, myz)));
  return m * kd_rcp(W) * 0.99999f;
}

// The exact cull's per-triangle decision for a (line, cluster) pair whose line misses the cluster's box by D
// (box_miss): may triangle tn (its float unit normal, w = 17.5 u rho, the u/v error coefficient; w < 0: never
// passes; w = +inf: may pass for any line) pass glm's u/v tests?  Its float determinant is below -|N| (N . d -
// beta) with beta = 5.8 u rho (1 + 1e-3) + 40 u (+ the float normal's and nd's rounding), so it cannot pass when
// nd > beta (back-facing); otherwise a passing point lies within K_t = w / g + c (times the margin's distance
// term) of the line, g = -nd - beta ("Cluster cull"), which needs K_t >= D, i.e. w >= (D - c) g.
// g <= 0: no bound, the triangle is tested.
KDPT_HD bool danger_needs_test(float4 tn, f3 d, float D, float c) {
  if (!(tn.w >= 0.0f)) return false;
  const float nd = tn.x * d.x + tn.y * d.y + tn.z * d.z;
  const float beta = 0.3318f * tn.w + 3.5e-6f;
  if (nd > beta) return false;
  const float g = -nd - beta;
  return !(g > 0.0f) || tn.w * 1.00001f >= (D - c) * g;
}

// One (bucket, cluster) cell of the masked cull (kdpt_clusters.h build_dir_masks on the host and k_build_masks on
// the device run this same code, -ffp-contract=off, so both give the same bits).  Per entry k of the cluster: its
// unit normal n_k, beta_k and dthr_k (kdpt_clusters.h mask_entries) and its rigorous coefficient krig_k; the
// bucket: its centre direction D[0..2] and radius D[3].  Entry k is in the danger mask when some direction of the
// bucket makes it front-facing (n_k . d <= beta_k) and needing more than Kf (n_k . d >= dthr_k), and its own
// direction-free rigorous coefficient K_t = 8.75 |e1||e2| + c exceeds Kf (a line glm's float u/v tests accept for
// t passes within K_t W of any region holding t -- DESIGN.md 4, "Cluster cull" -- so a pair that missed the box
// or the oriented box at Kf >= K_t cannot need t).
KDPT_HD unsigned long long dir_mask_cell(const double* nx, const double* ny, const double* nz, const double* beta,
                                         const double* dthr, const float* krig, const double* D, float Kf) {
  unsigned long long md = 0ull;
  for (int k = 0; k < 64; k++) {
    const double x = nx[k] * D[0] + ny[k] * D[1] + nz[k] * D[2];
    if (x - D[3] <= beta[k] && x + D[3] >= dthr[k] && krig[k] > Kf) md |= 1ull << k;
  }
  return md;
}

#if defined(__HIPCC__) || defined(__HIP__)
// ---------------------------------------------------------------------------
// Wave-cooperative form of traverseKD for gfx950 (64-lane waves).
//
// The per-ray algorithm and visited state are exactly traverseKD's; only the
// SIMT schedule changes ("while-while"): a node phase advances every lane until
// it reaches a leaf whose triangles must be tested (or finishes), then a leaf
// phase spreads ALL (ray, triangle) pairs of the lanes sitting on leaves over the
// 64 lanes.  A leaf's triangle tests are independent of each other; their
// sequential effects are recombined per ray through LDS:
//   bary.z        = that of the LAST triangle (in leaf order) passing the u/v tests
//   objMaterialIdx= mtlIdx of the LAST intersected triangle
//   hit record    = FIRST triangle reaching the minimum t with t > 0 && t_min > t
//   skip marks    = applied min(#intersected, 2) times (idempotent from the 2nd on)
// ---------------------------------------------------------------------------
// Trace-order class of a ray (a scheduling key only -- results never depend on it): rays that start
// inside the KD root's box first (they walk the dense part of the tree), then rays that cross it, then
// rays that miss it; within a class by direction octant so that a wave's rays step alike.
constexpr int TRACE_KEYS = 24;
__device__ inline int trace_class(const DevScene& S, f3 o, f3 d) {
  const float4 lo = S.rlo, hi = S.rhi;
  const bool inside = o.x >= lo.x && o.x <= hi.x && o.y >= lo.y && o.y <= hi.y && o.z >= lo.z && o.z <= hi.z;
  const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
  const float t1x = (lo.x - o.x) * ix, t2x = (hi.x - o.x) * ix;
  const float t1y = (lo.y - o.y) * iy, t2y = (hi.y - o.y) * iy;
  const float t1z = (lo.z - o.z) * iz, t2z = (hi.z - o.z) * iz;
  const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  const int cls = inside ? 0 : ((tmax >= tmin && tmax >= 0.0f) ? 1 : 2);
  const int oct = (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0);
  return S.trace_mode == 2 ? oct : (S.trace_mode == 3 ? cls : cls * 8 + oct);
}

// ---------------------------------------------------------------------------
// Node sources.  The traversal reads one node per step; where it reads it from
// is a template parameter:
//   NodesWide   : 64-byte records in HBM (any tree the validator accepts)
//   NodesPacked : 32-byte records (4 per 128-byte line), in HBM or -- when the
//                 kernel has copied the tree there -- in LDS.  Packing:
//     w0..w5 = min.xyz, max.xyz (float bits)
//     w6     = left | right << 16 (0xffff = -1), or triStart for a leaf with triangles
//     w7     = parent (16 bits, 0xffff = -1) | axis << 16 | hasTris << 18 | triSize << 19 (leaf with
//              triangles), else hasLeft << 19 | hasRight << 20 (the node step reads them as one field)
//   eligible when num_nodes < 65535, axis in 0..2, and every node with triangles
//   is childless with triSize < 8192 (checked on the host, else NodesWide).
// ---------------------------------------------------------------------------
struct NodeRec {
  float4 b0;     // min.xyz, max.x
  float4 b1;     // max.y, max.z, -, -
  int left, right, parent, axis, triStart, triSize;  // left / right: child index when hasL / hasR
  bool hasL, hasR;
  uint32_t has;  // hasL | hasR << 1
  bool tris;     // triSize > 0
  // NodesDerived only: the value both children write into their copy of this box (the centre along
  // `axis`), the value of the box coordinate this node changed in its parent's box, and that coordinate's
  // slot kc (0-2 min.xyz, 3-5 max.xyz; 7 for the root)
  float center, restore;
  uint32_t kc;
};

struct NodesWide {
  static constexpr bool kLeafHoldsCluster = false;  // big leaves: clusters from DevScene::leaf_cl
  static constexpr bool kDerivedBox = false;        // the record holds the node's box
  const int4* p;
  __device__ NodeRec operator()(int i) const {
    const int4 q0 = p[4 * i], q1 = p[4 * i + 1], q2 = p[4 * i + 2];
    NodeRec r;
    r.b0 = make_float4(ibits(q0.x), ibits(q0.y), ibits(q0.z), ibits(q0.w));
    r.b1 = make_float4(ibits(q1.x), ibits(q1.y), 0.0f, 0.0f);
    r.left = q1.z;
    r.right = q1.w;
    r.hasL = q1.z != -1;
    r.hasR = q1.w != -1;
    r.has = (r.hasL ? 1u : 0u) | (r.hasR ? 2u : 0u);
    r.parent = q2.x;
    r.triStart = q2.y;
    r.triSize = q2.z;
    r.tris = r.triSize > 0;
    r.axis = q2.w;
    return r;
  }
};

__device__ inline int link16(uint32_t v) { return v == 0xffffu ? -1 : (int)v; }

struct NodesPacked {
  static constexpr bool kLeafHoldsCluster = true;  // big leaves: triStart holds the first cluster
  static constexpr bool kDerivedBox = false;
  const int4* p;  // global or LDS (address space inferred after inlining)
  __device__ NodeRec operator()(int i) const {
    // two 16-byte vector loads (as int4 fields the compiler reads the record in four pieces)
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i q0 = reinterpret_cast<const v4i*>(p)[2 * i], q1 = reinterpret_cast<const v4i*>(p)[2 * i + 1];
    NodeRec r;
    r.b0 = make_float4(ibits(q0.x), ibits(q0.y), ibits(q0.z), ibits(q0.w));
    r.b1 = make_float4(ibits(q1.x), ibits(q1.y), 0.0f, 0.0f);
    const uint32_t w6 = (uint32_t)q1.z, w7 = (uint32_t)q1.w;
    const bool tris = (w7 >> 18) & 1u;
    r.left = (int)(w6 & 0xffffu);  // raw: only read when hasL / hasR
    r.right = (int)(w6 >> 16);
    r.has = tris ? 0u : (w7 >> 19) & 3u;
    r.hasL = (r.has & 1u) != 0u;
    r.hasR = (r.has & 2u) != 0u;
    r.tris = tris;
    r.parent = link16(w7 & 0xffffu);
    r.axis = (int)((w7 >> 16) & 3u);
    r.triStart = (int)w6;
    r.triSize = tris ? (int)(w7 >> 19) : 0;
    return r;
  }
};

// NodesDerived: 16-byte records (LDS), half of NodesPacked, so that two intersect workgroups share a CU and
// the C5 icosphere's tree fits in LDS.  The reference's builder gives every child its parent's box with ONE
// coordinate replaced by the parent's centre along the parent's axis (src/KDnode.cpp:209-213,235-239: max
// for the left child, min for the right), and the traversal only ever moves parent <-> child, so a lane
// keeps the current node's box in registers and updates that one coordinate per move -- the same float
// bits the record would have held (kdpt_create checks the derivation on every node, else no NodesDerived).
//     w0 = restore: the parent's value of the coordinate this node replaced (climbing puts it back)
//     w1 = centre along axis (the value a descent writes), or the first triangle / cluster of a leaf
//     w2 = left | right << 16 (0xffff = -1), or triSize of a leaf with triangles
//     w3 = parent (16 bits) | axis << 16 | hasTris << 18 | hasLeft << 19 | hasRight << 20 | kc << 21
struct NodesDerived {
  static constexpr bool kLeafHoldsCluster = true;
  static constexpr bool kDerivedBox = true;
  const int4* p;
  __device__ NodeRec operator()(int i) const {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i q = reinterpret_cast<const v4i*>(p)[i];  // one 16-byte load
    const uint32_t w2 = (uint32_t)q.z, w3 = (uint32_t)q.w;
    const bool tris = (w3 >> 18) & 1u;
    NodeRec r;
    r.b0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    r.b1 = r.b0;
    r.restore = ibits(q.x);
    r.center = ibits(q.y);
    r.triStart = q.y;
    r.left = (int)(w2 & 0xffffu);  // raw: only read when hasL / hasR
    r.right = (int)(w2 >> 16);
    r.triSize = tris ? (int)w2 : 0;
    r.has = tris ? 0u : (w3 >> 19) & 3u;
    r.hasL = (r.has & 1u) != 0u;
    r.hasR = (r.has & 2u) != 0u;
    r.tris = tris;
    r.parent = link16(w3 & 0xffffu);
    r.axis = (int)((w3 >> 16) & 3u);
    r.kc = (w3 >> 21) & 7u;
    return r;
  }
};

// wave-profile slots (count mode): trips / cycles of each part of the intersect kernel
enum ProfSlot {
  PROF_NODE_TRIPS, PROF_NODE_CYC, PROF_BIG_SWEEPS, PROF_BIG_CYC, PROF_SMALL_PHASES, PROF_SMALL_ROUNDS,
  PROF_SMALL_CYC, PROF_FINAL_CYC, PROF_SETUP_CYC, PROF_GEOM_CYC, PROF_POST_CYC, PROF_SPARE,
  PROF_BIG_LEAVES, PROF_BIG_CLUSTERS, PROF_BIG_PASS, PROF_BIG_MULTI, PROF_SMALL_PAIRS, PROF_NODE_LEAFWAIT,
  PROF_NODE_DONE, PROF_TAIL_CYC, PROF_TAIL_NODE_DONE, PROF_BIG_SUPERS, PROF_BIG_CULL_CYC, PROF_SLOTS
};

// Cluster boxes of the big leaves: separate lo/hi arrays (HBM) or interleaved lo, hi (LDS copy).
struct ClustersSplit {
  static constexpr bool kSuper = false;
  const float4* lo;
  const float4* hi;
  __device__ float4 lo_of(int c) const { return lo[c]; }
  __device__ float4 hi_of(int c) const { return hi[c]; }
};
struct ClustersInterleaved {
  static constexpr bool kSuper = false;
  const float4* p;
  __device__ float4 lo_of(int c) const { return p[2 * c]; }
  __device__ float4 hi_of(int c) const { return p[2 * c + 1]; }
};
// Two-level: the super-cluster records in LDS (16 bytes: half-precision box rounded outward, first cluster
// and count), the cluster boxes in HBM/L2.
struct ClustersSuper {
  static constexpr bool kSuper = true;
  const int4* sp;
  const float4* lo;
  const float4* hi;
  const float4* n;  // slab normals (DevScene::cl_n)
  const float4* u;  // the oriented box's in-plane slabs (DevScene::cl_u, cl_v, cl_w)
  const float4* v;
  const float4* w;
  __device__ float4 n_of(int c) const { return n[c]; }
  // box of super k, and its first cluster << 5 | count - 1
  __device__ uint32_t sup(int k, float4& l, float4& h) const {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i q = reinterpret_cast<const v4i*>(sp)[k];  // one 16-byte LDS load
    const uint32_t w0 = (uint32_t)q.x, w1 = (uint32_t)q.y, w2 = (uint32_t)q.z;
    l = make_float4(half_lo(w0), half_hi(w0), half_lo(w1), 0.0f);
    h = make_float4(half_hi(w1), half_lo(w2), half_hi(w2), 0.0f);
    return (uint32_t)q.w;
  }
  __device__ float4 lo_of(int c) const { return lo[c]; }
  __device__ float4 hi_of(int c) const { return hi[c]; }
};

struct WaveLeafLDS {
  int slot[64];    // pair_owner's scatter slots (all zero between calls)
  int tbase[64];   // item (cluster / triangle) index = tbase[owner] + pair index
  float4 od[64];   // ray origin.xyz, direction.x
  float2 dd[64];   // direction.y, direction.z
  unsigned long long lastPass[64];  // ((tri + 1) << 32) | bary.z bits, max
  int lastHit[64];
  int nhit[64];
  unsigned long long best[64];  // (t bits << 32) | triangle index, min
};

// Count mode only (the counting intersect kernel allocates one per wave, the others one unused record, so
// their LDS stays small enough for a shading workgroup to share the CU), kept by lane 0: slots PROF_*,
// the wave's clock when its ray queue ran dry, last timestamp.
struct WaveProf {
  unsigned long long prof[PROF_SLOTS];
  unsigned long long tail_t0;
  unsigned long long tlast;
};

__device__ inline void prof_add(WaveProf* P, int k, unsigned long long v) {
  if ((threadIdx.x & 63) == 0) P->prof[k] += v;
}
__device__ inline void prof_lap(WaveProf* P, int k) {  // cycles since the last lap into prof[k]
  const unsigned long long now = __builtin_readcyclecounter();
  if ((threadIdx.x & 63) == 0) {
    if (k >= 0) P->prof[k] += now - P->tlast;
    P->tlast = now;
  }
}


// number of set bits of mask below this lane
__device__ inline unsigned int lane_prefix(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__device__ inline float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Whole-wave reductions on DPP lane moves (VALU only; HIP's __shfl_* are ds_bpermute, an LDS round trip per
// step).  quad_perm xor 1 and xor 2, then the half-row and row mirrors give every lane its 16-lane row's
// result; row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the lower rows into row 3, so lane 63
// ends with the whole wave's, read into a scalar register.  Every lane of the wave must be active.
template <int CTRL, int ROWS>
__device__ inline uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ inline unsigned long long dpp_u64(unsigned long long v) {
  return ((unsigned long long)dpp_u32<CTRL, ROWS>((uint32_t)(v >> 32)) << 32) | dpp_u32<CTRL, ROWS>((uint32_t)v);
}
__device__ inline unsigned long long readlane_u64(unsigned long long v, int lane) {
  return ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
}
__device__ inline unsigned long long lane63_u64(unsigned long long v) {
  return ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}
#define KDPT_WAVE_REDUCE(STEP) STEP(0xB1, 0xF) STEP(0x4E, 0xF) STEP(0x141, 0xF) STEP(0x140, 0xF) \
                               STEP(0x142, 0xA) STEP(0x143, 0xC)

// Inclusive prefix sum / max over the wave on DPP row shifts and row broadcasts (VALU only): shr 1, 2, 4, 8
// within each 16-lane row, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the rows below.
// Lanes whose source is outside the row, or rows the row mask leaves out, add the identity 0 (values >= 0
// for the max).  Every lane of the wave must be active.
template <bool MAX>
__device__ inline int wave_incl_scan(int v) {
#define KDPT_SCAN(C, R)                                                   \
  {                                                                       \
    const int o = __builtin_amdgcn_update_dpp(0, v, C, R, 0xF, false);    \
    v = MAX ? max(v, o) : v + o;                                          \
  }
  KDPT_SCAN(0x111, 0xF) KDPT_SCAN(0x112, 0xF) KDPT_SCAN(0x114, 0xF) KDPT_SCAN(0x118, 0xF)
  KDPT_SCAN(0x142, 0xA) KDPT_SCAN(0x143, 0xC)
#undef KDPT_SCAN
  return v;
}

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#define KDPT_STEP(C, R) { const unsigned long long o = dpp_u64<C, R>(v); v = o < v ? o : v; }
  KDPT_WAVE_REDUCE(KDPT_STEP)
#undef KDPT_STEP
  return lane63_u64(v);
}

__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#define KDPT_STEP(C, R) { const unsigned long long o = dpp_u64<C, R>(v); v = o > v ? o : v; }
  KDPT_WAVE_REDUCE(KDPT_STEP)
#undef KDPT_STEP
  return lane63_u64(v);
}
__device__ inline int wave_max_i32(int v) {
#define KDPT_STEP(C, R) v = max(v, (int)dpp_u32<C, R>((uint32_t)v));
  KDPT_WAVE_REDUCE(KDPT_STEP)
#undef KDPT_STEP
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline float bpermute_f(float v, int src_lane) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_lane << 2, __float_as_int(v)));
}

// Position of the j-th (0-based) set bit of m (j < popcount(m)): a 6-step bisection on popcounts.
__device__ inline int select_bit(unsigned long long m, int j) {
  uint32_t x = (uint32_t)m;
  int base = 0, c = __popc(x);
  if (j >= c) {
    j -= c;
    x = (uint32_t)(m >> 32);
    base = 32;
  }
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    c = __popc(x & ((1u << w) - 1u));
    if (j >= c) {
      j -= c;
      x >>= w;
      base += w;
    }
  }
  return base;
}

// Owner lane of pair B + lane in a flattened (lane, item) enumeration where lane L owns pairs
// [excl_L, excl_L + cnt_L) (lanes in order, so starts increase with L).  The segment starts inside the
// window [B, B + 64) are scattered into slot[] (lane + 1), an inclusive max-scan fills the gaps, and a
// window position no start precedes belongs to the previous window's last owner (carry, updated).  Replaces
// a 6-step binary search (6 dependent LDS reads) by one LDS round trip plus DPP.  Wave-uniform call; slot[]
// is all zero on entry and on exit.
__device__ inline int pair_owner(int* slot, int excl, int cnt, int B, int& carry) {
  const int lane = threadIdx.x & 63;
  const int rel = excl - B;
  const bool mine = cnt > 0 && rel >= 0 && rel < 64;
  if (mine) slot[rel] = lane + 1;
  wave_lds_sync();
  const int v = wave_incl_scan<true>(slot[lane]);
  if (mine) slot[rel] = 0;  // after the read above (same wave: LDS operations stay in order)
  const int own = v > 0 ? v - 1 : carry;
  carry = __builtin_amdgcn_readlane(own, 63);
  return own;
}

__device__ inline TriData tri_load(const DevScene& S, int i) { return TriData{S.tv0[i], S.te1[i], S.te2[i]}; }


__device__ inline int tri_test(const DevScene& S, int i, f3 o, f3 d, float& bx, float& by, float& bz) {
  return tri_test_v(tri_load(S, i), o, d, bx, by, bz);
}


template <bool HYBRID>
__device__ inline float tri_hit_t_n(float4 n1v, float4 n2v, float4 n3v, f3 o, f3 d, float bx, float by, float bz,
                                    f3& hit, f3& norm) {
  const float w0 = 1 - bx - by;
  norm = normalize(add(add(scl(mk3(n1v.x, n1v.y, n1v.z), w0), scl(mk3(n2v.x, n2v.y, n2v.z), bx)),
                       scl(mk3(n3v.x, n3v.y, n3v.z), by)));
  hit = add(add(o, scl(d, bz)), scl(norm, HYBRID ? 0.0001f : 0.00001f));
  return distance(o, hit);
}

template <bool HYBRID>
__device__ inline float tri_hit_t(const DevScene& S, int i, f3 o, f3 d, float bx, float by, float bz, f3& hit,
                                  f3& norm) {
  return tri_hit_t_n<HYBRID>(S.tn0[i], S.tn1[i], S.tn2[i], o, d, bx, by, bz, hit, norm);
}

// One lane's ray and traversal state: exactly traverseKD's locals, kept across trace_phase calls so
// that the intersect kernel can give a lane a new ray whenever its previous one is finished.
struct WaveRay {
  f3 o, d, invdir;
  int cur, L;
  uint32_t cb, ps, g;
  bool rootv, sink, hitGeom, done, fault;
  float bz;
  int guard;
  Hit h;
  int objTri;  // the triangle whose hit record won (valid when h.obj_intersect)
  float lx, ly, lz, hx, hy, hz;  // NodesDerived: the box of node cur (min.xyz, max.xyz)
};

// Replace box slot k (0-2 min.xyz, 3-5 max.xyz; anything else: none) by v.
__device__ __attribute__((always_inline)) inline void box_set(WaveRay& R, uint32_t k, float v) {
  R.lx = k == 0u ? v : R.lx;
  R.ly = k == 1u ? v : R.ly;
  R.lz = k == 2u ? v : R.lz;
  R.hx = k == 3u ? v : R.hx;
  R.hy = k == 4u ? v : R.hy;
  R.hz = k == 5u ? v : R.hz;
}

// Start a ray: t_min / hit_geom_index come from the analytic geoms (k_geoms), tested first as in
// pathTraceOneBounceKDbare.
__device__ inline void wave_ray_start(const DevScene& S, WaveRay& R, f3 o, f3 d, float t_geom, int geom,
                                      WaveLeafLDS* W) {
  const int lane = threadIdx.x & 63;
  R.o = o;
  R.d = d;
  R.invdir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  R.cur = S.root;
  R.L = 0;
  R.cb = R.ps = R.g = 0;
  R.rootv = R.sink = R.hitGeom = R.done = R.fault = false;
  R.bz = FLT_MAXV;
  R.guard = 0;
  R.h.t_min = t_geom;
  R.h.hit_geom_index = geom;
  R.h.obj_intersect = false;
  R.h.objMaterialIdx = -1;
  R.h.ip = mk3(0, 0, 0);
  R.h.normal = mk3(0, 0, 0);
  R.objTri = -1;
  R.lx = S.rlo.x;  // the root's box (NodesDerived)
  R.ly = S.rlo.y;
  R.lz = S.rlo.z;
  R.hx = S.rhi.x;
  R.hy = S.rhi.y;
  R.hz = S.rhi.z;
  W->od[lane] = make_float4(o.x, o.y, o.z, d.x);
  W->dd[lane] = make_float2(d.y, d.z);
}

// One node phase and one leaf phase of traverseKD for every lane of the wave with an unfinished ray
// (R.done false); lanes finish by setting R.done.  fastAABB must be wave-uniform (every active lane's
// invdir finite).
template <bool HYBRID, bool COUNT, typename NodeSrc, typename ClusterSrc>
__device__ void trace_phase(const DevScene& S, const NodeSrc& nodes, const ClusterSrc& clusters, WaveRay& R,
                            bool fastAABB, int material_size, TraverseCounters& cnt, WaveLeafLDS* W,
                            WaveProf* WP) {
  const int lane = threadIdx.x & 63;
  const f3 o = R.o, d = R.d, invdir = R.invdir;
  int& cur = R.cur;
  int& L = R.L;
  uint32_t& cb = R.cb;
  uint32_t& ps = R.ps;
  uint32_t& g = R.g;
  bool& rootv = R.rootv;
  bool& sink = R.sink;
  bool& hitGeom = R.hitGeom;
  bool& done = R.done;
  bool& fault = R.fault;
  float& bz = R.bz;
  int& guard = R.guard;
  Hit& h = R.h;
  int& objTri = R.objTri;
  // ---------------- node phase ----------------
  bool leaf = false;
  bool lfirst = true;
  int trips = 0;
  if (COUNT) prof_lap(WP, -1);
  // One trip = one step of the reference's loop for every lane still walking nodes.  The
  // body runs for the whole wave and commits by selects on `walk`, and the per-lane flags
  // live in one register, so a trip carries no exec-mask bookkeeping.  Exact for a
  // validated tree (only the root has parentID == -1): at the root `up` ends the walk (the
  // reference exits before or after its test, or climbs to -1), so hitGeom only feeds the
  // AABB count.
  enum : uint32_t { F_ROOTV = 1, F_SINK = 2, F_HITGEOM = 4, F_DONE = 8, F_LEAF = 16, F_LFIRST = 32, F_FAULT = 64 };
  uint32_t fl = (rootv ? F_ROOTV : 0u) | (sink ? F_SINK : 0u) | (hitGeom ? F_HITGEOM : 0u) | (done ? F_DONE : 0u) |
                F_LFIRST;
  // leftFirst = d[axis] > 0 (comp: axis 0, 1, anything else z) as one bit test per trip
  const uint32_t dpos = (d.x > 0.0f ? 1u : 0u) | (d.y > 0.0f ? 2u : 0u) | (d.z > 0.0f ? 4u : 0u);
  while (true) {
    const bool walk = (fl & (F_DONE | F_LEAF)) == 0u;
    const unsigned long long wmask = __ballot(walk);
    if (!wmask) break;
    // Few lanes still walking and many waiting on leaves: test those leaves now; the walkers keep
    // their state and resume in the next node phase (their own sequence of steps is unchanged).
    if (__popcll(wmask) <= S.early_walk && __popcll(__ballot((fl & F_LEAF) != 0u)) >= S.early_leaf) break;
    if (COUNT) {
      trips += walk ? 1 : 0;
      prof_add(WP, PROF_SPARE, (unsigned long long)__popcll(wmask));  // lane-steps: SIMD efficiency
      prof_add(WP, PROF_NODE_LEAFWAIT, (unsigned long long)__popcll(__ballot((fl & F_LEAF) != 0u)));
      const unsigned long long nd_done = (unsigned long long)__popcll(__ballot((fl & F_DONE) != 0u));
      prof_add(WP, PROF_NODE_DONE, nd_done);
      if (WP->tail_t0) prof_add(WP, PROF_TAIL_NODE_DONE, nd_done);
    }
    const NodeRec nd = nodes(cur < 0 ? 0 : cur);
    const int left = nd.left, right = nd.right;
    const uint32_t Lu = (uint32_t)L;
    const uint32_t vb = (2u * Lu - 2u + ((ps >> ((Lu - 1u) & 31u)) & 1u)) & 31u;  // own flag (L > 0)
    const bool curVis = (L == 0) ? ((fl & F_ROOTV) != 0u) : (((cb >> vb) & 1u) != 0u);
    const bool isRoot = cur == S.root;
    const float4 nb0 = NodeSrc::kDerivedBox ? make_float4(R.lx, R.ly, R.lz, R.hx) : nd.b0;
    const float4 nb1 = NodeSrc::kDerivedBox ? make_float4(R.hy, R.hz, 0.0f, 0.0f) : nd.b1;
    float dd;
    const bool hg = fastAABB ? intersectAABB_fast(o, invdir, nb0, nb1, dd)
                             : intersectAABB(o, invdir, nb0, nb1, dd);
    const bool up = curVis || !hg || dd > bz;
    // Child choice on bit masks: `has` = children present (bit 0 left, bit 1 right), `avail` = present and not
    // yet visited at this level; the near side (fside: 0 left, 1 right) is taken when available, else the far
    // one.  takeFirst / takeSecond of traverseKDbareShortHybrid are avail's fside / far bits, so descend =
    // avail != 0 and the child is simply the one on side nside.
    const uint32_t fside = HYBRID ? (((dpos >> min((uint32_t)nd.axis, 2u)) & 1u) ^ 1u) : 0u;
    const uint32_t has = nd.has;
    const uint32_t sh2 = (2u * Lu) & 31u;
    const uint32_t avail = has & ~(cb >> sh2);  // (bits 0-1 only: has is)
    const uint32_t nside = ((avail >> fside) & 1u) ? fside : (fside ^ 1u);
    const bool descend = !up && avail != 0u;
    const bool lf = !up && avail == 0u && nd.tris;
    // "Mark and stay" on a node without triangles is always followed by a trip on the same
    // node that finds it visited and climbs (same box, so same hitGeom): do both now.
    const bool stay = !up && avail == 0u && !nd.tris;
    const bool climb = up || stay;
    if (COUNT && walk) cnt.aabb += (isRoot && curVis && !(fl & F_HITGEOM)) ? 0u : (stay ? 2u : 1u);
    // nodeIDs[ID] = true unless descending; nodeIDs[left] = nodeIDs[right] = true when climbing (neither
    // when descending: then only the new level's child flags are cleared, and the root's own flag moves
    // into g's slot)
    // (both forms computed, then one select: as an if/else the compiler branches on exec masks)
    const uint32_t cb_down = (cb & ~(3u << ((2u * Lu + 2u) & 31u))) | ((L == 0 && nside == 0u) ? (g << 2) : 0u);
    const uint32_t cb_here = cb | (L > 0 ? (1u << vb) : 0u) | (climb ? (has << sh2) : 0u);
    const uint32_t ncb = descend ? cb_down : cb_here;
    const bool runaway = guard >= S.trip_limit;
    uint32_t nfl = fl & ~(F_HITGEOM | F_LFIRST);
    nfl |= (!descend && L == 0) ? F_ROOTV : 0u;
    nfl |= (climb && has != 3u) ? F_SINK : 0u;
    nfl |= hg ? F_HITGEOM : 0u;
    nfl |= ((isRoot && climb) || runaway) ? F_DONE : 0u;
    nfl |= runaway ? F_FAULT : 0u;
    nfl |= lf ? F_LEAF : 0u;
    nfl |= fside == 0u ? F_LFIRST : 0u;
    if (walk) {  // commit (selects)
      cb = ncb;
      ps = descend ? ((ps & ~(1u << (Lu & 31u))) | (nside << (Lu & 31u))) : ps;
      cur = climb ? nd.parent : (descend ? (nside ? right : left) : cur);
      L += descend ? 1 : (climb ? -1 : 0);
      guard++;
      fl = nfl;
      if (NodeSrc::kDerivedBox) {
        // descending: the child's box is this one with max[axis] (left child) / min[axis] (right) set to the
        // centre; climbing: the parent's box is this one with the coordinate this node replaced put back
        const uint32_t kd = (nside ? 0u : 3u) + (uint32_t)nd.axis;
        box_set(R, descend ? kd : (climb ? nd.kc : 7u), descend ? nd.center : nd.restore);
      }
    }
  }
  rootv = (fl & F_ROOTV) != 0u;
  sink = (fl & F_SINK) != 0u;
  hitGeom = (fl & F_HITGEOM) != 0u;
  done = (fl & F_DONE) != 0u;
  leaf = (fl & F_LEAF) != 0u;
  lfirst = (fl & F_LFIRST) != 0u;
  fault = fault || (fl & F_FAULT) != 0u;
  if (COUNT) {
    prof_lap(WP, PROF_NODE_CYC);
    for (int off = 32; off > 0; off >>= 1) trips = max(trips, __shfl_xor(trips, off));
    prof_add(WP, PROF_NODE_TRIPS, (unsigned long long)trips);  // wave-level trips = the slowest lane's
  }
  if (__any(fault) && lane == 0) atomicOr(S.fault, 1);
  if (!__any(leaf)) return;
  // the leaf's own record, read once here rather than carried through every node trip (a lane that reaches
  // a leaf neither climbs nor descends, so cur is the leaf)
  const int lnode = cur;
  int lstart = 0, lsize = 0, lparent = -1, lclusters = 0;
  uint32_t lkc = 7u;
  float lrestore = 0.0f;
  if (leaf) {
    const NodeRec ln = nodes(cur);
    lstart = ln.triStart;
    lsize = ln.triSize;
    lparent = ln.parent;
    if (NodeSrc::kDerivedBox) {
      lkc = ln.kc;
      lrestore = ln.restore;
    }
    // a big leaf's cluster count: Morton runs of CLUSTER fill all but the last, unless the scene groups by
    // normal cones (S.cl_counts: the count from leaf_cl, requested here, read at the leaf phase)
    lclusters = (lsize + CLUSTER - 1) / CLUSTER;
    if (S.cl_counts && lsize >= BIG_LEAF) lclusters = S.leaf_cl[lnode].y;
  }
  // ---------------- leaf phase (wave-cooperative) ----------------
  // per lane results of this phase
  int r_pass = 0;          // 0 = none, else tri + 1 of the last u/v pass
  float r_bz = 0.0f;
  int r_lasthit = -1, r_nhit = 0;
  unsigned long long r_best = ~0ull;
  // Both leaf kinds enumerate (lane, item) pairs flattened over the wave: lane L owns pairs
  // [excl_L, excl_L + count_L), and lane k of a round takes pair B + k, whichever ray it belongs to.
  // (a) big leaves: the items are 64-triangle clusters.  One pass culls 64 (ray, cluster) pairs (clusters
  // whose box the ray's line misses, when every invdir is finite); each surviving cluster is then swept by
  // the whole wave with its ray, 64 triangles at a time, the next survivor's triangles fetched while this
  // one is tested.  Recombination by ORIGINAL index into the owner lane (order-free): last u/v pass = max
  // index, last hit = max, best = min (t, index).
  const bool big = leaf && lsize >= BIG_LEAF;
  if (__any(big)) {
    unsigned long long k_pass = 0ull, k_best = ~0ull;
    int k_lasthit = -1, k_nhit = 0;
    // Sweeps of the (ray, cluster) pairs `pass` marks: cluster c with the ray of lane own, each surviving
    // cluster by the whole wave, the next survivor's triangles fetched while this one is tested; the results
    // are folded into the owner lane's k_* (order-free).  Wave-uniform call.
    auto sweep64 = [&](bool pass, int c, int own) {
      unsigned long long sm = __ballot(pass);
      int s = -1;
      TriData T{};
      if (sm) {
        s = __builtin_ctzll(sm);
        sm &= sm - 1;
        const int ct = __builtin_amdgcn_readlane(c, s) * 64 + lane;
        T = TriData{S.c_v0[ct], S.c_e1[ct], S.c_e2[ct]};
      }
      while (s >= 0) {
        int sn = -1;
        TriData Tn{};
        if (sm) {
          sn = __builtin_ctzll(sm);
          sm &= sm - 1;
          const int ctn = __builtin_amdgcn_readlane(c, sn) * 64 + lane;
          Tn = TriData{S.c_v0[ctn], S.c_e1[ctn], S.c_e2[ctn]};
        }
        if (COUNT) prof_add(WP, PROF_BIG_SWEEPS, 1);
        const int j = __builtin_amdgcn_readlane(own, s);  // the cluster's ray: lane j's, wave-uniform
        const f3 jo = mk3(readlane_f(o.x, j), readlane_f(o.y, j), readlane_f(o.z, j));
        const f3 jd = mk3(readlane_f(d.x, j), readlane_f(d.y, j), readlane_f(d.z, j));
        const int orig = fbits(T.e1.w);
        float bx = 0, by = 0, bzk = 0;
        const int r = tri_test_v(T, jo, jd, bx, by, bzk);
        const unsigned long long m1 = __ballot(r >= 1);
        if (COUNT && m1) {
          prof_add(WP, PROF_BIG_PASS, 1);
          prof_add(WP, PROF_BIG_MULTI, (m1 & (m1 - 1)) ? 1 : 0);
        }
        if (m1) {
          const unsigned long long pk =
              r >= 1 ? ((unsigned long long)(unsigned int)(orig + 1) << 32) | f2u(bzk) : 0ull;
          // usually one lane of the cluster passes: read its key instead of reducing over the wave
          const unsigned long long wm = (m1 & (m1 - 1)) == 0ull ? readlane_u64(pk, __builtin_ctzll(m1))
                                                                : wave_max_u64(pk);
          if (lane == j) k_pass = wm > k_pass ? wm : k_pass;
          const unsigned long long m2 = __ballot(r == 2);
          if (m2) {
            const bool one = (m2 & (m2 - 1)) == 0ull;
            const int jh = __builtin_ctzll(m2);
            const int lh = one ? __builtin_amdgcn_readlane(orig, jh) : wave_max_i32(r == 2 ? orig : -1);
            unsigned long long key = ~0ull;
            if (r == 2) {
              f3 hp, nn;
              const float t = tri_hit_t<HYBRID>(S, orig, jo, jd, bx, by, bzk, hp, nn);
              if (t > 0.0f) key = ((unsigned long long)f2u(t) << 32) | (unsigned int)orig;
            }
            const unsigned long long wb = one ? readlane_u64(key, jh) : wave_min_u64(key);
            if (lane == j) {
              k_nhit += __builtin_popcountll(m2);
              k_lasthit = max(k_lasthit, lh);
              k_best = wb < k_best ? wb : k_best;
            }
          }
        }
        s = sn;
        T = Tn;
      }
    };
    // CLUSTER == 32: two (ray, cluster) pairs per round, lanes [0, 32) testing the first survivor's 32
    // triangles with its ray and lanes [32, 64) the second's with its own; the results of each half are folded
    // into that pair's owner lane as above (both halves may belong to one ray: the folds are order-free).
    auto sweep32 = [&](bool pass, int c, int own) {
      unsigned long long sm = __ballot(pass);
      const bool hi = lane >= 32;
      const unsigned long long hmask = hi ? 0xffffffff00000000ull : 0x00000000ffffffffull;
      auto take = [&]() {
        int t = -1;
        if (sm) {
          t = __builtin_ctzll(sm);
          sm &= sm - 1;
        }
        return t;
      };
      auto load = [&](int a, int b) {  // lane's half of survivors a (low) and b (high, -1: none)
        const int ca = a >= 0 ? __builtin_amdgcn_readlane(c, a) : -1;
        const int cb = b >= 0 ? __builtin_amdgcn_readlane(c, b) : -1;
        const int mc = hi ? cb : ca;
        TriData t{};  // zero edges fail glm's determinant test
        if (mc >= 0) {
          const int ct = mc * 32 + (lane & 31);
          t = TriData{S.c_v0[ct], S.c_e1[ct], S.c_e2[ct]};
        }
        return t;
      };
      int s0 = take(), s1 = take();
      TriData T{};
      if (s0 >= 0) T = load(s0, s1);
      while (s0 >= 0) {
        const int n0 = take(), n1 = take();
        TriData Tn{};
        if (n0 >= 0) Tn = load(n0, n1);
        if (COUNT) prof_add(WP, PROF_BIG_SWEEPS, 1);
        const int j0 = __builtin_amdgcn_readlane(own, s0);
        const int j1 = s1 >= 0 ? __builtin_amdgcn_readlane(own, s1) : j0;
        const f3 o0 = mk3(readlane_f(o.x, j0), readlane_f(o.y, j0), readlane_f(o.z, j0));
        const f3 d0 = mk3(readlane_f(d.x, j0), readlane_f(d.y, j0), readlane_f(d.z, j0));
        const f3 o1 = mk3(readlane_f(o.x, j1), readlane_f(o.y, j1), readlane_f(o.z, j1));
        const f3 d1 = mk3(readlane_f(d.x, j1), readlane_f(d.y, j1), readlane_f(d.z, j1));
        const f3 jo = hi ? o1 : o0, jd = hi ? d1 : d0;
        const int orig = fbits(T.e1.w);
        float bx = 0, by = 0, bzk = 0;
        const int r = tri_test_v(T, jo, jd, bx, by, bzk);
        const unsigned long long m1 = __ballot(r >= 1);
        if (COUNT && m1) {
          prof_add(WP, PROF_BIG_PASS, 1);
          prof_add(WP, PROF_BIG_MULTI, (m1 & (m1 - 1)) ? 1 : 0);
        }
        if (m1) {
          const unsigned long long pk =
              r >= 1 ? ((unsigned long long)(unsigned int)(orig + 1) << 32) | f2u(bzk) : 0ull;
          const unsigned long long m2 = __ballot(r == 2);
          unsigned long long key = ~0ull;
          if (r == 2) {
            f3 hp, nn;
            const float t = tri_hit_t<HYBRID>(S, orig, jo, jd, bx, by, bzk, hp, nn);
            if (t > 0.0f) key = ((unsigned long long)f2u(t) << 32) | (unsigned int)orig;
          }
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const unsigned long long hm = h ? 0xffffffff00000000ull : 0x00000000ffffffffull;
            const unsigned long long m1h = m1 & hm;
            if (!m1h) continue;
            const int jh = h ? j1 : j0;
            const bool mine = (hm & hmask) != 0ull;  // this lane is in half h
            const unsigned long long wm = (m1h & (m1h - 1)) == 0ull ? readlane_u64(pk, __builtin_ctzll(m1h))
                                                                    : wave_max_u64(mine ? pk : 0ull);
            if (lane == jh) k_pass = wm > k_pass ? wm : k_pass;
            const unsigned long long m2h = m2 & hm;
            if (m2h) {
              const bool one = (m2h & (m2h - 1)) == 0ull;
              const int lh2 = __builtin_ctzll(m2h);
              const int lh = one ? __builtin_amdgcn_readlane(orig, lh2)
                                 : wave_max_i32(mine && r == 2 ? orig : -1);
              const unsigned long long wb = one ? readlane_u64(key, lh2) : wave_min_u64(mine ? key : ~0ull);
              if (lane == jh) {
                k_nhit += __builtin_popcountll(m2h);
                k_lasthit = max(k_lasthit, lh);
                k_best = wb < k_best ? wb : k_best;
              }
            }
          }
        }
        s0 = n0;
        s1 = n1;
        T = Tn;
      }
    };
    auto sweep = [&](bool pass, int c, int own) {
      if constexpr (CLUSTER == 32) sweep32(pass, c, own);
      else sweep64(pass, c, own);
    };
    const int ncl = big ? lclusters : 0;
    if constexpr (ClusterSrc::kSuper) {
      // Two levels (leaves of thousands of triangles, e.g. the C5 icosphere's): the (ray, super-cluster) pairs
      // are culled first, 64 per pass, against the supers' boxes (LDS); each surviving super's SUPER clusters
      // are then culled against their own boxes, 64 / SUPER supers per round, and the survivors swept.  A
      // super's box holds its clusters' boxes, so the second level sees every cluster the one-level cull
      // would pass.
      const int nsp = (ncl + SUPER - 1) / SUPER;
      const int incl = wave_incl_scan<false>(nsp);
      const int P = __builtin_amdgcn_readlane(incl, 63);
      const int excl = incl - nsp;
      W->tbase[lane] = lstart - excl;  // super of pair q = tbase[owner] + q (lstart: the leaf's first super)
      wave_lds_sync();
      if (COUNT) {
        prof_add(WP, PROF_BIG_LEAVES, (unsigned long long)__popcll(__ballot(big)));
        prof_add(WP, PROF_BIG_SUPERS, (unsigned long long)P);
      }
      // one pass's surviving supers, {owner << 32 | first cluster << 5 | count - 1}, in W->best (the
      // small-leaf phase below initialises it afresh)
      static_assert(SUPER <= 32 && 64 % SUPER == 0, "super-cluster size");
      unsigned long long* slist = W->best;
      int carry = 0;
      for (int B = 0; B < P; B += 64) {
        const int own = pair_owner(W->slot, excl, nsp, B, carry);
        const int sp = W->tbase[own] + B + lane;
        bool pass = B + lane < P;
        float4 slo = make_float4(0.0f, 0.0f, 0.0f, 0.0f), shi = slo, sn = slo, sb = slo;
        uint32_t sinfo = 0u;
        // the super's slab record (L2) is requested for every pair before the box test, so its latency
        // overlaps the LDS record, the ray exchange and the box test
        if (fastAABB && S.sup_slab && pass) {
          sn = S.sup_n[sp];
          sb = S.sup_b[sp];
        }
        if (pass) sinfo = clusters.sup(sp, slo, shi);
        if (fastAABB) {
          const float4 od = W->od[own];  // the pair's ray from the wave's LDS copy (wave_ray_start)
          const f3 oo = mk3(od.x, od.y, od.z);
          const f3 ii = mk3(bpermute_f(invdir.x, own), bpermute_f(invdir.y, own), bpermute_f(invdir.z, own));
          if (pass) pass = cluster_may_pass(slo, shi, oo, ii, S.cl_margin);
          // the boxes' survivors against the super's slab (its record from L2), with the margin its normal
          // spread allows for this direction
          if (S.sup_slab && __any(pass)) {
            const float2 d2 = W->dd[own];
            const f3 dd = mk3(od.w, d2.x, d2.y);
            const CullK ck{S.cl_margin, S.cl_margin_lo, S.cull_a, S.cull_b, S.cull_c};
            if (pass) {
              pass = cluster_may_pass_slab(make_float4(slo.x, slo.y, slo.z, sb.x), make_float4(shi.x, shi.y, shi.z, sb.y),
                                           sn, oo, ii, dd, ck);
            }
          }
        }
        const unsigned long long sm = __ballot(pass);
        const int nsv = __popcll(sm);
        if (pass)
          slist[lane_prefix(sm)] = ((unsigned long long)(uint32_t)own << 32) | sinfo;
        wave_lds_sync();
        for (int q = 0; q < nsv; q += 64 / SUPER) {
          const int e = q + lane / SUPER, k = lane % SUPER;
          bool cp = e < nsv;
          int cown = 0, c = 0;
          if (cp) {
            const unsigned long long ent = slist[e];
            cown = (int)(ent >> 32);
            c = (int)((uint32_t)ent >> 5) + k;
            cp = k <= (int)((uint32_t)ent & 31u);
          }
          if (COUNT) prof_add(WP, PROF_BIG_CLUSTERS, (unsigned long long)__popcll(__ballot(cp)));
          if (fastAABB) {
            // the oriented-box records (L2) requested before the ray exchange, so their latency overlaps it
            const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            float4 rlo = z4, rhi = z4, rn = z4, ru = z4, rv = z4, rw = z4;
            if (S.cl_slab && S.cl_obb && cp) {
              rlo = clusters.lo_of(c);
              rhi = clusters.hi_of(c);
              rn = clusters.n_of(c);
              ru = clusters.u[c];
              rv = clusters.v[c];
              rw = clusters.w[c];
            }
            const float4 od = W->od[cown];
            const f3 oo = mk3(od.x, od.y, od.z);
            const f3 ii =
                mk3(bpermute_f(invdir.x, cown), bpermute_f(invdir.y, cown), bpermute_f(invdir.z, cown));
            if (S.cl_slab) {
              const CullK ck{S.cl_margin, S.cl_margin_lo, S.cull_a, S.cull_b, S.cull_c};
              const float2 d2 = W->dd[cown];
              const f3 dd = mk3(od.w, d2.x, d2.y);
              if (cp) {
                if (S.cl_obb)
                  cp = cluster_may_pass_obb(rlo, rhi, rn, ru, rv, rw, oo, ii, dd, ck);
                else
                  cp = cluster_may_pass_slab(clusters.lo_of(c), clusters.hi_of(c), clusters.n_of(c), oo, ii, dd, ck);
              }
            } else {
              if (cp) cp = cluster_may_pass(clusters.lo_of(c), clusters.hi_of(c), oo, ii, S.cl_margin);
            }
          }
          if (COUNT) prof_lap(WP, PROF_BIG_CULL_CYC);
          sweep(cp, c, cown);
          if (COUNT) prof_lap(WP, PROF_BIG_CYC);
        }
        wave_lds_sync();  // slist is rewritten by the next pass
      }
    } else {
      // One level: lane L owns the (ray, cluster) pairs [excl_L, excl_L + ncl_L); one pass culls 64 of them
      // against the cluster boxes (LDS) and the box survivors against the clusters' oriented boxes (L2), both
      // widened at the fast coefficient cl_margin; the hits are swept by the whole wave.
      // With direction masks (S.cl_mask: the exact cull, DESIGN.md 4 "Cluster cull") a miss may still hide a
      // u/v pass of a triangle nearly parallel to the line: the cluster's danger mask for the ray's direction
      // bucket (kdpt_clusters.h build_dir_masks) lists every triangle that can need more than cl_margin for
      // some direction of the bucket.  The mask is requested with the box test and read after the pass's
      // sweeps (its latency hidden behind them); the missed pair's lane then walks its bits, deciding each
      // triangle from its unit normal and the line's box_miss distance (danger_needs_test), and the rare one
      // that needs it gets glm's u/v tests.  A pass sweeps the whole cluster late, as the uncull'd walk would
      // have: the sweep's results fold by max / min / sum, so a late sweep is the same as an early one.
      const bool exact = S.cl_mask != nullptr;
      const int cfirst = big ? (NodeSrc::kLeafHoldsCluster ? lstart : S.leaf_cl[lnode].x) : 0;
      const int incl = wave_incl_scan<false>(ncl);
      const int P = __builtin_amdgcn_readlane(incl, 63);
      const int excl = incl - ncl;
      W->tbase[lane] = cfirst - excl;  // cluster of pair q = tbase[owner] + q
      wave_lds_sync();
      if (COUNT) {
        prof_add(WP, PROF_BIG_LEAVES, (unsigned long long)__popcll(__ballot(big)));
        prof_add(WP, PROF_BIG_CLUSTERS, (unsigned long long)P);
      }
      int carry = 0;
      for (int B = 0; B < P; B += 64) {
        const int own = pair_owner(W->slot, excl, ncl, B, carry);
        const int c = W->tbase[own] + B + lane;
        bool hit = B + lane < P;  // (no cull: every pair swept)
        unsigned long long m = 0ull;  // a missed pair's danger mask (exact cull)
        if (fastAABB) {
          const float4 od = W->od[own];  // the pair's ray from the wave's LDS copy (wave_ray_start)
          const float2 d2 = W->dd[own];
          const f3 oo = mk3(od.x, od.y, od.z), dd = mk3(od.w, d2.x, d2.y);
          const f3 ii = mk3(bpermute_f(invdir.x, own), bpermute_f(invdir.y, own), bpermute_f(invdir.z, own));
          float4 clo = make_float4(0.0f, 0.0f, 0.0f, 0.0f), chi = clo;
          unsigned long long dm = 0ull;
          const bool valid = hit;
          if (valid) {
            if (exact) dm = S.cl_mask[(uint32_t)dir_bucket(dd, S.mask_n) * (uint32_t)S.num_clusters + (uint32_t)c];
            clo = clusters.lo_of(c);
            chi = clusters.hi_of(c);
            hit = cluster_may_pass(clo, chi, oo, ii, S.cl_margin);
          }
          // the box's survivors against the cluster's oriented box (its slabs from L2)
          if (S.flat_obb && __any(hit)) {
            if (hit) {
              const float4 cn = S.cl_n[c];
              hit = cluster_may_pass_obb_k(clo, chi, cn, S.cl_u[c], S.cl_v[c], S.cl_w[c], oo, ii, dd,
                                           cn.x * dd.x + cn.y * dd.y + cn.z * dd.z, S.cl_margin);
            }
          }
          if (exact && valid && !hit) m = dm;
        }
        if (COUNT) prof_lap(WP, PROF_BIG_CULL_CYC);
        sweep(hit, c, own);
        if (COUNT) prof_lap(WP, PROF_BIG_CYC);
        if (!exact || !__any(m != 0ull)) continue;
        bool late = false;  // a danger triangle passed glm's u/v tests: sweep the cluster now
        {
          // (the line, its direction and its box recomputed rather than kept live across the sweep)
          const float4 od = W->od[own];  // the pair's ray from the wave's LDS copy (wave_ray_start)
          const float2 d2 = W->dd[own];
          const f3 oo = mk3(od.x, od.y, od.z), dd = mk3(od.w, d2.x, d2.y);
          const f3 ii = mk3(bpermute_f(invdir.x, own), bpermute_f(invdir.y, own), bpermute_f(invdir.z, own));
          unsigned long long nm = 0ull;  // the danger triangles danger_needs_test keeps
          if (m) {
            // one normal record per trip, the first requested before box_miss (the cluster box from LDS, the
            // line's reciprocal from its lane), so that its latency overlaps it (profiles/r06_ab_log.md r06l/r06m:
            // +1 % against two records per trip)
            const int e0 = c * 64;
            int k0 = __builtin_ctzll(m);
            m &= m - 1;
            float4 t0 = S.cl_tn[e0 + k0];
            const float D = box_miss(clusters.lo_of(c), clusters.hi_of(c), oo, ii);
            while (true) {
              if (danger_needs_test(t0, dd, D, S.cull_c)) nm |= 1ull << k0;
              if (!m) break;
              k0 = __builtin_ctzll(m);
              m &= m - 1;
              t0 = S.cl_tn[e0 + k0];
            }
          }
          if (__any(nm != 0ull)) {  // (rare) glm's u/v tests on the kept ones
            while (nm && !late) {
              const int e = c * 64 + __builtin_ctzll(nm);
              nm &= nm - 1;
              float bx, by, bz;
              late = tri_test_v(TriData{S.c_v0[e], S.c_e1[e], S.c_e2[e]}, oo, dd, bx, by, bz) >= 1;
            }
          }
        }
        if (COUNT) prof_lap(WP, PROF_BIG_CULL_CYC);
        if (__any(late)) sweep(late, c, own);
        if (COUNT) prof_lap(WP, PROF_BIG_CYC);
      }
    }
    if (big) {
      r_pass = (int)(k_pass >> 32);
      r_bz = u2f((uint32_t)(k_pass & 0xffffffffu));
      r_lasthit = k_lasthit;
      r_nhit = k_nhit;
      r_best = k_best;
    }
  }
  if (COUNT) prof_lap(WP, PROF_BIG_CYC);
  // (b) small leaves: the items are triangles, every (ray, triangle) pair tested by one lane; results
  // recombine through LDS atomics on the owner's slots
  const int sz = (leaf && !big) ? lsize : 0;
  if (__any(sz > 0)) {
    if (COUNT) prof_add(WP, PROF_SMALL_PHASES, 1);
    const int incl = wave_incl_scan<false>(sz);
    const int P = __builtin_amdgcn_readlane(incl, 63);
    const int excl = incl - sz;
    W->tbase[lane] = lstart - excl;  // triangle of pair q = tbase[owner] + q
    W->lastPass[lane] = 0ull;
    W->lastHit[lane] = -1;
    W->nhit[lane] = 0;
    W->best[lane] = ~0ull;
    wave_lds_sync();
    if (COUNT) {
      prof_add(WP, PROF_SMALL_ROUNDS, (unsigned long long)((P + 63) / 64));
      prof_add(WP, PROF_SMALL_PAIRS, (unsigned long long)P);
    }
    // the next round's owners are found and its triangles loaded while the current round is tested (two
    // rounds ahead spilled: -8 %, profiles/r04_ab_log.md)
    int carry = 0;
    int owner = pair_owner(W->slot, excl, sz, 0, carry);
    int tri = W->tbase[owner] + lane;
    TriData nxt{};
    if (lane < P) nxt = tri_load(S, tri);
    for (int B = 0; B < P; B += 64) {
      const TriData cur_t = nxt;
      const int cowner = owner, ctri = tri;
      const bool valid = B + lane < P;
      if (B + 64 < P) {
        owner = pair_owner(W->slot, excl, sz, B + 64, carry);
        tri = W->tbase[owner] + B + 64 + lane;
        if (B + 64 + lane < P) nxt = tri_load(S, tri);
      }
      if (valid) {
        const float4 q0 = W->od[cowner];
        const float2 q1 = W->dd[cowner];
        const f3 oo = mk3(q0.x, q0.y, q0.z), dd = mk3(q0.w, q1.x, q1.y);
        float bx, by, bzk;
        const int r = tri_test_v(cur_t, oo, dd, bx, by, bzk);
        if (r >= 1)
          atomicMax(&W->lastPass[cowner], ((unsigned long long)(unsigned int)(ctri + 1) << 32) | f2u(bzk));
        if (r == 2) {
          atomicMax(&W->lastHit[cowner], ctri);
          atomicAdd(&W->nhit[cowner], 1);
          f3 hp, nn;
          const float t = tri_hit_t<HYBRID>(S, ctri, oo, dd, bx, by, bzk, hp, nn);
          if (t > 0.0f) atomicMin(&W->best[cowner], ((unsigned long long)f2u(t) << 32) | (unsigned int)ctri);
        }
      }
    }
    wave_lds_sync();
    if (sz > 0) {
      const unsigned long long lp = W->lastPass[lane];
      r_pass = (int)(lp >> 32);
      r_bz = u2f((uint32_t)(lp & 0xffffffffu));
      r_lasthit = W->lastHit[lane];
      r_nhit = W->nhit[lane];
      r_best = W->best[lane];
    }
    wave_lds_sync();  // the LDS slots are rewritten by the next leaf phase
  }
  if (COUNT) prof_lap(WP, PROF_SMALL_CYC);
  if (leaf) {
    if (COUNT) cnt.tri += lsize;
    if (r_pass > 0) bz = r_bz;
    const int nh = r_nhit;
    if (nh > 0) {
      if (COUNT) cnt.hit += nh;
      h.objMaterialIdx = fbits(S.tv0[r_lasthit].w) + material_size - 1;
      if (HYBRID) {
        for (int rep = 0; rep < (nh > 1 ? 2 : 1); rep++) {
          const bool parVis = (L == 0) ? sink
                              : (L == 1 ? rootv
                                        : (((cb >> (2 * (L - 2) + (int)((ps >> (L - 2)) & 1u))) & 1u) != 0u));
          const int b = parVis ? 1 : 0;
          int target = -1;
          if (b < S.num_nodes) target = (b == 0) ? (lfirst ? S.n0_right : S.n0_left) : (lfirst ? S.n1_right : S.n1_left);
          if (target == -1) sink = true;
          else if (b == 0) cb |= 1u << (lfirst ? 1 : 0);
          else {
            const uint32_t bit = lfirst ? 1u : 0u;
            if (L >= 1 && (ps & 1u) == 0u) cb |= 1u << (2 + bit);
            else g |= 1u << bit;
          }
        }
      }
      if (r_best != ~0ull) {
        const float tb = u2f((uint32_t)(r_best >> 32));
        const int k = (int)(uint32_t)(r_best & 0xffffffffu);
        if (h.t_min > tb) {  // tb is tri_hit_t's value for triangle k (the winner's point and
          h.t_min = tb;        // normal are recomputed from k by the shading kernel)
          h.hit_geom_index = S.obj_material_offsets[fbits(S.tv0[k].w)];
          h.obj_intersect = true;
          objTri = k;
        }
      }
    }
    // The reference's next trip finds the leaf visited and climbs (leaves have no children,
    // validated: nodeIDs[-1] = true twice); do it here instead of in the node phase.
    if (COUNT) cnt.aabb++;
    sink = true;
    done = cur == S.root;
    cur = lparent;
    L--;
    if (NodeSrc::kDerivedBox) box_set(R, lkc, lrestore);  // back to the parent's box
  }
  if (COUNT) prof_lap(WP, PROF_FINAL_CYC);
}
#endif  // HIP

// ---------------- src/interactions.h ----------------
KDPT_HD f3 calculateRandomDirectionInHemisphere(f3 normal, Rng& rng) {  // :9-41
  float up = sqrtf(u01(rng));
  float over = sqrtf(1 - up * up);
  float around = u01(rng) * TWO_PI_F;
  f3 dnn;
  if (fabsf(normal.x) < SQRT_OF_ONE_THIRD_F) dnn = mk3(1, 0, 0);
  else if (fabsf(normal.y) < SQRT_OF_ONE_THIRD_F) dnn = mk3(0, 1, 0);
  else dnn = mk3(0, 0, 1);
  f3 p1 = normalize(cross(normal, dnn));
  f3 p2 = normalize(cross(normal, p1));
  float ca = kdpt_cosf(around), sa = kdpt_sinf(around);
  return add(add(scl(normal, up), scl(p1, ca * over)), scl(p2, sa * over));
}
KDPT_HD f3 rotateVector(f3 n1, f3 axis, float angle) {  // :44-65
  axis = normalize(axis);
  float u = axis.x, v = axis.y, w = axis.z, x = n1.x, y = n1.y, z = n1.z;
  float ca = kdpt_cosf(angle), sa = kdpt_sinf(angle);
  float dd = -u * x - v * y - w * z;
  return mk3((-u * dd) * (1 - ca) + x * ca + (-w * y + v * z) * sa,
             (-v * dd) * (1 - ca) + y * ca + (w * x - u * z) * sa,
             (-w * dd) * (1 - ca) + z * ca + (-v * x + u * y) * sa);
}
// :67-83.  theta and phi are float values widened to double; glm::cos/glm::sin on them are glibc's
// double cos/sin and glm::acos(float) is acosf -- all three restated bit-exactly (kdpt_math.h).
// Reached with default flags by any material with transmittance > 0 (e.g. the reference's own
// scenes/stanford_bunny.mtl, Tf 1.0 0.7 0.7) and by the soft lobes when softness > 0.
KDPT_HD f3 randSphericalVec(float angle, Rng& rng) {
  double theta = 2 * PI_F * u01(rng);
  double phi = kdpt_acosf((angle * PI_F * u01(rng) - 1.0f));
  f3 V = mk3((float)(kdpt_cos(theta) * kdpt_sin(phi)), (float)(kdpt_sin(theta) * kdpt_sin(phi)), (float)kdpt_cos(phi));
  return normalize(V);
}
KDPT_HD float getFresnelVal(f3 I, f3 N, float R0) {  // :127-133
  double F = (double)R0 + (double)(1.0f - R0) * pow5((double)(1.0f - dot(N, neg(I))));
  return (float)F;
}
KDPT_HD f3 soft_lobe(f3 dir, Rng& rng) {
  f3 v = randSphericalVec(0.02f, rng);
  float angle = kdpt_acosf(dot(mk3(0.0f, 0.0f, -1.0f), dir));
  f3 axis = normalize(cross(mk3(0.0f, 0.0f, -1.0f), dir));
  return rotateVector(v, axis, angle);
}
// :195-358
KDPT_HD void scatterRay(Ray& ray, f3 intersect, f3 normal, const DevMaterial& m, Rng& rng, float softness) {
  if (m.transmittance[0] > 0.0f || m.transmittance[1] > 0.0f || m.transmittance[2] > 0.0f) {
    float randval = u01(rng);
    if (randval < 0.5f && !ray.isinside) {
      f3 v = randSphericalVec(0.0001f, rng);
      float angle = kdpt_acosf(dot(mk3(0.0f, 0.0f, -1.0f), ray.direction));
      f3 axis = normalize(cross(mk3(0.0f, 0.0f, -1.0f), ray.direction));
      ray.direction = rotateVector(v, axis, angle);
      ray.origin = add(ray.origin, scl(ray.direction, 0.0001f));
      ray.sdepth = distance(ray.origin, intersect);
      ray.isinside = true;
    } else {
      ray.direction = calculateRandomDirectionInHemisphere(normal, rng);
      ray.origin = add(intersect, scl(normal, 0.00001f));
      ray.sdepth = 0.0f;
    }
  } else if (m.hasRefractive != 0.0f) {
    float randval = u01(rng);
    ray.direction = normalize(ray.direction);
    normal = normalize(normal);
    float fresn = getFresnelVal(ray.direction, normal, m.fresnel_R0);
    if (randval < 1.0f - fresn) {
      float ior = m.indexOfRefraction;
      if (!ray.isinside) ior = 1.0f / m.indexOfRefraction;
      double dd = (double)dot(normal, ray.direction);
      float angle = (float)(1.0f - ((double)ior * (double)ior) * (1.0f - dd * dd));
      if (angle < 0.0f) {
        float val = u01(rng);
        if (val < m.hasReflective) {
          ray.direction = reflect(ray.direction, normal);
          if (softness > 0.0f) ray.direction = soft_lobe(ray.direction, rng);
          ray.origin = add(intersect, scl(normal, 0.00001f));
        } else {
          ray.direction = calculateRandomDirectionInHemisphere(normal, rng);
          ray.origin = add(intersect, scl(normal, 0.00001f));
        }
      } else {
        float val = u01(rng);
        if (val < m.hasRefractive) {
          ray.direction = refract(ray.direction, normal, ior);
          if (softness > 0.0f) ray.direction = soft_lobe(ray.direction, rng);
          ray.origin = sub(intersect, scl(normal, 0.001f));
          ray.isinside = !ray.isinside;
        } else {
          ray.direction = calculateRandomDirectionInHemisphere(normal, rng);
          ray.origin = add(intersect, scl(normal, 0.00001f));
        }
      }
    } else {
      ray.direction = reflect(ray.direction, normal);
      ray.origin = add(intersect, scl(normal, 0.00001f));
      ray.isinside = false;
    }
  } else if (m.hasReflective != 0.0f) {
    float randval = u01(rng);
    if (randval < m.hasReflective) {
      ray.direction = reflect(ray.direction, normal);
      if (softness > 0.0f) ray.direction = soft_lobe(ray.direction, rng);
      ray.origin = add(intersect, scl(normal, 0.0001f));
      ray.isinside = false;
    } else {
      ray.direction = calculateRandomDirectionInHemisphere(normal, rng);
      ray.origin = add(intersect, scl(normal, 0.00001f));
    }
  } else {
    ray.direction = calculateRandomDirectionInHemisphere(normal, rng);
    ray.origin = add(intersect, scl(normal, 0.00001f));
    ray.isinside = false;
  }
}

// shadeMaterial body for a path with remainingBounces > 0 (src/pathtrace.cu:2318-2366)
KDPT_HD void shade(float t, int materialId, const DevMaterial* mats, bool enablesss, const Ray& ray, f3& color,
                   int& bounces) {
  if (t > 0.0f) {
    const DevMaterial& m = mats[materialId];
    f3 c = mk3(m.color[0], m.color[1], m.color[2]);
    f3 spec = mk3(m.spec_color[0], m.spec_color[1], m.spec_color[2]);
    if (m.emittance > 0.0f) {
      color = mul(color, scl(c, m.emittance));
      bounces = 0;
    } else {
      if (enablesss && (m.transmittance[0] > 0.0f || m.transmittance[1] > 0.0f || m.transmittance[2] > 0.0f)) {
        float scenescale = 1.0f;
        float sss = (double)(scenescale * ray.sdepth) > 1.0 ? 1.0f : ray.sdepth;
        sss = (double)(1.0f - sss) < 0.0 ? 0.0f : sss;
        sss = (float)((double)sss * (double)sss);
        f3 tr = mk3(m.transmittance[0], m.transmittance[1], m.transmittance[2]);
        color = mul(color, add(add(scl(c, 1.0f), scl(spec, m.hasRefractive)), scl(tr, sss)));
      } else if (m.hasRefractive > 0.0f) {
        color = mul(color, add(scl(c, 1.0f), scl(spec, m.hasRefractive)));
      } else if (m.hasReflective > 0.0f) {
        color = mul(color, add(scl(c, 1.0f), scl(spec, m.hasReflective)));
      } else {
        color = mul(color, scl(c, 1.0f));
      }
      bounces--;
    }
  } else {
    color = mk3(0.0f, 0.0f, 0.0f);
    bounces = 0;
  }
}

// Known answers for the glm pieces on the path, checked against the reference's vendored glm 0.9.6.3
// (oracle/ref) on the host and on gfx950 (kdpt_selftest_glm):
//   fn 0 intersectRayTriangle (gtx/intersect.inl:37-74) as tri_test_v runs it: in o, d, v0, v1, v2 (15
//        floats), out {passed, bary.x, bary.y, bary.z}; bary slots the test does not reach keep the
//        caller's values (out[1..3] are read first), which pins glm's partial writes;
//   fn 1 normalize (3 -> 3), fn 2 reflect (I, N -> 3), fn 3 refract (I, N, eta -> 3),
//   fn 4 glm::rotate(quat, vec3) (w, x, y, z, v -> 3).
KDPT_HD int glm_kat_inputs(int fn) {
  return fn == 0 ? 15 : fn == 1 ? 3 : fn == 2 ? 6 : fn == 3 ? 7 : fn == 4 ? 7 : 0;
}
KDPT_HD int glm_kat_outputs(int fn) { return fn == 0 ? 4 : (fn >= 1 && fn <= 4) ? 3 : 0; }
KDPT_HD void glm_kat(int fn, const float* in, float* out) {
  f3 r = mk3(0.0f, 0.0f, 0.0f);
  switch (fn) {
    case 0: {
      const TriData T{make_float4(in[6], in[7], in[8], 0.0f),
                      make_float4(in[9] - in[6], in[10] - in[7], in[11] - in[8], 0.0f),
                      make_float4(in[12] - in[6], in[13] - in[7], in[14] - in[8], 0.0f)};
      float bx = out[1], by = out[2], bz = out[3];
      const int k = tri_test_v(T, mk3(in[0], in[1], in[2]), mk3(in[3], in[4], in[5]), bx, by, bz);
      out[0] = k == 2 ? 1.0f : 0.0f;
      out[1] = bx;
      out[2] = by;
      out[3] = bz;
      return;
    }
    case 1: r = normalize(mk3(in[0], in[1], in[2])); break;
    case 2: r = reflect(mk3(in[0], in[1], in[2]), mk3(in[3], in[4], in[5])); break;
    case 3: r = refract(mk3(in[0], in[1], in[2]), mk3(in[3], in[4], in[5]), in[6]); break;
    case 4: r = quat_rotate(in[0], mk3(in[1], in[2], in[3]), mk3(in[4], in[5], in[6])); break;
    default: return;
  }
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

}  // namespace kdpt
