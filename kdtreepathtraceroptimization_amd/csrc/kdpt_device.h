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
};

struct DevScene {
  const DevGeom* geoms;
  int num_geoms;
  const DevMaterial* materials;
  int num_materials;
  int has_obj;
  int num_nodes;
  int root;
  // nodes: box0 = {minx,miny,minz,maxx}, box1 = {maxy,maxz,left,right}, meta = {parent,triStart,triSize,axis}
  const float4* nbox0;
  const float4* nbox1;
  const int4* nmeta;
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

// traverseKDbareShortHybrid (HYBRID) / traverseKDbare, with the compact visited state.
template <bool HYBRID, bool COUNT>
KDPT_HD void traverseKD(const DevScene& S, const Ray& ray, Hit& h, int material_size, TraverseCounters& cnt) {
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
    const float4 b0 = S.nbox0[cur];
    const float4 b1 = S.nbox1[cur];
    const int4 meta = S.nmeta[cur];
    const int left = fbits(b1.z), right = fbits(b1.w), parent = meta.x;
    const int lvlbit = (L > 0) ? (2 * (L - 1) + (int)((ps >> (L - 1)) & 1u)) : 0;
    const bool curVis = (L == 0) ? rootv : (((cb >> lvlbit) & 1u) != 0u);
    if (!hitGeom && parent == -1 && curVis) break;
    hitGeom = intersectAABB(o, invdir, b0, b1, dist);
    if (COUNT) cnt.aabb++;
    bool up = false;
    if (curVis) {
      up = true;
    } else {
      if (!hitGeom && parent == -1) break;
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
struct WaveLeafLDS {
  int pend[64];    // inclusive end of each lane's pair range
  int tbase[64];   // triangle index = tbase[owner] + pair index
  float4 od[64];   // ray origin.xyz, direction.x
  float2 dd[64];   // direction.y, direction.z
  unsigned long long lastPass[64];  // ((tri + 1) << 32) | bary.z bits, max
  int lastHit[64];
  int nhit[64];
  unsigned long long best[64];  // (t bits << 32) | triangle index, min
};

constexpr int BIG_LEAF = 64;  // leaves this size or larger are swept by the whole wave, one at a time

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  return v;
}

__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// glm::intersectRayTriangle on (o, d) and triangle i; returns 0 = miss before the u/v
// tests passed, 1 = passed u/v but t < 0 (bary.z still written), 2 = intersected.
__device__ inline int tri_test(const DevScene& S, int i, f3 o, f3 d, float& bx, float& by, float& bz) {
  const float4 tv = S.tv0[i];
  const float4 e1v = S.te1[i];
  const float4 e2v = S.te2[i];
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

template <bool HYBRID>
__device__ inline float tri_hit_t(const DevScene& S, int i, f3 o, f3 d, float bx, float by, float bz, f3& hit,
                                  f3& norm) {
  const float4 n1v = S.tn0[i], n2v = S.tn1[i], n3v = S.tn2[i];
  const float w0 = 1 - bx - by;
  norm = normalize(add(add(scl(mk3(n1v.x, n1v.y, n1v.z), w0), scl(mk3(n2v.x, n2v.y, n2v.z), bx)),
                       scl(mk3(n3v.x, n3v.y, n3v.z), by)));
  hit = add(add(o, scl(d, bz)), scl(norm, HYBRID ? 0.0001f : 0.00001f));
  return distance(o, hit);
}

template <bool HYBRID, bool COUNT>
__device__ void traverseKD_wave(const DevScene& S, const Ray& ray, bool active, Hit& h, int material_size,
                                TraverseCounters& cnt, WaveLeafLDS* W) {
  const int lane = threadIdx.x & 63;
  const f3 o = ray.origin, d = ray.direction;
  W->od[lane] = make_float4(o.x, o.y, o.z, d.x);
  W->dd[lane] = make_float2(d.y, d.z);
  const f3 invdir = active ? mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z) : mk3(0, 0, 0);
  int cur = S.root, L = 0;
  uint32_t cb = 0, ps = 0, g = 0;
  bool rootv = false, sink = false, hitGeom = false;
  bool done = !active;
  float dist = -1.0f, bz = FLT_MAXV;
  while (true) {
    // ---------------- node phase ----------------
    bool leaf = false;
    int lstart = 0, lsize = 0;
    bool lfirst = true;
    while (!done && !leaf) {
      if (cur == -1) { done = true; break; }
      const float4 b0 = S.nbox0[cur];
      const float4 b1 = S.nbox1[cur];
      const int4 meta = S.nmeta[cur];
      const int left = fbits(b1.z), right = fbits(b1.w), parent = meta.x;
      const int lvlbit = (L > 0) ? (2 * (L - 1) + (int)((ps >> (L - 1)) & 1u)) : 0;
      const bool curVis = (L == 0) ? rootv : (((cb >> lvlbit) & 1u) != 0u);
      if (!hitGeom && parent == -1 && curVis) { done = true; break; }
      hitGeom = intersectAABB(o, invdir, b0, b1, dist);
      if (COUNT) cnt.aabb++;
      bool up = curVis;
      if (!curVis) {
        if (!hitGeom && parent == -1) { done = true; break; }
        up = (!hitGeom || dist > bz);
      }
      if (up) {
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
        cb &= ~(3u << (2u * (uint32_t)(L + 1)));
        if (L == 0 && nside == 0u) cb |= g << 2;
        L++;
        cur = next;
        continue;
      }
      if (L == 0) rootv = true; else cb |= 1u << lvlbit;
      if (meta.z > 0) {
        leaf = true;
        lstart = meta.y;
        lsize = meta.z;
        lfirst = leftFirst;
      }
    }
    if (!__any(leaf)) break;
    // ---------------- leaf phase (wave-cooperative) ----------------
    // per lane results of this phase
    int r_pass = 0;          // 0 = none, else tri + 1 of the last u/v pass
    float r_bz = 0.0f;
    int r_lasthit = -1, r_nhit = 0;
    unsigned long long r_best = ~0ull;
    // (a) big leaves: the whole wave sweeps one leaf at a time with a uniform ray
    const bool big = leaf && lsize >= BIG_LEAF;
    unsigned long long bigmask = __ballot(big);
    while (bigmask) {
      const int j = __builtin_ctzll(bigmask);
      bigmask &= bigmask - 1;
      const int jstart = __shfl(lstart, j), jsize = __shfl(lsize, j);
      const f3 jo = mk3(__shfl(o.x, j), __shfl(o.y, j), __shfl(o.z, j));
      const f3 jd = mk3(__shfl(d.x, j), __shfl(d.y, j), __shfl(d.z, j));
      int u_pass = 0, u_lasthit = -1, u_nhit = 0;
      float u_bz = 0.0f;
      unsigned long long u_best = ~0ull;
      for (int base = 0; base < jsize; base += 64) {
        const int k = base + lane;
        const int tri = jstart + k;
        float bx = 0, by = 0, bzk = 0;
        const int r = (k < jsize) ? tri_test(S, tri, jo, jd, bx, by, bzk) : 0;
        const unsigned long long m1 = __ballot(r >= 1);
        if (m1) {
          const int last = 63 - __builtin_clzll(m1);
          u_pass = jstart + base + last + 1;
          u_bz = __shfl(bzk, last);
          const unsigned long long m2 = __ballot(r == 2);
          if (m2) {
            u_lasthit = jstart + base + 63 - __builtin_clzll(m2);
            u_nhit += __builtin_popcountll(m2);
            unsigned long long key = ~0ull;
            if (r == 2) {
              f3 hp, nn;
              const float t = tri_hit_t<HYBRID>(S, tri, jo, jd, bx, by, bzk, hp, nn);
              if (t > 0.0f) key = ((unsigned long long)f2u(t) << 32) | (unsigned int)tri;
            }
            const unsigned long long wm = wave_min_u64(key);
            u_best = wm < u_best ? wm : u_best;
          }
        }
      }
      if (lane == j) {
        r_pass = u_pass;
        r_bz = u_bz;
        r_lasthit = u_lasthit;
        r_nhit = u_nhit;
        r_best = u_best;
      }
    }
    // (b) small leaves: all (ray, triangle) pairs spread over the 64 lanes
    const int sz = (leaf && !big) ? lsize : 0;
    if (__any(sz > 0)) {
      int incl = sz;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
      }
      const int P = __shfl(incl, 63);
      W->pend[lane] = incl;
      W->tbase[lane] = lstart - (incl - sz);
      W->lastPass[lane] = 0ull;
      W->lastHit[lane] = -1;
      W->nhit[lane] = 0;
      W->best[lane] = ~0ull;
      wave_lds_sync();
      for (int pi = lane; pi < P; pi += 64) {
        int lo = 0, hi = 63;
#pragma unroll
        for (int st = 0; st < 6; st++) {
          const int mid = (lo + hi) >> 1;
          if (W->pend[mid] > pi) hi = mid; else lo = mid + 1;
        }
        const int owner = lo;
        const int tri = W->tbase[owner] + pi;
        const float4 q0 = W->od[owner];
        const float2 q1 = W->dd[owner];
        const f3 oo = mk3(q0.x, q0.y, q0.z), dd = mk3(q0.w, q1.x, q1.y);
        float bx, by, bzk;
        const int r = tri_test(S, tri, oo, dd, bx, by, bzk);
        if (r == 0) continue;
        atomicMax(&W->lastPass[owner], ((unsigned long long)(unsigned int)(tri + 1) << 32) | f2u(bzk));
        if (r == 1) continue;
        atomicMax(&W->lastHit[owner], tri);
        atomicAdd(&W->nhit[owner], 1);
        f3 hp, nn;
        const float t = tri_hit_t<HYBRID>(S, tri, oo, dd, bx, by, bzk, hp, nn);
        if (t > 0.0f) atomicMin(&W->best[owner], ((unsigned long long)f2u(t) << 32) | (unsigned int)tri);
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
          if (h.t_min > tb) {
            float bx, by, bzk;
            tri_test(S, k, o, d, bx, by, bzk);
            f3 hp, nn;
            h.t_min = tri_hit_t<HYBRID>(S, k, o, d, bx, by, bzk, hp, nn);
            h.hit_geom_index = S.obj_material_offsets[fbits(S.tv0[k].w)];
            h.ip = hp;
            h.normal = nn;
            h.obj_intersect = true;
          }
        }
      }
    }
  }
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
// :67-83 -- double cos/sin/acos: non-default (softness/SSS) branches only; device libm,
// equal to glibc up to the rare double->float rounding boundary (documented tolerance).
KDPT_HD f3 randSphericalVec(float angle, Rng& rng) {
  double theta = 2 * PI_F * u01(rng);
  double phi = acosf((angle * PI_F * u01(rng) - 1.0f));
  f3 V = mk3((float)(cos(theta) * sin(phi)), (float)(sin(theta) * sin(phi)), (float)cos(phi));
  return normalize(V);
}
KDPT_HD float getFresnelVal(f3 I, f3 N, float R0) {  // :127-133
  double F = (double)R0 + (double)(1.0f - R0) * pow5((double)(1.0f - dot(N, neg(I))));
  return (float)F;
}
KDPT_HD f3 soft_lobe(f3 dir, Rng& rng) {
  f3 v = randSphericalVec(0.02f, rng);
  float angle = acosf(dot(mk3(0.0f, 0.0f, -1.0f), dir));
  f3 axis = normalize(cross(mk3(0.0f, 0.0f, -1.0f), dir));
  return rotateVector(v, axis, angle);
}
// :195-358
KDPT_HD void scatterRay(Ray& ray, f3 intersect, f3 normal, const DevMaterial& m, Rng& rng, float softness) {
  if (m.transmittance[0] > 0.0f || m.transmittance[1] > 0.0f || m.transmittance[2] > 0.0f) {
    float randval = u01(rng);
    if (randval < 0.5f && !ray.isinside) {
      f3 v = randSphericalVec(0.0001f, rng);
      float angle = acosf(dot(mk3(0.0f, 0.0f, -1.0f), ray.direction));
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

}  // namespace kdpt
