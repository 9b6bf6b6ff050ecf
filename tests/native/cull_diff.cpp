// TEST INFRASTRUCTURE: differential test of the intersect kernel's cluster cull (kdpt_device.h
// cluster_may_pass / cluster_may_pass_slab, the half-precision super-cluster boxes, and the brute-force
// route's chunk boxes; all compiled here for the host) against glm's float u/v tests (tri_test_v, pinned
// bit for bit to the reference's glm::intersectRayTriangle, gtx/intersect.inl:37-74).
//
// The cull may drop a (line, cluster) pair only if no triangle of the cluster passes glm's u/v tests for
// that line -- with ANY t, since a pass with t < 0 still writes bary.z, which the reference's traversal
// reads (`dist > bary.z`, src/pathtrace.cu:1095).  A violation is a culled pair with such a triangle.
//
//   cull_diff TREE.bin NLINES SEED [MARGIN]
// TREE.bin: int32 num_nodes, int32 num_tris, kdpt_node_bare[num_nodes], kdpt_tri_bare[num_tris]
// (the product's host builder output).  MARGIN overrides the scene's margin coefficient (default: the one
// kdpt_create uses, cluster_margin()).  Prints one JSON line of counts per line generator.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define KDPT_RCP_ULP  // kd_rcp follows kdpt_rcp_ulp (the device reciprocal's 1-ulp error)
#include "../../kdtreepathtraceroptimization_amd/csrc/kdpt_clusters.h"

// the masked cull's box coefficient and mask resolution: the product's (cluster_margin, dir_mask_resolution)
// unless MASK_KF / MASK_N say otherwise
static float mask_kf() { return getenv("MASK_KF") ? (float)atof(getenv("MASK_KF")) : kdpt::CULL_MARGIN_MASKED; }
static int mask_res(int ncl) { return getenv("MASK_N") ? atoi(getenv("MASK_N")) : kdpt::dir_mask_resolution(ncl); }

using namespace kdpt;

namespace kdpt {
thread_local int kdpt_rcp_ulp = 0;  // kd_rcp's perturbation (KDPT_RCP_ULP): the lines are checked at -1, 0, +1
}

namespace {

enum Gen { G_RANDOM, G_GRAZE, G_GRAZE_EDGE, G_FACE, G_AXIS, G_SUPER_EDGE, G_ROUND, NGEN };
const char* kGenName[NGEN] = {"random", "graze", "graze_edge", "face", "axis", "super_edge", "round"};

struct Counts {
  long long lines = 0, pass = 0;           // lines tested, (line, cluster) pairs with a u/v pass
  long long culled_box = 0, viol_box = 0;  // one-level cull (dragon_5's LDS route)
  long long viol_slab = 0, viol_super = 0, viol_chunk = 0, viol_obb = 0;
  long long viol_mask = 0, mask_items = 0, mask_needed = 0;  // the exact one-level cull (build_dir_masks)
  long long nofast = 0;                    // some invdir component infinite: the wave does not cull
  long long margin_used = 0;               // passing pairs the box cull passes only thanks to the margin
  // over the passing (line, triangle) pairs: the largest distance of the line's exact crossing of the
  // triangle's plane outside the cluster's box, in margins (a violation needs about 1 or more)
  double worst = 0.0;
  double bound = 0.0;  // the largest distance / error bound over every pass (must be <= 1)
  void add(const Counts& o) {
    lines += o.lines; pass += o.pass; culled_box += o.culled_box; viol_box += o.viol_box;
    viol_slab += o.viol_slab; viol_super += o.viol_super; viol_chunk += o.viol_chunk; viol_obb += o.viol_obb;
    viol_mask += o.viol_mask; mask_items += o.mask_items; mask_needed += o.mask_needed;
    nofast += o.nofast; margin_used += o.margin_used; worst = std::max(worst, o.worst);
    bound = std::max(bound, o.bound);
  }
};

struct V3 { double x, y, z; };
V3 v3(double x, double y, double z) { return V3{x, y, z}; }
V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
double dotd(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 crossd(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
V3 unitd(V3 a) { return a * (1.0 / std::sqrt(dotd(a, a))); }
double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
void setc(V3& a, int i, double v) { (i == 0 ? a.x : (i == 1 ? a.y : a.z)) = v; }
V3 of4(float4 q) { return v3(q.x, q.y, q.z); }

// Where the float line (o, d) crosses the plane of the float triangle (v0, e1, e2), in long double (the
// inputs are exact floats; Cramer's rule with 64-bit mantissas), and how far that point lies outside the box
// [L, H] (infinity norm) in units of the cull's margin for that box.
double out_ratio(f3 o, f3 d, float4 v0, float4 e1, float4 e2, float4 L, float4 H, float K) {
  typedef long double ld;
  const ld ox = o.x, oy = o.y, oz = o.z, dx = d.x, dy = d.y, dz = d.z;
  const ld ax = e1.x, ay = e1.y, az = e1.z, bx = e2.x, by = e2.y, bz = e2.z;
  const ld sx = ox - (ld)v0.x, sy = oy - (ld)v0.y, sz = oz - (ld)v0.z;
  const ld px = dy * bz - dz * by, py = dz * bx - dx * bz, pz = dx * by - dy * bx;
  const ld a = ax * px + ay * py + az * pz;
  if (a == 0) return 1e30;
  const ld qx = sy * az - sz * ay, qy = sz * ax - sx * az, qz = sx * ay - sy * ax;
  const ld t = (bx * qx + by * qy + bz * qz) / a;
  const ld y[3] = {ox + t * dx, oy + t * dy, oz + t * dz};
  const ld lo[3] = {L.x, L.y, L.z}, hi[3] = {H.x, H.y, H.z};
  ld out = 0, dist = 1, size = 0;
  for (int k = 0; k < 3; k++) {
    out = std::max(out, std::max(lo[k] - y[k], y[k] - hi[k]));
    const ld c = 0.5L * (lo[k] + hi[k]);
    dist += std::fabs((k == 0 ? ox : (k == 1 ? oy : oz)) - c);
    size += hi[k] - lo[k];
  }
  return (double)(out / ((ld)K * (dist + size)));
}

// Rays of a real render (origin.xyz, direction.xyz as float32, e.g. the oracle's paths after each bounce):
// every ray against EVERY cluster (not only those its traversal reaches), each cull (box, box + slab, the
// super's half-precision box) that drops the pair checked against the 64 triangles' u/v tests.
int rays_check(const char* path, const ClusterSet& cs, float K, const CullK& ck) {
  FILE* f = fopen(path, "rb");
  if (!f) return 3;
  std::vector<float> r;
  float buf[6];
  while (fread(buf, sizeof(float), 6, f) == 6) r.insert(r.end(), buf, buf + 6);
  fclose(f);
  const long long nr = (long long)(r.size() / 6);
  const int ncl = (int)cs.info.size();
  std::vector<int> super_of(ncl, -1);
  for (size_t s = 0; s < cs.sup.size(); s++) {
    const uint32_t w = (uint32_t)cs.sup[s].w;
    for (uint32_t k = 0; k <= (w & 31u); k++) super_of[(w >> 5) + k] = (int)s;
  }
  long long pairs = 0, culled = 0, viol_box = 0, viol_slab = 0, viol_super = 0, viol_obb = 0, nofast = 0, passes = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : pairs, culled, viol_box, viol_slab, viol_super, viol_obb, nofast, passes)
  for (long long i = 0; i < nr; i++) {
    const f3 o = mk3(r[6 * i], r[6 * i + 1], r[6 * i + 2]), d = mk3(r[6 * i + 3], r[6 * i + 4], r[6 * i + 5]);
    const f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    if (!(fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV)) {
      nofast++;
      continue;
    }
    for (int c = 0; c < ncl; c++) {
      pairs++;
      const float4 L = cs.lo[c], H = cs.hi[c];
      const bool box = cluster_may_pass(L, H, o, inv, K);
      const bool slab = cluster_may_pass_slab(L, H, cs.nrm[c], o, inv, d, ck);
      const bool obb = cluster_may_pass_obb(L, H, cs.nrm[c], cs.obb_u[c], cs.obb_v[c], cs.obb_w[c], o, inv, d, ck);
      bool sup = true;
      if (super_of[c] >= 0) {
        const int4 q = cs.sup[super_of[c]];
        const float4 sl = make_float4(half_lo((uint32_t)q.x), half_hi((uint32_t)q.x), half_lo((uint32_t)q.y), 0);
        const float4 sh = make_float4(half_hi((uint32_t)q.y), half_lo((uint32_t)q.z), half_hi((uint32_t)q.z), 0);
        sup = cluster_may_pass(sl, sh, o, inv, K);
        const float4 sb = cs.sup_b[super_of[c]];
        sup = sup && cluster_may_pass_slab(make_float4(sl.x, sl.y, sl.z, sb.x), make_float4(sh.x, sh.y, sh.z, sb.y),
                                           cs.sup_n[super_of[c]], o, inv, d, ck);
      }
      if (box && slab && sup && obb) continue;
      culled++;
      const int2 inf = cs.info[c];
      bool pass = false;
      for (int k = 0; k < inf.y && !pass; k++) {
        float bx, by, bz;
        pass = tri_test_v(TriData{cs.cv0[inf.x + k], cs.ce1[inf.x + k], cs.ce2[inf.x + k]}, o, d, bx, by, bz) >= 1;
      }
      if (pass) {
        passes++;
        viol_box += !box;
        viol_slab += !slab;
        viol_super += !sup;
        viol_obb += !obb;
      }
    }
  }
  printf("{\"rays\": %lld, \"clusters\": %d, \"margin\": %.9g, \"pairs\": %lld, \"culled\": %lld, \"nofast\": %lld, "
         "\"viol_box\": %lld, \"viol_slab\": %lld, \"viol_super\": %lld, \"viol_obb\": %lld, \"violations\": %lld}\n",
         nr, ncl, (double)K, pairs, culled, nofast, viol_box, viol_slab, viol_super, viol_obb,
         viol_box + viol_slab + viol_super + viol_obb);
  return 0;
}

// The error bound of DESIGN.md 4 ("Cluster cull") for one passing (line, triangle): the distance from the
// line to the point v0 + u e1 + v e2 that glm's float test accepted, over the bound
// 17.34 u |o - v0| |e1| |e2| / a + 2.1 u max(|e1|, |e2|) + 2 u |o - v0| (a: glm's float determinant; the last
// term: the line through the float o - v0 instead of o).  Must stay <= 1.
double bound_ratio(f3 o, f3 d, float4 v0, float4 e1, float4 e2, float bx, float by) {
  typedef long double ld;
  const f3 p = cross(d, mk3(e2.x, e2.y, e2.z));
  const float a = dot(mk3(e1.x, e1.y, e1.z), p);  // the determinant as glm computes it
  const ld x[3] = {(ld)v0.x + (ld)bx * e1.x + (ld)by * e2.x, (ld)v0.y + (ld)bx * e1.y + (ld)by * e2.y,
                   (ld)v0.z + (ld)bx * e1.z + (ld)by * e2.z};
  const ld w[3] = {x[0] - o.x, x[1] - o.y, x[2] - o.z};
  const ld dd[3] = {d.x, d.y, d.z};
  const ld dl2 = dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2];
  const ld t = (w[0] * dd[0] + w[1] * dd[1] + w[2] * dd[2]) / dl2;
  ld dist2 = 0;
  for (int k = 0; k < 3; k++) dist2 += (w[k] - t * dd[k]) * (w[k] - t * dd[k]);
  const ld s = std::sqrt(((ld)o.x - v0.x) * ((ld)o.x - v0.x) + ((ld)o.y - v0.y) * ((ld)o.y - v0.y) +
                         ((ld)o.z - v0.z) * ((ld)o.z - v0.z));
  const ld l1 = std::sqrt((ld)e1.x * e1.x + (ld)e1.y * e1.y + (ld)e1.z * e1.z);
  const ld l2 = std::sqrt((ld)e2.x * e2.x + (ld)e2.y * e2.y + (ld)e2.z * e2.z);
  const ld u = 5.9604644775390625e-8L;
  const ld bound = 17.34L * u * s * l1 * l2 / (ld)a + 2.1L * u * std::max(l1, l2) + 2.0L * u * s;
  return (double)(std::sqrt(dist2) / bound);
}

// The product's masked cull (kdpt_device.h trace_phase, one-level route) for a (line, cluster) pair whose line
// missed the cluster's fast-margin box or oriented box: the pair's cell (dir_bucket) and its danger mask, and the
// mask's triangles that danger_needs_test keeps (those get glm's u/v tests).
struct MaskTables {
  int n = 0, ncl = 0;
  float c = 0.0f;
  std::vector<unsigned long long> masks;  // bucket-major, DevScene::cl_mask
  std::vector<float4> tn;                 // DevScene::cl_tn
  void build(const ClusterSet& cs, int res, float Kf, float cc) {
    n = res;
    ncl = (int)cs.info.size();
    c = cc;
    build_dir_masks(cs, n, Kf, masks);
    build_entry_normals(cs, tn);
  }
  unsigned long long needs(int cl, float4 L, float4 H, f3 o, f3 inv, f3 d, int& items) const {
    unsigned long long m = masks[(size_t)dir_bucket(d, n) * ncl + cl], nm = 0ull;
    items = 0;
    const float D = box_miss(L, H, o, inv);
    while (m) {
      const int k = __builtin_ctzll(m);
      m &= m - 1;
      items++;
      if (danger_needs_test(tn[64 * (size_t)cl + k], d, D, c)) nm |= 1ull << k;
    }
    return nm;
  }
  // the same with kd_rcp's quotient moved by -1, 0 and +1 ulp (v_rcp_f32's error): the triangles kept under
  // every one of them (a pass must be kept under each); the item count of the unperturbed one
  unsigned long long needs_all(int cl, float4 L, float4 H, f3 o, f3 inv, f3 d, int& items) const {
    unsigned long long all = ~0ull;
    for (int p : {0, -1, 1}) {
      kdpt_rcp_ulp = p;
      int it;
      all &= needs(cl, L, H, o, inv, d, it);
      if (p == 0) items = it;
    }
    kdpt_rcp_ulp = 0;
    return all;
  }
};

// Cull statistics of real rays through the traversal (--sim): each ray walks the tree (traverseKD, compiled
// here for the host); for every big leaf it tests, every cluster of the leaf is evaluated with the fast cull (box
// at the scene margin + oriented box at cull_margin_dir) and with the product's masked cull (box and oriented
// box at the masked cull's coefficient Kf; a missed pair's mask and danger_needs_test, under each of the three
// reciprocal perturbations).  A pair a cull drops while a triangle passes glm's u/v tests, or a
// passing triangle the masked cull does not test, is a violation.
int sim(const char* path, const kdpt_node_bare* nodes, int nn, const kdpt_tri_bare* tris, int nt,
        const std::vector<float4>& tv, const std::vector<float4>& e1, const std::vector<float4>& e2,
        const ClusterGrouping& grp) {
  FILE* f = fopen(path, "rb");
  if (!f) return 3;
  std::vector<float> r;
  float buf[6];
  while (fread(buf, sizeof(float), 6, f) == 6) r.insert(r.end(), buf, buf + 6);
  fclose(f);
  const long long nr = (long long)(r.size() / 6);
  ClusterSet cs;
  build_cluster_set(nodes, nn, tris, tv, e1, e2, cs, grp);
  const CullMargin cm = cluster_margin(cs.cv0, cs.ce1, cs.ce2);
  const CullK ck{cm.K, cm.K_lo, cm.a, cm.b, cm.c};
  std::vector<int4> nd4(4 * (size_t)nn);
  for (int i = 0; i < nn; i++) {
    const kdpt_node_bare& N = nodes[i];
    nd4[4 * i] = int4{fbits(N.mins[0]), fbits(N.mins[1]), fbits(N.mins[2]), fbits(N.maxs[0])};
    nd4[4 * i + 1] = int4{fbits(N.maxs[1]), fbits(N.maxs[2]), N.leftID, N.rightID};
    nd4[4 * i + 2] = int4{N.parentID, N.triIdStart, N.triIdSize, N.axis};
    nd4[4 * i + 3] = int4{0, 0, 0, 0};
  }
  std::vector<float4> n0(nt), n1(nt), n2(nt);
  for (int i = 0; i < nt; i++) {
    n0[i] = float4{tris[i].nx1, tris[i].ny1, tris[i].nz1, 0};
    n1[i] = float4{tris[i].nx2, tris[i].ny2, tris[i].nz2, 0};
    n2[i] = float4{tris[i].nx3, tris[i].ny3, tris[i].nz3, 0};
  }
  std::vector<int> offs(64, 0);
  DevScene S{};
  S.num_nodes = nn;
  S.root = 0;
  S.nodes = nd4.data();
  S.tv0 = tv.data(); S.te1 = e1.data(); S.te2 = e2.data();
  S.tn0 = n0.data(); S.tn1 = n1.data(); S.tn2 = n2.data();
  S.obj_material_offsets = offs.data();
  S.n0_left = nodes[0].leftID; S.n0_right = nodes[0].rightID;
  S.n1_left = nn > 1 ? nodes[1].leftID : -1; S.n1_right = nn > 1 ? nodes[1].rightID : -1;
  long long leaves = 0, pairs = 0, old_sw = 0, msk_sw = 0, prod = 0, viol_old = 0, nofast = 0, small_tris = 0,
            old_tris = 0, msk_missed = 0, msk_nonzero = 0, msk_items = 0, viol_msk = 0, msk_needed = 0;
  const float KF = mask_kf();
  MaskTables mt;
  mt.build(cs, mask_res((int)cs.info.size()), KF, cm.c);
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : leaves, pairs, old_sw, msk_sw, prod, viol_old, nofast, small_tris, old_tris, msk_missed, msk_nonzero, msk_items, viol_msk, msk_needed)
  for (long long i = 0; i < nr; i++) {
    const f3 o = mk3(r[6 * i], r[6 * i + 1], r[6 * i + 2]), d = mk3(r[6 * i + 3], r[6 * i + 4], r[6 * i + 5]);
    const f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const bool fast = fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV;
    if (!fast) nofast++;
    std::vector<int> visited;
    Ray ray;
    ray.origin = o;
    ray.direction = d;
    ray.isinside = false;
    ray.sdepth = 0;
    Hit h;
    h.t_min = FLT_MAXV; h.hit_geom_index = -1; h.obj_intersect = false; h.objMaterialIdx = -1;
    h.ip = mk3(0, 0, 0); h.normal = mk3(0, 0, 0);
    TraverseCounters cnt{0, 0, 0};
    traverseKD<true, false>(S, ray, h, 1, cnt, [&](int node) {
      if (nodes[node].triIdSize >= BIG_LEAF) visited.push_back(node);
      else small_tris += nodes[node].triIdSize;
    });
    for (int node : visited) {
      leaves++;
      const int2 lc = cs.leaf_cl[node];
      for (int c = lc.x; c < lc.x + lc.y; c++) {
        pairs++;
        const int2 inf = cs.info[c];
        unsigned long long passes = 0ull;  // the cluster's triangles that pass glm's u/v tests
        for (int k = 0; k < inf.y; k++) {
          float bx, by, bz;
          if (tri_test_v(TriData{cs.cv0[inf.x + k], cs.ce1[inf.x + k], cs.ce2[inf.x + k]}, o, d, bx, by, bz) >= 1)
            passes |= 1ull << k;
        }
        prod += passes != 0ull;
        if (!fast) {
          old_sw++;
          msk_sw++;
          continue;
        }
        const float4 L = cs.lo[c], H = cs.hi[c], n = cs.nrm[c];
        const bool ok_old = cluster_may_pass(L, H, o, inv, cm.K) &&
                            cluster_may_pass_obb(L, H, n, cs.obb_u[c], cs.obb_v[c], cs.obb_w[c], o, inv, d, ck);
        old_sw += ok_old;
        old_tris += ok_old ? inf.y : 0;
        viol_old += passes && !ok_old;
        const float ndv = n.x * d.x + n.y * d.y + n.z * d.z;
        const bool hit = cluster_may_pass(L, H, o, inv, KF) &&
                         cluster_may_pass_obb_k(L, H, n, cs.obb_u[c], cs.obb_v[c], cs.obb_w[c], o, inv, d, ndv, KF);
        if (hit) {
          msk_sw++;
          continue;
        }
        msk_missed++;
        int items;
        const unsigned long long nm = mt.needs_all(c, L, H, o, inv, d, items);
        msk_nonzero += items > 0;
        msk_items += items;
        msk_needed += __builtin_popcountll(nm);
        viol_msk += (passes & ~nm) != 0ull;
      }
    }
  }
  const double R = (double)std::max(1LL, nr);
  printf("{\"rays\": %lld, \"clusters\": %zu, \"mode\": %d, \"chord\": %g, \"big_leaves_per_ray\": %.4f, "
         "\"pairs_per_ray\": %.4f, \"sweeps_old\": %.4f, \"sweeps_masked\": %.4f, \"productive\": %.4f, "
         "\"viol_old\": %lld, \"nofast\": %lld, \"small_tris\": %.3f, \"old_tris\": %.3f, \"mask_n\": %d, "
         "\"msk_missed\": %.4f, \"msk_nonzero\": %.4f, \"msk_items\": %.4f, \"msk_needed\": %.4f, \"viol_msk\": %lld}\n",
         nr, cs.info.size(), grp.mode, grp.chord, leaves / R, pairs / R, old_sw / R, msk_sw / R, prod / R, viol_old,
         nofast, small_tris / R, old_tris / R, mt.n, msk_missed / R, msk_nonzero / R, msk_items / R, msk_needed / R,
         viol_msk);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: cull_diff TREE.bin NLINES SEED [MARGIN]\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 3;
  int nn = 0, nt = 0;
  if (fread(&nn, 4, 1, f) != 1 || fread(&nt, 4, 1, f) != 1 || nn <= 0 || nt <= 0) return 3;
  std::vector<kdpt_node_bare> nodes(nn);
  std::vector<kdpt_tri_bare> tris(nt);
  if (fread(nodes.data(), sizeof(kdpt_node_bare), nn, f) != (size_t)nn ||
      fread(tris.data(), sizeof(kdpt_tri_bare), nt, f) != (size_t)nt)
    return 3;
  fclose(f);
  const bool rays_mode = strcmp(argv[2], "--rays") == 0;
  const long long nlines = rays_mode ? 0 : atoll(argv[2]);
  const unsigned seed = (unsigned)atoi(argv[3]);
  // the triangle records exactly as kdpt_create forms them (e1 = v1 - v0, e2 = v2 - v0 in float)
  std::vector<float4> tv(nt), e1(nt), e2(nt);
  for (int i = 0; i < nt; i++) {
    const kdpt_tri_bare& T = tris[i];
    tv[i] = make_float4(T.x1, T.y1, T.z1, ibits(T.mtlIdx));
    e1[i] = make_float4(T.x2 - T.x1, T.y2 - T.y1, T.z2 - T.z1, 0.0f);
    e2[i] = make_float4(T.x3 - T.x1, T.y3 - T.y1, T.z3 - T.z1, 0.0f);
  }
  if (strcmp(argv[2], "--masks") == 0) {
    // cull_diff TREE --masks OUT.bin: the masks kdpt_create builds on the device for this tree (the scene's
    // masked-cull coefficient and resolution), from the host builder: int32 n, int32 num_clusters, float Kf,
    // uint64 masks[6 n^2][num_clusters]
    ClusterSet cs;
    build_cluster_set(nodes.data(), nn, tris.data(), tv, e1, e2, cs);
    const CullMargin cm = cluster_margin(cs.cv0, cs.ce1, cs.ce2);
    const int n = mask_res((int)cs.info.size()), ncl = (int)cs.info.size();
    std::vector<unsigned long long> masks;
    build_dir_masks(cs, n, cm.K, masks);
    FILE* g = fopen(argv[3], "wb");
    if (!g) return 3;
    const bool ok = fwrite(&n, 4, 1, g) == 1 && fwrite(&ncl, 4, 1, g) == 1 && fwrite(&cm.K, 4, 1, g) == 1 &&
                    fwrite(masks.data(), 8, masks.size(), g) == masks.size();
    fclose(g);
    long long nz = 0;
    for (size_t k = 0; k < masks.size(); k++) nz += masks[k] != 0ull;
    printf("{\"n\": %d, \"clusters\": %d, \"kf\": %.9g, \"exact\": %d, \"nonzero\": %lld, \"cells\": %zu}\n",
           n, ncl, (double)cm.K, (int)cm.exact, nz, masks.size());
    return ok ? 0 : 3;
  }
  if (strcmp(argv[2], "--sim") == 0) {
    ClusterGrouping grp;
    grp.mode = argc > 4 ? atoi(argv[4]) : 0;
    grp.chord = argc > 5 ? atof(argv[5]) : 0.5;
    grp.min_split = argc > 6 ? atoi(argv[6]) : 8;
    return sim(argv[3], nodes.data(), nn, tris.data(), nt, tv, e1, e2, grp);
  }
  ClusterSet cs;
  // CLUSTER_CHORD > 0: the normal-cone grouping kdpt_create uses for meshes with a rigorous margin
  // (kdpt_runtime.hip build_clusters, CLUSTER_CHORD_EXACT)
  ClusterGrouping grouping;
  if (getenv("CLUSTER_CHORD") && atof(getenv("CLUSTER_CHORD")) > 0) {
    grouping.mode = 1;
    grouping.chord = atof(getenv("CLUSTER_CHORD"));
  }
  build_cluster_set(nodes.data(), nn, tris.data(), tv, e1, e2, cs, grouping);
  std::vector<float4> clo, chi;
  build_chunk_boxes(tv, e1, e2, nt, clo, chi);
  const CullMargin cm = cluster_margin(cs.cv0, cs.ce1, cs.ce2);
  // the kernels' margins: the scene's (box-only levels cm.K, the slab level direction-dependent), or one
  // fixed coefficient for every level when MARGIN is given (tuning "cull_margin")
  const float K = argc > 4 ? (float)atof(argv[4]) : cm.K;
  const CullK ck = argc > 4 ? CullK{K, K, cm.a, cm.b, cm.c} : CullK{cm.K, cm.K_lo, cm.a, cm.b, cm.c};
  if (rays_mode) return rays_check(argv[3], cs, K, ck);
  const int ncl = (int)cs.info.size();
  if (ncl == 0) {
    printf("{\"clusters\": 0}\n");
    return 0;
  }
  // super of each cluster
  std::vector<int> super_of(ncl, -1);
  for (size_t s = 0; s < cs.sup.size(); s++) {
    const uint32_t w = (uint32_t)cs.sup[s].w;
    for (uint32_t k = 0; k <= (w & 31u); k++) super_of[(w >> 5) + k] = (int)s;
  }
  // chunk (brute-force route) of each triangle: chunks are file order; the test evaluates the chunk of the
  // triangle that generated the line, with that chunk's 64 triangles
  const float4 rlo = make_float4(nodes[0].mins[0], nodes[0].mins[1], nodes[0].mins[2], 0);
  const float4 rhi = make_float4(nodes[0].maxs[0], nodes[0].maxs[1], nodes[0].maxs[2], 0);
  const V3 slo = v3(rlo.x, rlo.y, rlo.z), shi = v3(rhi.x, rhi.y, rhi.z);
  const V3 sext = shi - slo;
  const double scale = std::max(sext.x, std::max(sext.y, sext.z));

  const float KF = mask_kf();
  MaskTables mt;
  mt.build(cs, mask_res((int)cs.info.size()), KF, cm.c);
  Counts tot[NGEN];
  const int nthreads = 1;
#pragma omp parallel
  {
    Counts loc[NGEN];
#pragma omp for schedule(dynamic, 4096)
    for (long long r = 0; r < nlines; r++) {
      std::mt19937_64 rng(seed * 0x9E3779B97F4A7C15ull + (unsigned long long)r);
      std::uniform_real_distribution<double> U(0.0, 1.0);
      auto logu = [&](double a, double b) { return std::pow(10.0, a + (b - a) * U(rng)); };
      auto sgn = [&]() { return U(rng) < 0.5 ? -1.0 : 1.0; };
      const int g = (int)(r % NGEN);
      const int c = (int)(U(rng) * ncl) % ncl;
      const int2 inf = cs.info[c];
      const int ent = inf.x + (int)(U(rng) * inf.y) % inf.y;  // a triangle of the cluster
      const V3 p0 = of4(cs.cv0[ent]), a1 = of4(cs.ce1[ent]), a2 = of4(cs.ce2[ent]);
      const V3 nrm = crossd(a1, a2);
      const double nl = std::sqrt(dotd(nrm, nrm));
      const float4 L = cs.lo[c], H = cs.hi[c];
      const V3 bl = of4(L), bh = of4(H), bc = (bl + bh) * 0.5, bs = bh - bl;
      V3 o, d;
      if (g == G_RANDOM || nl == 0.0) {
        // origin anywhere around the mesh, aimed at a point of the cluster's box grown by 50 %
        o = slo - sext * 0.5 + v3(sext.x * 2 * U(rng), sext.y * 2 * U(rng), sext.z * 2 * U(rng));
        const V3 t = bl - bs * 0.25 + v3(bs.x * 1.5 * U(rng), bs.y * 1.5 * U(rng), bs.z * 1.5 * U(rng));
        d = unitd(t - o);
      } else if (g == G_GRAZE || g == G_GRAZE_EDGE || g == G_SUPER_EDGE) {
        // nearly in the plane of the triangle: in-plane direction tilted by 1e-7.5 .. 1e-2 rad (or 0), through
        // a point of the plane near the triangle (G_GRAZE) or just outside the cluster's (super's) box near one
        // of the triangle's vertices (G_GRAZE_EDGE / G_SUPER_EDGE), offset off the plane by 0 .. 1e-3
        const V3 n = nrm * (1.0 / nl);
        const V3 ax = unitd(a1), ay = crossd(n, ax);
        const double phi = 2 * M_PI * U(rng);
        const V3 w = ax * std::cos(phi) + ay * std::sin(phi);
        const double th = U(rng) < 0.05 ? 0.0 : logu(-7.5, -2.0);
        d = w * std::cos(th) + n * (sgn() * std::sin(th));
        V3 x;
        if (g == G_GRAZE) {
          x = p0 + a1 * (-1.0 + 3.0 * U(rng)) + a2 * (-1.0 + 3.0 * U(rng));
        } else {
          const int vk = (int)(U(rng) * 3) % 3;
          x = vk == 0 ? p0 : (vk == 1 ? p0 + a1 : p0 + a2);
          V3 blo = bl, bhi = bh;
          if (g == G_SUPER_EDGE && super_of[c] >= 0) {
            const int4 q = cs.sup[super_of[c]];
            blo = v3(half_lo((uint32_t)q.x), half_hi((uint32_t)q.x), half_lo((uint32_t)q.y));
            bhi = v3(half_hi((uint32_t)q.y), half_lo((uint32_t)q.z), half_hi((uint32_t)q.z));
          }
          // push the point out through the box face nearest to the vertex, 0.2 .. 20 margins (at unit
          // distance) beyond it
          int best = 0;
          double bd = 1e300, side = 1;
          for (int a = 0; a < 3; a++) {
            const double dl = comp(x, a) - comp(blo, a), dh = comp(bhi, a) - comp(x, a);
            if (dl < bd) { bd = dl; best = a; side = -1; }
            if (dh < bd) { bd = dh; best = a; side = 1; }
          }
          const double mb = 1e-4 * (1.0 + scale) * logu(-0.7, 1.3);
          setc(x, best, (side < 0 ? comp(blo, best) : comp(bhi, best)) + side * mb);
        }
        const double h = U(rng) < 0.3 ? 0.0 : sgn() * logu(-9.0, -3.0) * scale;
        x = x + n * h;
        const double tau = sgn() * logu(-2.0, 1.2) * scale;  // origin on either side of the point
        o = x - d * tau;
      } else if (g == G_ROUND) {
        // rounding-induced passes: a line in the plane of the triangle, through a point beyond one of its
        // vertices and outside the cluster's box by 0.3 .. 30 margins, running parallel to that box face (so
        // the exact line stays outside the box), tilted so that glm's determinant is 1 .. 100 x FLT_EPSILON:
        // there the float u/v values carry errors of order |s| |e| u / a
        const V3 n = nrm * (1.0 / nl);
        const int vk = (int)(U(rng) * 3) % 3;
        V3 x = vk == 0 ? p0 : (vk == 1 ? p0 + a1 : p0 + a2);
        int best = 0;
        double bd = 1e300, side = 1;
        for (int a = 0; a < 3; a++) {
          const double dl = comp(x, a) - comp(bl, a), dh = comp(bh, a) - comp(x, a);
          if (dl < bd) { bd = dl; best = a; side = -1; }
          if (dh < bd) { bd = dh; best = a; side = 1; }
        }
        const double tau = sgn() * logu(-1.0, 0.7) * scale;
        const double mloc = 1e-4 * (1.0 + std::fabs(tau) + bs.x + bs.y + bs.z);
        // push the vertex out of the box within the plane: along the in-plane part of the face's axis, so
        // that the point stays in the plane and its coordinate on that axis clears the face by D
        V3 ea = v3(0, 0, 0);
        setc(ea, best, side);
        const V3 q = ea - n * dotd(n, ea);
        const double qa = std::fabs(comp(q, best));
        const double D = (side < 0 ? comp(x, best) - comp(bl, best) : comp(bh, best) - comp(x, best)) +
                         mloc * logu(-0.5, 1.5);
        if (qa > 1e-3) x = x + q * (D / qa);
        V3 w = crossd(n, ea);  // in the plane and parallel to the face: the line keeps its distance to it
        const double wl = std::sqrt(dotd(w, w));
        if (wl < 1e-3) { w = unitd(crossd(n, v3(0.3, 0.5, 0.7))); } else { w = w * (1.0 / wl); }
        const double sth = std::min(1.0, FLT_EPSILON * logu(0.0, 2.0) / nl);
        d = w * std::sqrt(1.0 - sth * sth) + n * (sgn() * sth);
        o = x - d * tau;
      } else if (g == G_FACE) {
        // origin on (or one float step off) a face of the cluster's box, random direction
        o = bl + v3(bs.x * U(rng), bs.y * U(rng), bs.z * U(rng));
        const int a = (int)(U(rng) * 3) % 3;
        double fv = U(rng) < 0.5 ? comp(bl, a) : comp(bh, a);
        const int step = (int)(U(rng) * 3) - 1;
        float ff = (float)fv;
        if (step) ff = std::nextafter(ff, step > 0 ? FLT_MAX : -FLT_MAX);
        setc(o, a, ff);
        d = unitd(v3(U(rng) - 0.5, U(rng) - 0.5, U(rng) - 0.5));
      } else {  // G_AXIS: a direction (nearly) along an axis, tiny, denormal or zero other components
        const int a = (int)(U(rng) * 3) % 3;
        const double tiny[6] = {0.0, 1e-40, 1e-38, 1e-30, 1e-10, 1e-4};
        d = v3(tiny[(int)(U(rng) * 6) % 6] * sgn(), tiny[(int)(U(rng) * 6) % 6] * sgn(),
               tiny[(int)(U(rng) * 6) % 6] * sgn());
        setc(d, a, sgn());
        const V3 t = bl - bs * 0.1 + v3(bs.x * 1.2 * U(rng), bs.y * 1.2 * U(rng), bs.z * 1.2 * U(rng));
        o = t - d * (sgn() * logu(-2.0, 1.0) * scale);
      }
      // the ray as the kernel holds it: float origin and direction (the renderer's directions are
      // normalised in float), invdir = 1 / d per component
      const f3 of = mk3((float)o.x, (float)o.y, (float)o.z);
      f3 df = mk3((float)d.x, (float)d.y, (float)d.z);
      if (g != G_AXIS) df = normalize(df);
      const f3 inv = mk3(1.0f / df.x, 1.0f / df.y, 1.0f / df.z);
      const bool fast = fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV;
      Counts& C = loc[g];
      C.lines++;
      auto any_pass = [&](const float4* v0, const float4* ea, const float4* eb, int n, const float4* bl4,
                          const float4* bh4) {
        bool any = false;
        for (int k = 0; k < n; k++) {
          float bx, by, bz;
          if (tri_test_v(TriData{v0[k], ea[k], eb[k]}, of, df, bx, by, bz) >= 1) {
            any = true;
            C.bound = std::max(C.bound, bound_ratio(of, df, v0[k], ea[k], eb[k], bx, by));
            if (bl4) C.worst = std::max(C.worst, out_ratio(of, df, v0[k], ea[k], eb[k], *bl4, *bh4, K > 0 ? K : 1e-4f));
          }
        }
        return any;
      };
      const bool pass = any_pass(&cs.cv0[inf.x], &cs.ce1[inf.x], &cs.ce2[inf.x], inf.y, &L, &H);
      if (!fast) {
        C.nofast++;
        continue;  // the wave runs no cull at all (kdpt_device.h trace_phase: fastAABB)
      }
      const bool box = cluster_may_pass(L, H, of, inv, K);
      if (!box) C.culled_box++;
      if (fast) {
        // the exact one-level cull: a line that misses the cluster's fast-margin box and oriented box tests only
        // the triangles of the cluster's danger mask that danger_needs_test keeps; every triangle passing glm's
        // u/v tests must be among them
        const float ndv = cs.nrm[c].x * df.x + cs.nrm[c].y * df.y + cs.nrm[c].z * df.z;
        const bool hit = cluster_may_pass(L, H, of, inv, KF) &&
                         cluster_may_pass_obb_k(L, H, cs.nrm[c], cs.obb_u[c], cs.obb_v[c], cs.obb_w[c], of, inv, df, ndv,
                                                KF);
        if (!hit) {
          int items;
          const unsigned long long nm = mt.needs_all(c, L, H, of, inv, df, items);
          C.mask_items += items;
          C.mask_needed += __builtin_popcountll(nm);
          for (int k = 0; k < inf.y; k++) {
            float bx, by, bz;
            if (tri_test_v(TriData{cs.cv0[inf.x + k], cs.ce1[inf.x + k], cs.ce2[inf.x + k]}, of, df, bx, by, bz) >= 1 &&
                !((nm >> k) & 1ull))
              C.viol_mask++;
          }
        }
      }
      if (pass) {
        C.pass++;
        if (!box) C.viol_box++;
        if (box && !cluster_may_pass(L, H, of, inv, 0.0f)) C.margin_used++;
        if (!cluster_may_pass_slab(L, H, cs.nrm[c], of, inv, df, ck)) C.viol_slab++;
        if (!cluster_may_pass_obb(L, H, cs.nrm[c], cs.obb_u[c], cs.obb_v[c], cs.obb_w[c], of, inv, df, ck)) C.viol_obb++;
        if (super_of[c] >= 0) {
          const int4 q = cs.sup[super_of[c]];
          const float4 sl = make_float4(half_lo((uint32_t)q.x), half_hi((uint32_t)q.x), half_lo((uint32_t)q.y), 0);
          const float4 sh = make_float4(half_hi((uint32_t)q.y), half_lo((uint32_t)q.z), half_hi((uint32_t)q.z), 0);
          if (!cluster_may_pass(sl, sh, of, inv, K)) C.viol_super++;
          const float4 sb = cs.sup_b[super_of[c]];
          if (!cluster_may_pass_slab(make_float4(sl.x, sl.y, sl.z, sb.x), make_float4(sh.x, sh.y, sh.z, sb.y),
                                     cs.sup_n[super_of[c]], of, inv, df, ck))
            C.viol_super++;
        }
      }
      // the brute-force route: the file-order chunk holding the line's triangle
      const int t0 = fbits(cs.ce1[ent].w), j = t0 >> 6, n64 = std::min(64, nt - 64 * j);
      if (any_pass(&tv[64 * j], &e1[64 * j], &e2[64 * j], n64, nullptr, nullptr) && !cluster_may_pass(clo[j], chi[j], of, inv, K))
        C.viol_chunk++;
    }
#pragma omp critical
    for (int g = 0; g < NGEN; g++) tot[g].add(loc[g]);
  }
  (void)nthreads;
  Counts all;
  printf("{\"clusters\": %d, \"supers\": %zu, \"margin\": %.9g, \"rigorous\": %.6g, \"exact\": %d, \"gens\": {", ncl,
         cs.sup.size(), (double)K, cm.rigorous, (int)(K >= cm.rigorous));
  for (int g = 0; g < NGEN; g++) {
    const Counts& C = tot[g];
    all.add(C);
    printf("%s\"%s\": {\"lines\": %lld, \"pass\": %lld, \"culled_box\": %lld, \"viol_box\": %lld, \"viol_slab\": %lld, "
           "\"viol_super\": %lld, \"viol_chunk\": %lld, \"viol_obb\": %lld, \"viol_mask\": %lld, \"mask_items\": %lld, "
           "\"mask_needed\": %lld, "
           "\"nofast\": %lld, \"margin_used\": %lld, \"worst\": %.4g, \"bound\": %.4g}",
           g ? ", " : "", kGenName[g], C.lines, C.pass, C.culled_box, C.viol_box, C.viol_slab, C.viol_super,
           C.viol_chunk, C.viol_obb, C.viol_mask, C.mask_items, C.mask_needed, C.nofast, C.margin_used, C.worst, C.bound);
  }
  printf("}, \"violations\": %lld, \"viol_mask\": %lld, \"lines\": %lld, \"pass\": %lld, \"margin_used\": %lld, "
         "\"worst\": %.4g, \"bound\": %.4g}\n",
         all.viol_box + all.viol_slab + all.viol_super + all.viol_chunk + all.viol_obb, all.viol_mask, all.lines, all.pass,
         all.margin_used, all.worst, all.bound);
  return 0;
}
