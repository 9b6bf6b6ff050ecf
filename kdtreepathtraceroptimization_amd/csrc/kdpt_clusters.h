// kdpt_clusters.h -- host-side construction of the big-leaf clusters, super-clusters and cluster slabs
// (DevScene::leaf_cl, cl_lo / cl_hi / cl_n, sup, c_v0 / c_e1 / c_e2).  Shared by the runtime
// (kdpt_runtime.hip build_clusters, which uploads the result) and the host differential test of the cluster
// cull (tests/native/cull_diff.cpp), so that the test checks exactly the boxes the kernels read.
//
// Only the order in which a wave tests a big leaf's triangles depends on this grouping (results are
// recombined by original index); the cull is conservative with respect to glm's float u/v tests
// ("Cluster cull"), which the margin coefficient (cluster_margin) guarantees.
#pragma once

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/kdpt.h"
#include "kdpt_device.h"

namespace kdpt {

// Half-precision bits of the largest half <= x (half_down) / the smallest half >= x (half_up); overflow goes
// to -inf / +inf, so the rounded value always bounds x (x finite).  Portable (no _Float16): round x to the
// nearest half through its float bits, then step outward when that rounded up (down).
inline uint32_t half_nearest(float x) {
  uint32_t b;
  memcpy(&b, &x, 4);
  const uint32_t s = (b >> 16) & 0x8000u;
  const uint32_t a = b & 0x7fffffffu;
  if (a >= 0x7f800000u) return s | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u);  // inf / nan
  if (a >= 0x477ff000u) return s | 0x7c00u;  // |x| >= 65520: rounds to inf
  if (a < 0x38800000u) {  // below the smallest normal half (2^-14): subnormal, units of 2^-24
    const float v = fabsf(x) * 16777216.0f;  // exact (power of two)
    const float r = nearbyintf(v);           // ties to even under the default rounding mode
    return s | (uint32_t)r;
  }
  const uint32_t e = (a >> 23) - 112u, m = a & 0x7fffffu;
  uint32_t h = (e << 10) | (m >> 13);
  const uint32_t rest = m & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) h++;  // to nearest, ties to even (may carry into e)
  return s | h;
}
inline uint32_t half_down(float x) {
  uint32_t b = half_nearest(x);
  if (half_to_float(b) > x) {  // one step towards -inf
    if (b == 0x0000u) b = 0x8001u;
    else if (b & 0x8000u) b = b + 1u;
    else b = b - 1u;
  }
  return b;
}
inline uint32_t half_up(float x) { return half_down(-x) ^ 0x8000u; }

constexpr double CULL_RHO_CAP = 64.0;  // |e1| |e2| / |e1 x e2| beyond which a triangle counts as a sliver

struct ClusterSet {
  std::vector<int2> leaf_cl, leaf_sp;  // per node: {first cluster, count} / {first super, count}
  std::vector<int4> sup;               // super-cluster records (DevScene::sup)
  std::vector<float4> sup_n, sup_b;    // the supers' slabs (DevScene::sup_n, sup_b)
  std::vector<float4> lo, hi, nrm;     // cluster boxes (w: slab bounds) and slab normals
  std::vector<float4> obb_u, obb_v, obb_w;  // the patch's in-plane slabs (DevScene::cl_u, cl_v, cl_w)
  std::vector<float4> kc;              // per cluster: the exact cull's {chord_eff, a, K_rig, c} (cull_k_exact)
  std::vector<float4> cv0, ce1, ce2;   // cluster-order triangles, CLUSTER per cluster (ce1.w = original index)
  std::vector<int2> info;              // {first entry in cv0, triangle count}
  bool supers_finite = true;           // every super box is finite in half precision
};

// How a big leaf's triangles are grouped into clusters (only the order in which a wave tests them changes).
struct ClusterGrouping {
  int mode = 0;         // 0: Morton runs of CLUSTER; 1: normal cones first, then balanced Morton runs per cone
  double chord = 0.5;   // mode 1: a cone is split while the chord of its unit normals about its axis exceeds this
  int min_split = 8;    // ... and it holds more than this many triangles
};

constexpr double ULP_HALF = 5.9604644775390625e-8;  // u = 2^-24
constexpr double CLUSTER_CHORD_EXACT = 0.03;  // the normal-cone chord of meshes whose cull margin is rigorous

// The exact cull's coefficients of one cluster (ClusterSet::kc, read by cull_k_exact), from the triangles glm
// tests (v0, e1, e2 as floats; products exact in double):
//   chord = max |N_t / |N_t| - n| over the triangles with N_t = e1 x e2 != 0 (n: the slab normal nf, as
//     stored); 4 -- never a usable bound -- when n = 0, or when an exactly degenerate triangle (N_t = 0) has
//     |e1||e2| > 0.3 (its float determinant can then reach FLT_EPSILON for any direction; below that
//     |a_t| <= 5.8 u |e1||e2| < FLT_EPSILON and it never passes);
//   rho = max(1, |e1||e2| / |N_t|) over the same triangles (slivers included: they only raise it);
//   chord_eff = chord (1 + 8u) + 5.8 u rho (1 + 1e-3) + 32 u, rounded up;
//   a = 17.5 u rho (1 + 1e-5); K_rig = 8.75 E + c; c = 64 u (1 + max|coord| + max|e|), E = max |e1||e2|
//   ("Cluster cull": the u/v error bound 17.34 u |s| |e1||e2| / a_t + 2.1 u max|e|).
inline float4 exact_cull_coef(const float4* e1, const float4* e2, const float4* v0, int n, bool has_n, const float* nf) {
  const double u = ULP_HALF;
  double chord = has_n ? 0.0 : 4.0, rho = 1.0, E = 0.0, emax = 0.0, cmax = 0.0;
  for (int k = 0; k < n; k++) {
    const double ax = e1[k].x, ay = e1[k].y, az = e1[k].z, bx = e2[k].x, by = e2[k].y, bz = e2[k].z;
    const double la = std::sqrt(ax * ax + ay * ay + az * az), lb = std::sqrt(bx * bx + by * by + bz * bz);
    const double Nx = ay * bz - az * by, Ny = az * bx - ax * bz, Nz = ax * by - ay * bx;
    const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
    E = std::max(E, la * lb);
    emax = std::max(emax, std::max(la, lb));
    cmax = std::max(cmax, std::max(std::fabs((double)v0[k].x), std::max(std::fabs((double)v0[k].y),
                                                                       std::fabs((double)v0[k].z))) + la + lb);
    if (Nl == 0.0) {
      if (la * lb > 0.3) chord = 4.0;
      continue;
    }
    rho = std::max(rho, la * lb / Nl);
    if (has_n) {
      const double cx = Nx / Nl - nf[0], cy = Ny / Nl - nf[1], cz = Nz / Nl - nf[2];
      chord = std::max(chord, std::sqrt(cx * cx + cy * cy + cz * cz));
    }
  }
  const double c = 64.0 * u * (1.0 + cmax + emax);
  const double ce = chord >= 2.0 ? 4.0 : chord * (1.0 + 8.0 * u) + 5.8 * u * rho * (1.0 + 1e-3) + 32.0 * u;
  auto up = [](double x) { return std::nextafter((float)x, FLT_MAX); };
  return make_float4(up(ce), up(17.5 * u * rho * (1.0 + 1e-5)), up(8.75 * E + c), up(c));
}

// Mode 1's cones: recursive median splits of the leaf's triangles along the principal axis of their unit
// normals (power iteration on the 3 x 3 second-moment matrix, in double; deterministic), until each cone's
// chord max |N_t / |N_t| - n| (n: the normalised sum of its area vectors, as the cluster slab forms it) is at
// most g.chord.  Exactly degenerate triangles (N_t = 0) have no normal and do not count towards a chord.
inline void normal_cones(const std::vector<std::array<double, 3>>& A, std::vector<int>& idx, int b, int e,
                         const ClusterGrouping& g, std::vector<std::pair<int, int>>& out) {
  double m[3] = {0, 0, 0};
  for (int k = b; k < e; k++)
    for (int a = 0; a < 3; a++) m[a] += A[idx[k]][a];
  const double ml = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
  double chord = ml > 0 ? 0.0 : 4.0;
  std::vector<std::array<double, 3>> un(e - b);
  for (int k = b; k < e; k++) {
    const std::array<double, 3>& q = A[idx[k]];
    const double l = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    un[k - b] = l > 0 ? std::array<double, 3>{q[0] / l, q[1] / l, q[2] / l} : std::array<double, 3>{0, 0, 0};
    if (l > 0 && ml > 0) {
      const double cx = un[k - b][0] - m[0] / ml, cy = un[k - b][1] - m[1] / ml, cz = un[k - b][2] - m[2] / ml;
      chord = std::max(chord, std::sqrt(cx * cx + cy * cy + cz * cz));
    }
  }
  if (chord <= g.chord || e - b <= g.min_split) {
    out.push_back({b, e});
    return;
  }
  double M[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, mu[3] = {0, 0, 0};
  for (const auto& q : un)
    for (int a = 0; a < 3; a++) mu[a] += q[a] / (e - b);
  for (const auto& q : un)
    for (int a = 0; a < 3; a++)
      for (int c = 0; c < 3; c++) M[a][c] += (q[a] - mu[a]) * (q[c] - mu[c]);
  int a0 = 0;
  for (int a = 1; a < 3; a++)
    if (M[a][a] > M[a0][a0]) a0 = a;
  double p[3] = {a0 == 0 ? 1.0 : 0.0, a0 == 1 ? 1.0 : 0.0, a0 == 2 ? 1.0 : 0.0};
  for (int it = 0; it < 32; it++) {
    double r[3];
    for (int a = 0; a < 3; a++) r[a] = M[a][0] * p[0] + M[a][1] * p[1] + M[a][2] * p[2];
    const double rl = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (!(rl > 0)) break;
    for (int a = 0; a < 3; a++) p[a] = r[a] / rl;
  }
  std::vector<std::pair<double, int>> key(e - b);
  for (int k = b; k < e; k++) key[k - b] = {p[0] * un[k - b][0] + p[1] * un[k - b][1] + p[2] * un[k - b][2], idx[k]};
  std::stable_sort(key.begin(), key.end(),
                   [](const std::pair<double, int>& x, const std::pair<double, int>& y) { return x.first < y.first; });
  for (int k = b; k < e; k++) idx[k] = key[k - b].second;
  const int mid = b + (e - b) / 2;
  normal_cones(A, idx, b, mid, g, out);
  normal_cones(A, idx, mid, e, g, out);
}

// Big leaves as clusters of <= CLUSTER triangles: Morton order of the triangle centroids inside the leaf's
// box (mode 1: within each normal cone), consecutive runs, each with its exact float box, the slab along its
// summed area vector, its oriented box and its exact-cull coefficients, and runs of SUPER clusters under one
// half-precision box rounded outward.
inline void build_cluster_set(const kdpt_node_bare* nodes, int nn, const kdpt_tri_bare* tris,
                              const std::vector<float4>& tv, const std::vector<float4>& e1,
                              const std::vector<float4>& e2, ClusterSet& cs,
                              const ClusterGrouping& grouping = ClusterGrouping{}) {
  cs = ClusterSet{};
  cs.leaf_cl.assign(nn, make_int2(0, 0));
  cs.leaf_sp.assign(nn, make_int2(0, 0));
  auto spread = [](uint32_t v) {
    uint32_t r = 0;
    for (int b = 0; b < 10; b++) r |= ((v >> b) & 1u) << (3 * b);
    return r;
  };
  for (int i = 0; i < nn; i++) {
    const kdpt_node_bare& N = nodes[i];
    if (N.triIdSize < BIG_LEAF) continue;
    const int start = N.triIdStart, size = N.triIdSize;
    std::vector<std::pair<uint32_t, int>> key(size);
    for (int k = 0; k < size; k++) {
      const kdpt_tri_bare& T = tris[start + k];
      const double cen[3] = {(T.x1 + (double)T.x2 + T.x3) / 3, (T.y1 + (double)T.y2 + T.y3) / 3,
                             (T.z1 + (double)T.z2 + T.z3) / 3};
      uint32_t m = 0;
      for (int a = 0; a < 3; a++) {
        const double ext = std::max((double)N.maxs[a] - N.mins[a], 1e-30);
        const double u = std::min(std::max((cen[a] - N.mins[a]) / ext, 0.0), 1.0);
        m |= spread((uint32_t)(u * 1023.0)) << a;
      }
      key[k] = {m, k};
    }
    auto by_morton = [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
      return a.first < b.first;
    };
    // ord: the leaf's triangles (leaf-local index) in cluster order; runs: each cluster's [begin, end) of ord
    std::vector<int> ord(size);
    std::vector<std::pair<int, int>> runs;
    if (grouping.mode == 0) {
      std::stable_sort(key.begin(), key.end(), by_morton);
      for (int k = 0; k < size; k++) ord[k] = key[k].second;
      for (int b = 0; b < size; b += CLUSTER) runs.push_back({b, std::min(size, b + CLUSTER)});
    } else {
      std::vector<std::array<double, 3>> A(size);
      for (int k = 0; k < size; k++) {
        const float4 a = e1[start + k], b = e2[start + k];  // glm's float edges, exact products in double
        A[k] = {(double)a.y * b.z - (double)a.z * b.y, (double)a.z * b.x - (double)a.x * b.z,
                (double)a.x * b.y - (double)a.y * b.x};
        ord[k] = k;
      }
      std::vector<std::pair<int, int>> cones;
      normal_cones(A, ord, 0, size, grouping, cones);
      for (const auto& cn : cones) {
        std::vector<std::pair<uint32_t, int>> ck;
        for (int k = cn.first; k < cn.second; k++) ck.push_back(key[ord[k]]);
        std::stable_sort(ck.begin(), ck.end(), by_morton);
        for (int k = cn.first; k < cn.second; k++) ord[k] = ck[k - cn.first].second;
        const int n = cn.second - cn.first, parts = (n + CLUSTER - 1) / CLUSTER;
        for (int q = 0; q < parts; q++)  // balanced runs: sizes differ by at most one
          runs.push_back({cn.first + (int)((long long)n * q / parts), cn.first + (int)((long long)n * (q + 1) / parts)});
      }
    }
    cs.leaf_cl[i] = make_int2((int)cs.info.size(), (int)runs.size());
    for (const auto& run : runs) {
      const int b = run.first, cnt = run.second - run.first;
      float l[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
      cs.info.push_back(make_int2((int)cs.cv0.size(), cnt));
      for (int k = b; k < b + cnt; k++) {
        const int t = start + ord[k];
        const kdpt_tri_bare& T = tris[t];
        const float vx[3] = {T.x1, T.x2, T.x3}, vy[3] = {T.y1, T.y2, T.y3}, vz[3] = {T.z1, T.z2, T.z3};
        for (int v = 0; v < 3; v++) {
          l[0] = std::min(l[0], vx[v]); h[0] = std::max(h[0], vx[v]);
          l[1] = std::min(l[1], vy[v]); h[1] = std::max(h[1], vy[v]);
          l[2] = std::min(l[2], vz[v]); h[2] = std::max(h[2], vz[v]);
        }
        cs.cv0.push_back(tv[t]);
        float4 q = e1[t];
        q.w = ibits(t);  // original triangle index
        cs.ce1.push_back(q);
        cs.ce2.push_back(e2[t]);
      }
      for (int k = cnt; k < CLUSTER; k++) {  // padding: e1 = e2 = 0 fails glm's determinant test
        cs.cv0.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
        cs.ce1.push_back(make_float4(0.0f, 0.0f, 0.0f, ibits(-1)));
        cs.ce2.push_back(make_float4(0.0f, 0.0f, 0.0f, 0.0f));
      }
      // the slab: n = the normalised sum of the triangles' (v1 - v0) x (v2 - v0), c as the kernel forms it,
      // [min, max] of n . (v - c) over the vertices in double, rounded outward to float
      const float cc[3] = {0.5f * (l[0] + h[0]), 0.5f * (l[1] + h[1]), 0.5f * (l[2] + h[2])};
      double ns[3] = {0, 0, 0};
      for (int k = b; k < b + cnt; k++) {
        const kdpt_tri_bare& T = tris[start + ord[k]];
        const double ax = (double)T.x2 - T.x1, ay = (double)T.y2 - T.y1, az = (double)T.z2 - T.z1;
        const double bx = (double)T.x3 - T.x1, by = (double)T.y3 - T.y1, bz = (double)T.z3 - T.z1;
        ns[0] += ay * bz - az * by;
        ns[1] += az * bx - ax * bz;
        ns[2] += ax * by - ay * bx;
      }
      const double nl = std::sqrt(ns[0] * ns[0] + ns[1] * ns[1] + ns[2] * ns[2]);
      float nf[3] = {0.0f, 0.0f, 0.0f};
      float dlo = -FLT_MAX, dhi = FLT_MAX;
      if (nl > 0 && std::isfinite(nl)) {
        for (int a = 0; a < 3; a++) nf[a] = (float)(ns[a] / nl);
        double mn = 1e300, mx = -1e300;
        for (int k = b; k < b + cnt; k++) {
          const kdpt_tri_bare& T = tris[start + ord[k]];
          const float vx[3] = {T.x1, T.x2, T.x3}, vy[3] = {T.y1, T.y2, T.y3}, vz[3] = {T.z1, T.z2, T.z3};
          for (int v = 0; v < 3; v++) {
            const double dv = (double)nf[0] * ((double)vx[v] - cc[0]) + (double)nf[1] * ((double)vy[v] - cc[1]) +
                              (double)nf[2] * ((double)vz[v] - cc[2]);
            mn = std::min(mn, dv);
            mx = std::max(mx, dv);
          }
        }
        dlo = std::nextafter((float)mn, -FLT_MAX);
        dhi = std::nextafter((float)mx, FLT_MAX);
      }
      // the spread of the triangles' normals about nf (slab level's direction-dependent margin,
      // cull_margin_dir): the largest chord |N_t / |N_t| - nf| over the cluster, N_t = e1 x e2 of glm's float
      // edges, rounded up; 4 (never a usable lower bound) when nf = 0, when a triangle is a sliver
      // (|e1| |e2| / |N_t| > CULL_RHO_CAP: the scene-wide rho of cull_margin_dir leaves it out, so only the
      // direction-free margin covers it), or when an exactly degenerate triangle has |e1||e2| > 0.3 (below that
      // its float determinant stays under FLT_EPSILON: it never passes)
      double spread = (nl > 0 && std::isfinite(nl)) ? 0.0 : 4.0;
      for (int k = b; k < b + cnt && spread < 4.0; k++) {
        const int e = cs.info.back().x + (k - b);
        const double ax = cs.ce1[e].x, ay = cs.ce1[e].y, az = cs.ce1[e].z;
        const double bx = cs.ce2[e].x, by = cs.ce2[e].y, bz = cs.ce2[e].z;
        const double Nx = ay * bz - az * by, Ny = az * bx - ax * bz, Nz = ax * by - ay * bx;
        const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
        const double E = std::sqrt(ax * ax + ay * ay + az * az) * std::sqrt(bx * bx + by * by + bz * bz);
        if (Nl == 0.0 ? E > 0.3 : E > CULL_RHO_CAP * Nl) {
          spread = 4.0;
          continue;
        }
        if (Nl == 0.0) continue;
        const double cx = Nx / Nl - nf[0], cy = Ny / Nl - nf[1], cz = Nz / Nl - nf[2];
        spread = std::max(spread, std::sqrt(cx * cx + cy * cy + cz * cz));
      }
      const float sf = std::nextafter((float)std::min(spread, 4.0), FLT_MAX);
      cs.kc.push_back(exact_cull_coef(&cs.ce1[cs.info.back().x], &cs.ce2[cs.info.back().x], &cs.cv0[cs.info.back().x],
                                      cnt, nl > 0 && std::isfinite(nl), nf));
      cs.lo.push_back(make_float4(l[0], l[1], l[2], dlo));
      cs.hi.push_back(make_float4(h[0], h[1], h[2], dhi));
      cs.nrm.push_back(make_float4(nf[0], nf[1], nf[2], sf));
      // the oriented box's in-plane directions: u along the principal axis of the vertices projected on
      // the plane, v = n x u (any unit directions would be valid slabs; these make the box tight), the
      // bounds of u . (q - c), v . (q - c) over the vertices in double, rounded outward to float
      float uf[3] = {0.0f, 0.0f, 0.0f}, vf[3] = {0.0f, 0.0f, 0.0f};
      float ulo = -FLT_MAX, uhi = FLT_MAX, vlo = -FLT_MAX, vhi = FLT_MAX;
      if (nl > 0 && std::isfinite(nl)) {
        const double n3[3] = {ns[0] / nl, ns[1] / nl, ns[2] / nl};
        const int amin = std::fabs(n3[0]) <= std::fabs(n3[1]) && std::fabs(n3[0]) <= std::fabs(n3[2]) ? 0
                         : (std::fabs(n3[1]) <= std::fabs(n3[2]) ? 1 : 2);
        const double ax[3] = {amin == 0 ? 1.0 : 0.0, amin == 1 ? 1.0 : 0.0, amin == 2 ? 1.0 : 0.0};
        double e1[3] = {n3[1] * ax[2] - n3[2] * ax[1], n3[2] * ax[0] - n3[0] * ax[2], n3[0] * ax[1] - n3[1] * ax[0]};
        const double e1l = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
        for (double& x : e1) x /= e1l;
        const double e2[3] = {n3[1] * e1[2] - n3[2] * e1[1], n3[2] * e1[0] - n3[0] * e1[2], n3[0] * e1[1] - n3[1] * e1[0]};
        double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
        int cntv = 0;
        for (int k = b; k < b + cnt; k++) {
          const kdpt_tri_bare& T = tris[start + ord[k]];
          const float vx[3] = {T.x1, T.x2, T.x3}, vy[3] = {T.y1, T.y2, T.y3}, vz[3] = {T.z1, T.z2, T.z3};
          for (int q = 0; q < 3; q++) {
            const double p[3] = {(double)vx[q] - cc[0], (double)vy[q] - cc[1], (double)vz[q] - cc[2]};
            const double x = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2], y = e2[0] * p[0] + e2[1] * p[1] + e2[2] * p[2];
            sx += x; sy += y; sxx += x * x; syy += y * y; sxy += x * y;
            cntv++;
          }
        }
        const double mx = sx / cntv, my = sy / cntv;
        const double cxx = sxx / cntv - mx * mx, cyy = syy / cntv - my * my, cxy = sxy / cntv - mx * my;
        const double th = 0.5 * std::atan2(2.0 * cxy, cxx - cyy);
        const double ud[3] = {std::cos(th) * e1[0] + std::sin(th) * e2[0], std::cos(th) * e1[1] + std::sin(th) * e2[1],
                              std::cos(th) * e1[2] + std::sin(th) * e2[2]};
        const double vd[3] = {n3[1] * ud[2] - n3[2] * ud[1], n3[2] * ud[0] - n3[0] * ud[2], n3[0] * ud[1] - n3[1] * ud[0]};
        for (int a = 0; a < 3; a++) {
          uf[a] = (float)ud[a];
          vf[a] = (float)vd[a];
        }
        double umn = 1e300, umx = -1e300, vmn = 1e300, vmx = -1e300;
        for (int k = b; k < b + cnt; k++) {
          const kdpt_tri_bare& T = tris[start + ord[k]];
          const float vx[3] = {T.x1, T.x2, T.x3}, vy[3] = {T.y1, T.y2, T.y3}, vz[3] = {T.z1, T.z2, T.z3};
          for (int q = 0; q < 3; q++) {
            const double p[3] = {(double)vx[q] - cc[0], (double)vy[q] - cc[1], (double)vz[q] - cc[2]};
            const double du = (double)uf[0] * p[0] + (double)uf[1] * p[1] + (double)uf[2] * p[2];
            const double dv = (double)vf[0] * p[0] + (double)vf[1] * p[1] + (double)vf[2] * p[2];
            umn = std::min(umn, du); umx = std::max(umx, du);
            vmn = std::min(vmn, dv); vmx = std::max(vmx, dv);
          }
        }
        ulo = std::nextafter((float)umn, -FLT_MAX);
        uhi = std::nextafter((float)umx, FLT_MAX);
        vlo = std::nextafter((float)vmn, -FLT_MAX);
        vhi = std::nextafter((float)vmx, FLT_MAX);
      }
      cs.obb_u.push_back(make_float4(uf[0], uf[1], uf[2], ulo));
      cs.obb_v.push_back(make_float4(vf[0], vf[1], vf[2], vlo));
      cs.obb_w.push_back(make_float4(uhi, vhi, 0.0f, 0.0f));
    }
    const int c0 = cs.leaf_cl[i].x, ncl = cs.leaf_cl[i].y;
    cs.leaf_sp[i] = make_int2((int)cs.sup.size(), (ncl + SUPER - 1) / SUPER);
    for (int b = 0; b < ncl; b += SUPER) {
      const int cnt = std::min(SUPER, ncl - b);
      float4 sl = cs.lo[c0 + b], sh = cs.hi[c0 + b];
      for (int k = c0 + b + 1; k < c0 + b + cnt; k++) {
        sl.x = std::min(sl.x, cs.lo[k].x); sl.y = std::min(sl.y, cs.lo[k].y); sl.z = std::min(sl.z, cs.lo[k].z);
        sh.x = std::max(sh.x, cs.hi[k].x); sh.y = std::max(sh.y, cs.hi[k].y); sh.z = std::max(sh.z, cs.hi[k].z);
      }
      // half precision rounded outward: the stored box holds the exact one
      const uint32_t lx = half_down(sl.x), ly = half_down(sl.y), lz = half_down(sl.z);
      const uint32_t hx = half_up(sh.x), hy = half_up(sh.y), hz = half_up(sh.z);
      for (uint32_t q : {lx, ly, lz, hx, hy, hz})
        if ((q & 0x7c00u) == 0x7c00u) cs.supers_finite = false;  // beyond the half range: no super route
      cs.sup.push_back(make_int4((int)(lx | ly << 16), (int)(lz | hx << 16), (int)(hy | hz << 16),
                                 (int)((uint32_t)(c0 + b) << 5 | (uint32_t)(cnt - 1))));
      // the super's own slab (the first cull level's direction-dependent test, DevScene::sup_n / sup_b): the
      // normalised sum of its triangles' area vectors, the largest chord to their unit normals (4 when a
      // sliver or a zero sum leaves no bound), and [min, max] of n . (q - c) over the triangles glm tests
      // (v0, v0 + e1, v0 + e2 exact in double), c the centre the kernel forms from the half-precision box
      const float cs0[3] = {0.5f * (half_to_float(lx) + half_to_float(hx)), 0.5f * (half_to_float(ly) + half_to_float(hy)),
                            0.5f * (half_to_float(lz) + half_to_float(hz))};
      double sn[3] = {0, 0, 0};
      const int e0 = cs.info[c0 + b].x, e1n = cs.info[c0 + b + cnt - 1].x + cs.info[c0 + b + cnt - 1].y;
      for (int e = e0; e < e1n; e++) {
        if (fbits(cs.ce1[e].w) < 0) continue;  // padding
        const double ax = cs.ce1[e].x, ay = cs.ce1[e].y, az = cs.ce1[e].z;
        const double bx = cs.ce2[e].x, by = cs.ce2[e].y, bz = cs.ce2[e].z;
        sn[0] += ay * bz - az * by;
        sn[1] += az * bx - ax * bz;
        sn[2] += ax * by - ay * bx;
      }
      const double snl = std::sqrt(sn[0] * sn[0] + sn[1] * sn[1] + sn[2] * sn[2]);
      float nfs[3] = {0.0f, 0.0f, 0.0f};
      double spread = 4.0, dmn = -1e300, dmx = 1e300;
      if (snl > 0 && std::isfinite(snl)) {
        for (int a = 0; a < 3; a++) nfs[a] = (float)(sn[a] / snl);
        spread = 0.0;
        dmn = 1e300;
        dmx = -1e300;
        for (int e = e0; e < e1n; e++) {
          if (fbits(cs.ce1[e].w) < 0) continue;
          const double ax = cs.ce1[e].x, ay = cs.ce1[e].y, az = cs.ce1[e].z;
          const double bx = cs.ce2[e].x, by = cs.ce2[e].y, bz = cs.ce2[e].z;
          const double Nx = ay * bz - az * by, Ny = az * bx - ax * bz, Nz = ax * by - ay * bx;
          const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
          const double E = std::sqrt(ax * ax + ay * ay + az * az) * std::sqrt(bx * bx + by * by + bz * bz);
          if (Nl == 0.0 ? E > 0.3 : E > CULL_RHO_CAP * Nl) {
            spread = 4.0;  // (as the clusters' spread: a sliver, or a degenerate triangle that can pass)
          } else if (Nl > 0.0 && spread < 4.0) {
            const double cx = Nx / Nl - nfs[0], cy = Ny / Nl - nfs[1], cz = Nz / Nl - nfs[2];
            spread = std::max(spread, std::sqrt(cx * cx + cy * cy + cz * cz));
          }
          const double v0[3] = {cs.cv0[e].x, cs.cv0[e].y, cs.cv0[e].z};
          for (int q = 0; q < 3; q++) {
            const double p[3] = {v0[0] + (q == 1 ? ax : (q == 2 ? bx : 0.0)) - cs0[0],
                                 v0[1] + (q == 1 ? ay : (q == 2 ? by : 0.0)) - cs0[1],
                                 v0[2] + (q == 1 ? az : (q == 2 ? bz : 0.0)) - cs0[2]};
            const double dv = (double)nfs[0] * p[0] + (double)nfs[1] * p[1] + (double)nfs[2] * p[2];
            dmn = std::min(dmn, dv);
            dmx = std::max(dmx, dv);
          }
        }
      }
      cs.sup_n.push_back(make_float4(nfs[0], nfs[1], nfs[2], std::nextafter((float)std::min(spread, 4.0), FLT_MAX)));
      cs.sup_b.push_back(make_float4(dmn < -1e38 ? -FLT_MAX : std::nextafter((float)dmn, -FLT_MAX),
                                     dmx > 1e38 ? FLT_MAX : std::nextafter((float)dmx, FLT_MAX), 0.0f, 0.0f));
    }
  }
}

// Direction masks of the exact one-level cull (DevScene::cl_mask).  For every cluster c and direction bucket b
// (dir_bucket: a cube map of n x n cells per face, nb = 6 n^2 buckets), masks[b ncl + c] = the danger mask over
// the cluster's 64 entries: the triangles that, for SOME direction of the bucket, are front-facing and need a
// margin above Kf -- the coefficient of the fast box test a pair's line missed (and whose rigorous coefficient
// exceeds Kf).  A triangle t needs the margin
// K_t(d) = 17.5 u rho_t / g_t + c (g_t = -N_t/|N_t| . d - beta_t; danger_needs_test), above Kf only when
// g_t < 17.5 u rho_t / (Kf - c).  Every other triangle of such a cluster is back-facing for the whole bucket
// (its float determinant negative) or lies farther from the line than its own error bound: it cannot pass glm's
// u/v tests ("Cluster cull").
// A bucket's directions d satisfy |d - d_b| <= r_b (d_b its normalised centre): the cell, grown by 1e-5 in u, v,
// lies on the face plane at |y| >= R, where radial projection is (1/R)-Lipschitz, so r_b = half diagonal / R.
// So |N . d - N . d_b| <= r_b (+ 1e-6 for the float d's length).  Exactly degenerate triangles are in every mask
// when |e1||e2| > 0.3 and in none otherwise (their float determinant stays below FLT_EPSILON).
constexpr int DIR_MASK_N = 256;  // finest cube-map cells per face edge (6 n^2 buckets; dir_mask_resolution)

// Per cluster entry of the masked cull (structure of arrays, 64 entries per cluster; dir_mask_cell): the unit
// normal and the two thresholds on x = N . d_b -- front when x - r <= beta, danger when also x + r >= dthr --
// and the rigorous coefficient krig = 8.75 |e1||e2| + c (c: the cluster's, ClusterSet::kc.w), rounded up.
// Entries in every mask get (0, inf, -inf), entries in none (padding, exactly degenerate with |e1||e2| <= 0.3)
// (0, -inf, -).
struct MaskEntries {
  std::vector<double> nx, ny, nz, beta, dthr;
  std::vector<float> krig;
};
inline void mask_entries(const ClusterSet& cs, float Kf, MaskEntries& me) {
  const int ncl = (int)cs.info.size();
  const size_t ne = 64 * (size_t)ncl;
  const double u = ULP_HALF;
  me.nx.assign(ne, 0.0);
  me.ny.assign(ne, 0.0);
  me.nz.assign(ne, 0.0);
  me.beta.assign(ne, -HUGE_VAL);
  me.dthr.assign(ne, HUGE_VAL);
  me.krig.assign(ne, 0.0f);
  for (int c = 0; c < ncl; c++) {
    const int2 inf = cs.info[c];
    const double gden = (double)Kf - cs.kc[c].w;
    for (int k = 0; k < inf.y; k++) {
      const size_t q = 64 * (size_t)c + k;
      const float4 e1 = cs.ce1[inf.x + k], e2 = cs.ce2[inf.x + k];
      const double Nx = (double)e1.y * e2.z - (double)e1.z * e2.y, Ny = (double)e1.z * e2.x - (double)e1.x * e2.z,
                   Nz = (double)e1.x * e2.y - (double)e1.y * e2.x;
      const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
      const double la = std::sqrt((double)e1.x * e1.x + (double)e1.y * e1.y + (double)e1.z * e1.z);
      const double lb = std::sqrt((double)e2.x * e2.x + (double)e2.y * e2.y + (double)e2.z * e2.z);
      me.krig[q] = std::nextafter((float)(8.75 * la * lb + (double)cs.kc[c].w), HUGE_VALF);
      if (Nl == 0.0) {
        if (la * lb > 0.3) {
          me.beta[q] = HUGE_VAL;
          me.dthr[q] = -HUGE_VAL;
        }
        continue;
      }
      const double rho = std::max(1.0, la * lb / Nl);
      me.nx[q] = Nx / Nl;
      me.ny[q] = Ny / Nl;
      me.nz[q] = Nz / Nl;
      me.beta[q] = 5.8 * u * rho * (1.0 + 1e-3) + 40.0 * u;
      const double gamma = gden > 0 ? 17.5 * u * rho * (1.0 + 1e-5) / gden : HUGE_VAL;
      me.dthr[q] = -me.beta[q] - gamma;
    }
  }
}

// The buckets' centre directions and radii (4 doubles per bucket, dir_mask_cell's D).
inline void mask_buckets(int n, std::vector<double>& bd) {
  const int nb = 6 * n * n;
  const double grow = 1e-5;
  bd.assign(4 * (size_t)nb, 0.0);
  for (int b = 0; b < nb; b++) {
    const int face = b / (n * n), j = (b / n) % n, i = b % n;
    const double a0 = -1.0 + 2.0 * i / n - grow, a1 = -1.0 + 2.0 * (i + 1) / n + grow;
    const double b0 = -1.0 + 2.0 * j / n - grow, b1 = -1.0 + 2.0 * (j + 1) / n + grow;
    const double ac = 0.5 * (a0 + a1), bc = 0.5 * (b0 + b1);
    const double amin = (a0 <= 0 && a1 >= 0) ? 0.0 : std::min(std::fabs(a0), std::fabs(a1));
    const double bmin = (b0 <= 0 && b1 >= 0) ? 0.0 : std::min(std::fabs(b0), std::fabs(b1));
    const double R = std::sqrt(1.0 + amin * amin + bmin * bmin);
    double* D = &bd[4 * (size_t)b];
    D[3] = 0.5 * std::sqrt((a1 - a0) * (a1 - a0) + (b1 - b0) * (b1 - b0)) / R * (1.0 + 1e-9) + 1e-6;
    const double sgn = (face & 1) ? -1.0 : 1.0;
    if (face < 2) { D[0] = sgn; D[1] = ac; D[2] = bc; }
    else if (face < 4) { D[0] = ac; D[1] = sgn; D[2] = bc; }
    else { D[0] = ac; D[1] = bc; D[2] = sgn; }
    const double dl = std::sqrt(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
    for (int a = 0; a < 3; a++) D[a] /= dl;
  }
}

// The masks on the host, bucket-major (masks[b ncl + c]: DevScene::cl_mask).  Test infrastructure: the product
// builds the same cells on the device (kdpt_runtime.hip k_build_masks, the same dir_mask_cell over the same
// entries and buckets; tests/test_gpu_masks.py compares the two).
inline void build_dir_masks(const ClusterSet& cs, int n, float Kf, std::vector<unsigned long long>& masks) {
  const int ncl = (int)cs.info.size(), nb = 6 * n * n;
  MaskEntries me;
  mask_entries(cs, Kf, me);
  std::vector<double> bd;
  mask_buckets(n, bd);
  masks.assign((size_t)nb * ncl, 0ull);
  auto work = [&](int c) {  // cluster by cluster: its 64 entries stay in cache over the buckets
    const size_t q0 = 64 * (size_t)c;
    for (int b = 0; b < nb; b++)
      masks[(size_t)b * ncl + c] = dir_mask_cell(&me.nx[q0], &me.ny[q0], &me.nz[q0], &me.beta[q0], &me.dthr[q0],
                                                 &me.krig[q0], &bd[4 * (size_t)b], Kf);
  };
  const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  int started = 0;
  try {
    for (; started < nth; started++)
      th.emplace_back([&, started]() {
        for (int c = started; c < ncl; c += nth) work(c);
      });
  } catch (...) {  // no thread could be started: the remaining residues run here
  }
  for (int t = started; t < nth; t++)
    for (int c = t; c < ncl; c += nth) work(c);
  for (auto& x : th) x.join();
}

// Per cluster entry (DevScene::cl_tn): the triangle's unit normal, rounded to float, and w = 17.5 u rho rounded
// up (danger_needs_test); w = -1 for padding and for exactly degenerate triangles with |e1||e2| <= 0.3 (never
// pass), w = +inf for larger exactly degenerate ones (may pass for any line).
inline void build_entry_normals(const ClusterSet& cs, std::vector<float4>& out) {
  const int ncl = (int)cs.info.size();
  out.assign(64 * (size_t)ncl, make_float4(0.0f, 0.0f, 0.0f, -1.0f));
  const double u = ULP_HALF;
  for (int c = 0; c < ncl; c++) {
    const int2 inf = cs.info[c];
    for (int k = 0; k < inf.y; k++) {
      const float4 e1 = cs.ce1[inf.x + k], e2 = cs.ce2[inf.x + k];
      const double Nx = (double)e1.y * e2.z - (double)e1.z * e2.y, Ny = (double)e1.z * e2.x - (double)e1.x * e2.z,
                   Nz = (double)e1.x * e2.y - (double)e1.y * e2.x;
      const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
      const double la = std::sqrt((double)e1.x * e1.x + (double)e1.y * e1.y + (double)e1.z * e1.z);
      const double lb = std::sqrt((double)e2.x * e2.x + (double)e2.y * e2.y + (double)e2.z * e2.z);
      float4& o = out[64 * (size_t)c + k];
      if (Nl == 0.0) {
        if (la * lb > 0.3) o.w = HUGE_VALF;
        continue;
      }
      const double rho = std::max(1.0, la * lb / Nl);
      o = make_float4((float)(Nx / Nl), (float)(Ny / Nl), (float)(Nz / Nl),
                      std::nextafter((float)(17.5 * u * rho * (1.0 + 1e-5)), HUGE_VALF));
    }
  }
}

// The cube-map resolution of the masks: the finest of DIR_MASK_N, 128, 64, ... 4 cells per face edge whose masks
// (8 bytes per cluster and bucket) fit in `budget` bytes, else 2.  A danger mask holds the triangles whose plane
// passes within the bucket's radius (plus a band of 17.5 u rho / (Kf - c)) of its directions, so its bit count
// falls with the bucket size: on C3 (dragon_5, 181 clusters, 569 MB at 256) the danger items per path halve with
// each doubling of the resolution and the rate rises by ~120 Mrays/s per item: 4 967 / 5 412 / 5 668 / 5 780 /
// 5 839 Mrays/s at 16 / 32 / 64 / 128 / 256 cells (profiles/r06_ab_log.md, sessions r06j, r06k).  Device memory
// is plentiful (288 GB); the budget keeps a scene of many clusters to a coarser table.
inline int dir_mask_resolution(int ncl, size_t budget = (size_t)640 << 20) {
  for (int n : {DIR_MASK_N, 128, 64, 32, 16, 8, 4})
    if ((size_t)ncl * 6 * n * n * 8 <= budget) return n;
  return 2;
}

// The brute-force route's boxes of 64 file-order triangles [64j, 64j + 64): the triangles glm tests,
// v0, v0 + e1, v0 + e2, exact in double and rounded outward to float (BruteArgs::chunk_lo / chunk_hi).
inline void build_chunk_boxes(const std::vector<float4>& tv, const std::vector<float4>& e1,
                              const std::vector<float4>& e2, int nt, std::vector<float4>& clo,
                              std::vector<float4>& chi) {
  const int nch = std::max(1, (nt + 63) / 64);
  clo.assign(nch, make_float4(0, 0, 0, 0));
  chi.assign(nch, make_float4(0, 0, 0, 0));
  for (int j = 0; j < nch; j++) {
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int k = 64 * j; k < std::min(nt, 64 * j + 64); k++) {
      const double v[3] = {tv[k].x, tv[k].y, tv[k].z}, a[3] = {e1[k].x, e1[k].y, e1[k].z},
                   b[3] = {e2[k].x, e2[k].y, e2[k].z};
      for (int r = 0; r < 3; r++) {  // the triangle glm tests: v0 + u e1 + v e2, exact in double
        lo[r] = std::min({lo[r], v[r], v[r] + a[r], v[r] + b[r]});
        hi[r] = std::max({hi[r], v[r], v[r] + a[r], v[r] + b[r]});
      }
    }
    float l[3], h[3];
    for (int r = 0; r < 3; r++) {
      if (lo[r] > hi[r]) lo[r] = hi[r] = 0.0;  // empty chunk (no triangles)
      l[r] = (float)lo[r];
      if ((double)l[r] > lo[r]) l[r] = std::nextafter(l[r], -FLT_MAX);
      h[r] = (float)hi[r];
      if ((double)h[r] < hi[r]) h[r] = std::nextafter(h[r], FLT_MAX);
    }
    clo[j] = make_float4(l[0], l[1], l[2], 0.0f);
    chi[j] = make_float4(h[0], h[1], h[2], 0.0f);
  }
}

// The cluster cull's margin coefficient K (DevScene::cl_margin; cluster_may_pass widens a box by
// K (1 + |o - c|_1 + size_1)).  A triangle can pass glm's float u/v tests for a line that misses it: the
// computed (u, v) carry rounding errors of order u |o - v0| |e1| |e2| / a (a: glm's determinant), and a may
// be as small as FLT_EPSILON.  DESIGN.md 4 ("Cluster cull") bounds the distance from the line to the point
// v0 + u e1 + v e2 the float test accepts by 17.34 u |o - v0| |e1| |e2| / a + 2.1 u max|e|; with a >= FLT_EPSILON
// = 2u that is 8.67 |o - v0| E + ..., E = |e1| |e2|.  So K_rigorous = 8.75 E_max + 64 u (1 + max|coord| +
// max|e|) makes the cull conservative for EVERY line (the constant term covers the box and slab tests' own
// rounding).  Meshes of small triangles (the C5 icosphere: E_max = 1.07e-4, K = 9.4e-4) get it; for meshes of
// large triangles it would cull nothing (dragon_5: E_max = 0.2), so their box levels use K = CULL_MARGIN_MASKED
// (1e-3) and the masked cull (build_dir_masks, mask_bound_code) decides a missed pair's near-parallel triangles:
// exact as well.  The box coefficient alone (knob "cull_exact" = 0, and the brute-force route's chunk cull) is
// conservative except for lines lying within ~17 u |o - v0| of a triangle's plane and within ~17 u rho / K of
// parallel to it (tests/native/cull_diff.cpp constructs such lines); the "cluster_cull" knob = 0 removes the cull.
struct CullMargin {
  float K;          // the box-only tests' coefficient (DevScene::cl_margin)
  float K_lo;       // the slab level's floor (cl_margin_lo)
  float a, b, c;    // the slab level's direction-dependent bound (cull_a, cull_b, cull_c)
  double rigorous;  // K_rigorous for these triangles
  bool exact;       // K >= K_rigorous: the cull never drops a triangle that passes glm's u/v tests
};
constexpr float CULL_MARGIN_FAST = 1e-4f;  // the slab level's floor (K_lo)
// the box coefficient of meshes whose K_rigorous exceeds the cap (their masked cull): 10x the floor narrows the
// danger band of their direction masks tenfold and costs no measurable sweeps (profiles/r05_ab_log.md)
constexpr float CULL_MARGIN_MASKED = 1e-3f;
constexpr double CULL_MARGIN_CAP = 2e-3;   // largest K_rigorous worth using (beyond it the cull loses its bite)
inline CullMargin cluster_margin(const std::vector<float4>& v0, const std::vector<float4>& e1,
                                 const std::vector<float4>& e2) {
  double emax = 0.0, pmax = 0.0, cmax = 0.0, rho = 1.0;
  for (size_t i = 0; i < e1.size(); i++) {
    const double ax = e1[i].x, ay = e1[i].y, az = e1[i].z, bx = e2[i].x, by = e2[i].y, bz = e2[i].z;
    const double a = std::sqrt(ax * ax + ay * ay + az * az), b = std::sqrt(bx * bx + by * by + bz * bz);
    const double Nx = ay * bz - az * by, Ny = az * bx - ax * bz, Nz = ax * by - ay * bx;
    const double Nl = std::sqrt(Nx * Nx + Ny * Ny + Nz * Nz);
    emax = std::max(emax, std::max(a, b));
    pmax = std::max(pmax, a * b);
    if (Nl > 0.0 && a * b <= CULL_RHO_CAP * Nl) rho = std::max(rho, a * b / Nl);  // slivers: spread 4
    cmax = std::max(cmax, std::max(std::fabs((double)v0[i].x), std::max(std::fabs((double)v0[i].y),
                                                                           std::fabs((double)v0[i].z))) + a + b);
  }
  const double u = 5.9604644775390625e-8;  // 2^-24
  CullMargin r;
  r.rigorous = 8.75 * pmax + 64.0 * u * (1.0 + cmax + emax);
  r.exact = r.rigorous <= CULL_MARGIN_CAP;
  r.K_lo = CULL_MARGIN_FAST;
  r.K = r.exact ? std::max(std::nextafter((float)r.rigorous, FLT_MAX), CULL_MARGIN_FAST) : CULL_MARGIN_MASKED;
  r.a = std::nextafter((float)(17.5 * u * rho * (1.0 + 1e-5)), FLT_MAX);
  r.b = std::nextafter((float)(5.8 * u * rho + 10.0 * u), FLT_MAX);
  r.c = std::nextafter((float)(64.0 * u * (1.0 + cmax + emax)), FLT_MAX);
  return r;
}

}  // namespace kdpt
