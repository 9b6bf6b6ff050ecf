// kd_build.hip -- the reference's host KD-tree build (Scene::loadObj's KD section, src/scene.cpp:866-968:
// KDtree(triangles) -> rootNode->updateBbox() -> split(13) -> cacheTriangles_ / cacheNodesBare) on the GPU,
// byte-identical to it (and to csrc/scene_host.cpp's host restatement).
//
// The reference builds depth-first and numbers nodes in pre-order (a file-static counter incremented as
// each child is created, left subtree before right).  Here the tree is built level by level, breadth first,
// with one pass over all (node, triangle) pairs of a level per kernel:
//   k_side      per pair: does the triangle go left (mins[axis] < centre + 0.0001) / right
//               (maxs[axis] >= centre - 0.0001)?  (KDnode.cpp:177-186, the comparisons in double)
//   scans       of the two flags over the level's pairs (pairs are grouped by node, in the node's
//               triangle order, so a node's side counts are differences of the scans)
//   k_decide    per node: split when it has > 2 triangles, its level <= maxdepth and neither side takes
//               every triangle (KDnode.cpp:160-193); else it is a leaf and keeps its triangles
//   scans       of the per-node split flags / children's pair counts / leaf sizes
//   k_children  per split node: both children (box = the parent's with maxs[axis] (left) or mins[axis]
//               (right) set to the parent's centre, centre recomputed, splitPos, axis; KDnode.cpp:195-246)
//   k_scatter   per pair: into the left and/or right child's pair list, STABLY (the reference's
//               leftSide/rightSide keep the parent's order), or into the leaf store
// After the last level, subtree sizes (bottom-up) give every node its pre-order ID (ID(left) = ID + 1,
// ID(right) = ID + 1 + size(left)), the leaves' triangle lists are laid out in ID order (cacheTriangles_,
// src/scene.cpp:409-459; duplicates included) and NodeBare[] is written in ID order (cacheNodesBare,
// :905-932).  The root box (KDnode::updateBbox, KDnode.cpp:112-149) is a first-occurrence min/max over the
// triangles' bounds -- the reference's `a > b ? b : a` fold keeps the earliest of equal values (+0 / -0)
// -- plus the 0.001 pad, which does not refresh the centre.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kdpt.h"
#include "kd_build.h"

namespace {

// (the failing call and HIP's reason on stderr: the scene-build entry points return only the code)
#define KD_TRY(x)                                                                                       \
  do {                                                                                                  \
    hipError_t e_ = (x);                                                                                \
    if (e_ != hipSuccess) {                                                                             \
      fprintf(stderr, "[kdpt] device KD build: %s failed: %s\n", #x, hipGetErrorString(e_));           \
      return KDPT_ERR_HIP;                                                                              \
    }                                                                                                   \
  } while (0)

constexpr int BLK = 256;
inline int blocks(long long n) { return (int)std::max(1ll, (n + BLK - 1) / BLK); }

// Triangle::computeBounds (KDnode.h:216-225): the nested ternaries, component by component
__device__ inline float tmin3(float a, float b, float c) { return a < b ? (a < c ? a : c) : (b < c ? b : c); }
__device__ inline float tmax3(float a, float b, float c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }

__global__ void k_tri_bounds(const float* __restrict__ v9, int n, float4* __restrict__ lo, float4* __restrict__ hi) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= n) return;
  const float* v = v9 + 9 * (size_t)i;  // x1 y1 z1 x2 y2 z2 x3 y3 z3
  lo[i] = make_float4(tmin3(v[0], v[3], v[6]), tmin3(v[1], v[4], v[7]), tmin3(v[2], v[5], v[8]), 0.0f);
  hi[i] = make_float4(tmax3(v[0], v[3], v[6]), tmax3(v[1], v[4], v[7]), tmax3(v[2], v[5], v[8]), 0.0f);
}

// Order-preserving 32-bit key of a float with +0 and -0 equal (they compare equal in the reference's fold).
__device__ inline uint32_t fkey(float f) {
  uint32_t u = __float_as_uint(f);
  if (f == 0.0f) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Root box: per component the FIRST triangle (in order) holding the minimum (maximum): min over
// (key << 32 | index) resp. max over (key << 32 | ~index).  NaNs never win (the fold's comparisons are
// false for them) unless triangle 0 holds one, which the host handles.
__global__ void k_root_keys(const float4* __restrict__ lo, const float4* __restrict__ hi, int n,
                            unsigned long long* keys) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  unsigned long long kmin[3] = {~0ull, ~0ull, ~0ull}, kmax[3] = {0ull, 0ull, 0ull};
  if (i < n) {
    const float4 a = lo[i], b = hi[i];
    const float la[3] = {a.x, a.y, a.z}, hb[3] = {b.x, b.y, b.z};
    for (int c = 0; c < 3; c++) {
      if (la[c] == la[c]) kmin[c] = ((unsigned long long)fkey(la[c]) << 32) | (uint32_t)i;
      if (hb[c] == hb[c]) kmax[c] = ((unsigned long long)fkey(hb[c]) << 32) | (uint32_t)~(uint32_t)i;
    }
  }
  for (int c = 0; c < 3; c++) {
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long om = __shfl_xor(kmin[c], off), ox = __shfl_xor(kmax[c], off);
      kmin[c] = om < kmin[c] ? om : kmin[c];
      kmax[c] = ox > kmax[c] ? ox : kmax[c];
    }
  }
  if ((threadIdx.x & 63) == 0) {
    for (int c = 0; c < 3; c++) {
      atomicMin(&keys[c], kmin[c]);
      atomicMax(&keys[3 + c], kmax[c]);
    }
  }
}

struct LevelArgs {
  int level, ax, maxdepth;
  int lvl_begin, nlvl;  // this level's nodes: global BFS indices [lvl_begin, lvl_begin + nlvl)
  long long npairs;
};

// Node store (global BFS index): box, centre, links, build results.
struct Nodes {
  float4 *lo, *hi, *ctr;   // box mins / maxs / centre (w unused)
  int* parent;
  int* left;
  int* right;
  int* axis;
  float* split_pos;
  int* pstart;             // this node's pair range in the level's pair list (its level only)
  int* pcnt;
  int* leaf_start;         // leaves: range in the leaf store; -1 for split nodes
  int* leaf_cnt;
  int* size;               // subtree size (nodes)
  int* id;                 // pre-order ID
};

__global__ void k_side(LevelArgs L, const int* __restrict__ ptri, const int* __restrict__ pnode, Nodes N,
                       const float4* __restrict__ tlo, const float4* __restrict__ thi, int* __restrict__ fl,
                       int* __restrict__ fr) {
  const long long p = (long long)blockIdx.x * BLK + threadIdx.x;
  if (p >= L.npairs) {
    if (p == L.npairs) fl[p] = fr[p] = 0;  // the scans' total slot
    return;
  }
  const int t = ptri[p], k = pnode[p];
  const float4 c4 = N.ctr[k], a = tlo[t], b = thi[t];
  const float c = L.ax == 0 ? c4.x : (L.ax == 1 ? c4.y : c4.z);
  const float mn = L.ax == 0 ? a.x : (L.ax == 1 ? a.y : a.z);
  const float mx = L.ax == 0 ? b.x : (L.ax == 1 ? b.y : b.z);
  fl[p] = ((double)mn < (double)c + 0.0001) ? 1 : 0;
  fr[p] = ((double)mx >= (double)c - 0.0001) ? 1 : 0;
}

__global__ void k_decide(LevelArgs L, Nodes N, const int* __restrict__ sl, const int* __restrict__ sr,
                         int* __restrict__ nsplit, int* __restrict__ npair_next, int* __restrict__ nleaf,
                         int* __restrict__ cl, int* __restrict__ cr) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= L.nlvl) {
    if (i == L.nlvl) nsplit[i] = npair_next[i] = nleaf[i] = 0;
    return;
  }
  const int k = L.lvl_begin + i;
  const int s = N.pstart[k], num = N.pcnt[k];
  const int l = sl[s + num] - sl[s], r = sr[s + num] - sr[s];
  const bool split = num > 2 && L.level <= L.maxdepth && l != num && r != num;
  nsplit[i] = split ? 1 : 0;
  npair_next[i] = split ? l + r : 0;
  nleaf[i] = split ? 0 : num;
  cl[i] = l;
  cr[i] = r;
}

__device__ inline void set_comp(float4& v, int ax, float x) {
  if (ax == 0) v.x = x; else if (ax == 1) v.y = x; else v.z = x;
}
__device__ inline float comp4(const float4& v, int ax) { return ax == 0 ? v.x : (ax == 1 ? v.y : v.z); }
// BoundingBox::updateCentroid (KDnode.h:279-285): (mins + maxs) in float, / 2.0 in double
__device__ inline float4 centroid(const float4& lo, const float4& hi) {
  return make_float4((float)((double)(lo.x + hi.x) / 2.0), (float)((double)(lo.y + hi.y) / 2.0),
                     (float)((double)(lo.z + hi.z) / 2.0), 0.0f);
}

__global__ void k_children(LevelArgs L, Nodes N, const int* __restrict__ nsplit_ex, const int* __restrict__ npair_ex,
                           const int* __restrict__ nleaf_ex, const int* __restrict__ nsplit_in,
                           const int* __restrict__ cl, const int* __restrict__ cr, int leaf_base) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= L.nlvl) return;
  const int k = L.lvl_begin + i;
  if (!nsplit_in[i]) {  // a leaf: keeps its triangles (triIdStart / triIdSize are set when laid out)
    N.left[k] = N.right[k] = -1;
    N.leaf_start[k] = leaf_base + nleaf_ex[i];
    N.leaf_cnt[k] = N.pcnt[k];
    return;
  }
  const int next_begin = L.lvl_begin + L.nlvl;
  const int lk = next_begin + 2 * nsplit_ex[i], rk = lk + 1;
  N.left[k] = lk;
  N.right[k] = rk;
  N.leaf_start[k] = -1;
  N.leaf_cnt[k] = 0;
  const float4 plo = N.lo[k], phi = N.hi[k], pc = N.ctr[k];
  const int ax = L.ax, cax = (ax + 1) % 3;
  {  // left: setBounds(parent) then maxs[axis] = parent centre; splitPos = parent maxs[axis]
    float4 lo = plo, hi = phi;
    set_comp(hi, ax, comp4(pc, ax));
    N.lo[lk] = lo;
    N.hi[lk] = hi;
    N.ctr[lk] = centroid(lo, hi);
    N.split_pos[lk] = comp4(phi, ax);
    N.axis[lk] = cax;
    N.parent[lk] = k;
    N.pstart[lk] = npair_ex[i];
    N.pcnt[lk] = cl[i];
  }
  {  // right: mins[axis] = parent centre; splitPos = parent mins[axis]
    float4 lo = plo, hi = phi;
    set_comp(lo, ax, comp4(pc, ax));
    N.lo[rk] = lo;
    N.hi[rk] = hi;
    N.ctr[rk] = centroid(lo, hi);
    N.split_pos[rk] = comp4(plo, ax);
    N.axis[rk] = cax;
    N.parent[rk] = k;
    N.pstart[rk] = npair_ex[i] + cl[i];
    N.pcnt[rk] = cr[i];
  }
}

__global__ void k_scatter(LevelArgs L, Nodes N, const int* __restrict__ ptri, const int* __restrict__ pnode,
                          const int* __restrict__ fl, const int* __restrict__ fr, const int* __restrict__ sl,
                          const int* __restrict__ sr, const int* __restrict__ nsplit_in, int* __restrict__ ntri,
                          int* __restrict__ nnode, int* __restrict__ leaf_tri, int* __restrict__ leaf_node) {
  const long long p = (long long)blockIdx.x * BLK + threadIdx.x;
  if (p >= L.npairs) return;
  const int t = ptri[p], k = pnode[p], i = k - L.lvl_begin;
  const int s = N.pstart[k];
  if (nsplit_in[i]) {
    const int lk = N.left[k], rk = N.right[k];
    if (fl[p]) {
      const int q = N.pstart[lk] + (sl[p] - sl[s]);
      ntri[q] = t;
      nnode[q] = lk;
    }
    if (fr[p]) {
      const int q = N.pstart[rk] + (sr[p] - sr[s]);
      ntri[q] = t;
      nnode[q] = rk;
    }
  } else {
    const int q = N.leaf_start[k] + (int)(p - s);
    leaf_tri[q] = t;
    leaf_node[q] = k;
  }
}

__global__ void k_sizes(Nodes N, int begin, int count) {  // one level, deepest first
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= count) return;
  const int k = begin + i;
  const int l = N.left[k], r = N.right[k];
  N.size[k] = 1 + (l >= 0 ? N.size[l] : 0) + (r >= 0 ? N.size[r] : 0);
}

__global__ void k_ids(Nodes N, int begin, int count) {  // one level, root first; ID[root] set before
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= count) return;
  const int k = begin + i;
  const int l = N.left[k], r = N.right[k];
  if (l >= 0) N.id[l] = N.id[k] + 1;
  if (r >= 0) N.id[r] = N.id[k] + 1 + (l >= 0 ? N.size[l] : 0);
}

__global__ void k_leaf_sizes_by_id(Nodes N, int nnodes, int* __restrict__ by_id) {
  const int k = blockIdx.x * BLK + threadIdx.x;
  if (k > nnodes) return;
  if (k == nnodes) {
    by_id[k] = 0;
    return;
  }
  by_id[N.id[k]] = N.leaf_cnt[k];
}

__global__ void k_write_nodes(Nodes N, int nnodes, const int* __restrict__ tstart_by_id,
                              kdpt_node_bare* __restrict__ out) {
  const int k = blockIdx.x * BLK + threadIdx.x;
  if (k >= nnodes) return;
  const int id = N.id[k];
  kdpt_node_bare o;
  o.axis = N.axis[k];
  o.splitPos = N.split_pos[k];
  const float4 lo = N.lo[k], hi = N.hi[k];
  o.mins[0] = lo.x; o.mins[1] = lo.y; o.mins[2] = lo.z;
  o.maxs[0] = hi.x; o.maxs[1] = hi.y; o.maxs[2] = hi.z;
  o.ID = id;
  o.parentID = N.parent[k] >= 0 ? N.id[N.parent[k]] : -1;
  o.leftID = N.left[k] >= 0 ? N.id[N.left[k]] : -1;
  o.rightID = N.right[k] >= 0 ? N.id[N.right[k]] : -1;
  const int cnt = N.leaf_cnt[k];
  o.triIdStart = cnt > 0 ? tstart_by_id[id] : -1;
  o.triIdSize = cnt > 0 ? cnt : -1;
  o.tmin = 0.0f;
  o.tmax = 0.0f;
  out[id] = o;
}

__global__ void k_write_tris(Nodes N, long long nleafpairs, const int* __restrict__ leaf_tri,
                             const int* __restrict__ leaf_node, const int* __restrict__ tstart_by_id,
                             const float* __restrict__ v9, const float* __restrict__ n9, const int* __restrict__ mtl,
                             kdpt_tri_bare* __restrict__ out) {
  const long long q = (long long)blockIdx.x * BLK + threadIdx.x;
  if (q >= nleafpairs) return;
  const int k = leaf_node[q], t = leaf_tri[q];
  const int pos = tstart_by_id[N.id[k]] + (int)(q - N.leaf_start[k]);
  const float* v = v9 + 9 * (size_t)t;
  const float* n = n9 + 9 * (size_t)t;
  kdpt_tri_bare o;
  o.x1 = v[0]; o.y1 = v[1]; o.z1 = v[2];
  o.x2 = v[3]; o.y2 = v[4]; o.z2 = v[5];
  o.x3 = v[6]; o.y3 = v[7]; o.z3 = v[8];
  o.nx1 = n[0]; o.ny1 = n[1]; o.nz1 = n[2];
  o.nx2 = n[3]; o.ny2 = n[4]; o.nz2 = n[5];
  o.nx3 = n[6]; o.ny3 = n[7]; o.nz3 = n[8];
  o.mtlIdx = mtl[t];
  out[pos] = o;
}

__global__ void k_iota(int* a, int n) {
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i < n) a[i] = i;
}

// Device memory owned by one build; freed on every exit path.
struct Arena {
  std::vector<void*> p;
  ~Arena() {
    for (void* q : p) (void)hipFree(q);
  }
  template <typename T>
  hipError_t alloc(T** out, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) p.push_back(q);
    *out = (T*)q;
    return e;
  }
  // frees one of the arena's buffers now (the caller has synchronised every use of it)
  hipError_t release(void* q) {
    auto it = std::find(p.begin(), p.end(), q);
    if (it == p.end()) return hipErrorInvalidValue;
    p.erase(it);
    return hipFree(q);
  }
};

struct Scanner {
  void* tmp = nullptr;
  size_t bytes = 0;
  hipStream_t st;
  Arena* arena;
  hipError_t exclusive(const int* in, int* out, long long n) {  // n items (the last one the total slot)
    size_t need = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (int)n, st);
    if (e != hipSuccess) return e;
    if (need > bytes) {
      if ((e = arena->alloc((char**)&tmp, need)) != hipSuccess) return e;
      bytes = need;
    }
    return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, out, (int)n, st);
  }
};

int read_int(const int* d, int* h, hipStream_t st) {
  KD_TRY(hipMemcpyAsync(h, d, sizeof(int), hipMemcpyDeviceToHost, st));
  KD_TRY(hipStreamSynchronize(st));
  return KDPT_OK;
}

}  // namespace

namespace kdpt_host {

int build_kd_device(const float* v9, const float* n9, const int* mtl, int ntri, int maxdepth, int device,
                    std::vector<kdpt_node_bare>& nodes_out, std::vector<kdpt_tri_bare>& tris_out, double* ms) {
  nodes_out.clear();
  tris_out.clear();
  if (ntri <= 0) return KDPT_OK;
  const auto t0 = std::chrono::steady_clock::now();
  KD_TRY(hipSetDevice(device));
  hipStream_t st;
  KD_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{st};
  Arena A;
  float *d_v9, *d_n9;
  int* d_mtl;
  float4 *d_tlo, *d_thi;
  KD_TRY(A.alloc(&d_v9, 9 * (size_t)ntri));
  KD_TRY(A.alloc(&d_n9, 9 * (size_t)ntri));
  KD_TRY(A.alloc(&d_mtl, (size_t)ntri));
  KD_TRY(A.alloc(&d_tlo, (size_t)ntri));
  KD_TRY(A.alloc(&d_thi, (size_t)ntri));
  KD_TRY(hipMemcpyAsync(d_v9, v9, 36 * (size_t)ntri, hipMemcpyHostToDevice, st));
  KD_TRY(hipMemcpyAsync(d_n9, n9, 36 * (size_t)ntri, hipMemcpyHostToDevice, st));
  KD_TRY(hipMemcpyAsync(d_mtl, mtl, 4 * (size_t)ntri, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_tri_bounds, dim3(blocks(ntri)), dim3(BLK), 0, st, d_v9, ntri, d_tlo, d_thi);
  KD_TRY(hipGetLastError());
  // ---- root box (KDnode::updateBbox): first-occurrence min / max, then the pad (centre not refreshed)
  unsigned long long* d_keys;
  KD_TRY(A.alloc(&d_keys, 6));
  {
    const unsigned long long init[6] = {~0ull, ~0ull, ~0ull, 0ull, 0ull, 0ull};
    KD_TRY(hipMemcpyAsync(d_keys, init, sizeof init, hipMemcpyHostToDevice, st));
  }
  hipLaunchKernelGGL(k_root_keys, dim3(blocks(ntri)), dim3(BLK), 0, st, d_tlo, d_thi, ntri, d_keys);
  KD_TRY(hipGetLastError());
  unsigned long long keys[6];
  float4 lo0, hi0;
  KD_TRY(hipMemcpyAsync(keys, d_keys, sizeof keys, hipMemcpyDeviceToHost, st));
  KD_TRY(hipMemcpyAsync(&lo0, d_tlo, sizeof lo0, hipMemcpyDeviceToHost, st));
  KD_TRY(hipMemcpyAsync(&hi0, d_thi, sizeof hi0, hipMemcpyDeviceToHost, st));
  KD_TRY(hipStreamSynchronize(st));
  float rmin[3], rmax[3];
  {
    const float l0[3] = {lo0.x, lo0.y, lo0.z}, h0[3] = {hi0.x, hi0.y, hi0.z};
    for (int c = 0; c < 3; c++) {
      // the fold starts from triangle 0 and replaces only on a strict improvement: a NaN at triangle 0
      // stays; otherwise the first triangle holding the extreme value
      if (l0[c] != l0[c] || keys[c] == ~0ull) {
        rmin[c] = l0[c];
      } else {
        float4 v;
        KD_TRY(hipMemcpy(&v, d_tlo + (uint32_t)keys[c], sizeof v, hipMemcpyDeviceToHost));
        rmin[c] = c == 0 ? v.x : (c == 1 ? v.y : v.z);
      }
      if (h0[c] != h0[c] || keys[3 + c] == 0ull) {
        rmax[c] = h0[c];
      } else {
        float4 v;
        KD_TRY(hipMemcpy(&v, d_thi + (uint32_t)~(uint32_t)keys[3 + c], sizeof v, hipMemcpyDeviceToHost));
        rmax[c] = c == 0 ? v.x : (c == 1 ? v.y : v.z);
      }
    }
  }
  float4 rlo, rhi, rctr;
  {
    float ctr[3];
    for (int c = 0; c < 3; c++) ctr[c] = (float)((double)(rmin[c] + rmax[c]) / 2.0);  // before the pad
    const float pad = (float)0.001;
    rlo = make_float4(rmin[0] - pad, rmin[1] - pad, rmin[2] - pad, 0.0f);
    rhi = make_float4(rmax[0] + pad, rmax[1] + pad, rmax[2] + pad, 0.0f);
    rctr = make_float4(ctr[0], ctr[1], ctr[2], 0.0f);
  }
  // ---- node store: at most 2 children per split node; a level's node count and pair count are known
  // before its children are made, so the store grows per level (capacity doubling)
  // every split makes two non-empty children and levels stop past maxdepth: < 2^(maxdepth + 2) nodes
  long long cap = std::max<long long>(1024, std::min<long long>(4ll * ntri + 16, 1ll << std::min(maxdepth + 2, 20)));
  Nodes N{};
  KD_TRY(A.alloc(&N.lo, cap));
  KD_TRY(A.alloc(&N.hi, cap));
  KD_TRY(A.alloc(&N.ctr, cap));
  KD_TRY(A.alloc(&N.parent, cap));
  KD_TRY(A.alloc(&N.left, cap));
  KD_TRY(A.alloc(&N.right, cap));
  KD_TRY(A.alloc(&N.axis, cap));
  KD_TRY(A.alloc(&N.split_pos, cap));
  KD_TRY(A.alloc(&N.pstart, cap));
  KD_TRY(A.alloc(&N.pcnt, cap));
  KD_TRY(A.alloc(&N.leaf_start, cap));
  KD_TRY(A.alloc(&N.leaf_cnt, cap));
  KD_TRY(A.alloc(&N.size, cap));
  KD_TRY(A.alloc(&N.id, cap));
  {  // root: KDnode defaults (axis 0, splitPos 0, parent -1), all triangles in file order
    const int m1 = -1, z = 0, nt = ntri;
    const float zf = 0.0f;
    KD_TRY(hipMemcpyAsync(N.lo, &rlo, sizeof rlo, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.hi, &rhi, sizeof rhi, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.ctr, &rctr, sizeof rctr, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.parent, &m1, 4, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.axis, &z, 4, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.split_pos, &zf, 4, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.pstart, &z, 4, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.pcnt, &nt, 4, hipMemcpyHostToDevice, st));
    KD_TRY(hipMemcpyAsync(N.id, &z, 4, hipMemcpyHostToDevice, st));
  }
  // pairs of the current and next level (grown as needed), leaf store
  long long pcap = std::max<long long>(3 * (long long)ntri, 1024), lcap = std::max<long long>(3 * (long long)ntri, 1024);
  int *ptri, *pnode, *ntri_, *nnode, *fl, *fr, *sl, *sr, *leaf_tri, *leaf_node;
  KD_TRY(A.alloc(&ptri, pcap));
  KD_TRY(A.alloc(&pnode, pcap));
  KD_TRY(A.alloc(&ntri_, pcap));
  KD_TRY(A.alloc(&nnode, pcap));
  KD_TRY(A.alloc(&fl, pcap + 1));
  KD_TRY(A.alloc(&fr, pcap + 1));
  KD_TRY(A.alloc(&sl, pcap + 1));
  KD_TRY(A.alloc(&sr, pcap + 1));
  KD_TRY(A.alloc(&leaf_tri, lcap));
  KD_TRY(A.alloc(&leaf_node, lcap));
  hipLaunchKernelGGL(k_iota, dim3(blocks(ntri)), dim3(BLK), 0, st, ptri, ntri);
  KD_TRY(hipMemsetAsync(pnode, 0, 4 * (size_t)ntri, st));
  // per-level node scratch (sized for the widest level: < number of nodes)
  int *nsplit, *npair, *nleaf, *nsplit_ex, *npair_ex, *nleaf_ex, *cl, *cr;
  KD_TRY(A.alloc(&nsplit, cap + 1));
  KD_TRY(A.alloc(&npair, cap + 1));
  KD_TRY(A.alloc(&nleaf, cap + 1));
  KD_TRY(A.alloc(&nsplit_ex, cap + 1));
  KD_TRY(A.alloc(&npair_ex, cap + 1));
  KD_TRY(A.alloc(&nleaf_ex, cap + 1));
  KD_TRY(A.alloc(&cl, cap));
  KD_TRY(A.alloc(&cr, cap));
  Scanner scan{nullptr, 0, st, &A};
  std::vector<int> lvl_begin{0}, lvl_count{1};
  long long npairs = ntri, leaf_total = 0;
  int nnodes = 1;
  for (int level = 0;; level++) {
    const int nl = lvl_count.back(), lb = lvl_begin.back();
    if (nl == 0) break;
    LevelArgs L{level, level % 3, maxdepth, lb, nl, npairs};
    hipLaunchKernelGGL(k_side, dim3(blocks(npairs + 1)), dim3(BLK), 0, st, L, ptri, pnode, N, d_tlo, d_thi, fl, fr);
    KD_TRY(hipGetLastError());
    KD_TRY(scan.exclusive(fl, sl, npairs + 1));
    KD_TRY(scan.exclusive(fr, sr, npairs + 1));
    hipLaunchKernelGGL(k_decide, dim3(blocks(nl + 1)), dim3(BLK), 0, st, L, N, sl, sr, nsplit, npair, nleaf, cl, cr);
    KD_TRY(hipGetLastError());
    KD_TRY(scan.exclusive(nsplit, nsplit_ex, nl + 1));
    KD_TRY(scan.exclusive(npair, npair_ex, nl + 1));
    KD_TRY(scan.exclusive(nleaf, nleaf_ex, nl + 1));
    int tot[3];
    KD_TRY(hipMemcpyAsync(&tot[0], nsplit_ex + nl, 4, hipMemcpyDeviceToHost, st));
    KD_TRY(hipMemcpyAsync(&tot[1], npair_ex + nl, 4, hipMemcpyDeviceToHost, st));
    KD_TRY(hipMemcpyAsync(&tot[2], nleaf_ex + nl, 4, hipMemcpyDeviceToHost, st));
    KD_TRY(hipStreamSynchronize(st));
    const int nsplit_tot = tot[0];
    const long long npairs_next = tot[1], nleaf_tot = tot[2];
    if (nnodes + 2ll * nsplit_tot > cap || npairs_next > pcap || leaf_total + nleaf_tot > lcap) {
      // grow the buffers and carry on with this level: the level's flags and scans are already in place,
      // only the next level's outputs need the larger capacity (rare: the initial capacities cover the
      // reference meshes).  Each replaced buffer is freed once its copy has run, so the peak device
      // memory is the new capacity plus one old buffer, not the sum of every size.
      auto grow = [&](auto*& ptr, long long oldn, long long newn) -> hipError_t {
        using T = std::remove_reference_t<decltype(*ptr)>;
        T* q;
        hipError_t e = A.alloc(&q, (size_t)newn);
        if (e != hipSuccess) return e;
        e = hipMemcpyAsync(q, ptr, sizeof(T) * (size_t)oldn, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess) e = A.release(ptr);
        ptr = q;
        return e;
      };
      if (nnodes + 2ll * nsplit_tot > cap) {
        const long long nc = std::max(2 * cap, nnodes + 2ll * nsplit_tot + 16);
        KD_TRY(grow(N.lo, cap, nc)); KD_TRY(grow(N.hi, cap, nc)); KD_TRY(grow(N.ctr, cap, nc));
        KD_TRY(grow(N.parent, cap, nc)); KD_TRY(grow(N.left, cap, nc)); KD_TRY(grow(N.right, cap, nc));
        KD_TRY(grow(N.axis, cap, nc)); KD_TRY(grow(N.split_pos, cap, nc)); KD_TRY(grow(N.pstart, cap, nc));
        KD_TRY(grow(N.pcnt, cap, nc)); KD_TRY(grow(N.leaf_start, cap, nc)); KD_TRY(grow(N.leaf_cnt, cap, nc));
        KD_TRY(grow(N.size, cap, nc)); KD_TRY(grow(N.id, cap, nc));
        KD_TRY(grow(nsplit, cap + 1, nc + 1)); KD_TRY(grow(npair, cap + 1, nc + 1)); KD_TRY(grow(nleaf, cap + 1, nc + 1));
        KD_TRY(grow(nsplit_ex, cap + 1, nc + 1)); KD_TRY(grow(npair_ex, cap + 1, nc + 1));
        KD_TRY(grow(nleaf_ex, cap + 1, nc + 1)); KD_TRY(grow(cl, cap, nc)); KD_TRY(grow(cr, cap, nc));
        cap = nc;
      }
      if (npairs_next > pcap) {
        const long long nc = std::max(2 * pcap, npairs_next + 16);
        KD_TRY(grow(ntri_, pcap, nc)); KD_TRY(grow(nnode, pcap, nc));
        KD_TRY(grow(ptri, pcap, nc)); KD_TRY(grow(pnode, pcap, nc));
        KD_TRY(grow(fl, pcap + 1, nc + 1)); KD_TRY(grow(fr, pcap + 1, nc + 1));
        KD_TRY(grow(sl, pcap + 1, nc + 1)); KD_TRY(grow(sr, pcap + 1, nc + 1));
        pcap = nc;
      }
      if (leaf_total + nleaf_tot > lcap) {
        const long long nc = std::max(2 * lcap, leaf_total + nleaf_tot + 16);
        KD_TRY(grow(leaf_tri, lcap, nc)); KD_TRY(grow(leaf_node, lcap, nc));
        lcap = nc;
      }
    }
    hipLaunchKernelGGL(k_children, dim3(blocks(nl)), dim3(BLK), 0, st, L, N, nsplit_ex, npair_ex, nleaf_ex, nsplit,
                       cl, cr, (int)leaf_total);
    KD_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_scatter, dim3(blocks(npairs)), dim3(BLK), 0, st, L, N, ptri, pnode, fl, fr, sl, sr, nsplit,
                       ntri_, nnode, leaf_tri, leaf_node);
    KD_TRY(hipGetLastError());
    std::swap(ptri, ntri_);
    std::swap(pnode, nnode);
    npairs = npairs_next;
    leaf_total += nleaf_tot;
    lvl_begin.push_back(lb + nl);
    lvl_count.push_back(2 * nsplit_tot);
    nnodes += 2 * nsplit_tot;
  }
  // ---- pre-order IDs: subtree sizes bottom-up, then IDs top-down
  const int nlev = (int)lvl_count.size();
  for (int l = nlev - 1; l >= 0; l--)
    if (lvl_count[l] > 0)
      hipLaunchKernelGGL(k_sizes, dim3(blocks(lvl_count[l])), dim3(BLK), 0, st, N, lvl_begin[l], lvl_count[l]);
  for (int l = 0; l < nlev; l++)
    if (lvl_count[l] > 0)
      hipLaunchKernelGGL(k_ids, dim3(blocks(lvl_count[l])), dim3(BLK), 0, st, N, lvl_begin[l], lvl_count[l]);
  KD_TRY(hipGetLastError());
  // ---- leaves' triangles in ID order, then the NodeBare / TriBare arrays
  int *by_id, *tstart;
  KD_TRY(A.alloc(&by_id, (size_t)nnodes + 1));
  KD_TRY(A.alloc(&tstart, (size_t)nnodes + 1));
  hipLaunchKernelGGL(k_leaf_sizes_by_id, dim3(blocks(nnodes + 1)), dim3(BLK), 0, st, N, nnodes, by_id);
  KD_TRY(hipGetLastError());
  KD_TRY(scan.exclusive(by_id, tstart, nnodes + 1));
  kdpt_node_bare* d_nodes;
  kdpt_tri_bare* d_tris;
  KD_TRY(A.alloc(&d_nodes, (size_t)nnodes));
  KD_TRY(A.alloc(&d_tris, (size_t)leaf_total));
  hipLaunchKernelGGL(k_write_nodes, dim3(blocks(nnodes)), dim3(BLK), 0, st, N, nnodes, tstart, d_nodes);
  if (leaf_total > 0)
    hipLaunchKernelGGL(k_write_tris, dim3(blocks(leaf_total)), dim3(BLK), 0, st, N, leaf_total, leaf_tri, leaf_node,
                       tstart, d_v9, d_n9, d_mtl, d_tris);
  KD_TRY(hipGetLastError());
  nodes_out.resize(nnodes);
  tris_out.resize((size_t)leaf_total);
  KD_TRY(hipMemcpyAsync(nodes_out.data(), d_nodes, sizeof(kdpt_node_bare) * (size_t)nnodes, hipMemcpyDeviceToHost, st));
  if (leaf_total > 0)
    KD_TRY(hipMemcpyAsync(tris_out.data(), d_tris, sizeof(kdpt_tri_bare) * (size_t)leaf_total, hipMemcpyDeviceToHost,
                          st));
  KD_TRY(hipStreamSynchronize(st));
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return KDPT_OK;
}

}  // namespace kdpt_host
