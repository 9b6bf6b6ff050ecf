// kdpt_runtime.hip -- gfx950 kernels and the C-ABI (include/kdpt.h) for the
// reference's per-sample hot path (src/pathtrace.cu:2405-2635 `pathtrace`).
//
// One iteration = k_gen_rays, then per bounce (cap 8, src/pathtrace.cu:2608):
//   k_trace    : the intersect kernel -- 6 analytic geoms + KD traversal, one lane
//                per live path, persistent waves pulling 64-path chunks, the KD
//                tree read from LDS when it fits (32-byte packed nodes)
//   k_shade    : scatterRay + shadeMaterial + partialGather, writes the path in
//                place and the tile's survivor count
//   k_scan     : exclusive scan of tile counts (key-major when iter == 2 sorts)
//   k_scatter  : stable compaction (thrust::remove_if) -- and on iter 2 the
//                stable sort by materialIdHit (thrust::sort, a merge sort) --
//                into the other path buffer.
// No host synchronisation inside an iteration: the live-path count lives on
// the device and kernels past the end of the live range exit at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include "../../include/kdpt.h"
#include "kdpt_device.h"
#include "kdpt_clusters.h"

using namespace kdpt;

namespace kdpt_host {
void node_box_matrices(const float* mins, const float* maxs, float* transform16, float* inverse16);
}

namespace {

constexpr int TILE = 256;  // paths per workgroup (4 waves of 64)
constexpr int MAX_KEYS = 64;

thread_local std::string g_last_error;
double g_reduce_spin_us = 0;  // kdpt_set_tuning(NULL, "reduce_spin_us", v): the default of new contexts
double g_cluster_chord = -1;   // kdpt_set_tuning(NULL, "cluster_chord", v): big-leaf grouping of new contexts
bool g_cu_mask_streams = true;  // kdpt_set_tuning(NULL, "cu_mask_streams", v): ... and their stream kind

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(KDPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));        \
  } while (0)

// Path state, structure of arrays of float4 (coalesced 1 KiB per wave load):
//   p0 = {origin.xyz, sdepth}
//   p1 = {direction.xyz, pixelIndex | isinside << 31}
//   p2 = {color.rgb, remainingBounces}
//   pm = materialIdHit
struct PathBuf {
  float4* p0;
  float4* p1;
  float4* p2;
  int* pm;
};

struct Counters {
  unsigned long long aabb, tri, hit;
  unsigned long long aabb_prep;  // root-box tests of rays that end before the intersect kernel (k_geoms/k_shade)
  unsigned long long cand;       // rays handed to the intersect kernel
  unsigned long long wave[PROF_SLOTS + 2];  // WaveLeafLDS::prof summed over chunks, then chunks, cycles
  unsigned long long life[64];  // count mode: wave lifetimes in the intersect kernel, 10 us bins (s_memrealtime)
  unsigned long long steps[64];  // count mode: node steps per ray, bins of 4
  unsigned long long chord_steps[8], chord_n[8];  // ... summed by the ray's chord through the root box (8ths of
                                                  // the box diagonal): does the chord predict a ray's cost?
};

// ---------------------------------------------------------------------------
// generateRayFromCamera (src/pathtrace.cu:315-397)
// ---------------------------------------------------------------------------
__device__ __attribute__((always_inline)) inline bool gen_rays_body(
    const kdpt_camera& cam, int iter, int traceDepth, PathBuf out, float focalLength, float dofAngle, int antialias,
    int* counts, int ncounts, int* work, int nwork, unsigned long long* trace_t, unsigned long long* lb, int nlb,
    float* zero_image, f3& ray_o, f3& ray_d) {
  const int W = cam.resolution[0], H = cam.resolution[1];
  const int index = blockIdx.x * blockDim.x + threadIdx.x;
  if (index == 0) {
    counts[0] = W * H;
    for (int k = 1; k < ncounts; k++) counts[k] = 0;
    for (int k = 0; k < nwork; k++) {
      work[k] = 0;
      work[nwork + k] = 0;  // candidate counts (k_geoms), stored after the work counters
      work[2 * nwork + k] = 0;  // k_shade_fused's tile tickets
      trace_t[2 * k] = ~0ull;  // k_trace span of bounce k, then (at 2*nwork) k_geoms' span
      trace_t[2 * k + 1] = 0ull;
      trace_t[2 * nwork + 2 * k] = ~0ull;
      trace_t[2 * nwork + 2 * k + 1] = 0ull;
    }
  }
  for (int e = index; e < nlb; e += gridDim.x * blockDim.x) lb[e] = 0ull;  // k_shade_fused's look-back records
  if (index >= W * H) return false;
  if (zero_image) {  // batched iterations: this iteration's partial image starts at zero (no separate fill)
    zero_image[3 * index] = 0.0f;
    zero_image[3 * index + 1] = 0.0f;
    zero_image[3 * index + 2] = 0.0f;
  }
  const int x = index % W, y = index / W;
  const f3 view = mk3(cam.view[0], cam.view[1], cam.view[2]);
  const f3 right = mk3(cam.right[0], cam.right[1], cam.right[2]);
  const f3 upv = mk3(cam.up[0], cam.up[1], cam.up[2]);
  Ray ray;
  ray.origin = mk3(cam.position[0], cam.position[1], cam.position[2]);
  ray.isinside = false;
  // cam.right * cam.pixelLength.x * (...): (vec * float) * float
  f3 a = scl(scl(right, cam.pixelLength[0]), ((float)x - (float)W * 0.5f));
  f3 b = scl(scl(upv, cam.pixelLength[1]), ((float)y - (float)H * 0.5f));
  ray.direction = normalize(sub(sub(view, a), b));
  Rng rng = rng_seed(utilhash((uint32_t)iter));  // same stream for every pixel (:334)
  if (antialias) {
    const float jitterscale = (float)0.002;
    float j0 = u01(rng), j1 = u01(rng), j2 = u01(rng);
    f3 v3a = normalize(mk3(j0, j1, j2));
    ray.direction = add(ray.direction, scl(v3a, jitterscale));
    ray.direction = normalize(ray.direction);
  }
  float u = kdpt_cosf(PI_F * u01(rng));
  float u2 = u * u;
  float sq = sqrtf(1 - u2);
  float theta = 2 * PI_F * u01(rng);
  f3 vv = normalize(mk3(sq * kdpt_cosf(theta), sq * kdpt_sinf(theta), u));
  (void)u01(rng);  // R1
  (void)u01(rng);  // R2
  float randangle = u01(rng) * PI_F * dofAngle;
  float qw = kdpt_cosf(randangle / 2.0f);
  float sh = kdpt_sinf(randangle / 2.0f);
  f3 qv = mk3(vv.x * sh, vv.y * sh, vv.z * sh);
  const f3 randrot = quat_rotate(qw, qv, ray.direction);  // glm::rotate(Q1, direction)
  ray.origin = sub(add(ray.origin, scl(ray.direction, focalLength)), scl(randrot, focalLength));
  ray.direction = normalize(randrot);
  out.p0[index] = make_float4(ray.origin.x, ray.origin.y, ray.origin.z, 0.0f);
  out.p1[index] = make_float4(ray.direction.x, ray.direction.y, ray.direction.z, ibits(index));
  out.p2[index] = make_float4(1.0f, 1.0f, 1.0f, ibits(traceDepth));
  ray_o = ray.origin;
  ray_d = ray.direction;
  return true;
}

// Launched for a whole batch of iterations at once (k_gen_rays_b, blockIdx.y = iteration).
struct GenIter {
  int iter;
  PathBuf out;
  int* counts;
  int* work;
  unsigned long long* trace_t;
  unsigned long long* lb;
  float* zero_image;
};

// ---------------------------------------------------------------------------
// pathTraceOneBounceKDbare (src/pathtrace.cu:1489-1662): the intersect kernel.
//
// Persistent: one 1024-thread workgroup per CU slot; every wave repeatedly takes
// the next 64 live paths from a device counter, so a wave that drew heavy rays
// never holds a CU idle.  With MODE == TREE_LDS the workgroup first copies the
// packed KD tree into LDS and every node step is an LDS read.
// Output per path: hit code (-1 none, g >= 0 analytic geom g, -(k + 2) triangle k)
// and objMaterialIdx; k_shade recomputes the winner's point and normal with the
// same functions, so nothing else needs to travel.
// ---------------------------------------------------------------------------
// TREE_LDS: 32-byte NodesPacked records in LDS (+ the cluster boxes); TREE_LDS16: 16-byte NodesDerived
// records + cluster boxes in LDS; TREE_LDS16G: NodesDerived in LDS, cluster boxes in HBM/L2 (trees whose
// clusters do not fit, e.g. the C5 icosphere: 2 655 nodes = 41 KB, 22 848 clusters = 714 KB); TREE_LDS16S:
// NodesDerived + the super-cluster boxes in LDS, cluster boxes in HBM/L2, two-level cull (the C5 icosphere:
// 1 430 supers of 16 clusters = 45 KB)
enum TreeMode { TREE_WIDE = 0, TREE_PACKED = 1, TREE_LDS = 2, TREE_LDS16 = 3, TREE_LDS16G = 4, TREE_LDS16S = 5 };
#ifndef KDPT_TRACE_BLOCK
#define KDPT_TRACE_BLOCK 1024  // tools/build_variant.sh experiments only
#endif
constexpr int TRACE_BLOCK = KDPT_TRACE_BLOCK;  // LDS mode: one workgroup per CU shares the tree copy
#ifndef KDPT_SRUN_SPREAD
#define KDPT_SRUN_SPREAD 0  // 1: static runs of ceil(n / waves) instead of 64 (experiment)
#endif
// workgroup size of the intersect kernel: with the tree in LDS every wave of a CU must share the copy,
// otherwise small workgroups let the tail of one launch hold only a quarter of a CU
// NodesDerived halves the tree copy.  Two 512-thread workgroups per CU (30 KB of per-wave leaf scratch + 46 KB
// of tree and cluster boxes each for dragon_5), so that one workgroup's launch tail would overlap the next
// one's start, measured 5.5 % slower than one 1024-thread workgroup (profiles/r03_ab_log.md)
#ifndef KDPT_TRACE_BLOCK16
#define KDPT_TRACE_BLOCK16 1024  // tools/build_variant.sh experiments only
#endif
constexpr int TRACE_BLOCK16 = KDPT_TRACE_BLOCK16;
constexpr bool tree_in_lds(int mode) { return mode >= 2; }
template <int MODE>
constexpr int trace_block() { return MODE == 2 ? TRACE_BLOCK : (MODE >= 3 ? TRACE_BLOCK16 : 256); }

// Up to MAXB iterations (each its own path buffers) at the same bounce share one intersect launch:
// more rays per launch keep the lanes of the persistent waves busy.
#ifndef KDPT_MAXB
#define KDPT_MAXB 16  // tools/build_variant.sh experiments only
#endif
constexpr int MAXB = KDPT_MAXB;
struct TraceIter {
  const int* cand;      // k_geoms' list of the paths whose ray meets the KD root box (queue slot -> path)
  const int* ccount;    // ... and its length per bounce
  const float4* cray;   // ... and their rays in queue order: [2 slot] = {origin, t_min}, [2 slot + 1] = {dir, geom}
  int2* hits;
};

struct TraceArgs {
  DevScene S;
  TraceIter it[MAXB];
  int nb;
  int prof_steps;  // count mode, "profile_batches" = 2: per-ray node-step histogram
  int* work;  // chunk counters, zeroed by k_gen_rays (of iteration 0 of the batch)
  int depth;
  Counters* counters;
  unsigned long long* trace_t;  // [4 * cap]: per bounce first block start / last block end (s_memrealtime)
                                // of k_trace, then of k_geoms (at 2 * cap)
};

struct GenBatch {
  GenIter it[MAXB];
  kdpt_camera cam;
  int traceDepth, antialias, ncounts, nwork, nlb;
  float focalLength, dofAngle;
};
__global__ __launch_bounds__(256) void k_gen_rays_b(GenBatch B) {
  const GenIter& g = B.it[blockIdx.y];
  f3 o, d;
  (void)gen_rays_body(B.cam, g.iter, B.traceDepth, g.out, B.focalLength, B.dofAngle, B.antialias, g.counts,
                      B.ncounts, g.work, B.nwork, g.trace_t, g.lb, B.nlb, g.zero_image, o, d);
}

__device__ inline void flush_counters(Counters* C, const TraverseCounters& cnt, WaveProf* W,
                                      unsigned long long t_k0) {
  unsigned int a = cnt.aabb, tr = cnt.tri, hi = cnt.hit;
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_down(a, off);
    tr += __shfl_down(tr, off);
    hi += __shfl_down(hi, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&C->aabb, (unsigned long long)a);
    atomicAdd(&C->tri, (unsigned long long)tr);
    atomicAdd(&C->hit, (unsigned long long)hi);
    for (int k = 0; k < PROF_SLOTS; k++) {
      atomicAdd(&C->wave[k], W->prof[k]);
      W->prof[k] = 0;
    }
    atomicAdd(&C->wave[PROF_SLOTS], 1ull);
    atomicAdd(&C->wave[PROF_SLOTS + 1], __builtin_readcyclecounter() - t_k0);
  }
}

// The intersect stage's first part for one ray: the analytic geoms of pathTraceOneBounceKDbare (tested
// before the KD tree; src/pathtrace.cu:1600-1640) -> t_min / hit, and the traversal's first step, the
// KD root's box (same intersectAABB, same invdir): false = the traversal ends there.
constexpr int ORDERED_GEOMS = 8;  // scenes with at most this many analytic geoms test them nearest-first
__device__ __attribute__((always_inline)) inline bool prep_ray(const DevScene& S, bool kd, f3 o, f3 d, float& t_min, int& hit) {
  Ray ray;
  ray.origin = o;
  ray.direction = d;
  ray.isinside = false;
  ray.sdepth = 0.0f;
  t_min = FLT_MAXV;
  hit = -1;
  f3 tmp_i = mk3(0, 0, 0), tmp_n = mk3(0, 0, 0);
  const f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const bool finite = fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV;
  const int ng = S.num_geoms;
  if (finite && ng <= ORDERED_GEOMS) {
    // Nearest-first: the reference keeps the first geom (index order) reaching the smallest t > 0; here
    // the geoms whose bounds the ray enters are tested in order of their entry bound, stopping once that
    // bound exceeds the best t, and ties go to the lower index -- the same winner and the same t, with
    // typically one or two exact tests per ray instead of one per geom the wave's rays come near.
    float lo[ORDERED_GEOMS];
    uint32_t pending = 0;
#pragma unroll
    for (int g = 0; g < ORDERED_GEOMS; g++) {
      lo[g] = FLT_INFV;
      if (g < ng && geom_entry_bound(S.geoms[g], o, inv, lo[g])) pending |= 1u << g;
    }
    while (pending) {
      int gb = 0;
      float lb = FLT_INFV;
#pragma unroll
      for (int g = 0; g < ORDERED_GEOMS; g++)
        if (((pending >> g) & 1u) && lo[g] < lb) {
          lb = lo[g];
          gb = g;
        }
      if (lb > t_min) break;  // every remaining geom's exact t exceeds the best
      pending &= ~(1u << gb);
      const DevGeom& G = S.geoms[gb];
      const float t = G.type == 1 ? boxIntersectionTest(G, ray, tmp_i, tmp_n)
                                  : sphereIntersectionTest(G, ray, tmp_i, tmp_n);
      if (t > 0.0f && (t < t_min || (t == t_min && gb < hit))) {
        t_min = t;
        hit = gb;
      }
    }
  } else {
    float t = 0;
    for (int g = 0; g < ng; g++) {
      const DevGeom& G = S.geoms[g];
      if (finite && !geom_may_hit(G, o, inv)) {
        t = -1.0f;  // the exact test would miss
      } else if (G.type == 1) {
        t = boxIntersectionTest(G, ray, tmp_i, tmp_n);
      } else if (G.type == 0) {
        t = sphereIntersectionTest(G, ray, tmp_i, tmp_n);
      }
      if (t > 0.0f && t_min > t) {
        t_min = t;
        hit = g;
      }
    }
  }
  if (!kd) return false;
  float dist;
  return intersectAABB(o, inv, make_float4(S.rlo.x, S.rlo.y, S.rlo.z, S.rhi.x),
                       make_float4(S.rhi.y, S.rhi.z, 0.0f, 0.0f), dist);
}

// The analytic geoms of pathTraceOneBounceKDbare (tested before the KD tree; src/pathtrace.cu:1600-1640),
// one lane per live path, consecutive paths per wave: {t_min bits, geom index} for k_trace.
//
// The KD traversal's first step tests the root's box, and a ray that misses it ends there with no other
// effect (traverseKDbareShortHybrid: `!hitGeom && parentID == -1` -> break), so such a ray's hit record
// is final here: it is written now, and only the rays that meet the root box are listed (cand, ccount)
// for the intersect kernel -- whose lanes then all hold rays that actually walk the tree.
// k_gen_geoms_b / k_geoms_b: 256-thread workgroups (one wave per SIMD), one candidate-list atomic per
// workgroup.  A 1024-thread workgroup needs 4 waves x 88 VGPRs on every SIMD of a CU, which a CU running an
// intersect workgroup (4 x 96 of 512) never has, so the batch's first launch waited for CUs free of k_trace:
// 0.93 ms per launch in the pipelined bench against 0.18 ms alone (profiles/r03_ab_log.md); one 88-VGPR
// wave fits beside the intersect workgroup
#ifndef KDPT_GEN_BLOCK
#define KDPT_GEN_BLOCK 256  // tools/build_variant.sh experiments only
#endif
constexpr int GEN_BLOCK = KDPT_GEN_BLOCK;
// One workgroup's part: the analytic geoms + root-box test of its paths (live: the lane holds a path still
// bouncing), the final hit record of the rays that end there, and the others appended to the candidate list
// through *ccnt (one atomic per workgroup; a single counter hit once per wave by ~10k waves serialises for
// ~100 us at 800x800).  Every thread of the workgroup must call it.
template <int TB = GEN_BLOCK>
__device__ __attribute__((always_inline)) inline void geoms_core(const DevScene& S, bool live, int i, f3 o, f3 d,
                                                                 float4* __restrict__ cray, int2* __restrict__ hits,
                                                                 int* __restrict__ cand, int* __restrict__ ccnt,
                                                                 Counters* count_aabb) {
  const bool kd = S.has_obj && S.num_nodes > 0;
  bool tested = false, walk = false;  // traversed at all / goes on to the intersect kernel
  float t_min = 0.0f;
  int hit = -1;
  if (live) {
    tested = kd;
    walk = prep_ray(S, kd, o, d, t_min, hit);
    if (!walk) hits[i] = make_int2(hit, -1);  // final: the analytic geoms' hit (code -1: none)
  }
  __shared__ int s_wcount[TB / 64], s_base;
  const unsigned long long wm = __ballot(walk);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s_wcount[wv] = __popcll(wm);
  if (count_aabb) {  // count mode: the root test of the rays that end here, and the candidates
    const unsigned long long miss = __ballot(tested && !walk);
    if (lane == 0 && miss) {
      atomicAdd(&count_aabb->aabb, (unsigned long long)__popcll(miss));
      atomicAdd(&count_aabb->aabb_prep, (unsigned long long)__popcll(miss));
    }
    if (lane == 0 && wm) atomicAdd(&count_aabb->cand, (unsigned long long)__popcll(wm));
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < TB / 64; w++) {
      const int c = s_wcount[w];
      s_wcount[w] = tot;
      tot += c;
    }
    s_base = tot ? atomicAdd(ccnt, tot) : 0;
  }
  __syncthreads();
  if (walk) {
    const int slot = s_base + s_wcount[wv] + (int)lane_prefix(wm);
    cand[slot] = i;
    cray[2 * slot] = make_float4(o.x, o.y, o.z, t_min);
    cray[2 * slot + 1] = make_float4(d.x, d.y, d.z, ibits(hit));
  }
}

__device__ __attribute__((always_inline)) inline void geoms_body(const DevScene& S, PathBuf paths, const int* counts,
                                                                 int depth, float4* __restrict__ cray,
                                                                 int2* __restrict__ hits, int* __restrict__ cand,
                                                                 int* __restrict__ ccount, Counters* count_aabb,
                                                                 unsigned long long* gspan) {
  const int n = counts[depth];
  if ((int)(blockIdx.x * blockDim.x) >= n) return;  // uniform per block
  if (threadIdx.x == 0) atomicMin(&gspan[2 * depth], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // finished paths (compaction off) are skipped, as pathTraceOneBounce* skips them
  const bool live = i < n && fbits(paths.p2[i].w) > 0;
  f3 o = mk3(0, 0, 0), d = mk3(0, 0, 1);
  if (live) {
    const float4 q0 = paths.p0[i], q1 = paths.p1[i];
    o = mk3(q0.x, q0.y, q0.z);
    d = mk3(q1.x, q1.y, q1.z);
  }
  geoms_core<GEN_BLOCK>(S, live, i, o, d, cray, hits, cand, ccount + depth, count_aabb);
  if (threadIdx.x == 0) atomicMax(&gspan[2 * depth + 1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// Launched for a whole batch of iterations at once (blockIdx.y = iteration).
struct GeomsIter {
  PathBuf paths;
  const int* counts;
  float4* cray;
  int2* hits;
  int* cand;
  int* ccount;
};
struct GeomsBatch {
  DevScene S;
  GeomsIter it[MAXB];
  int depth;
  Counters* count_aabb;
  unsigned long long* gspan;
};
__global__ __launch_bounds__(GEN_BLOCK) void k_geoms_b(GeomsBatch B) {
  const GeomsIter& g = B.it[blockIdx.y];
  geoms_body(B.S, g.paths, g.counts, B.depth, g.cray, g.hits, g.cand, g.ccount, B.count_aabb, B.gspan);
}

// A batch's camera rays and their bounce-0 intersect-stage first part in one launch (blockIdx.y = iteration):
// each lane generates its pixel's ray (written out for the shading) and tests it against the analytic geoms
// and the KD root box straight from registers.  The bounce-0 candidate counter cannot be the one the
// generation zeroes (other workgroups of this launch already add to it), so bounce 0 counts into
// ccount0[parity] of the context, and the launch zeroes ccount0[!parity] for the context's next use (always
// on the same stream, so nothing still reads it).
struct GenGeomsIter {
  int* ccount0;       // this use's bounce-0 candidate counter
  int* ccount0_next;  // the next use's (zeroed here)
  float4* cray;
  int2* hits;
  int* cand;
};
struct GenGeomsBatch {
  GenBatch g;
  DevScene S;
  GenGeomsIter it[MAXB];
  Counters* count_aabb;
};
__global__ __launch_bounds__(GEN_BLOCK) void k_gen_geoms_b(GenGeomsBatch B) {
  const GenIter& g = B.g.it[blockIdx.y];
  const GenGeomsIter& q = B.it[blockIdx.y];
  f3 o = mk3(0, 0, 0), d = mk3(0, 0, 1);
  const bool valid = gen_rays_body(B.g.cam, g.iter, B.g.traceDepth, g.out, B.g.focalLength, B.g.dofAngle,
                                   B.g.antialias, g.counts, B.g.ncounts, g.work, B.g.nwork, g.trace_t, g.lb, B.g.nlb,
                                   g.zero_image, o, d);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *q.ccount0_next = 0;
  geoms_core<GEN_BLOCK>(B.S, valid && B.g.traceDepth > 0, i, o, d, q.cray, q.hits, q.cand, q.ccount0,
                        B.count_aabb);
}

#ifdef KDPT_TAIL_PROF  // tools/build_variant.sh experiments only: intersect workgroup life / tail (ticks)
__device__ unsigned long long g_tail_prof[4];
#endif

// KD traversal of every live path.  Each lane holds one ray; whenever rays finish, the idle lanes take
// the next paths of the bounce from a device counter, so a wave stays full until the bounce runs out
// of paths (the per-ray algorithm is unchanged -- only which lane runs it, and when).
// Compiled for 5 waves per SIMD although a workgroup brings only 4 (its LDS tree copy keeps it alone on the
// CU): the cap (96 VGPRs instead of 108, a few spilled to scratch outside the hot loops) leaves 128 VGPRs per
// SIMD, room for a fused-shading wave of another batch on the same CU while the traversal runs -- and its LDS
// (WaveProf only in the counting kernel) leaves room for that workgroup's 4.2 KB.  A/B +2.8 %.
#ifndef KDPT_TRACE_WAVES
#define KDPT_TRACE_WAVES 5  // tools/build_variant.sh experiments
#endif
// (only with the tree in LDS: the 256-thread workgroups of the other modes share CUs anyway, and the C5
// icosphere, whose tree lives in HBM, lost 3.5 % to the cap)
#define KDPT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(tree_in_lds(MODE) ? KDPT_TRACE_WAVES : 1)))
template <bool HYBRID, bool COUNT, int MODE>
__global__ __launch_bounds__(trace_block<MODE>()) KDPT_TRACE_ATTR void k_trace(TraceArgs A) {
  constexpr int TB = trace_block<MODE>();
  extern __shared__ int4 s_tree[];
  __shared__ WaveLeafLDS s_leaf[TB / 64];
  __shared__ WaveProf s_prof[COUNT ? TB / 64 : 1];
  const DevScene& S = A.S;
  int pre[MAXB + 1];  // the batch's paths, concatenated: iteration b owns queue slots [pre[b], pre[b+1])
  pre[0] = 0;
#pragma unroll
  for (int b = 0; b < MAXB; b++) pre[b + 1] = pre[b] + (b < A.nb ? A.it[b].ccount[A.depth] : 0);
  const int n = pre[MAXB];
  // tree copy: NodesPacked (2 x 16 bytes per node) or NodesDerived (16 bytes), then the cluster boxes
  constexpr int NODE_WORDS = MODE == TREE_LDS ? 2 : 1;
  if (tree_in_lds(MODE)) {
    if (n == 0) return;  // uniform: nothing to trace
    const int words = NODE_WORDS * S.num_nodes;
    const int4* src = MODE == TREE_LDS ? S.pnodes : (MODE == TREE_LDS16S ? S.snodes : S.dnodes);
    for (int k = threadIdx.x; k < words; k += TB) s_tree[k] = src[k];
    if (MODE == TREE_LDS16S) {
      for (int k = threadIdx.x; k < S.num_supers; k += TB) s_tree[words + k] = S.sup[k];
    } else if (MODE != TREE_LDS16G) {
      float4* s_cl = reinterpret_cast<float4*>(s_tree + words);
      for (int k = threadIdx.x; k < S.num_clusters; k += TB) {
        s_cl[2 * k] = S.cl_lo[k];
        s_cl[2 * k + 1] = S.cl_hi[k];
      }
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  WaveLeafLDS* W = &s_leaf[threadIdx.x >> 6];
  WaveProf* P = &s_prof[COUNT ? (threadIdx.x >> 6) : 0];
  if (COUNT && lane < PROF_SLOTS) P->prof[lane] = 0;
  if (COUNT && lane == 0) P->tail_t0 = 0;
  W->slot[lane] = 0;  // pair_owner's invariant
  // launch duration on the device clock (first block start .. last block end); the HIP events around
  // the launch also count time spent queued behind other streams' kernels when iterations overlap
  __shared__ int s_waves_done;
#ifdef KDPT_TAIL_PROF
  __shared__ unsigned long long s_t0, s_tex;
#endif
  if (threadIdx.x == 0) {
    s_waves_done = 0;
    atomicMin(&A.trace_t[2 * A.depth], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#ifdef KDPT_TAIL_PROF
    s_t0 = __builtin_amdgcn_s_memrealtime();
    s_tex = ~0ull;
#endif
  }
  __syncthreads();
  int* work = A.work + A.depth;
  const unsigned long long rt0 = COUNT ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const unsigned long long t_k0 = COUNT ? __builtin_readcyclecounter() : 0ull;
  TraverseCounters cnt{};
  WaveRay R;  // every field defined: idle lanes take part in the wave-level code with a finished ray
  wave_ray_start(S, R, mk3(0.0f, 0.0f, 0.0f), mk3(0.0f, 0.0f, 1.0f), FLT_MAXV, -1, W);
  R.done = true;
  int pidx = -1;  // the lane's path (-1: idle)
  int pb = 0;     // ... and the batch iteration it belongs to
  // Path slots: each wave first takes a static run of 64 consecutive slots, the runs dealt out wave-major
  // across the workgroups (run r goes to wave r / grid of workgroup r % grid): a bounce with few rays then
  // still fills every CU (the kernel is issue-bound: rays piled onto a few CUs would leave the others idle)
  // while each wave stays dense (a node trip costs the same whatever the number of walking lanes).  A device
  // counter hands out the rest, exactly as many as the wave has idle lanes, so the tail stays balanced.
  const int nwaves = gridDim.x * (TB / 64);
  const int wid = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
  const int srun = KDPT_SRUN_SPREAD ? min(64, max(1, (n + nwaves - 1) / nwaves)) : 64;
  bool first = true, exhausted = false;
  long long rounds = 0;
#ifdef KDPT_TAIL_PROF
  unsigned long long tex_seen = 0;
#endif
  while (true) {
    if (__ballot(1) != ~0ull) {  // the refill protocol needs the whole wave here
      atomicOr(S.fault, 4);
      break;
    }
    // ---- refill idle lanes ----
    if (COUNT) prof_lap(P, -1);
    const unsigned long long im = exhausted ? 0ull : __ballot(pidx < 0);
    if (im) {
      const int p = (int)lane_prefix(im);
      int k;
      if (first) {  // static run: slots [wid*srun, wid*srun + srun)
        first = false;
        k = p < srun ? wid * srun + p : n;
        exhausted = (long long)nwaves * srun >= n;
      } else {
        int b = 0;
        if (lane == 0) b = nwaves * srun + atomicAdd(work, __popcll(im));
        const int base = __builtin_amdgcn_readfirstlane(b);  // lane 0 is active: the whole wave is here
        k = base + p;
        exhausted = base + __popcll(im) >= n;  // the counter only grows: later rounds find nothing
      }
      if (COUNT && exhausted && lane == 0 && !P->tail_t0) P->tail_t0 = __builtin_readcyclecounter();
#ifdef KDPT_TAIL_PROF
      if (exhausted && !tex_seen) tex_seen = __builtin_amdgcn_s_memrealtime();
#endif
      if (pidx < 0 && k < n) {
        int b = 0;
#pragma unroll
        for (int q = 1; q < MAXB; q++) b += k >= pre[q];
        const int* cand = A.it[0].cand;
        const float4* cray = A.it[0].cray;
        int local = k;
#pragma unroll
        for (int q = 1; q < MAXB; q++)
          if (b == q) {
            cand = A.it[q].cand;
            cray = A.it[q].cray;
            local = k - pre[q];
          }
        // the slot's path index and its ray (written in queue order with the slot): three independent loads
        // of consecutive slots, not a slot load followed by scattered path loads
        const int i = cand[local];
        const float4 q0 = cray[2 * local], q1 = cray[2 * local + 1];
        pidx = i;
        pb = b;
        wave_ray_start(S, R, mk3(q0.x, q0.y, q0.z), mk3(q1.x, q1.y, q1.z), q0.w, fbits(q1.w), W);
      }
    }
    if (COUNT) prof_lap(P, PROF_SETUP_CYC);
    const bool busy = pidx >= 0 && !R.done;
    if (__any(busy)) {
      const bool fastAABB = __all(!busy || (fabsf(R.invdir.x) < FLT_INFV && fabsf(R.invdir.y) < FLT_INFV &&
                                            fabsf(R.invdir.z) < FLT_INFV));
      if (MODE == TREE_LDS)
        trace_phase<HYBRID, COUNT>(S, NodesPacked{s_tree},
                                   ClustersInterleaved{reinterpret_cast<const float4*>(s_tree + 2 * S.num_nodes)}, R,
                                   fastAABB, S.num_materials, cnt, W, P);
      else if (MODE == TREE_LDS16)
        trace_phase<HYBRID, COUNT>(S, NodesDerived{s_tree},
                                   ClustersInterleaved{reinterpret_cast<const float4*>(s_tree + S.num_nodes)}, R,
                                   fastAABB, S.num_materials, cnt, W, P);
      else if (MODE == TREE_LDS16G)
        trace_phase<HYBRID, COUNT>(S, NodesDerived{s_tree}, ClustersSplit{S.cl_lo, S.cl_hi}, R, fastAABB,
                                   S.num_materials, cnt, W, P);
      else if (MODE == TREE_LDS16S)
        trace_phase<HYBRID, COUNT>(
            S, NodesDerived{s_tree},
            ClustersSuper{s_tree + S.num_nodes, S.cl_lo, S.cl_hi, S.cl_n, S.cl_u, S.cl_v, S.cl_w}, R, fastAABB,
            S.num_materials, cnt, W, P);
      else if (MODE == TREE_PACKED)
        trace_phase<HYBRID, COUNT>(S, NodesPacked{S.pnodes}, ClustersSplit{S.cl_lo, S.cl_hi}, R, fastAABB,
                                   S.num_materials, cnt, W, P);
      else
        trace_phase<HYBRID, COUNT>(S, NodesWide{S.nodes}, ClustersSplit{S.cl_lo, S.cl_hi}, R, fastAABB,
                                   S.num_materials, cnt, W, P);
    }
    // ---- finished rays: their hit record (what ShadeableIntersection would carry) ----
    if (pidx >= 0 && R.done) {
      if (COUNT && A.prof_steps) {  // (its atomics distort the cycle profile: a separate run)
        const int st = R.guard;
        atomicAdd(&A.counters->steps[min(st >> 2, 63)], 1ull);
        const float4 lo = S.rlo, hi = S.rhi;
        const float ax = (lo.x - R.o.x) * R.invdir.x, bx = (hi.x - R.o.x) * R.invdir.x;
        const float ay = (lo.y - R.o.y) * R.invdir.y, by = (hi.y - R.o.y) * R.invdir.y;
        const float az = (lo.z - R.o.z) * R.invdir.z, bz2 = (hi.z - R.o.z) * R.invdir.z;
        const float t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz2), 0.0f));
        const float t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz2));
        const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
        const float diag = sqrtf(dx * dx + dy * dy + dz * dz);
        const float f = diag > 0.0f ? 8.0f * fmaxf(t1 - t0, 0.0f) / diag : 0.0f;
        const int cb = f >= 7.0f || !(f == f) ? 7 : (int)f;
        atomicAdd(&A.counters->chord_steps[cb], (unsigned long long)st);
        atomicAdd(&A.counters->chord_n[cb], 1ull);
      }
      const Hit& h = R.h;
      const int code = h.hit_geom_index == -1 ? -1 : (h.obj_intersect ? -(R.objTri + 2) : h.hit_geom_index);
      int2* hits = A.it[0].hits;
#pragma unroll
      for (int q = 1; q < MAXB; q++)
        if (pb == q) hits = A.it[q].hits;
      hits[pidx] = make_int2(code, h.objMaterialIdx);
      pidx = -1;
    }
    if (exhausted && !__any(pidx >= 0)) break;
    if (++rounds > (1ll << 20)) {  // unreachable: every round finishes or advances some ray
      if (lane == 0) atomicOr(S.fault, 8);
      break;
    }
  }
  if (COUNT) {
    prof_lap(P, PROF_POST_CYC);
    if (lane == 0 && P->tail_t0) P->prof[PROF_TAIL_CYC] += __builtin_readcyclecounter() - P->tail_t0;
    flush_counters(A.counters, cnt, P, t_k0);
    if (lane == 0) {
      const unsigned long long us10 = (__builtin_amdgcn_s_memrealtime() - rt0) / 1000;  // 100 MHz ticks
      atomicAdd(&A.counters->life[us10 < 63 ? us10 : 63], 1ull);
    }
  }
#ifdef KDPT_TAIL_PROF
  if (lane == 0 && tex_seen) atomicMin(&s_tex, tex_seen);
#endif
  if (lane == 0 && atomicAdd(&s_waves_done, 1) == TB / 64 - 1) {
    atomicMax(&A.trace_t[2 * A.depth + 1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#ifdef KDPT_TAIL_PROF
    // this workgroup's life, and its part after its first wave found the ray queue empty
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long tex = s_tex == ~0ull ? t1 : s_tex;
    atomicAdd(&g_tail_prof[0], t1 - s_t0);
    atomicAdd(&g_tail_prof[1], t1 - (tex < s_t0 ? s_t0 : tex));
    atomicAdd(&g_tail_prof[2], 1ull);
#endif
  }
}

// ---------------------------------------------------------------------------
// pathTraceOneBounce (src/pathtrace.cu:402-628, enable_kd = false): the brute-force intersect kernel,
// the reference's "bruteforce" / "bbox" benchmark columns.  One lane per live path, consecutive paths
// per wave; the analytic geoms, then every OBJ triangle in file order, shape after shape.
//
// The triangle index is wave-uniform (every lane of a wave tests the same triangle), so the triangle
// is fetched with scalar loads once per wave.  Each lane first evaluates, without the division,
// the exact values the reference's Moller-Trumbore divides (a, u = dot(s,p), v = dot(d,q),
// w = dot(e2,q): same operations, same order, so the same bits) and rejects the triangle when the
// decision is certain whatever f = 1/a rounds to; only the remaining lanes (the line crosses the
// triangle, or a decision sits within a few ulps of its threshold) run the reference's exact test and
// hit point.  Output: the same hit record as k_trace (code, objMaterialIdx).
// ---------------------------------------------------------------------------
struct BruteShape {
  float4 lo;  // bbox min (the reference's float(obj_polysbboxes[i + k] - 0.01)), w = index count bits
  float4 hi;  // bbox max (+ 0.01), w = obj_materialOffsets[i] bits
};

struct BruteArgs {
  DevScene S;  // tv0/te1/te2/tn0..2: the OBJ triangles in file order
  PathBuf paths;
  const int* counts;
  int depth;
  int2* hits;
  const BruteShape* shapes;
  int num_shapes;
  const float4* chunk_lo;  // boxes of the file-order triangles [64j, 64j + 64) (the tested triangles
  const float4* chunk_hi;  // v0, v0 + e1, v0 + e2, rounded outward)
  Counters* counters;
  unsigned long long* trace_t;
};

// intersectBbox (src/interactions.h:136-165), std::min/max as in intersectAABBarrays
__device__ inline float intersectBbox(f3 o, f3 d, float4 lo, float4 hi) {
  const f3 invdir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float v1 = (lo.x - o.x) * invdir.x, v2 = (hi.x - o.x) * invdir.x;
  const float v3 = (lo.y - o.y) * invdir.y, v4 = (hi.y - o.y) * invdir.y;
  const float v5 = (lo.z - o.z) * invdir.z, v6 = (hi.z - o.z) * invdir.z;
  const float dmin = std_max(std_max(std_min(v1, v2), std_min(v3, v4)), std_min(v5, v6));
  const float dmax = std_min(std_min(std_max(v1, v2), std_max(v3, v4)), std_max(v5, v6));
  if (dmax < 0) return dmax;
  if (dmin > dmax) return dmax;
  return dmin;
}

// Is glm::intersectRayTriangle certain to return false?  a, u, v, w are the reference's exact values;
// f = RN(1/a) > 0 (a >= eps).  bx = RN(f*u) < 0 for u < -a*2^-100 (|f*u| >= 2^-101, far from rounding
// to -0); bx > 1 for u > RN(a*(1+2^-20)) (then u/a > 1 + 2^-21 and two roundings cannot bring it to 1);
// likewise by, the sum (u + v > a*(1+2^-18) with u, v >= 0) and bz = RN(f*w) < 0.
__device__ inline bool tri_certain_miss(float a, float u, float v, float w) {
  const float tiny = a * 0x1p-100f;
  const float one_u = a * 1.00000095367431640625f;  // a * (1 + 2^-20)
  const float one_s = a * 1.000003814697265625f;    // a * (1 + 2^-18)
  return !(a >= FLT_EPS) || u < -tiny || u > one_u || v < -tiny || w < -tiny ||
         (u >= 0.0f && v >= 0.0f && u + v > one_s);
}

template <bool COUNT>
__device__ inline void brute_triangle(const DevScene& S, int k, const TriData& T, f3 o, f3 d, float& t_min, int& best,
                                      bool take, TraverseCounters& cnt) {
  const f3 v0 = mk3(T.v0.x, T.v0.y, T.v0.z), e1 = mk3(T.e1.x, T.e1.y, T.e1.z), e2 = mk3(T.e2.x, T.e2.y, T.e2.z);
  const f3 p = cross(d, e2);
  const float a = dot(e1, p);
  const f3 s = sub(o, v0);
  const float u = dot(s, p);
  const f3 q = cross(s, e1);
  const float v = dot(d, q);
  const float w = dot(e2, q);
  if (take && !tri_certain_miss(a, u, v, w)) {
    float bx, by, bz;
    if (tri_test_v(T, o, d, bx, by, bz) == 2) {  // intersected: bary.z >= 0
      if (COUNT) cnt.hit++;
      f3 hp, nn;
      const float t = tri_hit_t<true>(S, k, o, d, bx, by, bz, hp, nn);  // hit += norm * 0.0001f
      if (t > 0.0f && t_min > t) {
        t_min = t;
        best = k;
      }
    }
  }
}

template <bool USEBBOX, bool COUNT>
__global__ __launch_bounds__(TILE) void k_brute(BruteArgs A) {
  const int n = A.counts[A.depth];
  if ((int)blockIdx.x * TILE >= n) return;  // uniform per block
  if (threadIdx.x == 0) atomicMin(&A.trace_t[2 * A.depth], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  const DevScene& S = A.S;
  const int i = blockIdx.x * TILE + threadIdx.x;
  bool live = false;
  f3 o = mk3(0.0f, 0.0f, 0.0f), d = mk3(0.0f, 0.0f, 1.0f);
  if (i < n) {
    const float4 q0 = A.paths.p0[i], q1 = A.paths.p1[i];
    live = fbits(A.paths.p2[i].w) > 0;
    o = mk3(q0.x, q0.y, q0.z);
    d = mk3(q1.x, q1.y, q1.z);
  }
  // the analytic geoms (src/pathtrace.cu:461-483)
  float t_min = FLT_MAXV;
  int geom = -1;
  if (live) {
    Ray ray;
    ray.origin = o;
    ray.direction = d;
    ray.isinside = false;
    ray.sdepth = 0.0f;
    f3 tmp_i, tmp_n;
    float t = 0;
    const f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const bool finite = fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV;
    for (int g = 0; g < S.num_geoms; g++) {
      const DevGeom& G = S.geoms[g];
      if (finite && !geom_may_hit(G, o, inv)) t = -1.0f;
      else if (G.type == 1) t = boxIntersectionTest(G, ray, tmp_i, tmp_n);
      else if (G.type == 0) t = sphereIntersectionTest(G, ray, tmp_i, tmp_n);
      if (t > 0.0f && t_min > t) {
        t_min = t;
        geom = g;
      }
    }
  }
  // the polygon loop (src/pathtrace.cu:485-576)
  const f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const bool cull = __all(!live || (fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV));
  TraverseCounters cnt{};
  int best = -1;
  int objMat = -1;
  int iterator = 0;  // in vertex indices, like the reference; advances only past shapes whose bbox passed
  if (S.has_obj) {
    for (int sh = 0; sh < A.num_shapes; sh++) {
      const BruteShape B = A.shapes[sh];
      objMat = fbits(B.hi.w);
      const int nidx = fbits(B.lo.w);
      bool take = live;
      if (USEBBOX) take = live && intersectBbox(o, d, B.lo, B.hi) > -1.0f;
      const unsigned long long tm = __ballot(take);
      if (tm) {
        const int it0 = __shfl(iterator, __builtin_ctzll(tm));
        if (__all(!take || iterator == it0)) {
          // every lane that tests this shape starts at the same triangle: scalar triangle fetches
          const int k0 = __builtin_amdgcn_readfirstlane(it0 / 3);
          const int nt = nidx / 3;
          // 64-triangle chunks: no triangle of a chunk whose box the lane's line misses (box widened as in
          // cluster_may_pass) passes the u/v tests, so those lanes skip it, and the wave skips a chunk no lane
          // can hit; the others test its triangles in file order as before
          for (int k = k0; k < k0 + nt;) {
            const int j = k >> 6, kend = min(k0 + nt, (j + 1) << 6);
            const bool may = take && (!cull || cluster_may_pass(A.chunk_lo[j], A.chunk_hi[j], o, inv, S.cl_margin));
            if (__any(may)) {
              for (; k < kend; k++) {
                const TriData T = tri_load(S, k);
                brute_triangle<COUNT>(S, k, T, o, d, t_min, best, may, cnt);
              }
            }
            k = kend;
          }
        } else {
          const int nt = nidx / 3;
          for (int j = 0; j < nt; j++) {
            const int k = iterator / 3 + j;
            if (take) {
              const TriData T = tri_load(S, k);
              brute_triangle<COUNT>(S, k, T, o, d, t_min, best, true, cnt);
            }
          }
        }
        if (COUNT && take) cnt.tri += nidx / 3;
      }
      if (take) iterator += nidx;
    }
  }
  if (i < n && live) {
    const int code = best >= 0 ? -(best + 2) : geom;
    A.hits[i] = make_int2(code, objMat);
  }
  if (COUNT) {
    unsigned int tr = cnt.tri, hi = cnt.hit;
    for (int off = 32; off > 0; off >>= 1) {
      tr += __shfl_down(tr, off);
      hi += __shfl_down(hi, off);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&A.counters->tri, (unsigned long long)tr);
      atomicAdd(&A.counters->hit, (unsigned long long)hi);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&A.trace_t[2 * A.depth + 1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------------------
// pathTraceOneBounceKDbareBoxes (src/pathtrace.cu:1738-1885, viz_kd): the analytic geoms, then every KD
// node's box as a box (boxIntersectionTestBox = boxIntersectionTest of the node's unit-cube transform).
// One lane per path; the node index is wave-uniform, so each box's matrices are scalar loads.  A winning
// node box k is reported as geom num_geoms + k (its record carries material num_materials - 1), which
// k_shade recomputes like any analytic geom.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TILE) void k_viz(DevScene S, PathBuf paths, const int* counts, int depth, int2* hits,
                                               unsigned long long* trace_t) {
  const int n = counts[depth];
  if ((int)blockIdx.x * TILE >= n) return;
  if (threadIdx.x == 0) atomicMin(&trace_t[2 * depth], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int i = blockIdx.x * TILE + threadIdx.x;
  if (i < n && fbits(paths.p2[i].w) > 0) {
    const float4 q0 = paths.p0[i], q1 = paths.p1[i];
    Ray ray;
    ray.origin = mk3(q0.x, q0.y, q0.z);
    ray.direction = mk3(q1.x, q1.y, q1.z);
    ray.isinside = false;
    ray.sdepth = q0.w;
    const f3 inv = mk3(1.0f / ray.direction.x, 1.0f / ray.direction.y, 1.0f / ray.direction.z);
    const bool finite = fabsf(inv.x) < FLT_INFV && fabsf(inv.y) < FLT_INFV && fabsf(inv.z) < FLT_INFV;
    float t_min = FLT_MAXV, t = 0;
    int hit = -1;
    f3 tmp_i, tmp_n;
    const int total = S.num_geoms + (S.has_obj ? S.num_boxes : 0);
    for (int g = 0; g < total; g++) {
      const DevGeom& G = S.geoms[g];
      if (finite && !geom_may_hit(G, ray.origin, inv)) t = -1.0f;
      else if (G.type == 1) t = boxIntersectionTest(G, ray, tmp_i, tmp_n);
      else if (G.type == 0) t = sphereIntersectionTest(G, ray, tmp_i, tmp_n);
      if (t > 0.0f && t_min > t) {
        t_min = t;
        hit = g;
      }
    }
    hits[i] = make_int2(hit, -1);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&trace_t[2 * depth + 1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------------------
// shadeMaterial + scatterRay (src/pathtrace.cu:1885-2100, src/interactions.h) +
// partialGather, one lane per live path; writes the path in place and the tile's
// survivor count (or, when sorting, its per-material histogram).
// ---------------------------------------------------------------------------
struct ShadeArgs {
  DevScene S;
  PathBuf paths;
  const int2* hits;
  float* image;
  const int* counts;
  int depth;
  int iter;
  float softness;
  int enable_sss;
  int* tile_counts;  // [ntiles] or key-major [MAX_KEYS][ntiles] when sorting
  int* tile_kcounts;  // key-major [TRACE_KEYS][ntiles] survivors per trace-order class, or null
  int ntiles;
  int nkeys;
  unsigned long long* total_segments;  // running sum of paths launched into the intersect kernel
  const unsigned long long* trace_t;   // this bounce's intersect launch record (see TraceArgs)
  const unsigned long long* gspan;     // ... and the k_geoms launches' record
  unsigned long long* trace_total;     // [2]: summed launch ticks, launches (the batch's first iteration only)
  unsigned long long* trace_rays;      // rays handed to the intersect kernel, summed (every iteration)
  const int* ccount;                   // ... per bounce (this iteration's candidate counts)
  // next bounce's intersect-stage first part (prep_ray) for every surviving path, fused here instead of a
  // k_geoms pass: {t_min bits, (geom + 1) | walks << 16} at the path's current slot (k_scatter moves it)
  int image_zeroed;  // `image` is this iteration's partial image, zeroed by its camera-ray launch: a pixel's
                     // partialGather then reads +0 (each pixel's path ends once), so its load is skipped
  int prep_on;
  int2* prep;
  int* tile_ccounts;   // [ntiles] walking survivors per tile
  Counters* count_aabb;  // count mode: root tests of the rays that end there
};

// One path's shading (shadeMaterial + scatterRay, src/pathtrace.cu), the partialGather of a path that ends
// here, and, when the hand-off runs, the next bounce's intersect-stage first part (prep_ray).
struct ShadeOut {
  float4 q0, q1, q2;
  int pm;
  bool changed, alive, walk, tested;
  float tm;
  int gh;
};

// Everything one path's shading reads from memory, loaded in one go: the path, its hit record, the pixel's
// accumulated value (COMPACT: partialGather) and the hit triangle's vertex, edge and normal records (all in
// flight together; k_shade_fused issues them before its publication barrier, and must read the hit record
// before it lets later tiles write the next bounce's records into the same array).
struct ShadeIn {
  float4 q0, q1, q2;
  int pm;
  int2 hr;
  float3 px_old;
  TriData T;
  float4 n1v, n2v, n3v;
};

template <bool COMPACT>
__device__ __attribute__((always_inline)) inline void shade_load(const ShadeArgs& A, const DevScene& S, int i,
                                                                 ShadeIn& in) {
  in.q0 = A.paths.p0[i];
  in.q1 = A.paths.p1[i];
  in.q2 = A.paths.p2[i];
  in.pm = A.paths.pm[i];
  in.hr = A.hits[i];
  in.px_old = make_float3(0.0f, 0.0f, 0.0f);
  if (COMPACT && !A.image_zeroed) {
    const float* px = A.image + 3 * (size_t)(fbits(in.q1.w) & 0x7fffffff);
    in.px_old = make_float3(px[0], px[1], px[2]);
  }
  if (in.hr.x < -1 && fbits(in.q2.w) > 0) {
    const int k = -in.hr.x - 2;
    in.T = TriData{S.tv0[k], S.te1[k], S.te2[k]};
    in.n1v = S.tn0[k];
    in.n2v = S.tn1[k];
    in.n3v = S.tn2[k];
  }
}

template <bool HYBRID, bool COMPACT>
__device__ __attribute__((always_inline)) inline void shade_one(const ShadeArgs& A, const DevScene& S, int i,
                                                                const ShadeIn& in, ShadeOut& o) {
  const float4 q0 = in.q0, q1 = in.q1, q2 = in.q2;
  int matHit = in.pm;
  const int2 hr = in.hr;
  const int pw = fbits(q1.w);
  const int pix = pw & 0x7fffffff;
  Ray ray;
  ray.origin = mk3(q0.x, q0.y, q0.z);
  ray.direction = mk3(q1.x, q1.y, q1.z);
  ray.isinside = (pw >> 31) & 1;
  ray.sdepth = q0.w;
  f3 color = mk3(q2.x, q2.y, q2.z);
  int bounces = fbits(q2.w);
  o.changed = bounces > 0;
  const float3 px_old = in.px_old;
  if (bounces > 0) {
    float isect_t = -1.0f;
    int isect_mat = 0;
    if (hr.x != -1) {
      f3 ip, nrm;
      float t;
      int mid;
      if (hr.x < -1) {  // triangle: the traversal's final recomputation, repeated
        float bx, by, bzk;
        tri_test_v(in.T, ray.origin, ray.direction, bx, by, bzk);
        t = tri_hit_t_n<HYBRID>(in.n1v, in.n2v, in.n3v, ray.origin, ray.direction, bx, by, bzk, ip, nrm);
        mid = hr.y;
      } else {
        const DevGeom& G = S.geoms[hr.x];
        t = G.type == 1 ? boxIntersectionTest(G, ray, ip, nrm) : sphereIntersectionTest(G, ray, ip, nrm);
        mid = G.materialid;
      }
      Rng rng = seeded_rng(A.iter, i, A.depth);
      matHit = mid;
      scatterRay(ray, ip, nrm, S.materials[mid], rng, A.softness);
      isect_t = t;
      isect_mat = mid;
    }
    shade(isect_t, isect_mat, S.materials, A.enable_sss != 0, ray, color, bounces);
  }
  o.q0 = make_float4(ray.origin.x, ray.origin.y, ray.origin.z, ray.sdepth);
  o.q1 = make_float4(ray.direction.x, ray.direction.y, ray.direction.z, ibits(pix | ((ray.isinside ? 1 : 0) << 31)));
  o.q2 = make_float4(color.x, color.y, color.z, ibits(bounces));
  o.pm = matHit;
  if (COMPACT && bounces == 0) {
    // partialGather: one live path per pixel, so this read-modify-write never collides
    float* px = A.image + 3 * (size_t)pix;
    px[0] = px_old.x + color.x;
    px[1] = px_old.y + color.y;
    px[2] = px_old.z + color.z;
  }
  o.alive = COMPACT ? (bounces != 0) : true;
  o.walk = o.tested = false;
  o.tm = 0.0f;
  o.gh = -1;
  if (COMPACT && A.prep_on && bounces != 0) {
    o.walk = prep_ray(S, S.has_obj && S.num_nodes > 0, ray.origin, ray.direction, o.tm, o.gh);
    o.tested = S.has_obj && S.num_nodes > 0;
  }
}

__device__ inline void shade_stats(const ShadeArgs& A, int n) {
  atomicAdd(A.total_segments, (unsigned long long)n);
  // the intersect kernel of this bounce on the device clock (first block start .. last block end; a
  // launch that had nothing to do left its record empty)
  const unsigned long long t0 = A.trace_t[2 * A.depth], t1 = A.trace_t[2 * A.depth + 1];
  const unsigned long long span = t1 > t0 ? t1 - t0 : 0ull;
  if (A.trace_total && span) {
    atomicAdd(&A.trace_total[0], span);
    atomicAdd(&A.trace_total[1], 1ull);
  }
  if (A.trace_rays) atomicAdd(A.trace_rays, (unsigned long long)A.ccount[A.depth]);
}

__device__ inline void count_prep(const ShadeArgs& A, bool tested, bool walk) {
  const unsigned long long miss = __ballot(tested && !walk), wm = __ballot(walk);
  if ((threadIdx.x & 63) == 0 && miss) {
    atomicAdd(&A.count_aabb->aabb, (unsigned long long)__popcll(miss));
    atomicAdd(&A.count_aabb->aabb_prep, (unsigned long long)__popcll(miss));
  }
  if ((threadIdx.x & 63) == 0 && wm) atomicAdd(&A.count_aabb->cand, (unsigned long long)__popcll(wm));
}

// Shading in place, then k_scan + k_scatter (the material sort of iteration 2, no compaction, or the
// trace-order classes).
template <bool HYBRID, bool COMPACT, bool SORT>
__global__ __launch_bounds__(TILE) void k_shade(ShadeArgs A) {
  const int n = A.counts[A.depth];
  const int tile = blockIdx.x;
  if (tile * TILE >= n) return;  // uniform per block
  const int i = tile * TILE + threadIdx.x;
  if (i == 0) shade_stats(A, n);
  __shared__ int s_hist[MAX_KEYS];
  __shared__ int s_khist[TRACE_KEYS];
  if (SORT) {
    for (int k = threadIdx.x; k < MAX_KEYS; k += TILE) s_hist[k] = 0;
  }
  if (COMPACT && A.tile_kcounts && threadIdx.x < TRACE_KEYS) s_khist[threadIdx.x] = 0;
  if (SORT || (COMPACT && A.tile_kcounts)) __syncthreads();
  const DevScene& S = A.S;
  bool alive = false, walk = false, tested = false;
  int key = 0;
  if (i < n) {
    ShadeOut o;
    ShadeIn in;
    shade_load<COMPACT>(A, A.S, i, in);
    shade_one<HYBRID, COMPACT>(A, A.S, i, in, o);
    if (o.changed) {
      A.paths.p0[i] = o.q0;
      A.paths.p1[i] = o.q1;
      A.paths.p2[i] = o.q2;
      A.paths.pm[i] = o.pm;
    }
    alive = o.alive;
    walk = o.walk;
    tested = o.tested;
    key = o.pm;
    if (COMPACT && A.prep_on && alive) A.prep[i] = make_int2(fbits(o.tm), (o.gh + 1) | (walk ? 0x10000 : 0));
    if (COMPACT && A.tile_kcounts && alive)
      atomicAdd(&s_khist[trace_class(S, mk3(o.q0.x, o.q0.y, o.q0.z), mk3(o.q1.x, o.q1.y, o.q1.z))], 1);
  }
  if (COMPACT && A.tile_kcounts) {
    __syncthreads();
    if (threadIdx.x < TRACE_KEYS) A.tile_kcounts[threadIdx.x * A.ntiles + tile] = s_khist[threadIdx.x];
  }
  if (SORT) {
    if (alive) atomicAdd(&s_hist[key], 1);
    __syncthreads();
    for (int k = threadIdx.x; k < A.nkeys; k += TILE) A.tile_counts[k * A.ntiles + tile] = s_hist[k];
  } else {
    const int c = __syncthreads_count(alive);
    if (threadIdx.x == 0) A.tile_counts[tile] = c;
  }
  if (COMPACT && A.prep_on) {
    const int cw = __syncthreads_count(walk);
    if (threadIdx.x == 0) A.tile_ccounts[tile] = cw;
    if (A.count_aabb) count_prep(A, tested, walk);
  }
}

// Single-pass shading + stable stream compaction (the usual case: compaction on, no material sort).
// Tiles take tickets in arrival order, publish their survivor / walker counts and find their offsets by a
// decoupled look-back over the earlier tiles' records (lb: flag << 62 | survivors << 31 | walkers; flag 1 =
// this tile's counts, 2 = inclusive prefix), then write the survivors straight into the other path buffer in
// the order the scan + scatter would give, with the next bounce's hand-off records.  A tile writes only
// after every earlier tile has published, i.e. has read its inputs, and its own slots are >= the ones it
// writes, so the hit records can be compacted in place.
struct FuseArgs {
  PathBuf dst;
  int* tickets;               // [cap] tile tickets per bounce
  unsigned long long* lb;     // [cap][ntiles] look-back records
  int* counts;                // [cap + 2] live paths per bounce
  int* ccount;                // [cap] candidates per bounce
  float4* cray;
  int2* hits;
  int* cand;
};

__device__ inline unsigned long long lb_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void lb_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long lb_pack(unsigned long long flag, unsigned s, unsigned w) {
  return (flag << 62) | ((unsigned long long)s << 31) | (unsigned long long)w;
}

constexpr int STAGE_MATS = 32;
#ifdef KDPT_SHADE_PROF  // tools/build_variant.sh experiments only: shading phase times (s_memrealtime ticks)
__device__ unsigned long long g_shade_prof[8];
#endif
#ifndef KDPT_SHADE_TB
#define KDPT_SHADE_TB 256  // tools/build_variant.sh experiments only
#endif
#ifndef KDPT_SHADE_WAVES
#define KDPT_SHADE_WAVES 6  // fused shading: waves per SIMD it is compiled for (caps its VGPRs at 80)
#endif
constexpr int SHADE_TB = KDPT_SHADE_TB;  // paths per fused-shading workgroup (one tile ticket each)

// The LDS a shading workgroup uses: staged geoms/materials and the per-tile compaction scratch.
template <bool STAGE, int TB = TILE>
struct ShadeLDS {
  int tile, b;
  unsigned cnt[2][TB / 64];
  unsigned ex[2];
  uint32_t geoms[STAGE ? ORDERED_GEOMS * sizeof(DevGeom) / 4 : 1];
  uint32_t mats[STAGE ? STAGE_MATS * sizeof(DevMaterial) / 4 : 1];
};

// what a fused-shading workgroup needs beside a resident intersect workgroup (the LDS16S route leaves it free)
constexpr size_t SHADE_LDS_RESERVE = sizeof(ShadeLDS<true, SHADE_TB>);

// STAGE: the analytic geoms and the materials copied into LDS (small scenes: their per-lane reads, indexed
// by hit and by nearest-first order, are then LDS reads instead of L2 round trips)
// (SYNC false: the caller's next __syncthreads publishes the copy -- k_shade_fused overlaps it with the
// tile ticket's atomic round trip)
template <bool STAGE, int TB, bool SYNC = true>
__device__ __attribute__((always_inline)) inline DevScene stage_scene(const DevScene& S0, ShadeLDS<STAGE, TB>& L) {
  static_assert(sizeof(DevGeom) % 4 == 0 && sizeof(DevMaterial) % 4 == 0, "staged as dwords");
  DevScene S = S0;
  if (STAGE) {
    const int gw = S0.num_geoms * (int)(sizeof(DevGeom) / 4), mw = S0.num_materials * (int)(sizeof(DevMaterial) / 4);
    for (int k = threadIdx.x; k < gw; k += TB) L.geoms[k] = reinterpret_cast<const uint32_t*>(S0.geoms)[k];
    for (int k = threadIdx.x; k < mw; k += TB) L.mats[k] = reinterpret_cast<const uint32_t*>(S0.materials)[k];
    if (SYNC) __syncthreads();
    S.geoms = reinterpret_cast<const DevGeom*>(L.geoms);
    S.materials = reinterpret_cast<const DevMaterial*>(L.mats);
  }
  return S;
}

// shade()'s outcome for path i ahead of the shading: bounces left after this bounce != 0.  A listed hit
// has t > 0 (the traversal and k_geoms/prep_ray keep only t > 0, and shade_one recomputes the same t), so
// the path survives iff it has bounces left, hit something, the hit material does not emit, and one bounce
// remains after this one.
__device__ __attribute__((always_inline)) inline bool survives(const DevScene& S, int bounces, int2 hr) {
  if (bounces <= 0) return bounces != 0;
  if (hr.x == -1) return false;
  const int mid = hr.x < -1 ? hr.y : S.geoms[hr.x].materialid;
  return !(S.materials[mid].emittance > 0.0f) && bounces - 1 != 0;
}

// One 256-path tile of one iteration: shading, the survivors' stable compaction into the other path buffer
// (decoupled look-back over the earlier tiles' records), the next bounce's intersect-stage hand-off.  Tiles
// of an iteration must be started in increasing order (tickets), so every earlier tile is already running.
template <bool HYBRID, bool STAGE, int TB>
__device__ __attribute__((always_inline)) inline void shade_tile(const ShadeArgs& A, const FuseArgs& F, const DevScene& S, int tile, int n,
                                  ShadeLDS<STAGE, TB>& L, unsigned long long t_wg = 0ull) {
  const int i = tile * TB + threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#ifdef KDPT_SHADE_PROF
  const unsigned long long pt0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (i == 0) shade_stats(A, n);
  unsigned long long* lb = F.lb + (size_t)A.depth * A.ntiles;
  // (1) Which paths survive this bounce follows from the hit record and the hit material alone, so the
  // tile's survivor count is published (look-back aggregate) before the shading: later tiles' look-backs
  // then wait on this tile's two loads, not on its whole shading (measured: the look-back wait had grown
  // as long as the shading itself, the slowest of 64 predecessors' shading each time).
  // the hit record is read once, here: once this tile's aggregate is out, later tiles may finish their
  // look-back and write the next bounce's records (F.hits == A.hits) into this tile's index range
  ShadeIn in;
  in.hr = make_int2(-1, -1);
  if (i < n) shade_load<true>(A, S, i, in);
  const bool pred = i < n && survives(S, fbits(in.q2.w), in.hr);
  const unsigned long long ms = __ballot(pred);
#ifdef KDPT_SHADE_PROF
  const unsigned long long pa = __builtin_amdgcn_s_memrealtime();
#endif
  if (lane == 0) L.cnt[0][wid] = (unsigned)__popcll(ms);
  __syncthreads();
#ifdef KDPT_SHADE_PROF
  const unsigned long long pb = __builtin_amdgcn_s_memrealtime();
#endif
  if (wid == 0) {
    unsigned aS = 0;
    for (int w = 0; w < TB / 64; w++) aS += L.cnt[0][w];
    if (lane == 0) lb_store(lb + tile, lb_pack(tile == 0 ? 2 : 1, aS, 0));
  }
  // (2) the shading
  ShadeOut o;
  o.alive = o.walk = o.tested = false;
  if (i < n) shade_one<HYBRID, true>(A, S, i, in, o);
  if (o.alive != pred) atomicOr(S.fault, 32);  // unreachable: survives() restates shade()'s outcome
  const unsigned long long mw = __ballot(o.walk);
  if (A.count_aabb && A.prep_on) count_prep(A, o.tested, o.walk);
  if (lane == 0) L.cnt[1][wid] = (unsigned)__popcll(mw);
  __syncthreads();
#ifdef KDPT_SHADE_PROF
  const unsigned long long pt1 = __builtin_amdgcn_s_memrealtime();
#endif
  // (3) the survivors' exclusive prefix (look-back), the walkers' place in the next bounce's candidate
  // list (one counter add per tile: the list's order only decides which lane traces which ray)
  if (wid == 0) {
    unsigned aS = 0, aW = 0;
    for (int w = 0; w < TB / 64; w++) {
      aS += L.cnt[0][w];
      aW += L.cnt[1][w];
    }
    unsigned eS = 0;
    if (tile != 0) {
      for (int base = tile - 1;; base -= 64) {
        const int j = base - lane;
        unsigned long long v = j >= 0 ? lb_load(lb + j) : lb_pack(2, 0, 0);
        while (__ballot((v >> 62) == 0)) {
          __builtin_amdgcn_s_sleep(1);
          if ((v >> 62) == 0) v = lb_load(lb + j);
        }
        const unsigned long long pre = __ballot((v >> 62) == 2);
        const int upto = pre ? __ffsll((long long)pre) - 1 : 63;  // nearest inclusive prefix, and the counts before it
        unsigned sm = lane <= upto ? (unsigned)(v >> 31) & 0x7fffffffu : 0u;
        for (int off = 32; off > 0; off >>= 1) sm += __shfl_xor(sm, off);
        eS += sm;
        if (pre) break;
      }
      if (lane == 0) lb_store(lb + tile, lb_pack(2, eS + aS, 0));
    }
    if (lane == 0) {
      L.ex[0] = eS;
      L.ex[1] = (A.prep_on && aW) ? (unsigned)atomicAdd(&F.ccount[A.depth + 1], (int)aW) : 0u;
      if (tile == (n - 1) / TB) F.counts[A.depth + 1] = (int)(eS + aS);  // the last tile: the next bounce's paths
    }
  }
  __syncthreads();
#ifdef KDPT_SHADE_PROF
  const unsigned long long pt2 = __builtin_amdgcn_s_memrealtime();
#endif
  if (o.alive) {
    unsigned bS = L.ex[0], bW = L.ex[1];
    for (int w = 0; w < wid; w++) {
      bS += L.cnt[0][w];
      bW += L.cnt[1][w];
    }
    const int d = (int)(bS + lane_prefix(ms));
    F.dst.p0[d] = o.q0;
    F.dst.p1[d] = o.q1;
    F.dst.p2[d] = o.q2;
    F.dst.pm[d] = o.pm;
    if (A.prep_on) {
      if (o.walk) {
        const int slot = (int)(bW + lane_prefix(mw));
        F.cand[slot] = d;
        F.cray[2 * slot] = make_float4(o.q0.x, o.q0.y, o.q0.z, o.tm);
        F.cray[2 * slot + 1] = make_float4(o.q1.x, o.q1.y, o.q1.z, ibits(o.gh));
      } else {
        F.hits[d] = make_int2(o.gh, -1);  // final: the analytic geoms' hit (code -1: none)
      }
    }
  }
#ifdef KDPT_SHADE_PROF
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long pt3 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&g_shade_prof[0], pt1 - pt0);
    atomicAdd(&g_shade_prof[1], pt2 - pt1);
    atomicAdd(&g_shade_prof[2], pt3 - pt2);
    atomicAdd(&g_shade_prof[3], 1ull);
    atomicAdd(&g_shade_prof[4], (unsigned long long)min(TB, n - tile * TB));
    atomicAdd(&g_shade_prof[5], pt0 - t_wg);  // ticket + staging
    atomicAdd(&g_shade_prof[6], pa - pt0);    // the path / hit-record loads (thread 0's wave)
    atomicAdd(&g_shade_prof[7], pb - pa);     // the publication barrier (the tile's slowest wave)
  }
#endif
}

// One launch per bounce and iteration: tile = ticket (tickets start the tiles in order).
template <bool HYBRID, bool STAGE>
__device__ __attribute__((always_inline)) inline void shade_fused_body(const ShadeArgs& A, const FuseArgs& F) {
  const int n = A.counts[A.depth];
  // the grid covers every pixel, so past the first bounces most workgroups have no tile: exactly the first
  // ceil(n / SHADE_TB) take tickets (one contended atomic per tile, not per workgroup), the rest leave at once
  if ((int)blockIdx.x * SHADE_TB >= n) return;
#ifdef KDPT_SHADE_PROF
  const unsigned long long t_wg = __builtin_amdgcn_s_memrealtime();
#else
  const unsigned long long t_wg = 0ull;
#endif
  __shared__ ShadeLDS<STAGE, SHADE_TB> L;
  // the ticket's device-scope atomic and the staging copy are in flight together; one barrier for both
  if (threadIdx.x == 0) L.tile = atomicAdd(&F.tickets[A.depth], 1);
  const DevScene S = stage_scene<STAGE, SHADE_TB, false>(A.S, L);
  __syncthreads();
  const int tile = L.tile;
  shade_tile<HYBRID, STAGE, SHADE_TB>(A, F, S, tile, n, L, t_wg);
}

template <bool HYBRID, bool STAGE>
__global__ __launch_bounds__(SHADE_TB) __attribute__((amdgpu_waves_per_eu(KDPT_SHADE_WAVES))) void k_shade_fused(ShadeArgs A, FuseArgs F) {
  shade_fused_body<HYBRID, STAGE>(A, F);
}

// The same for every fused iteration of a batch in one launch (blockIdx.y = iteration): the batch's
// shading no longer runs iteration after iteration on its stream.
struct ShadeBatch {
  ShadeArgs a[MAXB];
  FuseArgs f[MAXB];
};
template <bool HYBRID, bool STAGE>
__global__ __launch_bounds__(SHADE_TB) __attribute__((amdgpu_waves_per_eu(KDPT_SHADE_WAVES))) void k_shade_fused_b(ShadeBatch B) {
  shade_fused_body<HYBRID, STAGE>(B.a[blockIdx.y], B.f[blockIdx.y]);
}

// Exclusive scan of the tile counts (one workgroup; <= MAX_KEYS * ntiles entries).
// One workgroup per scan job: job 0 = the survivors (or, when sorting, the per-material histogram),
// job 1 = the walking survivors of the intersect-stage hand-off (launched only when it runs).
struct ScanJob {
  const int* tile_counts;
  int* tile_off;
  int nkeys;
  int* total_out;
};
// 256 threads: every kernel a batch launches fits beside a resident intersect workgroup (4 waves x 96 VGPRs per
// SIMD, 150 KB of LDS per CU), which a 1024-thread workgroup never does
constexpr int SCAN_TB = 256;
__global__ __launch_bounds__(SCAN_TB) void k_scan(ScanJob j0, ScanJob j1, const int* counts, int depth,
                                                  int ntiles_alloc) {
  const ScanJob& J = blockIdx.x == 0 ? j0 : j1;
  const int* __restrict__ tile_counts = J.tile_counts;
  int* __restrict__ tile_off = J.tile_off;
  const int nkeys = J.nkeys;
  int* total_out = J.total_out;
  const int n = counts[depth];
  const int ntiles = (n + TILE - 1) / TILE;
  const int total_entries = nkeys * ntiles;
  __shared__ int s_wave[SCAN_TB / 64];
  __shared__ int s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < total_entries; base += SCAN_TB) {
    const int e = base + threadIdx.x;
    int v = 0;
    int k = 0, t = 0;
    if (e < total_entries) {
      k = e / ntiles;
      t = e - k * ntiles;
      v = tile_counts[k * ntiles_alloc + t];
    }
    // inclusive wave scan
    int x = v;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
      int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    __syncthreads();
    if (wid == 0) {
      int w = lane < SCAN_TB / 64 ? s_wave[lane] : 0;
      for (int off = 1; off < SCAN_TB / 64; off <<= 1) {
        int y = __shfl_up(w, off);
        if (lane >= off) w += y;
      }
      if (lane < SCAN_TB / 64) s_wave[lane] = w;
    }
    __syncthreads();
    const int carry = s_carry;
    const int excl = carry + (wid > 0 ? s_wave[wid - 1] : 0) + x - v;
    if (e < total_entries) tile_off[k * ntiles_alloc + t] = excl;
    __syncthreads();
    if (threadIdx.x == SCAN_TB - 1) s_carry = excl + v;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total_out) *total_out = s_carry;
}

// Stable compaction (and, on iter 2, the stable sort by materialIdHit).
// The next bounce's intersect-stage hand-off, moved with the survivors by k_scatter: walking rays get their
// geoms record at the new slot and a candidate-list entry (stable: tile order, offsets from k_scan), the
// others their final hit record.
struct ScatterPrep {
  int on;
  const int2* prep;
  float4* cray;
  int2* hits;
  int* cand;
  const int* tile_coff;
};

template <bool SORT>
__global__ __launch_bounds__(TILE) void k_scatter(PathBuf src, PathBuf dst, const int* __restrict__ tile_off,
                                                  const int* counts, int depth, int ntiles_alloc, int compact,
                                                  ScatterPrep P) {
  const int n = counts[depth];
  const int tile = blockIdx.x;
  if (tile * TILE >= n) return;
  const int i = tile * TILE + threadIdx.x;
  const bool valid = i < n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float4 q0, q1, q2;
  int pm = 0;
  bool alive = false;
  if (valid) {
    q0 = src.p0[i];
    q1 = src.p1[i];
    q2 = src.p2[i];
    pm = src.pm[i];
    alive = compact ? (fbits(q2.w) != 0) : true;
  }
  int dst_i;
  if (!SORT) {
    __shared__ int s_wave[TILE / 64];
    const unsigned long long m = __ballot(alive);
    if (lane == 0) s_wave[wid] = __popcll(m);
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wid; w++) before += s_wave[w];
    dst_i = tile_off[tile] + before + (int)lane_prefix(m);
  } else {
    __shared__ int s_key[TILE];
    s_key[threadIdx.x] = alive ? pm : -0x7fffffff;
    __syncthreads();
    int r = 0;
    for (int j = 0; j < (int)threadIdx.x; j++) r += (s_key[j] == pm);
    dst_i = tile_off[pm * ntiles_alloc + tile] + r;
  }
  if (alive) {
    dst.p0[dst_i] = q0;
    dst.p1[dst_i] = q1;
    dst.p2[dst_i] = q2;
    dst.pm[dst_i] = pm;
  }
  if (P.on) {
    __shared__ int s_walk[TILE / 64];
    const int2 pr = alive ? P.prep[i] : make_int2(0, 0);
    const bool w = alive && (pr.y & 0x10000);
    const int geom = (pr.y & 0xffff) - 1;
    const unsigned long long m = __ballot(w);
    if (lane == 0) s_walk[wid] = __popcll(m);
    __syncthreads();
    if (alive) {
      if (w) {
        int before = 0;
        for (int k = 0; k < wid; k++) before += s_walk[k];
        const int slot = P.tile_coff[tile] + before + (int)lane_prefix(m);
        P.cand[slot] = dst_i;
        P.cray[2 * slot] = make_float4(q0.x, q0.y, q0.z, u2f((uint32_t)pr.x));
        P.cray[2 * slot + 1] = make_float4(q1.x, q1.y, q1.z, ibits(geom));
      } else {
        P.hits[dst_i] = make_int2(geom, -1);  // final: the analytic geoms' hit (code -1: none)
      }
    }
  }
}

// finalGather (src/pathtrace.cu:2373-2383), including index = paths[index].pixelIndex
__global__ void k_final_gather(PathBuf paths, const int* counts, int depth, float* image) {
  const int n = counts[depth];
  const int index = blockIdx.x * blockDim.x + threadIdx.x;
  if (index >= n) return;
  const int j = fbits(paths.p1[index].w) & 0x7fffffff;
  const float4 c = paths.p2[j];
  const int pix = fbits(paths.p1[j].w) & 0x7fffffff;
  image[3 * (size_t)pix + 0] += c.x;
  image[3 * (size_t)pix + 1] += c.y;
  image[3 * (size_t)pix + 2] += c.z;
}

// sendImageToPBO (src/pathtrace.cu:69-89)
__global__ void k_pbo(const float* image, int npix, int iter, uchar4* pbo) {
  const int index = blockIdx.x * blockDim.x + threadIdx.x;
  if (index >= npix) return;
  int c[3];
  for (int k = 0; k < 3; k++) {
    int v = (int)((double)(image[3 * (size_t)index + k] / iter) * 255.0);
    c[k] = v < 0 ? 0 : (v > 255 ? 255 : v);
  }
  pbo[index] = make_uchar4((unsigned char)c[0], (unsigned char)c[1], (unsigned char)c[2], 0);
}

// saveImage (src/main.cpp:1087-1108): x-flip and divide by the sample count, then image::savePNG's
// bytes (src/image.cpp:22-35): glm::clamp(pix, 0, 1) * 255.f truncated to unsigned char.  `lin`
// (optional) receives the flipped, divided float image that image::saveHDR writes.
__global__ void k_save_image(const float* __restrict__ image, int W, int H, float samples, uint8_t* __restrict__ rgb,
                             float* __restrict__ lin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  const int y = i / W, X = i - y * W;
  const size_t src = 3 * ((size_t)(W - 1 - X) + (size_t)y * W);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float v = image[src + k] / samples;
    if (lin) lin[3 * (size_t)i + k] = v;
    const float cl = glm_min(glm_max(v, 0.0f), 1.0f) * 255.f;
    rgb[3 * (size_t)i + k] = (uint8_t)cl;
  }
}

// debug: unpack the live path array into the reference PathSegment layout
__global__ void k_unpack(PathBuf src, const int* counts, int depth, kdpt_path_segment* out) {
  const int n = counts[depth];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 q0 = src.p0[i], q1 = src.p1[i], q2 = src.p2[i];
  kdpt_path_segment s;
  s.origin[0] = q0.x; s.origin[1] = q0.y; s.origin[2] = q0.z;
  s.direction[0] = q1.x; s.direction[1] = q1.y; s.direction[2] = q1.z;
  const int pw = fbits(q1.w);
  s.isinside = (uint8_t)((pw >> 31) & 1);
  s.pad_[0] = s.pad_[1] = s.pad_[2] = 0;
  s.sdepth = q0.w;
  s.color[0] = q2.x; s.color[1] = q2.y; s.color[2] = q2.z;
  s.pixelIndex = pw & 0x7fffffff;
  s.remainingBounces = fbits(q2.w);
  s.materialIdHit = src.pm[i];
  out[i] = s;
}

__global__ void k_selftest_math(const float* x, int n, float* so, float* co) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { so[i] = kdpt_sinf(x[i]); co[i] = kdpt_cosf(x[i]); }
}
// glibc acosf / sin / cos restatements (kdpt_math.h): fn 0 acosf(x), 1 sin((double)x), 2 cos((double)x)
__device__ inline uint64_t libm_bits(int fn, float x) {
  if (fn == 0) return f2u(kdpt_acosf(x));
  return d2u(fn == 1 ? kdpt_sin((double)x) : kdpt_cos((double)x));
}
__device__ inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ void k_selftest_libm(int fn, const float* x, int n, double* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t b = libm_bits(fn, x[i]);
  out[i] = fn == 0 ? (double)u2f((uint32_t)b) : u2d(b);
}
__global__ void k_selftest_libm_digest(int fn, uint32_t first, uint64_t count, unsigned long long* acc) {
  uint64_t sum = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += stride) {
    const uint32_t xb = (uint32_t)(first + k);
    sum += splitmix64(libm_bits(fn, u2f(xb)) ^ splitmix64(xb));
  }
  atomicAdd(acc, (unsigned long long)sum);
}
__global__ void k_selftest_rng(const int* iid, int n, int k, float* u) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rng r = seeded_rng(iid[3 * i], iid[3 * i + 1], iid[3 * i + 2]);
  float v = 0;
  for (int j = 0; j <= k; j++) v = u01(r);
  u[i] = v;
}
__global__ void k_selftest_rng_draws(int mode, const uint32_t* in, int n, int k, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rng r = mode == 0 ? seeded_rng((int)in[3 * i], (int)in[3 * i + 1], (int)in[3 * i + 2])
        : mode == 1 ? rng_seed(utilhash(in[i])) : rng_seed(in[i]);
  for (int j = 0; j < k; j++) out[(size_t)i * k + j] = u01(r);
}
__global__ void k_selftest_glm(int fn, const float* in, int n, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  glm_kat(fn, in + (size_t)glm_kat_inputs(fn) * i, out + (size_t)glm_kat_outputs(fn) * i);
}
__global__ void k_selftest_fresnel(const float* c, int n, float R0, float* f) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // getFresnelVal with dot(N,-I) == c[i]: F = R0 + (1-R0) * pow(1 - c, 5)
  double F = (double)R0 + (double)(1.0f - R0) * pow5((double)(1.0f - c[i]));
  f[i] = (float)F;
}

}  // namespace

// ---------------------------------------------------------------------------
// Context
// ---------------------------------------------------------------------------
struct kdpt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool owns_stream = true;  // false: a pipeline group member, running on its group leader's stream
  kdpt_options opt{};
  kdpt_camera cam{};
  int traceDepth = 0;
  int W = 0, H = 0, npix = 0, ntiles = 0, nkeys = 1;
  int cap = 8;
  DevScene S{};
  // owned device memory
  std::vector<void*> allocs;
  uchar4* pbo_staging = nullptr;  // kdpt_write_pbo into host memory
  PathBuf buf[2]{};
  int cur = 0;
  float* image = nullptr;
  bool image_external = false;
  int* counts = nullptr;  // [cap + 2] live paths per bounce, [cap + 2] fault flag, then [cap] work counters
  int* work = nullptr;
  int2* hits = nullptr;   // [npix] hit code + objMaterialIdx from the intersect kernel
  float4* cray = nullptr;   // [2 npix] the candidates' rays in queue order (k_geoms / shading -> k_trace)
  int* cand = nullptr;      // [npix] paths whose ray meets the KD root box (k_geoms -> k_trace)
  int2* prep = nullptr;     // [npix] next bounce's geoms record + walk flag (k_shade -> k_scatter)
  int* tile_ccounts = nullptr;  // [ntiles] walking survivors per tile, and their offsets
  int* tile_coff = nullptr;
  int* ccount = nullptr;    // [cap] their number per bounce (inside the counts allocation)
  int* tickets = nullptr;   // [cap] k_shade_fused's tile tickets (inside the counts allocation)
  unsigned long long* lb = nullptr;  // [cap][ntiles] k_shade_fused's look-back records
  int tree_mode = 0;      // TreeMode
  int trace_grid = 0;     // persistent intersect workgroups
  int full_trace_grid = 0;  // the occupancy-derived grid (trace_grid before a "trace_grid_frac" knob)
  bool grid_env = false;  // trace_grid fixed by the "trace_grid_frac" tuning knob
  bool force_global_tree = false;  // "tree_global" tuning knob: keep the tree in HBM/L2
  bool super_cull = true;          // "super_cull" tuning knob: 0 = no TREE_LDS16S route (one-level cull)
  CullMargin cull{};                // the scene's cluster-cull margins (kdpt_clusters.h cluster_margin)
  // the exact one-level cull's direction masks (kdpt_clusters.h build_dir_masks), built when the scene's rigorous
  // margin is above the cap; S.cl_mask points at them unless a knob chose another cull
  unsigned long long* mask_dev = nullptr;
  float4* tn_dev = nullptr;  // the clusters' per-entry normal records (DevScene::cl_tn)
  int mask_n = 0;
  bool cull_exact = true;   // "cull_exact" knob: 0 = the fast-margin cull (not exact for such scenes)
  double create_ms = 0, mask_build_ms = 0;  // kdpt_create's host wall time, and the masks' (kdpt_stats)
  bool cu_mask_streams = false;  // batch and reduce streams created with an all-CU mask (create_stream)
  bool cull_scene = true;   // false after "cluster_cull" = 0 or a fixed "cull_margin"
  std::unique_ptr<ClusterSet> mask_cs;  // the clusters the masks were built from ("cull_mask_n" rebuilds)
  int tree_format = 0;             // "tree_format" knob: 16 / 32 = LDS node records of that size only
  size_t tree_lds = 0;    // dynamic LDS bytes of the intersect kernel (TREE_LDS)
  int* tile_counts = nullptr;
  int* tile_off = nullptr;
  int* tile_kcounts = nullptr;  // trace-order class counts per tile [TRACE_KEYS][ntiles]
  int* tile_koff = nullptr;
  int* perm = nullptr;          // trace order of the next bounce
  bool trace_order = true;      // KDPT_TRACE_ORDER=0 disables (identity order)
  bool no_fuse = false;         // "shade_fused" = 0: k_shade + k_scan + k_scatter instead of k_shade_fused
  bool shade_batch = true;      // "shade_batch": a batch's fused shading in one launch (k_shade_fused_b)
  bool gen_geoms = true;        // "gen_geoms": camera rays + bounce-0 k_geoms in one launch (k_gen_geoms_b)
  int* ccount0 = nullptr;       // [2] bounce-0 candidate counters of k_gen_geoms_b (alternating uses)
  int gen_parity = 0;           // which of them the next use counts into
  int* cc0_cur = nullptr;       // this use's (bounce 0 reads it instead of ccount[0])
  bool zero_partial = false;    // k_gen_rays zeroes `image` (a pipeline slot's per-iteration partial image)
  int chunk_width[3] = {16, 64, 64};
  Counters* counters = nullptr;
  Counters last_profile{};
  unsigned long long* total_segments = nullptr;  // device running total (async use)
  unsigned long long* trace_t = nullptr;         // per-bounce intersect launch record (per slot)
  unsigned long long* trace_total = nullptr;     // [3] device-clock intersect ticks, launches, rays (shared)
  double wall_khz = 100000.0;                    // s_memrealtime frequency
  int* h_counts = nullptr;  // pinned
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> bounce_ev;
  kdpt_stats stats{};
  bool count_mode = false;
  bool sync_debug = false;  // "sync_debug" = 1: synchronise and log after every launch
  // Pipelined iterations (kdpt_trace_iterations): extra slots, each a context sharing this one's
  // scene upload but owning its per-iteration buffers, stream and partial image; the partial
  // images are added into `image` in iteration order, each batch's add on the batch's own stream after the
  // previous batch's add (acc_ev / acc_last: the chain).
  kdpt_ctx* parent = nullptr;
  std::vector<kdpt_ctx*> slots;
  int slot_batch = 1;
  int next_group = 0;  // the slot group the next batch goes to
  bool profile_batches = false;
  bool profile_steps = false;  // "profile_batches" = 2
  std::vector<hipEvent_t> acc_ev;  // per slot group: its last batch's add into the target done
  hipEvent_t acc_last = nullptr;   // the most recent add (one of acc_ev): the next add follows it
  hipEvent_t img_last = nullptr;   // the most recent frame reduce + image add (one of frame_ev)
  // intersect-kernel timing (testing_mode) of every iteration, read back at synchronisation
  std::vector<std::vector<hipEvent_t>> pending_ev;  // per launched iteration: 2 events per bounce
  std::vector<hipEvent_t> free_ev;
  std::vector<hipEvent_t>* rec_ev = nullptr;  // when set, launch_iteration records the bounce events here
  double intersect_ms_total = 0;
  long long intersect_launches_total = 0;
  // enable_kd = 0: brute-force intersect kernel over the OBJ triangles in file order
  bool brute = false;
  bool viz = false;  // viz_kd: the KD node boxes drawn as boxes (k_viz)
  BruteShape* shapes = nullptr;
  int num_shapes = 0;
  float4* chunk_lo = nullptr;  // brute force: boxes of 64 file-order triangles
  float4* chunk_hi = nullptr;
  // spp-sharded frames (kdpt_comm_init / kdpt_render_frames / kdpt_render_sharded): this context's rank, the
  // RCCL communicator (null: one rank, or the in-process copy reduce of kdpt_render_sharded), two frame
  // buffers (frame f accumulates into frame_buf[f & 1] while f - 1 is reduced) and rank 0's reduced frame
  int nranks = 1, rank = 0;
  void* comm = nullptr;  // ncclComm_t
  bool owns_comm = false;
  bool external_reduce = false;  // kdpt_comm_init without an id: each rank hands its frame shares out
  float* frame_buf[2] = {nullptr, nullptr};
  float* frame_sum = nullptr;
  hipEvent_t frame_ev[2] = {nullptr, nullptr};      // frame_buf[k] consumed by its reduce
  hipStream_t reduce_stream = nullptr;  // the frames' reduces and image adds, beside the accumulation stream
  double reduce_spin_us = 0;  // "reduce_spin_us" knob: a device spin before every frame's reduce (a slow peer)
  std::vector<void*> host_reg;  // pageable host `out` ranges pinned for kdpt_render_frames (released at synchronize)
};

namespace {

// A context's streams (its own, the batch groups' and the frame reduce's): created with a mask of every CU, which
// gives each a hardware queue of its own instead of one of the GPU_MAX_HW_QUEUES (4 by default) in-order queues
// HIP multiplexes a process's plain streams onto -- where a waiting or long-running command of one stream holds
// the others on its queue.  C4's 32-spp frames: 6.49 -> 5.68 ms with 24 queues, and a 5 ms reduce delay per frame
// costs nothing at 4 or 24 queues (profiles/r06_ab_log.md).  Knob "cu_mask_streams" = 0 (process default):
// plain non-blocking streams; a failed creation falls back to one.
int create_stream(kdpt_ctx* c, hipStream_t* st) {
  if (c->cu_mask_streams) {
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c->device));
    const int n = std::max(1, prop.multiProcessorCount);
    std::vector<uint32_t> mask((n + 31) / 32, 0xffffffffu);
    if (n % 32) mask.back() = (1u << (n % 32)) - 1u;
    if (hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()) == hipSuccess) return KDPT_OK;
    (void)hipGetLastError();
  }
  HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
  return KDPT_OK;
}

template <typename T>
int dalloc(kdpt_ctx* c, T** p, size_t n) {
  void* q = nullptr;
  HIP_TRY(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)));
  c->allocs.push_back(q);
  *p = (T*)q;
  return KDPT_OK;
}

template <typename T>
int dupload(kdpt_ctx* c, T** p, const T* src, size_t n) {
  int rc = dalloc(c, p, n);
  if (rc) return rc;
  if (n) HIP_TRY(hipMemcpy(*p, src, n * sizeof(T), hipMemcpyHostToDevice));
  return KDPT_OK;
}

int launch_iteration(kdpt_ctx* c, int iter, int stop_depth, bool count);
void release_comm(kdpt_ctx* c);  // (multi-GPU section, end of file)
void unregister_host(kdpt_ctx* c);
int launch_batch(kdpt_ctx* const* cs, const int* iters, int nb, hipStream_t st, int stop_depth, bool count,
                 std::vector<hipEvent_t>* bev);

// Work queued on the context's own stream that reads or writes `image` must follow the pipelined
// accumulation (kdpt_trace_iterations adds partial images on the batch streams without a host sync) and the
// frames' image adds (kdpt_render_frames, on the reduce stream).
int join_accum(kdpt_ctx* c) {
  if (c->acc_last) HIP_TRY(hipStreamWaitEvent(c->stream, c->acc_last, 0));
  if (c->img_last) HIP_TRY(hipStreamWaitEvent(c->stream, c->img_last, 0));
  return KDPT_OK;
}


// stats.segments / seg_per_bounce / bounces of the iteration whose counts are in h_counts
int segments_from_counts(kdpt_ctx* c) {
  long long seg = 0;
  int bounces = 0;
  for (int d = 0; d < 32; d++) c->stats.seg_per_bounce[d] = 0;
  for (int d = 0; d < c->cap; d++) {
    const int nd = c->h_counts[d];
    if (d > 0 && c->h_counts[d] <= 0) break;  // the reference stops once num_paths <= 0
    seg += nd;
    if (d < 32) c->stats.seg_per_bounce[d] = nd;
    bounces = d + 1;
    if (c->opt.compaction && c->h_counts[d + 1] <= 0) break;
  }
  c->stats.segments = seg;
  c->stats.bounces = bounces;
  return bounces;
}

// Per-iteration device state: two path buffers, hit records, trace order, tile counts/offsets,
// live counts + fault word + work counters.  (The scene, image and counters live elsewhere.)
// The zero fills go on the context's own stream and are waited for: every kernel of the context runs on a
// non-blocking stream, which does not order itself after the null stream, so a plain hipMemset there could
// land after the first iteration's camera-ray kernel had set its path count (that iteration would vanish).
int alloc_iteration_buffers(kdpt_ctx* c) {
  int rc;
  for (int b = 0; b < 2; b++) {
    if ((rc = dalloc(c, &c->buf[b].p0, c->npix)) || (rc = dalloc(c, &c->buf[b].p1, c->npix)) ||
        (rc = dalloc(c, &c->buf[b].p2, c->npix)) || (rc = dalloc(c, &c->buf[b].pm, c->npix)))
      return rc;
    HIP_TRY(hipMemsetAsync(c->buf[b].pm, 0, sizeof(int) * c->npix, c->stream));
  }
  // counts[0..cap+1]: live paths per bounce (rewritten every iteration); counts[cap+2]: fault flag;
  // counts[cap+3 ..]: work counters of the persistent intersect kernel
  if ((rc = dalloc(c, &c->trace_t, 4 * (size_t)c->cap))) return rc;
  HIP_TRY(hipMemsetAsync(c->trace_t, 0, sizeof(unsigned long long) * 4 * c->cap, c->stream));
  if ((rc = dalloc(c, &c->counts, 4 * (size_t)c->cap + 5)) || (rc = dalloc(c, &c->lb, (size_t)c->cap * c->ntiles)) || (rc = dalloc(c, &c->hits, (size_t)c->npix)) ||
      (rc = dalloc(c, &c->cand, (size_t)c->npix)) || (rc = dalloc(c, &c->prep, (size_t)c->npix)) ||
      (rc = dalloc(c, &c->tile_ccounts, (size_t)c->ntiles)) || (rc = dalloc(c, &c->tile_coff, (size_t)c->ntiles)) ||
      (rc = dalloc(c, &c->cray, 2 * (size_t)c->npix)) ||
      (rc = dalloc(c, &c->perm, (size_t)c->npix)) ||
      (rc = dalloc(c, &c->tile_kcounts, (size_t)TRACE_KEYS * c->ntiles)) ||
      (rc = dalloc(c, &c->tile_koff, (size_t)TRACE_KEYS * c->ntiles)) ||
      (rc = dalloc(c, &c->tile_counts, (size_t)MAX_KEYS * c->ntiles)) ||
      (rc = dalloc(c, &c->tile_off, (size_t)MAX_KEYS * c->ntiles)))
    return rc;
  if (hipHostMalloc((void**)&c->h_counts, sizeof(int) * (c->cap + 3), hipHostMallocDefault) != hipSuccess)
    return fail(KDPT_ERR_HIP, "hipHostMalloc");
  HIP_TRY(hipMemsetAsync(c->counts, 0, sizeof(int) * (4 * c->cap + 5), c->stream));
  HIP_TRY(hipMemsetAsync(c->lb, 0, sizeof(unsigned long long) * c->cap * c->ntiles, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->S.fault = c->counts + c->cap + 2;
  c->work = c->counts + c->cap + 3;
  c->ccount = c->work + c->cap;
  c->tickets = c->ccount + c->cap;
  c->ccount0 = c->tickets + c->cap;  // 2 entries, zero
  c->gen_parity = 0;
  return KDPT_OK;
}

int alloc_iteration_events(kdpt_ctx* c) {
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  c->bounce_ev.resize(2 * (size_t)c->cap);
  for (auto& e : c->bounce_ev) HIP_TRY(hipEventCreate(&e));
  return KDPT_OK;
}

// A pipeline slot: shares p's scene upload and counters, owns its iteration buffers, its stream
// and a partial image that k_gen_rays' iteration accumulates into.
// Pipeline slots, members before their group leader (the leader owns the stream they share).
void destroy_slots(kdpt_ctx* c) {
  for (size_t k = c->slots.size(); k-- > 0;) kdpt_destroy(c->slots[k]);
}

// Drop the pipeline slots (their streams drained by the caller) and the add chain's events.
void drop_slots(kdpt_ctx* c) {
  destroy_slots(c);
  for (auto e : c->acc_ev) (void)hipEventDestroy(e);
  c->slots.clear();
  c->acc_ev.clear();
  c->acc_last = nullptr;
}

// share: the stream of the slot's group leader (a group's batches all run on the leader's stream), or null
// for a leader, which creates its own
int make_slot(kdpt_ctx* p, kdpt_ctx** out, hipStream_t share = nullptr) {
  kdpt_ctx* c = new kdpt_ctx();
  c->parent = p;
  c->device = p->device;
  c->opt = p->opt;
  c->opt.external_image = nullptr;
  c->cam = p->cam;
  c->traceDepth = p->traceDepth;
  c->W = p->W;
  c->H = p->H;
  c->npix = p->npix;
  c->ntiles = p->ntiles;
  c->nkeys = p->nkeys;
  c->cap = p->cap;
  c->S = p->S;
  c->tree_mode = p->tree_mode;
  c->trace_grid = p->trace_grid;
  c->tree_lds = p->tree_lds;
  c->trace_order = p->trace_order;
  c->no_fuse = p->no_fuse;
  c->shade_batch = p->shade_batch;
  c->gen_geoms = p->gen_geoms;
  for (int k = 0; k < 3; k++) c->chunk_width[k] = p->chunk_width[k];
  c->counters = p->counters;
  c->total_segments = p->total_segments;
  c->trace_total = p->trace_total;
  c->wall_khz = p->wall_khz;
  c->sync_debug = p->sync_debug;
  c->brute = p->brute;
  c->viz = p->viz;
  c->shapes = p->shapes;
  c->num_shapes = p->num_shapes;
  c->chunk_lo = p->chunk_lo;
  c->chunk_hi = p->chunk_hi;
  c->cu_mask_streams = p->cu_mask_streams;
  int rc;
  if (share) {
    c->stream = share;
    c->owns_stream = false;
  } else if (create_stream(c, &c->stream) != KDPT_OK) {
    kdpt_destroy(c);
    return fail(KDPT_ERR_HIP, "hipStreamCreate failed");
  }
  if ((rc = alloc_iteration_buffers(c)) || (rc = dalloc(c, &c->image, 3 * (size_t)c->npix)) ||
      (rc = alloc_iteration_events(c))) {
    kdpt_destroy(c);
    return rc;
  }
  *out = c;
  return KDPT_OK;
}

// A batch's partial images added in iteration order (one add per pixel and iteration, as partialGather
// does), with one read and one write of the accumulation image per batch instead of one per iteration.
struct PartialImages {
  const float* p[MAXB];
  int nb;
};
__global__ void k_accumulate_batch(float* __restrict__ image, PartialImages parts, int n3) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n3) return;
  float v = image[i];
  for (int b = 0; b < parts.nb; b++) v += parts.p[b][i];
  image[i] = v;
}

// Read back the intersect-kernel events of finished iterations (testing_mode).
int drain_intersect_events(kdpt_ctx* c) {
  for (auto& evs : c->pending_ev) {
    for (size_t k = 0; k + 1 < evs.size(); k += 2) {
      float ms = 0;
      HIP_TRY(hipEventSynchronize(evs[k + 1]));
      if (hipEventElapsedTime(&ms, evs[k], evs[k + 1]) == hipSuccess) {
        c->intersect_ms_total += ms;
        c->intersect_launches_total++;
      }
    }
    for (auto e : evs) c->free_ev.push_back(e);
  }
  c->pending_ev.clear();
  return KDPT_OK;
}

// The scene's cull margins (kdpt_clusters.h cluster_margin) into the context and its DevScene; fixed: one
// direction-free coefficient for every level (tuning "cull_margin" / "cluster_cull" = 0, which passes inf).
void set_cull(kdpt_ctx* c, const CullMargin& cm) {
  c->cull = cm;
  c->S.cl_margin = cm.K;
  c->S.cl_margin_lo = cm.K_lo;
  c->S.cull_a = cm.a;
  c->S.cull_b = cm.b;
  c->S.cull_c = cm.c;
}
void fix_cull(kdpt_ctx* c, float K) {
  c->S.cl_margin = c->S.cl_margin_lo = K;
}
// The one-level route's cull: the exact masked one when the scene has masks and the knobs leave the scene's
// margins in place, else the margin-only cull.
void apply_cull_route(kdpt_ctx* c) {
  c->S.cl_mask = (c->mask_dev && c->cull_exact && c->cull_scene) ? c->mask_dev : nullptr;
  c->S.mask_n = c->mask_n;
  c->S.cl_tn = c->tn_dev;
}
// The masked cull's cells on the device (kdpt_device.h dir_mask_cell, the code the host builder runs): one
// workgroup per (cluster, 256 buckets), the cluster's 64 entries staged in LDS (every lane reads the same entry:
// a broadcast), one mask per lane, written bucket-major.
__global__ void __launch_bounds__(256) k_build_masks(const double* __restrict__ ent, const float* __restrict__ krig,
                                                     const double* __restrict__ bd, int ncl, int nb, float Kf,
                                                     unsigned long long* __restrict__ masks) {
  __shared__ double se[5][64];
  __shared__ float sk[64];
  const int c = blockIdx.x;
  const size_t ne = 64 * (size_t)ncl;
  if (threadIdx.x < 64) {
    for (int f = 0; f < 5; f++) se[f][threadIdx.x] = ent[f * ne + 64 * (size_t)c + threadIdx.x];
    sk[threadIdx.x] = krig[64 * (size_t)c + threadIdx.x];
  }
  __syncthreads();
  const int b = blockIdx.y * 256 + threadIdx.x;
  if (b >= nb) return;
  masks[(size_t)b * ncl + c] = dir_mask_cell(se[0], se[1], se[2], se[3], se[4], sk, bd + 4 * (size_t)b, Kf);
}

// Release one of the context's device allocations before kdpt_destroy (a rebuilt table).
void dfree(kdpt_ctx* c, void* p) {
  if (!p) return;
  auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
  if (it != c->allocs.end()) c->allocs.erase(it);
  (void)hipFree(p);
}

// The direction masks of the scene's clusters at resolution n (cube-map cells per face edge), built on the device (k_build_masks) from the per-entry records and the bucket directions the host
// computes (kdpt_clusters.h mask_entries / mask_buckets; tests/test_gpu_parity.py checks the cells against the
// host builder).  A rebuild (knobs "cull_mask_n", "cull_fast_k") frees the previous tables.
int build_masks(kdpt_ctx* c, int n) {
  const auto t0 = std::chrono::steady_clock::now();
  const ClusterSet& cs = *c->mask_cs;
  const int ncl = (int)cs.info.size(), nb = 6 * n * n;
  const float Kf = c->cull.K;
  MaskEntries me;
  mask_entries(cs, Kf, me);
  std::vector<double> bd;
  mask_buckets(n, bd);
  const size_t ne = 64 * (size_t)ncl;
  std::vector<double> ent(5 * ne);
  for (size_t k = 0; k < ne; k++) {
    ent[k] = me.nx[k];
    ent[ne + k] = me.ny[k];
    ent[2 * ne + k] = me.nz[k];
    ent[3 * ne + k] = me.beta[k];
    ent[4 * ne + k] = me.dthr[k];
  }
  dfree(c, c->mask_dev);
  c->mask_dev = nullptr;
  c->S.cl_mask = nullptr;
  unsigned long long* dm = nullptr;
  int rc;
  if ((rc = dalloc(c, &dm, (size_t)nb * ncl))) return rc;
  c->mask_dev = dm;
  double* d_ent = nullptr;
  float* d_krig = nullptr;
  double* d_bd = nullptr;
  auto release = [&]() {
    (void)hipFree(d_ent);
    (void)hipFree(d_krig);
    (void)hipFree(d_bd);
  };
  // (the uploads on the context's stream, ahead of the kernel; pageable sources are staged before each call
  // returns, and the stream is drained before the temporaries go)
  if (hipMalloc(&d_ent, ent.size() * sizeof(double)) != hipSuccess ||
      hipMalloc(&d_krig, me.krig.size() * sizeof(float)) != hipSuccess ||
      hipMalloc(&d_bd, bd.size() * sizeof(double)) != hipSuccess ||
      hipMemcpyAsync(d_ent, ent.data(), ent.size() * sizeof(double), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(d_krig, me.krig.data(), me.krig.size() * sizeof(float), hipMemcpyHostToDevice, c->stream) !=
          hipSuccess ||
      hipMemcpyAsync(d_bd, bd.data(), bd.size() * sizeof(double), hipMemcpyHostToDevice, c->stream) != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    release();
    return fail(KDPT_ERR_HIP, "mask build: device buffers");
  }
  hipLaunchKernelGGL(k_build_masks, dim3(ncl, (nb + 255) / 256), dim3(256), 0, c->stream, d_ent, d_krig, d_bd, ncl,
                     nb, Kf, dm);
  const hipError_t e1 = hipGetLastError(), e2 = hipStreamSynchronize(c->stream);
  release();
  if (e1 != hipSuccess || e2 != hipSuccess) return fail(KDPT_ERR_HIP, "k_build_masks failed");
  if (!c->tn_dev) {
    std::vector<float4> tn;
    build_entry_normals(cs, tn);
    if ((rc = dupload(c, &c->tn_dev, tn.data(), tn.size()))) return rc;
  }
  c->mask_n = n;
  c->mask_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  apply_cull_route(c);
  return KDPT_OK;
}

// Big leaves as clusters of <= 64 triangles, super-clusters and slabs (kdpt_clusters.h), uploaded.
int build_clusters(kdpt_ctx* c, const kdpt_scene* sc, const std::vector<float4>& tv, const std::vector<float4>& e1,
                   const std::vector<float4>& e2, std::vector<int2>& leaf_cl, std::vector<int2>& leaf_sp) {
  ClusterSet cs;
  build_cluster_set(sc->nodes, sc->num_nodes, sc->tris, tv, e1, e2, cs);
  // Meshes of small triangles (a rigorous margin: the two-level cull of the C5 icosphere) group each big leaf's
  // triangles into normal cones of chord CLUSTER_CHORD_EXACT first, then Morton runs per cone: flatter clusters
  // whose oriented boxes the lines miss more often -- C5's sweeps per ray 1.83 -> 1.30 (host simulation), C5
  // 4 568 / 4 377 -> 5 110 / 5 087 Mrays/s (profiles/r06_ab_log.md).  Only the order of a leaf's sweeps changes
  // (the results fold order-free); such leaves hold more clusters than ceil(size / 64) (S.cl_counts).  Not for meshes of large triangles: dragon_5's leaves split into 4-8x as many
  // clusters.  Kept only while the super-clusters grow by at most 40 % (they must fit the LDS route); knob
  // "cluster_chord" (process default): 0 = Morton runs only, > 0 = that chord for every mesh.
  {
    const double chord = g_cluster_chord >= 0 ? g_cluster_chord
                                             : (cluster_margin(cs.cv0, cs.ce1, cs.ce2).exact ? CLUSTER_CHORD_EXACT : 0.0);
    if (chord > 0 && !cs.info.empty()) {
      ClusterGrouping g;
      g.mode = 1;
      g.chord = chord;
      ClusterSet cones;
      build_cluster_set(sc->nodes, sc->num_nodes, sc->tris, tv, e1, e2, cones, g);
      if (g_cluster_chord > 0 || cones.sup.size() * 10 <= cs.sup.size() * 14) cs = std::move(cones);
    }
  }
  leaf_cl = cs.leaf_cl;
  leaf_sp = cs.leaf_sp;
  const std::vector<int4>& sp = cs.sup;
  const std::vector<float4>&lo = cs.lo, &hi = cs.hi, &nrm = cs.nrm, &cv0 = cs.cv0, &ce1 = cs.ce1, &ce2 = cs.ce2;
  const std::vector<int2>& info = cs.info;
  int2 *dl, *di;
  float4 *dlo, *dhi, *dv0, *de1, *de2;
  int rc;
  if ((rc = dupload(c, &dl, leaf_cl.data(), leaf_cl.size())) || (rc = dupload(c, &di, info.data(), info.size())) ||
      (rc = dupload(c, &dlo, lo.data(), lo.size())) || (rc = dupload(c, &dhi, hi.data(), hi.size())) ||
      (rc = dupload(c, &dv0, cv0.data(), cv0.size())) || (rc = dupload(c, &de1, ce1.data(), ce1.size())) ||
      (rc = dupload(c, &de2, ce2.data(), ce2.size())))
    return rc;
  int4* dsp;
  float4 *dn, *du, *dv, *dw;
  if ((rc = dupload(c, &dsp, sp.data(), sp.size())) || (rc = dupload(c, &dn, nrm.data(), nrm.size())) ||
      (rc = dupload(c, &du, cs.obb_u.data(), cs.obb_u.size())) ||
      (rc = dupload(c, &dv, cs.obb_v.data(), cs.obb_v.size())) ||
      (rc = dupload(c, &dw, cs.obb_w.data(), cs.obb_w.size())))
    return rc;
  c->S.cl_n = dn;
  c->S.cl_slab = 1;
  c->S.cl_u = du;
  c->S.cl_v = dv;
  c->S.cl_w = dw;
  c->S.cl_obb = 1;
  c->S.flat_obb = 1;
  float4 *dsn, *dsb;
  if ((rc = dupload(c, &dsn, cs.sup_n.data(), cs.sup_n.size())) || (rc = dupload(c, &dsb, cs.sup_b.data(), cs.sup_b.size())))
    return rc;
  c->S.sup_n = dsn;
  c->S.sup_b = dsb;
  c->S.sup_slab = 1;
  set_cull(c, cluster_margin(cv0, ce1, ce2));
  // no margin makes the cull exact for these triangles: the masked one-level cull (its direction masks for the
  // fast margin the box levels use)
  if (!c->cull.exact && !info.empty()) {
    c->mask_cs.reset(new ClusterSet(cs));
    if ((rc = build_masks(c, dir_mask_resolution((int)info.size())))) return rc;
  }
  c->S.sup = dsp;
  // a super box past the half range (+-65504) would be infinite, its centre NaN and the cull wrong: such a
  // scene gets no super-cluster route (TREE_LDS16S needs num_supers > 0)
  c->S.num_supers = cs.supers_finite ? (int)sp.size() : 0;
  c->S.leaf_cl = dl;
  c->S.num_clusters = (int)info.size();
  c->S.cl_counts = 0;
  for (int i = 0; i < sc->num_nodes; i++)
    if (leaf_cl[i].y != 0 && leaf_cl[i].y != (sc->nodes[i].triIdSize + CLUSTER - 1) / CLUSTER) c->S.cl_counts = 1;
  c->S.cl_info = di;
  c->S.cl_lo = dlo;
  c->S.cl_hi = dhi;
  c->S.c_v0 = dv0;
  c->S.c_e1 = de1;
  c->S.c_e2 = de2;
  return KDPT_OK;
}

// NodesPacked records (kdpt_device.h); false when the tree does not fit the format.
bool pack_nodes(const kdpt_node_bare* N, int nn, const std::vector<int2>& leaf_cl, std::vector<int4>& out) {
  if (nn >= 0xffff) return false;
  out.assign(2 * (size_t)nn, make_int4(0, 0, 0, 0));
  auto l16 = [](int v) { return v == -1 ? 0xffffu : (uint32_t)v; };
  for (int i = 0; i < nn; i++) {
    const kdpt_node_bare& n = N[i];
    const bool tris = n.triIdSize > 0;
    if (tris && (n.leftID != -1 || n.rightID != -1 || n.triIdSize >= (1 << 13))) return false;
    const uint32_t axis = n.axis == 0 ? 0u : (n.axis == 1 ? 1u : 2u);  // comp(): anything else reads z
    // a big leaf keeps its first cluster instead of its first triangle (its clusters carry the triangles)
    const uint32_t first = n.triIdSize >= BIG_LEAF ? (uint32_t)leaf_cl[i].x : (uint32_t)n.triIdStart;
    const uint32_t w6 = tris ? first : (l16(n.leftID) | (l16(n.rightID) << 16));
    const uint32_t kids = (n.leftID != -1 ? 1u : 0u) | (n.rightID != -1 ? 2u : 0u);
    const uint32_t w7 = l16(n.parentID) | (axis << 16) | ((tris ? 1u : 0u) << 18) |
                        ((tris ? (uint32_t)n.triIdSize : kids) << 19);
    out[2 * i] = make_int4(fbits(n.mins[0]), fbits(n.mins[1]), fbits(n.mins[2]), fbits(n.maxs[0]));
    out[2 * i + 1] = make_int4(fbits(n.maxs[1]), fbits(n.maxs[2]), (int)w6, (int)w7);
  }
  return true;
}

// NodesDerived records (kdpt_device.h); false unless every node's box is its parent's with exactly the one
// coordinate the reference's split replaces (checked bit for bit), both children write the same centre, and
// the tree fits the 16-bit links.
bool pack_nodes16(const kdpt_node_bare* N, int nn, const std::vector<int2>& leaf_cl, std::vector<int4>& out) {
  if (nn < 1 || nn >= 0xffff || N[0].parentID != -1) return false;
  out.assign((size_t)nn, make_int4(0, 0, 0, 0));
  auto l16 = [](int v) { return v == -1 ? 0xffffu : (uint32_t)v; };
  auto same = [](float a, float b) { return fbits(a) == fbits(b); };
  for (int i = 0; i < nn; i++) {
    const kdpt_node_bare& n = N[i];
    const bool tris = n.triIdSize > 0;
    if (tris && (n.leftID != -1 || n.rightID != -1)) return false;
    if (n.axis < 0 || n.axis > 2) return false;
    for (int ch : {n.leftID, n.rightID})
      if (ch != -1 && (ch <= 0 || ch >= nn || N[ch].parentID != i)) return false;
    uint32_t kc = 7u;
    float restore = 0.0f;
    if (i > 0) {
      const int p = n.parentID;
      if (p < 0 || p >= nn) return false;
      const kdpt_node_bare& P = N[p];
      const bool isL = P.leftID == i, isR = P.rightID == i;
      if (isL == isR) return false;
      const int a = P.axis;
      for (int k = 0; k < 3; k++) {
        if (!(k == a && isR) && !same(n.mins[k], P.mins[k])) return false;
        if (!(k == a && isL) && !same(n.maxs[k], P.maxs[k])) return false;
      }
      kc = isR ? (uint32_t)a : 3u + (uint32_t)a;
      restore = isR ? P.mins[a] : P.maxs[a];
    }
    float center = 0.0f;
    if (n.leftID != -1) center = N[n.leftID].maxs[n.axis];
    if (n.rightID != -1) {
      if (n.leftID != -1 && !same(center, N[n.rightID].mins[n.axis])) return false;
      center = N[n.rightID].mins[n.axis];
    }
    const uint32_t first = n.triIdSize >= BIG_LEAF ? (uint32_t)leaf_cl[i].x : (uint32_t)n.triIdStart;
    const uint32_t w1 = tris ? first : fbits(center);
    const uint32_t w2 = tris ? (uint32_t)n.triIdSize : (l16(n.leftID) | (l16(n.rightID) << 16));
    const uint32_t kids = (n.leftID != -1 ? 1u : 0u) | (n.rightID != -1 ? 2u : 0u);
    const uint32_t w3 = l16(n.parentID) | ((uint32_t)n.axis << 16) | ((tris ? 1u : 0u) << 18) |
                        ((tris ? 0u : kids) << 19) | (kc << 21);
    out[i] = make_int4(fbits(restore), (int)w1, (int)w2, (int)w3);
  }
  return true;
}

template <bool HYBRID, bool COUNT, int MODE>
int trace_occupancy(kdpt_ctx* c, size_t lds, int* blocks) {
  if (lds > 0)
    HIP_TRY(hipFuncSetAttribute((const void*)k_trace<HYBRID, COUNT, MODE>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, k_trace<HYBRID, COUNT, MODE>, trace_block<MODE>(), lds));
  return KDPT_OK;
}

template <int MODE>
int trace_occupancy_all(kdpt_ctx* c, size_t lds, int* blocks) {
  int best = 0, rc = KDPT_OK;
  for (int hyb = 0; hyb < 2 && !rc; hyb++)
    for (int cnt = 0; cnt < 2 && !rc; cnt++) {
      int b = 0;
      rc = hyb ? (cnt ? trace_occupancy<true, true, MODE>(c, lds, &b) : trace_occupancy<true, false, MODE>(c, lds, &b))
               : (cnt ? trace_occupancy<false, true, MODE>(c, lds, &b) : trace_occupancy<false, false, MODE>(c, lds, &b));
      if (!rc && (best == 0 || b < best)) best = b;
    }
  *blocks = best;
  return rc;
}

// Pick where the intersect kernel reads the tree from, and its persistent grid: in LDS when it fits (the
// "tree_format" knob limits the LDS records to one size) -- the candidate that keeps the most intersect waves
// on a CU wins, ties in the order below.
int setup_trace(kdpt_ctx* c) {
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, c->device));
  const size_t lds_max = prop.sharedMemPerBlock > 0 ? prop.sharedMemPerBlock : 65536;
  // (the counting kernel's per-wave WaveProf too: the tree must fit next to either kernel's static part)
  const size_t per_wave = sizeof(WaveLeafLDS) + sizeof(WaveProf);
  const size_t cl_bytes = 32 * (size_t)c->S.num_clusters;
  struct Cand { int mode; size_t lds; };
  std::vector<Cand> cands;
  // (in order of preference at equal occupancy: the 32-byte records need no box bookkeeping on the walk, which
  // costs the derived form 6 % on dragon_5; the derived form is what fits the C5 icosphere's tree)
  if (!c->force_global_tree) {
    if (c->S.pnodes && c->tree_format != 16) {
      const size_t t32 = 32 * (size_t)c->S.num_nodes + cl_bytes, st32 = per_wave * (TRACE_BLOCK / 64);
      if (st32 + t32 <= lds_max) cands.push_back({TREE_LDS, t32});
    }
    if (c->S.dnodes && c->tree_format != 32) {
      const size_t t16 = 16 * (size_t)c->S.num_nodes, st16 = per_wave * (TRACE_BLOCK16 / 64);
      if (st16 + t16 + cl_bytes <= lds_max) cands.push_back({TREE_LDS16, t16 + cl_bytes});
      // (leaving room for a fused-shading workgroup's LDS beside the intersect workgroup)
      const size_t sp_bytes = 16 * (size_t)c->S.num_supers;
      // (not when the one-level cull is the masked exact one: the supers' margins are not rigorous for it)
      if (c->S.snodes && c->super_cull && !c->S.cl_mask && st16 + t16 + sp_bytes + SHADE_LDS_RESERVE <= lds_max)
        cands.push_back({TREE_LDS16S, t16 + sp_bytes});
      if (st16 + t16 <= lds_max) cands.push_back({TREE_LDS16G, t16});
    }
  }
  c->tree_mode = c->S.pnodes ? TREE_PACKED : TREE_WIDE;
  c->tree_lds = 0;
  int blocks = 0, best_waves = 0, rc = KDPT_OK;
  for (const Cand& k : cands) {
    int b = 0;
    rc = k.mode == TREE_LDS16 ? trace_occupancy_all<TREE_LDS16>(c, k.lds, &b)
       : k.mode == TREE_LDS16G ? trace_occupancy_all<TREE_LDS16G>(c, k.lds, &b)
       : k.mode == TREE_LDS16S ? trace_occupancy_all<TREE_LDS16S>(c, k.lds, &b)
                                : trace_occupancy_all<TREE_LDS>(c, k.lds, &b);
    if (rc) return rc;
    const int waves = b * (k.mode == TREE_LDS ? TRACE_BLOCK : TRACE_BLOCK16) / 64;
    if (b > 0 && waves > best_waves) {
      best_waves = waves;
      blocks = b;
      c->tree_mode = k.mode;
      c->tree_lds = k.lds;
    }
  }
  if (c->tree_lds == 0) {
    rc = c->tree_mode == TREE_PACKED ? trace_occupancy_all<TREE_PACKED>(c, 0, &blocks)
                                     : trace_occupancy_all<TREE_WIDE>(c, 0, &blocks);
    if (rc) return rc;
  }
  if (blocks < 1) return fail(KDPT_ERR_UNSUPPORTED, "intersect kernel does not fit on a CU");
  c->trace_grid = blocks * prop.multiProcessorCount;
  c->full_trace_grid = c->trace_grid;
  return KDPT_OK;
}

// A ray that needs more node steps than any valid tree allows sets the fault word and stops;
// the iteration then reports an error instead of returning a silently wrong image.
int fault_error(kdpt_ctx* c, int code) {
  (void)hipMemsetAsync(c->counts + c->cap + 2, 0, sizeof(int), c->stream);
  (void)hipStreamSynchronize(c->stream);
  if (code & 32)
    return fail(KDPT_ERR_HIP, "shading: a path's survival differed from its hit record's prediction, code " +
                                  std::to_string(code));
  return fail(KDPT_ERR_HIP, "KD traversal exceeded its step bound (inconsistent tree), code " + std::to_string(code));
}

int check_fault(kdpt_ctx* c) {
  int f = 0;
  HIP_TRY(hipMemcpy(&f, c->counts + c->cap + 2, sizeof(int), hipMemcpyDeviceToHost));
  return f ? fault_error(c, f) : KDPT_OK;
}

}  // namespace

#ifdef KDPT_TAIL_PROF
extern "C" int kdpt_debug_tail_prof(unsigned long long* out) {  // sums, then zeroes, the counters
  const unsigned long long zero[4] = {0, 0, 0, 0};
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_prof), sizeof(zero)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tail_prof), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef KDPT_SHADE_PROF
extern "C" int kdpt_debug_shade_prof(unsigned long long* out) {  // sums, then zeroes, the counters
  const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_shade_prof), sizeof(zero)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_shade_prof), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
extern "C" {

void kdpt_default_options(kdpt_options* o) {
  memset(o, 0, sizeof *o);
  o->focal_length = 6.0f;
  o->dof_angle = 0.0f;
  o->softness = 0.0f;
  o->cacherays = 0;
  o->antialias = 1;
  o->enable_sss = 0;
  o->testing_mode = 0;
  o->compaction = 1;
  o->enable_kd = 1;
  o->viz_kd = 0;
  o->use_bbox = 0;
  o->short_stack = 1;
  o->bounce_cap = 8;
  o->block_size = 0;
  o->external_image = nullptr;
}

const char* kdpt_last_error(void) { return g_last_error.c_str(); }

int kdpt_create(const kdpt_scene* sc, const kdpt_options* opt, int device, kdpt_ctx** out) {
  const auto t_create = std::chrono::steady_clock::now();
  if (!sc || !out) return fail(KDPT_ERR_ARG, "null scene/out");
  *out = nullptr;
  kdpt_options o;
  if (opt) o = *opt; else kdpt_default_options(&o);
  if (o.bounce_cap <= 0) o.bounce_cap = 8;
  if (o.bounce_cap > 30) return fail(KDPT_ERR_ARG, "bounce_cap > 30");
  if (o.block_size && o.block_size != TILE) return fail(KDPT_ERR_UNSUPPORTED, "block_size must be 0 or 256");
  const int W = sc->camera.resolution[0], H = sc->camera.resolution[1];
  if (W <= 0 || H <= 0 || (long long)W * H >= (1ll << 30)) return fail(KDPT_ERR_ARG, "bad resolution");
  if (sc->num_materials > MAX_KEYS) return fail(KDPT_ERR_UNSUPPORTED, "more than 64 materials");
  // The compact visited-state traversal needs the reference builder's shape:
  // nodes[i].ID == i, root == node 0, node 1 == root's left child, <= 15 levels.
  std::vector<int> level;
  const bool brute = !o.enable_kd && sc->has_obj;
  if (brute) {
    // the arrays pathTraceOneBounce reads (src/pathtrace.cu:485-576) must be in bounds
    if (sc->num_shapes < 1 || !sc->obj_materialOffsets || !sc->obj_polyoffsets || !sc->obj_polysidxflat ||
        !sc->obj_verts || !sc->obj_norms)
      return fail(KDPT_ERR_ARG, "enable_kd=0 needs the OBJ arrays (obj_verts, obj_norms, obj_polysidxflat, ...)");
    long long total = 0;
    for (int i = 0; i < sc->num_shapes; i++) {
      if (sc->obj_polyoffsets[i] < 0 || sc->obj_polyoffsets[i] % 3)
        return fail(KDPT_ERR_UNSUPPORTED, "OBJ shapes must be triangulated (index counts multiple of 3)");
      if (sc->obj_materialOffsets[i] < 0 || sc->obj_materialOffsets[i] >= sc->num_materials)
        return fail(KDPT_ERR_ARG, "obj_materialOffsets out of range");
      total += sc->obj_polyoffsets[i];
    }
    if (total != sc->polyidxcount) return fail(KDPT_ERR_ARG, "obj_polyoffsets do not sum to polyidxcount");
    for (int j = 0; j < sc->polyidxcount; j++) {
      const long long v = sc->obj_polysidxflat[j];
      if (v < 0 || 3 * v + 2 >= sc->num_obj_verts || 3 * v + 2 >= sc->num_obj_norms)
        return fail(KDPT_ERR_ARG, "OBJ vertex index out of range (vertex or normal array)");
    }
    if (o.use_bbox && (!sc->obj_bboxes || sc->num_bbox_floats < sc->num_shapes + 5))
      return fail(KDPT_ERR_ARG, "use_bbox needs obj_bboxes[num_shapes + 5]");
  }
  if (sc->has_obj && sc->num_nodes > 0 && !brute) {
    const kdpt_node_bare* N = sc->nodes;
    int root = -1;
    for (int i = 0; i < sc->num_nodes; i++)
      if (N[i].parentID == -1) { root = N[i].ID; break; }
    if (root != 0) return fail(KDPT_ERR_UNSUPPORTED, "root must be node 0");
    for (int i = 0; i < sc->num_nodes; i++) {
      if (N[i].ID != i) return fail(KDPT_ERR_UNSUPPORTED, "nodes must be stored in ID order");
      for (int ch : {N[i].leftID, N[i].rightID})
        if (ch != -1 && (ch <= i || ch >= sc->num_nodes || N[ch].parentID != i))
          return fail(KDPT_ERR_ARG, "inconsistent KD node links");
      if (N[i].triIdSize > 0 && (N[i].triIdStart < 0 || N[i].triIdStart + N[i].triIdSize > sc->num_tris))
        return fail(KDPT_ERR_ARG, "triangle range out of bounds");
      if (N[i].triIdSize > 0 && (N[i].leftID != -1 || N[i].rightID != -1))
        return fail(KDPT_ERR_UNSUPPORTED, "KD node with both triangles and children");
    }
    if (sc->num_nodes > 1 && N[0].leftID != 1) return fail(KDPT_ERR_UNSUPPORTED, "node 1 must be root's left child");
    level.assign(sc->num_nodes, 0);
    for (int i = 1; i < sc->num_nodes; i++) {
      // only the root has no parent (the traversal tests `parentID == -1` as `cur == root`)
      if (N[i].parentID < 0 || N[i].parentID >= i) return fail(KDPT_ERR_ARG, "inconsistent KD parent links");
      level[i] = level[N[i].parentID] + 1;
      if (level[i] > 15) return fail(KDPT_ERR_UNSUPPORTED, "KD tree deeper than 15 levels");
    }
    for (int i = 0; i < sc->num_tris; i++) {
      int m = sc->tris[i].mtlIdx;
      if (m < 0 || m >= sc->num_shapes) return fail(KDPT_ERR_ARG, "triangle mtlIdx out of range");
    }
  }
  kdpt_ctx* c = new kdpt_ctx();
  c->device = device;
  c->opt = o;
  c->cam = sc->camera;
  c->traceDepth = sc->traceDepth;
  c->W = W;
  c->H = H;
  c->npix = W * H;
  c->ntiles = (c->npix + TILE - 1) / TILE;
  c->cap = o.bounce_cap;
  c->nkeys = std::max(1, sc->num_materials);
  auto bail = [&](int rc) {
    kdpt_destroy(c);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(fail(KDPT_ERR_HIP, "hipSetDevice failed"));
  c->cu_mask_streams = g_cu_mask_streams;
  if (create_stream(c, &c->stream) != KDPT_OK) return bail(fail(KDPT_ERR_HIP, "hipStreamCreate failed"));
  int rc;
  // geoms / materials (viz_kd: the KD node boxes follow the analytic geoms, as boxes with the last material,
  // src/pathtrace.cu:1813-1831)
  const bool viz = o.viz_kd && o.enable_kd && sc->has_obj && sc->num_nodes > 0;
  std::vector<kdpt_geom> allg(sc->geoms, sc->geoms + sc->num_geoms);
  if (viz) {
    if (sc->num_materials < 1) return fail(KDPT_ERR_ARG, "viz_kd needs a material");
    for (int k = 0; k < sc->num_nodes; k++) {
      kdpt_geom g{};
      g.type = 1;
      g.materialid = sc->num_materials - 1;
      kdpt_host::node_box_matrices(sc->nodes[k].mins, sc->nodes[k].maxs, g.transform, g.inverseTransform);
      allg.push_back(g);
    }
  }
  std::vector<DevGeom> dg(allg.size());
  for (size_t i = 0; i < allg.size(); i++) {
    dg[i].type = allg[i].type;
    dg[i].materialid = allg[i].materialid;
    memcpy(dg[i].transform, allg[i].transform, 64);
    memcpy(dg[i].inverseTransform, allg[i].inverseTransform, 64);
    memcpy(dg[i].invTranspose, allg[i].invTranspose, 64);
    {  // world bounds of the transformed unit cube (contains the transformed unit sphere), + margin
      const float* m = allg[i].transform;  // column-major
      double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
      for (int k = 0; k < 8; k++) {
        const double v[3] = {(k & 1) ? 0.5 : -0.5, (k & 2) ? 0.5 : -0.5, (k & 4) ? 0.5 : -0.5};
        for (int r = 0; r < 3; r++) {
          const double w = (double)m[r] * v[0] + (double)m[4 + r] * v[1] + (double)m[8 + r] * v[2] + (double)m[12 + r];
          lo[r] = std::min(lo[r], w);
          hi[r] = std::max(hi[r], w);
        }
      }
      const double ext = std::max(std::max(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
      const double margin = 1e-3 * ext + 1e-3;
      for (int r = 0; r < 3; r++) {
        dg[i].wlo[r] = (float)(lo[r] - margin);
        dg[i].whi[r] = (float)(hi[r] + margin);
      }
      dg[i].wlo[3] = dg[i].whi[3] = 0.0f;
    }
    if (dg[i].type != 0 && dg[i].type != 1)  // SPHERE / CUBE: the only types the scene parser creates
      return bail(fail(KDPT_ERR_UNSUPPORTED, "geom type other than sphere (0) or cube (1)"));
    if (dg[i].materialid < 0 || dg[i].materialid >= sc->num_materials)
      return bail(fail(KDPT_ERR_ARG, "geom materialid out of range"));
  }
  std::vector<DevMaterial> dm(sc->num_materials);
  for (int i = 0; i < sc->num_materials; i++) {
    const kdpt_material& m = sc->materials[i];
    DevMaterial& d = dm[i];
    memcpy(d.color, m.color, 12);
    d.spec_exponent = m.specular_exponent;
    memcpy(d.spec_color, m.specular_color, 12);
    d.hasReflective = m.hasReflective;
    d.hasRefractive = m.hasRefractive;
    d.indexOfRefraction = m.indexOfRefraction;
    d.emittance = m.emittance;
    memcpy(d.transmittance, m.transmittance, 12);
    // glm::pow((1.0f - ior) / (1.0f + ior), 2.0f): powf(x, 2) folds to x * x
    float rr = (1.0f - m.indexOfRefraction) / (1.0f + m.indexOfRefraction);
    d.fresnel_R0 = rr * rr;
    d.pad_[0] = d.pad_[1] = d.pad_[2] = 0;
  }
  DevGeom* d_geoms;
  DevMaterial* d_mats;
  if ((rc = dupload(c, &d_geoms, dg.data(), dg.size()))) return bail(rc);
  if ((rc = dupload(c, &d_mats, dm.data(), dm.size()))) return bail(rc);
  c->S.geoms = d_geoms;
  c->S.num_geoms = sc->num_geoms;
  c->S.num_boxes = viz ? sc->num_nodes : 0;
  c->viz = viz;
  c->S.materials = d_mats;
  c->S.num_materials = sc->num_materials;
  c->S.has_obj = sc->has_obj ? 1 : 0;
  c->S.num_nodes = sc->has_obj ? sc->num_nodes : 0;
  c->S.root = 0;
  c->S.n0_left = c->S.n0_right = c->S.n1_left = c->S.n1_right = -1;
  set_cull(c, cluster_margin({}, {}, {}));  // (no triangles: the fast margin; replaced below)
  if (sc->has_obj && sc->num_nodes > 0 && !brute) {
    const int nn = sc->num_nodes, nt = sc->num_tris;
    std::vector<int4> nodes(4 * (size_t)nn);
    std::vector<float4> tv(nt), e1(nt), e2(nt), n0(nt), n1(nt), n2(nt);
    for (int i = 0; i < nn; i++) {  // one 64-byte record per node (one cache line per visit)
      const kdpt_node_bare& N = sc->nodes[i];
      nodes[4 * i + 0] = make_int4(fbits(N.mins[0]), fbits(N.mins[1]), fbits(N.mins[2]), fbits(N.maxs[0]));
      nodes[4 * i + 1] = make_int4(fbits(N.maxs[1]), fbits(N.maxs[2]), N.leftID, N.rightID);
      nodes[4 * i + 2] = make_int4(N.parentID, N.triIdStart, N.triIdSize, N.axis);
      nodes[4 * i + 3] = make_int4(0, 0, 0, 0);
    }
    for (int i = 0; i < nt; i++) {
      const kdpt_tri_bare& T = sc->tris[i];
      // glm::intersectRayTriangle's e1 = v1 - v0, e2 = v2 - v0 in float: same bits here
      tv[i] = make_float4(T.x1, T.y1, T.z1, ibits(T.mtlIdx));
      e1[i] = make_float4(T.x2 - T.x1, T.y2 - T.y1, T.z2 - T.z1, 0.0f);
      e2[i] = make_float4(T.x3 - T.x1, T.y3 - T.y1, T.z3 - T.z1, 0.0f);
      n0[i] = make_float4(T.nx1, T.ny1, T.nz1, 0.0f);
      n1[i] = make_float4(T.nx2, T.ny2, T.nz2, 0.0f);
      n2[i] = make_float4(T.nx3, T.ny3, T.nz3, 0.0f);
    }
    int4* dnodes;
    float4 *dtv, *de1, *de2, *dn0, *dn1, *dn2;
    int* doff;
    if ((rc = dupload(c, &dnodes, nodes.data(), nodes.size())) || (rc = dupload(c, &dtv, tv.data(), nt)) ||
        (rc = dupload(c, &de1, e1.data(), nt)) || (rc = dupload(c, &de2, e2.data(), nt)) ||
        (rc = dupload(c, &dn0, n0.data(), nt)) || (rc = dupload(c, &dn1, n1.data(), nt)) ||
        (rc = dupload(c, &dn2, n2.data(), nt)) ||
        (rc = dupload(c, &doff, sc->obj_materialOffsets, (size_t)sc->num_shapes)))
      return bail(rc);
    c->S.nodes = dnodes;
    c->S.pnodes = nullptr;
    std::vector<int2> leaf_cl, leaf_sp;
    if ((rc = build_clusters(c, sc, tv, e1, e2, leaf_cl, leaf_sp))) return bail(rc);
    std::vector<int4> packed;
    if (pack_nodes(sc->nodes, nn, leaf_cl, packed)) {
      int4* dp;
      if ((rc = dupload(c, &dp, packed.data(), packed.size()))) return bail(rc);
      c->S.pnodes = dp;
    }
    c->S.dnodes = nullptr;
    c->S.snodes = nullptr;
    if (pack_nodes16(sc->nodes, nn, leaf_cl, packed)) {
      int4* dp;
      if ((rc = dupload(c, &dp, packed.data(), packed.size()))) return bail(rc);
      c->S.dnodes = dp;
      // the same records with a big leaf's first super-cluster (TREE_LDS16S), when the scene has supers
      if (c->S.num_supers > 0 && pack_nodes16(sc->nodes, nn, leaf_sp, packed)) {
        if ((rc = dupload(c, &dp, packed.data(), packed.size()))) return bail(rc);
        c->S.snodes = dp;
      }
    }
    c->S.tv0 = dtv;
    c->S.te1 = de1;
    c->S.te2 = de2;
    c->S.tn0 = dn0;
    c->S.tn1 = dn1;
    c->S.tn2 = dn2;
    c->S.obj_material_offsets = doff;
    c->S.rlo = make_float4(sc->nodes[0].mins[0], sc->nodes[0].mins[1], sc->nodes[0].mins[2], 0.0f);
    c->S.rhi = make_float4(sc->nodes[0].maxs[0], sc->nodes[0].maxs[1], sc->nodes[0].maxs[2], 0.0f);
    c->S.n0_left = sc->nodes[0].leftID;
    c->S.n0_right = sc->nodes[0].rightID;
    if (nn > 1) {
      c->S.n1_left = sc->nodes[1].leftID;
      c->S.n1_right = sc->nodes[1].rightID;
    }
  } else if (brute) {
    // pathTraceOneBounce's triangles: the file-order OBJ triangles (vertex/normal gathers done here
    // once; the values are the ones the reference's kernel gathers per test)
    const int nt = sc->polyidxcount / 3;
    std::vector<float4> tv(nt), e1(nt), e2(nt), n0(nt), n1(nt), n2(nt);
    for (int k = 0; k < nt; k++) {
      const int* ix = sc->obj_polysidxflat + 3 * (size_t)k;
      const float* a = sc->obj_verts + 3 * (size_t)ix[0];
      const float* b = sc->obj_verts + 3 * (size_t)ix[1];
      const float* cc = sc->obj_verts + 3 * (size_t)ix[2];
      tv[k] = make_float4(a[0], a[1], a[2], 0.0f);
      e1[k] = make_float4(b[0] - a[0], b[1] - a[1], b[2] - a[2], 0.0f);
      e2[k] = make_float4(cc[0] - a[0], cc[1] - a[1], cc[2] - a[2], 0.0f);
      const float* na = sc->obj_norms + 3 * (size_t)ix[0];
      const float* nb = sc->obj_norms + 3 * (size_t)ix[1];
      const float* nc = sc->obj_norms + 3 * (size_t)ix[2];
      n0[k] = make_float4(na[0], na[1], na[2], 0.0f);
      n1[k] = make_float4(nb[0], nb[1], nb[2], 0.0f);
      n2[k] = make_float4(nc[0], nc[1], nc[2], 0.0f);
    }
    std::vector<float4> clo, chi;
    build_chunk_boxes(tv, e1, e2, nt, clo, chi);
    set_cull(c, cluster_margin(tv, e1, e2));
    std::vector<BruteShape> shp(sc->num_shapes);
    for (int i = 0; i < sc->num_shapes; i++) {
      // glm::vec3(obj_polysbboxes[i] - 0.01, ...): double arithmetic, rounded to float by the constructor
      const float* bb = sc->obj_bboxes;
      float l[3] = {0, 0, 0}, h[3] = {0, 0, 0};
      if (o.use_bbox)
        for (int k = 0; k < 3; k++) {
          l[k] = (float)((double)bb[i + k] - 0.01);
          h[k] = (float)((double)bb[i + 3 + k] + 0.01);
        }
      shp[i].lo = make_float4(l[0], l[1], l[2], ibits(sc->obj_polyoffsets[i]));
      shp[i].hi = make_float4(h[0], h[1], h[2], ibits(sc->obj_materialOffsets[i]));
    }
    float4 *dtv, *de1, *de2, *dn0, *dn1, *dn2;
    if ((rc = dupload(c, &dtv, tv.data(), nt)) || (rc = dupload(c, &de1, e1.data(), nt)) ||
        (rc = dupload(c, &de2, e2.data(), nt)) || (rc = dupload(c, &dn0, n0.data(), nt)) ||
        (rc = dupload(c, &dn1, n1.data(), nt)) || (rc = dupload(c, &dn2, n2.data(), nt)) ||
        (rc = dupload(c, &c->shapes, shp.data(), shp.size())) ||
        (rc = dupload(c, &c->chunk_lo, clo.data(), clo.size())) || (rc = dupload(c, &c->chunk_hi, chi.data(), chi.size())))
      return bail(rc);
    c->S.tv0 = dtv;
    c->S.te1 = de1;
    c->S.te2 = de2;
    c->S.tn0 = dn0;
    c->S.tn1 = dn1;
    c->S.tn2 = dn2;
    c->S.num_nodes = 0;
    c->num_shapes = sc->num_shapes;
    c->brute = true;
  } else {
    c->S.has_obj = 0;
  }
  if ((rc = alloc_iteration_buffers(c))) return bail(rc);
  if (o.external_image) {
    c->image = o.external_image;
    c->image_external = true;
  } else if ((rc = dalloc(c, &c->image, 3 * (size_t)c->npix))) {
    return bail(rc);
  }
  if ((rc = dalloc(c, &c->counters, 1)) || (rc = dalloc(c, &c->total_segments, 1)) ||
      (rc = dalloc(c, &c->trace_total, 3)))
    return bail(rc);
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
      c->wall_khz = khz;
  }
  // The product reads no environment variables: every route is the tested default unless a caller
  // changes it explicitly with kdpt_set_tuning (A/B experiments, the three-kernel compaction test).
  c->S.trace_mode = 0;
  // leave the node phase early once at most early_walk lanes still walk and at least early_leaf wait on a
  // leaf (the walkers resume after the leaf phase; first A/B at 32 / 24: 3 390 -> 3 540 Mrays/s; 0 / 65 =
  // never)
  // re-swept after the flattened leaf phase made leaf phases cheaper (32 / 24 before: 4 505-4 530 -> 4 659-4 704
  // Mrays/s, k_trace launch 0.85 -> 0.80 ms), and again with round 5's exact cull (24 -> 16: C3 5 747-5 756 ->
  // 5 798-5 802, C5 4 487 -> 4 544; 8 / 12 / 20 / 32 below 16, early_leaf 8 / 24 neutral; profiles/r05_ab_log.md)
  c->S.early_walk = 16;
  c->S.early_leaf = 1;
  c->trace_order = false;  // superseded by k_geoms' candidate lists
  if ((rc = setup_trace(c))) return bail(rc);
  c->S.trip_limit = 8 * std::max(c->S.num_nodes, 1) + 64;
  if ((rc = alloc_iteration_events(c))) return bail(rc);
  // the scene's uploads (hipMemcpy) complete before any kernel of the context's non-blocking streams
  HIP_TRY(hipDeviceSynchronize());
  if ((rc = kdpt_reset(c))) return bail(rc);
  c->reduce_spin_us = g_reduce_spin_us;
  c->create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_create).count();
  *out = c;
  return KDPT_OK;
}

int kdpt_set_options(kdpt_ctx* c, const kdpt_options* o) {
  if (!c || !o) return fail(KDPT_ERR_ARG, "null arg");
  if (c->parent) return fail(KDPT_ERR_ARG, "not a top-level context");
  const kdpt_options& p = c->opt;
  // these select what is uploaded or how much is allocated: a new context is needed
  if (o->enable_kd != p.enable_kd || o->viz_kd != p.viz_kd || o->use_bbox != p.use_bbox ||
      (o->bounce_cap > 0 ? o->bounce_cap : 8) != c->cap || o->block_size != p.block_size ||
      o->external_image != p.external_image)
    return fail(KDPT_ERR_UNSUPPORTED, "enable_kd, viz_kd, use_bbox, bounce_cap, block_size and external_image "
                                      "are fixed at kdpt_create");
  HIP_TRY(hipSetDevice(c->device));
  if (!c->slots.empty()) {  // iterations in flight keep the options they were enqueued with
    int rc = kdpt_synchronize(c);
    if (rc) return rc;
  }
  auto apply = [o](kdpt_options& d) {
    d.focal_length = o->focal_length;
    d.dof_angle = o->dof_angle;
    d.softness = o->softness;
    d.cacherays = o->cacherays;
    d.antialias = o->antialias;
    d.enable_sss = o->enable_sss;
    d.testing_mode = o->testing_mode;
    d.compaction = o->compaction;
    d.short_stack = o->short_stack;
  };
  apply(c->opt);
  for (auto sl : c->slots) apply(sl->opt);
  return KDPT_OK;
}

int kdpt_set_tuning(kdpt_ctx* c, const char* name, double value) {
  if (!c && name && std::string(name) == "reduce_spin_us") {  // the process default of contexts created later
    if (!(value >= 0.0 && value <= 1e6)) return fail(KDPT_ERR_ARG, "reduce_spin_us must be in [0, 1e6]");
    g_reduce_spin_us = value;
    return KDPT_OK;
  }
  if (!c && name && std::string(name) == "cu_mask_streams") {  // ... the kind of their batch / reduce streams
    g_cu_mask_streams = value != 0.0;
    return KDPT_OK;
  }
  if (!c && name && std::string(name) == "cluster_chord") {  // ... and their big-leaf cluster grouping
    if (!(value >= -1.0 && value <= 4.0)) return fail(KDPT_ERR_ARG, "cluster_chord must be in [-1, 4]");
    g_cluster_chord = value;
    return KDPT_OK;
  }
  if (!c || !name) return fail(KDPT_ERR_ARG, "null arg");
  if (c->parent) return fail(KDPT_ERR_ARG, "not a top-level context");
  HIP_TRY(hipSetDevice(c->device));
  // pipeline slots copy the knobs when they are made: drop them so the next kdpt_trace_iterations
  // makes new ones
  if (!c->slots.empty()) {
    int rc = kdpt_synchronize(c);
    if (rc) return rc;
    drop_slots(c);
  }
  const std::string k(name);
  const int v = (int)value;
  if (k == "shade_fused") {
    c->no_fuse = v == 0;
  } else if (k == "early_walk") {
    c->S.early_walk = v;
  } else if (k == "early_leaf") {
    c->S.early_leaf = v;
  } else if (k == "shade_batch") {
    c->shade_batch = v != 0;
  } else if (k == "gen_geoms") {
    c->gen_geoms = v != 0;
  } else if (k == "chunk_width0" || k == "chunk_width1" || k == "chunk_width2") {
    c->chunk_width[k.back() - '0'] = std::min(64, std::max(1, v));
  } else if (k == "trace_grid_frac") {
    if (!(value > 0.0 && value <= 1.0)) return fail(KDPT_ERR_ARG, "trace_grid_frac must be in (0, 1]");
    c->trace_grid = std::max(1, (int)(c->full_trace_grid * value));
    c->grid_env = value < 1.0;
  } else if (k == "cluster_obb") {
    c->S.cl_obb = v != 0;
  } else if (k == "flat_obb") {
    c->S.flat_obb = v != 0;
  } else if (k == "super_slab") {
    c->S.sup_slab = v != 0;
  } else if (k == "tree_format" || k == "tree_global" || k == "super_cull" || k == "cluster_slab") {
    if (k == "tree_format") {
      if (v != 0 && v != 16 && v != 32) return fail(KDPT_ERR_ARG, "tree_format must be 0 (best), 16 or 32");
      c->tree_format = v;
    } else if (k == "super_cull") {
      c->super_cull = v != 0;
    } else if (k == "cluster_slab") {
      c->S.cl_slab = v != 0;
      return KDPT_OK;
    } else {
      c->force_global_tree = v != 0;
    }
    const double frac = (double)c->trace_grid / std::max(1, c->full_trace_grid);
    int rc = setup_trace(c);
    if (rc) return rc;
    if (c->grid_env) c->trace_grid = std::max(1, (int)(c->full_trace_grid * frac));
  } else if (k == "cluster_cull" || k == "cull_margin" || k == "cull_exact" || k == "cull_mask_n" ||
             k == "cull_fast_k") {
    if (k == "cluster_cull") {
      // 0: no cluster / chunk cull at all (every big-leaf cluster swept: exact by construction, whatever the
      // scene's margin); 1: the scene's margins (and masks)
      c->cull_scene = v != 0;
      if (v != 0) set_cull(c, c->cull);
      else fix_cull(c, __builtin_inff());
    } else if (k == "cull_margin") {
      // > 0: one fixed margin coefficient for every level (no masks: not exact in general); 0: the scene's
      if (!(value >= 0.0)) return fail(KDPT_ERR_ARG, "cull_margin must be >= 0 (0: the scene's)");
      c->cull_scene = value == 0.0;
      if (value > 0.0) fix_cull(c, (float)value);
      else set_cull(c, c->cull);
    } else if (k == "cull_exact") {
      // 0: the fast-margin one-level cull instead of the masked exact one (A/B; not exact for such scenes)
      c->cull_exact = v != 0;
    } else if (k == "cull_fast_k") {
      // the masked cull's box coefficient (default CULL_MARGIN_MASKED), its direction masks rebuilt for it: a
      // wider box sweeps more clusters, a narrower one leaves more danger triangles to decide
      if (!(value > 0.0 && value < 1.0)) return fail(KDPT_ERR_ARG, "cull_fast_k must be in (0, 1)");
      if (!c->mask_cs) return fail(KDPT_ERR_ARG, "cull_fast_k: this scene has no direction masks");
      c->cull.K = c->cull.K_lo = (float)value;
      if (c->cull_scene) set_cull(c, c->cull);
      int rc = build_masks(c, c->mask_n);
      if (rc) return rc;
    } else {
      if (v < 1 || v > 512) return fail(KDPT_ERR_ARG, "cull_mask_n must be in 1 .. 512");
      if (!c->mask_cs) return fail(KDPT_ERR_ARG, "cull_mask_n: this scene has no direction masks");
      int rc = build_masks(c, v);
      if (rc) return rc;
    }
    apply_cull_route(c);
    const double frac = (double)c->trace_grid / std::max(1, c->full_trace_grid);
    int rc = setup_trace(c);  // the route may change (no super-cluster route under the masked cull)
    if (rc) return rc;
    if (c->grid_env) c->trace_grid = std::max(1, (int)(c->full_trace_grid * frac));
  } else if (k == "profile_batches") {
    c->profile_batches = v != 0;
    c->profile_steps = v >= 2;
  } else if (k == "sync_debug") {
    c->sync_debug = v != 0;
  } else if (k == "reduce_spin_us") {
    if (!(value >= 0.0 && value <= 1e6)) return fail(KDPT_ERR_ARG, "reduce_spin_us must be in [0, 1e6]");
    c->reduce_spin_us = value;
  } else {
    return fail(KDPT_ERR_ARG, "unknown tuning knob " + k);
  }
  return KDPT_OK;
}

int kdpt_reset(kdpt_ctx* c) {
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  for (auto sl : c->slots) HIP_TRY(hipStreamSynchronize(sl->stream));
  if (c->reduce_stream) HIP_TRY(hipStreamSynchronize(c->reduce_stream));
  drain_intersect_events(c);
  c->intersect_ms_total = 0;
  c->intersect_launches_total = 0;
  HIP_TRY(hipMemsetAsync(c->image, 0, sizeof(float) * 3 * (size_t)c->npix, c->stream));
  HIP_TRY(hipMemsetAsync(c->total_segments, 0, sizeof(unsigned long long), c->stream));
  HIP_TRY(hipMemsetAsync(c->trace_total, 0, 3 * sizeof(unsigned long long), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  memset(&c->stats, 0, sizeof c->stats);
  c->stats.intersect_grid_share = 1.0f;
  return KDPT_OK;
}

int kdpt_trace_iteration_async(kdpt_ctx* c, int frame, int iter) {
  (void)frame;  // unused by the reference too
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  return launch_iteration(c, iter, -1, false);
}

int kdpt_synchronize(kdpt_ctx* c) {
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto sl : c->slots) {
    HIP_TRY(hipStreamSynchronize(sl->stream));
    int rc = check_fault(sl);
    if (rc) return rc;
  }
  if (c->reduce_stream) HIP_TRY(hipStreamSynchronize(c->reduce_stream));
  unregister_host(c);
  int rc = drain_intersect_events(c);
  if (rc) return rc;
  if (c->profile_batches) HIP_TRY(hipMemcpy(&c->last_profile, c->counters, sizeof(Counters), hipMemcpyDeviceToHost));
  return check_fault(c);
}

int kdpt_trace_iteration(kdpt_ctx* c, int frame, int iter) {
  (void)frame;
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventRecord(c->ev0, c->stream));
  int rc = launch_iteration(c, iter, -1, c->count_mode);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->ev1, c->stream));
  HIP_TRY(hipMemcpyAsync(c->h_counts, c->counts, sizeof(int) * (c->cap + 3), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->h_counts[c->cap + 2]) return fault_error(c, c->h_counts[c->cap + 2]);
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->stats.ms_last_iteration = ms;
  c->stats.iterations++;
  const int bounces = segments_from_counts(c);
  if (c->opt.testing_mode) {
    float tot = 0;
    for (int d = 0; d < bounces; d++) {
      float b = 0;
      if (hipEventElapsedTime(&b, c->bounce_ev[2 * d], c->bounce_ev[2 * d + 1]) == hipSuccess) tot += b;
    }
    c->stats.ms_intersect = tot;
    c->intersect_ms_total += tot;
    c->intersect_launches_total += bounces;
  }
  return KDPT_OK;
}

// Iterations first_iter + k * stride (k < count) in batches of `batch`, `pipeline` batches in flight, their
// partial images added into `target` (the context's image, or a frame buffer of kdpt_render_frames) in
// iteration order.  Each batch's add runs on the batch's own stream, after the previous batch's add (the one
// cross-stream wait of the pipeline, normally satisfied by the time it is reached): no stream ever waits for a
// whole batch, so none holds an in-order hardware queue that batch streams share (HIP multiplexes a process's
// streams onto GPU_MAX_HW_QUEUES queues, 4 by default).  zero_after: the target is first zeroed, after that
// event (a frame buffer after its previous reduce).  Returns once everything is queued.
int enqueue_iterations(kdpt_ctx* c, int first_iter, int count, int stride, int pipeline, int batch, float* target,
                       hipEvent_t zero_after = nullptr) {
  const int depth = std::min(16, std::max(1, pipeline));
  const int B = std::min(MAXB, std::max(1, batch));
  // the first add follows everything already queued on the context's own stream (reset, ...)
  hipEvent_t entry;
  HIP_TRY(hipEventCreateWithFlags(&entry, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(entry, c->stream));
  // slots: `depth` groups of B iteration contexts; a group runs one batch at a time on its first
  // context's stream
  if ((int)c->slots.size() < depth * B || c->slot_batch != B) {
    if (!c->slots.empty()) {
      int rc = kdpt_synchronize(c);
      if (rc) return rc;
      drop_slots(c);
    }
    c->slot_batch = B;
    c->next_group = 0;
    // Only the group leaders create streams, one after another: HIP maps streams onto its hardware queues
    // (GPU_MAX_HW_QUEUES) in creation order, reusing the least-used queue once all exist, so a stream per
    // slot context (8 x 4) had put pairs of leaders -- two batches' chains -- on one in-order queue.
    while ((int)c->slots.size() < depth * B) {
      kdpt_ctx* sl = nullptr;
      const bool leader = c->slots.size() % B == 0;
      int rc = make_slot(c, &sl, leader ? nullptr : c->slots[c->slots.size() / B * B]->stream);
      if (rc) return rc;
      c->slots.push_back(sl);
    }
    for (int g = 0; g < depth; g++) {
      hipEvent_t d;
      HIP_TRY(hipEventCreateWithFlags(&d, hipEventDisableTiming));
      c->acc_ev.push_back(d);
    }
  }
  const int ngroups = (int)c->acc_ev.size();
  // With several batches in flight each intersect launch gets a share of the chip (2/depth of the
  // persistent grid, all of it for depth <= 2, a quarter from depth 8 on): a launch's length is set by its
  // heaviest rays, so concurrent launches on disjoint CU subsets overlap those tails instead of queueing
  // behind them.  (Sweep with every batch on its own hardware queue: a quarter is best at depths 8-12.)
  for (auto sl : c->slots)
    sl->trace_grid =
        c->grid_env ? c->trace_grid : std::max(1, c->trace_grid * 2 / std::min(8, std::max(2, depth)));
  c->stats.intersect_grid_share =
      c->slots.empty() ? 1.0f : (float)c->slots[0]->trace_grid / (float)std::max(1, c->full_trace_grid);
  // diagnostic ("profile_batches" knob): the counting intersect kernel (kdpt_wave_profile after sync)
  if (c->profile_batches) HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(Counters), c->stream));
  bool first = true;
  for (int kb = 0; kb < count; kb += B) {
    const int nb = std::min(B, count - kb);
    // groups in turn, continuing across calls: kdpt_render_frames queues one call per frame, and a frame
    // shorter than the pipeline must not restart at group 0 (it would wait on that group's previous batch)
    const int g = c->next_group % ngroups;
    c->next_group = (g + 1) % ngroups;
    kdpt_ctx* const* grp = &c->slots[(size_t)g * B];
    hipStream_t st = grp[0]->stream;
    // (the group's previous batch's partial images were added on this stream, before this batch's camera rays
    // clear them)
    int iters[MAXB];
    for (int b = 0; b < nb; b++) {
      iters[b] = first_iter + (kb + b) * stride;
      grp[b]->zero_partial = true;  // k_gen_rays clears the partial image
    }
    std::vector<hipEvent_t>* bev = nullptr;
    if (c->opt.testing_mode) {
      std::vector<hipEvent_t> evs;
      for (int e = 0; e < 2 * c->cap; e++) {
        hipEvent_t ev;
        if (!c->free_ev.empty()) { ev = c->free_ev.back(); c->free_ev.pop_back(); }
        else HIP_TRY(hipEventCreate(&ev));
        evs.push_back(ev);
      }
      c->pending_ev.push_back(evs);
      bev = &c->pending_ev.back();
    }
    int rc = launch_batch(grp, iters, nb, st, -1, c->profile_batches, bev);
    if (rc) return rc;
    // the add: after the previous add (the chain), and for the call's first batch after the context's stream,
    // the frames' image adds (when the target is the image) and the target's zeroing
    if (c->acc_last) HIP_TRY(hipStreamWaitEvent(st, c->acc_last, 0));
    if (first) {
      HIP_TRY(hipStreamWaitEvent(st, entry, 0));
      if (c->img_last && target == c->image) HIP_TRY(hipStreamWaitEvent(st, c->img_last, 0));
      if (zero_after) {
        HIP_TRY(hipStreamWaitEvent(st, zero_after, 0));
        HIP_TRY(hipMemsetAsync(target, 0, sizeof(float) * 3 * (size_t)c->npix, st));
      }
      first = false;
    }
    const int n3 = 3 * c->npix;
    PartialImages parts{};
    parts.nb = nb;
    for (int b = 0; b < nb; b++) parts.p[b] = grp[b]->image;  // in iteration order
    hipLaunchKernelGGL(k_accumulate_batch, dim3((n3 + 255) / 256), dim3(256), 0, st, target, parts, n3);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->acc_ev[g], st));
    c->acc_last = c->acc_ev[g];
  }
  HIP_TRY(hipEventDestroy(entry));
  c->stats.iterations += count;
  return KDPT_OK;
}

int kdpt_trace_iterations(kdpt_ctx* c, int frame, int first_iter, int count, int stride, int pipeline, int batch) {
  (void)frame;
  if (!c || count < 0 || first_iter < 1 || stride < 1) return fail(KDPT_ERR_ARG, "bad arguments");
  if (c->parent) return fail(KDPT_ERR_ARG, "not a top-level context");
  HIP_TRY(hipSetDevice(c->device));
  return enqueue_iterations(c, first_iter, count, stride, pipeline, batch, c->image);
}

int kdpt_read_image(kdpt_ctx* c, float* rgb) {
  if (!c || !rgb) return fail(KDPT_ERR_ARG, "null arg");
  HIP_TRY(hipSetDevice(c->device));
  int rc = join_accum(c);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(rgb, c->image, sizeof(float) * 3 * (size_t)c->npix, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return KDPT_OK;
}

int kdpt_trace_config(kdpt_ctx* c, int* tree_mode, int* block, int* grid, long long* lds_bytes) {
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  const int m = c->tree_mode;
  if (tree_mode) *tree_mode = m;
  if (block)
    *block = m == TREE_LDS ? trace_block<TREE_LDS>() : (m >= TREE_LDS16 ? trace_block<TREE_LDS16>() : trace_block<TREE_PACKED>());
  if (grid) *grid = c->full_trace_grid;
  if (lds_bytes) *lds_bytes = (long long)c->tree_lds;
  return KDPT_OK;
}

int kdpt_cull_margin(kdpt_ctx* c, float* margin, double* rigorous, int* exact) {
  if (!c) return fail(KDPT_ERR_ARG, "null ctx");
  if (margin) *margin = c->S.cl_margin;
  if (rigorous) *rigorous = c->cull.rigorous;
  // the box-only levels use cl_margin; the slab level's margin is rigorous by construction whenever that is;
  // the masked one-level cull is exact whatever the margin (its masks hold every triangle that can pass)
  if (exact) *exact = ((double)c->S.cl_margin >= c->cull.rigorous || c->S.cl_mask) ? 1 : 0;
  return KDPT_OK;
}

int kdpt_write_pbo(kdpt_ctx* c, int iter, uint8_t* rgba) {
  if (!c || !rgba || iter == 0) return fail(KDPT_ERR_ARG, "bad arg");
  HIP_TRY(hipSetDevice(c->device));
  int rc = join_accum(c);
  if (rc) return rc;
  // The reference's pbo is the GL-mapped device buffer (src/main.cpp runCuda); a headless caller passes host
  // memory.  Memory of this context's device is written by the kernel directly; anything else (host memory,
  // another device's buffer) through the context's staging buffer and a copy.
  hipPointerAttribute_t attr{};
  const bool on_device = hipPointerGetAttributes(&attr, rgba) == hipSuccess && attr.type == hipMemoryTypeDevice &&
                         attr.device == c->device;
  (void)hipGetLastError();  // a plain host pointer is an error for hipPointerGetAttributes on some runtimes
  uchar4* d = reinterpret_cast<uchar4*>(rgba);
  if (!on_device) {
    if (!c->pbo_staging) HIP_TRY(hipMalloc((void**)&c->pbo_staging, sizeof(uchar4) * (size_t)c->npix));
    d = c->pbo_staging;
  }
  hipLaunchKernelGGL(k_pbo, dim3((c->npix + 255) / 256), dim3(256), 0, c->stream, c->image, c->npix, iter, d);
  HIP_TRY(hipGetLastError());
  if (!on_device)
    HIP_TRY(hipMemcpyAsync(rgba, d, sizeof(uchar4) * (size_t)c->npix, hipMemcpyDefault, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return KDPT_OK;
}

// The saveImage pixel pass on the device; rgb (host, 3*W*H) and/or lin (host, 3*W*H floats).
static int save_image_pass(kdpt_ctx* c, float samples, uint8_t* rgb, float* lin) {
  HIP_TRY(hipSetDevice(c->device));
  for (auto sl : c->slots) HIP_TRY(hipStreamSynchronize(sl->stream));
  if (c->reduce_stream) HIP_TRY(hipStreamSynchronize(c->reduce_stream));
  const size_t n3 = 3 * (size_t)c->npix;
  uint8_t* d_rgb = nullptr;
  float* d_lin = nullptr;
  HIP_TRY(hipMalloc((void**)&d_rgb, n3));
  if (lin && hipMalloc((void**)&d_lin, n3 * sizeof(float)) != hipSuccess) {
    (void)hipFree(d_rgb);
    return fail(KDPT_ERR_HIP, "hipMalloc");
  }
  hipLaunchKernelGGL(k_save_image, dim3((c->npix + 255) / 256), dim3(256), 0, c->stream, c->image, c->W, c->H,
                     samples, d_rgb, d_lin);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && rgb) e = hipMemcpyAsync(rgb, d_rgb, n3, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && lin) e = hipMemcpyAsync(lin, d_lin, n3 * sizeof(float), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_rgb);
  if (d_lin) (void)hipFree(d_lin);
  if (e != hipSuccess) return fail(KDPT_ERR_HIP, std::string("save image: ") + hipGetErrorString(e));
  return KDPT_OK;
}

int kdpt_save_rgb8(kdpt_ctx* c, float samples, uint8_t* rgb) {
  if (!c || !rgb) return fail(KDPT_ERR_ARG, "null arg");
  return save_image_pass(c, samples, rgb, nullptr);
}

int kdpt_save_png(kdpt_ctx* c, const char* path, float samples) {
  if (!c || !path) return fail(KDPT_ERR_ARG, "null arg");
  std::vector<uint8_t> rgb(3 * (size_t)c->npix);
  int rc = save_image_pass(c, samples, rgb.data(), nullptr);
  if (rc) return rc;
  rc = kdpt_write_png(path, rgb.data(), c->W, c->H);
  return rc ? fail(rc, std::string("cannot write ") + path) : KDPT_OK;
}

int kdpt_save_hdr(kdpt_ctx* c, const char* path, float samples) {
  if (!c || !path) return fail(KDPT_ERR_ARG, "null arg");
  std::vector<float> lin(3 * (size_t)c->npix);
  int rc = save_image_pass(c, samples, nullptr, lin.data());
  if (rc) return rc;
  rc = kdpt_write_hdr(path, lin.data(), c->W, c->H);
  return rc ? fail(rc, std::string("cannot write ") + path) : KDPT_OK;
}

int kdpt_cull_masks(kdpt_ctx* c, int* mask_n, int* num_clusters, unsigned long long* masks) {
  if (!c || !mask_n || !num_clusters) return fail(KDPT_ERR_ARG, "null arg");
  HIP_TRY(hipSetDevice(c->device));
  *mask_n = c->mask_dev ? c->mask_n : 0;
  *num_clusters = c->S.num_clusters;
  if (!c->mask_dev) return KDPT_OK;
  const size_t cells = 6 * (size_t)c->mask_n * c->mask_n * (size_t)c->S.num_clusters;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (masks)
    HIP_TRY(hipMemcpyAsync(masks, c->mask_dev, cells * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return KDPT_OK;
}

int kdpt_get_stats(kdpt_ctx* c, kdpt_stats* st) {
  if (!c || !st) return fail(KDPT_ERR_ARG, "null arg");
  HIP_TRY(hipSetDevice(c->device));
  unsigned long long tot = 0, tt[3] = {0, 0, 0};
  HIP_TRY(hipMemcpyAsync(&tot, c->total_segments, sizeof tot, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(tt, c->trace_total, sizeof tt, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->stats.intersect_device_ms_total = (double)tt[0] / c->wall_khz;
  c->stats.intersect_device_launches_total = (long long)tt[1];
  c->stats.total_trace_rays = (long long)tt[2];
  c->stats.total_segments = (long long)tot;
  c->stats.intersect_ms_total = c->intersect_ms_total;
  c->stats.intersect_launches_total = c->intersect_launches_total;
  c->stats.create_ms = c->create_ms;
  c->stats.mask_build_ms = c->mask_build_ms;
  *st = c->stats;
  return KDPT_OK;
}

int kdpt_image_device_ptr(kdpt_ctx* c, void** p) {
  if (!c || !p) return fail(KDPT_ERR_ARG, "null arg");
  *p = c->image;
  return KDPT_OK;
}

int kdpt_destroy(kdpt_ctx* c) {
  if (!c) return KDPT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  drop_slots(c);  // (each slot drains its stream)
  for (auto& evs : c->pending_ev)
    for (auto e : evs) (void)hipEventDestroy(e);
  for (auto e : c->free_ev) (void)hipEventDestroy(e);
  // (a kdpt_render_frames that failed partway may have left a reduce queued: drain it before the communicator
  // and the frame buffers go)
  if (c->reduce_stream) (void)hipStreamSynchronize(c->reduce_stream);
  release_comm(c);
  unregister_host(c);
  for (auto e : c->frame_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->reduce_stream) (void)hipStreamDestroy(c->reduce_stream);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->pbo_staging) (void)hipFree(c->pbo_staging);
  if (c->h_counts) (void)hipHostFree(c->h_counts);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (auto e : c->bounce_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream && c->owns_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return KDPT_OK;
}

int kdpt_debug_paths(kdpt_ctx* c, int iter, int stop_depth, kdpt_path_segment* out, int* npaths) {
  if (!c || !out || stop_depth < 0 || stop_depth >= c->cap) return fail(KDPT_ERR_ARG, "bad arg");
  HIP_TRY(hipSetDevice(c->device));
  // run on a scratch image so the accumulation buffer is untouched
  float* saved = c->image;
  float* scratch = nullptr;
  HIP_TRY(hipMalloc((void**)&scratch, sizeof(float) * 3 * (size_t)c->npix));
  HIP_TRY(hipMemsetAsync(scratch, 0, sizeof(float) * 3 * (size_t)c->npix, c->stream));
  c->image = scratch;
  unsigned long long* saved_tot = c->total_segments;
  c->total_segments = reinterpret_cast<unsigned long long*>(c->counters);  // scratch word
  int rc = launch_iteration(c, iter, stop_depth, false);
  c->total_segments = saved_tot;
  c->image = saved;
  if (rc) { (void)hipFree(scratch); return rc; }
  kdpt_path_segment* d = nullptr;
  HIP_TRY(hipMalloc((void**)&d, sizeof(kdpt_path_segment) * (size_t)c->npix));
  const int depth_slot = stop_depth + 1;
  hipLaunchKernelGGL(k_unpack, dim3((c->npix + 255) / 256), dim3(256), 0, c->stream, c->buf[c->cur], c->counts,
                     depth_slot, d);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(c->h_counts, c->counts, sizeof(int) * (c->cap + 2), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if ((rc = check_fault(c))) { (void)hipFree(d); (void)hipFree(scratch); return rc; }
  const int n = c->h_counts[depth_slot];
  *npaths = n;
  HIP_TRY(hipMemcpy(out, d, sizeof(kdpt_path_segment) * (size_t)n, hipMemcpyDeviceToHost));
  (void)hipFree(d);
  (void)hipFree(scratch);
  return KDPT_OK;
}

// Roofline counters: one extra (untimed) iteration with per-path AABB/triangle/hit counts.
int kdpt_count_iteration(kdpt_ctx* c, int iter, unsigned long long* aabb_tri_hit) {
  if (!c || !aabb_tri_hit) return fail(KDPT_ERR_ARG, "null arg");
  HIP_TRY(hipSetDevice(c->device));
  float* saved = c->image;
  float* scratch = nullptr;
  HIP_TRY(hipMalloc((void**)&scratch, sizeof(float) * 3 * (size_t)c->npix));
  HIP_TRY(hipMemsetAsync(scratch, 0, sizeof(float) * 3 * (size_t)c->npix, c->stream));
  HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(Counters), c->stream));
  c->image = scratch;
  unsigned long long* saved_tot = c->total_segments;
  unsigned long long* scratch_tot = nullptr;
  HIP_TRY(hipMalloc((void**)&scratch_tot, sizeof(unsigned long long)));
  c->total_segments = scratch_tot;
  int rc = launch_iteration(c, iter, -1, true);
  c->total_segments = saved_tot;
  c->image = saved;
  Counters h{};
  if (!rc) {
    HIP_TRY(hipMemcpyAsync(&h, c->counters, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_counts, c->counts, sizeof(int) * (c->cap + 3), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    segments_from_counts(c);  // stats.segments / seg_per_bounce now describe the counting iteration
    rc = check_fault(c);
  }
  (void)hipFree(scratch);
  (void)hipFree(scratch_tot);
  aabb_tri_hit[0] = h.aabb;
  aabb_tri_hit[1] = h.tri;
  aabb_tri_hit[2] = h.hit;
  c->last_profile = h;
  return rc;
}

int kdpt_count_split(kdpt_ctx* c, unsigned long long* aabb_prep_cand) {
  if (!c || !aabb_prep_cand) return fail(KDPT_ERR_ARG, "null arg");
  aabb_prep_cand[0] = c->last_profile.aabb_prep;
  aabb_prep_cand[1] = c->last_profile.cand;
  return KDPT_OK;
}

int kdpt_wave_profile(kdpt_ctx* c, unsigned long long* out, int n) {
  if (!c || !out) return fail(KDPT_ERR_ARG, "null arg");
  unsigned long long v[PROF_SLOTS + 5];
  for (int k = 0; k < PROF_SLOTS + 2; k++) v[k] = c->last_profile.wave[k];
  v[PROF_SLOTS + 2] = c->last_profile.aabb;
  v[PROF_SLOTS + 3] = c->last_profile.tri;
  v[PROF_SLOTS + 4] = c->last_profile.hit;
  int k = 0;
  for (; k < n && k < PROF_SLOTS + 5; k++) out[k] = v[k];
  for (int b = 0; b < 64 && k < n; b++, k++) out[k] = c->last_profile.life[b];
  for (int b = 0; b < 64 && k < n; b++, k++) out[k] = c->last_profile.steps[b];
  for (int b = 0; b < 8 && k < n; b++, k++) out[k] = c->last_profile.chord_steps[b];
  for (int b = 0; b < 8 && k < n; b++, k++) out[k] = c->last_profile.chord_n[b];
  return PROF_SLOTS + 5 + 64 + 64 + 16;
}

int kdpt_selftest_math(const float* x, int n, float* so, float* co) {
  float *dx, *ds, *dc;
  HIP_TRY(hipMalloc((void**)&dx, sizeof(float) * n));
  HIP_TRY(hipMalloc((void**)&ds, sizeof(float) * n));
  HIP_TRY(hipMalloc((void**)&dc, sizeof(float) * n));
  HIP_TRY(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, ds, dc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(so, ds, sizeof(float) * n, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(co, dc, sizeof(float) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx); (void)hipFree(ds); (void)hipFree(dc);
  return KDPT_OK;
}

int kdpt_selftest_libm(int fn, const float* x, int n, double* out) {
  if (fn < 0 || fn > 2 || n < 0 || (n && (!x || !out))) return fail(KDPT_ERR_ARG, "kdpt_selftest_libm: bad arguments");
  if (n == 0) return KDPT_OK;
  float* dx;
  double* dout;
  HIP_TRY(hipMalloc((void**)&dx, sizeof(float) * n));
  HIP_TRY(hipMalloc((void**)&dout, sizeof(double) * n));
  HIP_TRY(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_libm, dim3((n + 255) / 256), dim3(256), 0, 0, fn, dx, n, dout);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx); (void)hipFree(dout);
  return KDPT_OK;
}

int kdpt_selftest_libm_digest(int fn, uint32_t first, unsigned long long count, unsigned long long* digest) {
  if (fn < 0 || fn > 2 || !digest || count > (1ull << 32) || first + count > (1ull << 32))
    return fail(KDPT_ERR_ARG, "kdpt_selftest_libm_digest: bad arguments");
  unsigned long long* dacc;
  HIP_TRY(hipMalloc((void**)&dacc, sizeof(unsigned long long)));
  HIP_TRY(hipMemset(dacc, 0, sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_selftest_libm_digest, dim3(4096), dim3(256), 0, 0, fn, first, (uint64_t)count, dacc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(digest, dacc, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  (void)hipFree(dacc);
  return KDPT_OK;
}

int kdpt_selftest_rng(const int* iid, int n, int k, float* u) {
  int* di;
  float* du;
  HIP_TRY(hipMalloc((void**)&di, sizeof(int) * 3 * n));
  HIP_TRY(hipMalloc((void**)&du, sizeof(float) * n));
  HIP_TRY(hipMemcpy(di, iid, sizeof(int) * 3 * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_rng, dim3((n + 255) / 256), dim3(256), 0, 0, di, n, k, du);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(u, du, sizeof(float) * n, hipMemcpyDeviceToHost));
  (void)hipFree(di); (void)hipFree(du);
  return KDPT_OK;
}

int kdpt_selftest_rng_draws(int mode, const uint32_t* in, int n, int k, float* out) {
  if (mode < 0 || mode > 2 || n < 0 || k < 0 || (n && k && (!in || !out)))
    return fail(KDPT_ERR_ARG, "bad rng selftest arguments");
  if (!n || !k) return KDPT_OK;
  const size_t nin = (size_t)n * (mode == 0 ? 3 : 1), nout = (size_t)n * k;
  uint32_t* di;
  float* dout;
  HIP_TRY(hipMalloc((void**)&di, sizeof(uint32_t) * nin));
  if (hipMalloc((void**)&dout, sizeof(float) * nout) != hipSuccess) {
    (void)hipFree(di);
    return fail(KDPT_ERR_HIP, "hipMalloc failed");
  }
  int rc = KDPT_OK;
  if (hipMemcpy(di, in, sizeof(uint32_t) * nin, hipMemcpyHostToDevice) != hipSuccess) rc = KDPT_ERR_HIP;
  if (rc == KDPT_OK) {
    hipLaunchKernelGGL(k_selftest_rng_draws, dim3((n + 255) / 256), dim3(256), 0, 0, mode, di, n, k, dout);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpy(out, dout, sizeof(float) * nout, hipMemcpyDeviceToHost) != hipSuccess)
      rc = KDPT_ERR_HIP;
  }
  (void)hipFree(di);
  (void)hipFree(dout);
  return rc == KDPT_OK ? KDPT_OK : fail(rc, "rng selftest failed");
}

int kdpt_selftest_glm(int fn, const float* in, int n, float* out) {
  const int ni = glm_kat_inputs(fn), no = glm_kat_outputs(fn);
  if (!ni || n < 0 || (n && (!in || !out))) return fail(KDPT_ERR_ARG, "bad glm selftest arguments");
  if (!n) return KDPT_OK;
  float *din, *dout;
  HIP_TRY(hipMalloc((void**)&din, sizeof(float) * ni * (size_t)n));
  HIP_TRY(hipMalloc((void**)&dout, sizeof(float) * no * (size_t)n));
  HIP_TRY(hipMemcpy(din, in, sizeof(float) * ni * (size_t)n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dout, out, sizeof(float) * no * (size_t)n, hipMemcpyHostToDevice));  // sentinels
  hipLaunchKernelGGL(k_selftest_glm, dim3((n + 255) / 256), dim3(256), 0, 0, fn, din, n, dout);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(out, dout, sizeof(float) * no * (size_t)n, hipMemcpyDeviceToHost));
  (void)hipFree(din); (void)hipFree(dout);
  return KDPT_OK;
}

int kdpt_selftest_fresnel(const float* cs, int n, float ior, float* f) {
  float *dc, *df;
  HIP_TRY(hipMalloc((void**)&dc, sizeof(float) * n));
  HIP_TRY(hipMalloc((void**)&df, sizeof(float) * n));
  HIP_TRY(hipMemcpy(dc, cs, sizeof(float) * n, hipMemcpyHostToDevice));
  float rr = (1.0f - ior) / (1.0f + ior);
  hipLaunchKernelGGL(k_selftest_fresnel, dim3((n + 255) / 256), dim3(256), 0, 0, dc, n, rr * rr, df);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(f, df, sizeof(float) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dc); (void)hipFree(df);
  return KDPT_OK;
}

}  // extern "C"

namespace {

template <bool HYBRID, bool COUNT>
void launch_trace_mode(kdpt_ctx* c, const TraceArgs& a, hipStream_t st) {
  const dim3 g(c->trace_grid);
  if (c->tree_mode == TREE_LDS)
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_LDS>), g, dim3(trace_block<TREE_LDS>()), c->tree_lds, st, a);
  else if (c->tree_mode == TREE_LDS16)
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_LDS16>), g, dim3(trace_block<TREE_LDS16>()), c->tree_lds, st, a);
  else if (c->tree_mode == TREE_LDS16G)
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_LDS16G>), g, dim3(trace_block<TREE_LDS16G>()), c->tree_lds, st, a);
  else if (c->tree_mode == TREE_LDS16S)
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_LDS16S>), g, dim3(trace_block<TREE_LDS16S>()), c->tree_lds, st, a);
  else if (c->tree_mode == TREE_PACKED)
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_PACKED>), g, dim3(trace_block<TREE_PACKED>()), 0, st, a);
  else
    hipLaunchKernelGGL((k_trace<HYBRID, COUNT, TREE_WIDE>), g, dim3(trace_block<TREE_WIDE>()), 0, st, a);
}

void launch_trace(kdpt_ctx* c, const TraceArgs& a, bool count, hipStream_t st) {
  const bool hyb = c->opt.short_stack != 0;
  if (hyb) { if (count) launch_trace_mode<true, true>(c, a, st); else launch_trace_mode<true, false>(c, a, st); }
  else { if (count) launch_trace_mode<false, true>(c, a, st); else launch_trace_mode<false, false>(c, a, st); }
}

template <bool HYBRID>
void launch_shade_h(kdpt_ctx* c, const ShadeArgs& a, bool compact, bool sort, hipStream_t st) {
  const dim3 g(c->ntiles), b(TILE);
  if (compact) {
    if (sort) hipLaunchKernelGGL((k_shade<HYBRID, true, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_shade<HYBRID, true, false>), g, b, 0, st, a);
  } else {
    if (sort) hipLaunchKernelGGL((k_shade<HYBRID, false, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_shade<HYBRID, false, false>), g, b, 0, st, a);
  }
}

// One iteration of each context in cs (nb <= MAXB; all share the scene and options), in lockstep on
// stream st: per bounce the analytic geoms of each, one intersect launch over all of them, then each
// one's shading and compaction.  The iterations stay independent: only the intersect launch is shared.
int launch_batch(kdpt_ctx* const* cs, const int* iters, int nb, hipStream_t st, int stop_depth, bool count,
                 std::vector<hipEvent_t>* bev) {
  kdpt_ctx* c0 = cs[0];
  // camera rays and bounce 0's analytic geoms + root-box test in one launch (not for the brute-force and box-view
  // intersect kernels, which have no first part)
  const bool gen_geoms = c0->gen_geoms && !c0->brute && !c0->viz;
  {  // the batch's camera rays in one launch (blockIdx.y = iteration)
    GenBatch gb;
    gb.cam = c0->cam;
    gb.traceDepth = c0->traceDepth;
    gb.focalLength = c0->opt.focal_length;
    gb.dofAngle = c0->opt.dof_angle;
    gb.antialias = c0->opt.antialias;
    gb.ncounts = c0->cap + 2;
    gb.nwork = c0->cap;
    gb.nlb = c0->cap * c0->ntiles;
    for (int b = 0; b < nb; b++) {
      kdpt_ctx* c = cs[b];
      c->cur = 0;
      gb.it[b] = GenIter{c->opt.cacherays ? 1 : iters[b], c->buf[0], c->counts, c->work, c->trace_t, c->lb,
                         c->zero_partial ? c->image : nullptr};
    }
    if (gen_geoms) {
      GenGeomsBatch gg;
      gg.g = gb;
      gg.S = c0->S;
      gg.count_aabb = count ? c0->counters : nullptr;
      for (int b = 0; b < nb; b++) {
        kdpt_ctx* c = cs[b];
        c->cc0_cur = c->ccount0 + c->gen_parity;
        gg.it[b] = GenGeomsIter{c->cc0_cur, c->ccount0 + (c->gen_parity ^ 1), c->cray, c->hits, c->cand};
        c->gen_parity ^= 1;
      }
      hipLaunchKernelGGL(k_gen_geoms_b, dim3((c0->npix + GEN_BLOCK - 1) / GEN_BLOCK, nb), dim3(GEN_BLOCK), 0, st,
                         gg);
    } else {
      hipLaunchKernelGGL(k_gen_rays_b, dim3((c0->npix + 255) / 256, nb), dim3(256), 0, st, gb);
    }
    HIP_TRY(hipGetLastError());
  }
  const bool compact = c0->opt.compaction != 0;
  bool prep_ready = false;  // this bounce's intersect-stage first part came with the previous scatter
  for (int depth = 0; depth < c0->cap; depth++) {
    const bool prep_next = compact && depth + 1 < c0->cap && !c0->brute && !c0->viz;
    if (c0->opt.testing_mode && bev) HIP_TRY(hipEventRecord((*bev)[2 * depth], st));
    TraceArgs t;
    t.S = c0->S;
    t.nb = nb;
    t.prof_steps = (c0->parent ? c0->parent : c0)->profile_steps ? 1 : 0;
    for (int b = 0; b < MAXB; b++) {
      kdpt_ctx* c = cs[b < nb ? b : 0];
      t.it[b].cand = c->cand;
      t.it[b].ccount = (depth == 0 && gen_geoms) ? c->cc0_cur : c->ccount;  // indexed by depth (0 here)
      t.it[b].cray = c->cray;
      t.it[b].hits = c->hits;
    }
    t.work = c0->work;
    t.depth = depth;
    t.counters = c0->counters;
    t.trace_t = c0->trace_t;
    if (c0->viz) {
      for (int b = 0; b < nb; b++) {
        kdpt_ctx* c = cs[b];
        hipLaunchKernelGGL(k_viz, dim3(c->ntiles), dim3(TILE), 0, st, c->S, c->buf[c->cur], c->counts, depth, c->hits,
                           c0->trace_t);
        HIP_TRY(hipGetLastError());
      }
    } else if (c0->brute) {
      for (int b = 0; b < nb; b++) {
        kdpt_ctx* c = cs[b];
        BruteArgs ba;
        ba.S = c->S;
        ba.paths = c->buf[c->cur];
        ba.counts = c->counts;
        ba.depth = depth;
        ba.hits = c->hits;
        ba.shapes = c->shapes;
        ba.num_shapes = c->num_shapes;
        ba.chunk_lo = c->chunk_lo;
        ba.chunk_hi = c->chunk_hi;
        ba.counters = c0->counters;
        ba.trace_t = c0->trace_t;
        const dim3 g(c->ntiles), bl(TILE);
        if (c->opt.use_bbox) {
          if (count) hipLaunchKernelGGL((k_brute<true, true>), g, bl, 0, st, ba);
          else hipLaunchKernelGGL((k_brute<true, false>), g, bl, 0, st, ba);
        } else {
          if (count) hipLaunchKernelGGL((k_brute<false, true>), g, bl, 0, st, ba);
          else hipLaunchKernelGGL((k_brute<false, false>), g, bl, 0, st, ba);
        }
        HIP_TRY(hipGetLastError());
        if (c0->sync_debug) {
          BruteShape h0;
          HIP_TRY(hipStreamSynchronize(st));  // (the null-stream copy below does not order after st)
          HIP_TRY(hipMemcpy(&h0, c->shapes, sizeof h0, hipMemcpyDeviceToHost));
          fprintf(stderr, "[kdpt] brute depth %d use_bbox %d shapes %d lo %g %g %g hi %g %g %g n %d mat %d\n", depth,
                  c->opt.use_bbox, c->num_shapes, h0.lo.x, h0.lo.y, h0.lo.z, h0.hi.x, h0.hi.y, h0.hi.z, fbits(h0.lo.w),
                  fbits(h0.hi.w));
        }
      }
    } else {
      // the intersect stage's first part: already done by the previous bounce's k_shade/k_scatter when it
      // ran with the hand-off (prep_ready), else here
      if (!prep_ready && !(depth == 0 && gen_geoms)) {  // the batch's iterations in one launch (blockIdx.y = iteration)
        GeomsBatch gb;
        gb.S = c0->S;
        gb.depth = depth;
        gb.count_aabb = count ? c0->counters : nullptr;
        gb.gspan = c0->trace_t + 2 * c0->cap;
        for (int b = 0; b < nb; b++) {
          kdpt_ctx* c = cs[b];
          gb.it[b] = GeomsIter{c->buf[c->cur], c->counts, c->cray, c->hits, c->cand, c->ccount};
        }
        hipLaunchKernelGGL(k_geoms_b, dim3((c0->npix + GEN_BLOCK - 1) / GEN_BLOCK, nb), dim3(GEN_BLOCK), 0, st, gb);
        HIP_TRY(hipGetLastError());
      }
      launch_trace(c0, t, count, st);
      HIP_TRY(hipGetLastError());
    }
    if (c0->sync_debug) {
      fprintf(stderr, "[kdpt] trace depth %d launched (grid %d, mode %d, lds %zu, batch %d)\n", depth,
              c0->trace_grid, c0->tree_mode, c0->tree_lds, nb);
      HIP_TRY(hipStreamSynchronize(st));
      fprintf(stderr, "[kdpt] trace depth %d done\n", depth);
    }
    if (c0->opt.testing_mode && bev) HIP_TRY(hipEventRecord((*bev)[2 * depth + 1], st));
    ShadeBatch sbatch;
    int nfused = 0, fused_grid = 0;
    bool fused_hyb = false, fused_stage = false;
    for (int b = 0; b < nb; b++) {
      kdpt_ctx* c = cs[b];
      const bool sort = (iters[b] == 2);
      ShadeArgs a;
      a.S = c->S;
      a.paths = c->buf[c->cur];
      a.hits = c->hits;
      a.image = c->image;
      a.image_zeroed = c->zero_partial ? 1 : 0;
      a.counts = c->counts;
      a.depth = depth;
      a.iter = iters[b];
      a.softness = c->opt.softness;
      a.enable_sss = c->opt.enable_sss;
      a.tile_counts = c->tile_counts;
      a.tile_kcounts = (compact && c->trace_order) ? c->tile_kcounts : nullptr;
      a.ntiles = c->ntiles;
      a.nkeys = c->nkeys;
      a.total_segments = c->total_segments;
      a.trace_t = c0->trace_t;
      a.gspan = c0->trace_t + 2 * c0->cap;
      a.trace_total = b == 0 ? c->trace_total : nullptr;
      a.trace_rays = (c0->brute || c0->viz) ? nullptr : c->trace_total + 2;
      a.ccount = (depth == 0 && gen_geoms) ? c->cc0_cur : c->ccount;
      a.prep_on = prep_next ? 1 : 0;
      a.prep = c->prep;
      a.tile_ccounts = c->tile_ccounts;
      a.count_aabb = count ? c0->counters : nullptr;
      if (compact && !sort && !a.tile_kcounts && !c->no_fuse) {
        // single pass: shading, compaction into the other buffer and the hand-off (k_shade_fused)
        const int nxt = c->cur ^ 1;
        const FuseArgs f{c->buf[nxt], c->tickets, c->lb, c->counts, c->ccount, c->cray, c->hits, c->cand};
        const bool stage = c->S.num_geoms + c->S.num_boxes <= ORDERED_GEOMS && c->S.num_materials <= STAGE_MATS;
        const bool hyb = c->opt.short_stack || c->brute;
        const int shade_grid = (c->npix + SHADE_TB - 1) / SHADE_TB;
        if (c0->shade_batch) {  // launched below, with the batch's other fused iterations
          sbatch.a[nfused] = a;
          sbatch.f[nfused] = f;
          nfused++;
          fused_hyb = hyb;
          fused_stage = stage;
          fused_grid = shade_grid;
          c->cur = nxt;
          continue;
        }
        if (hyb && stage) hipLaunchKernelGGL((k_shade_fused<true, true>), dim3(shade_grid), dim3(SHADE_TB), 0, st, a, f);
        else if (hyb) hipLaunchKernelGGL((k_shade_fused<true, false>), dim3(shade_grid), dim3(SHADE_TB), 0, st, a, f);
        else if (stage) hipLaunchKernelGGL((k_shade_fused<false, true>), dim3(shade_grid), dim3(SHADE_TB), 0, st, a, f);
        else hipLaunchKernelGGL((k_shade_fused<false, false>), dim3(shade_grid), dim3(SHADE_TB), 0, st, a, f);
        HIP_TRY(hipGetLastError());
        c->cur = nxt;
        continue;
      }
      // hit point offset: 1e-4 for the hybrid traversal and the brute-force kernel, 1e-5 for traverseKDbare
      if (c->opt.short_stack || c->brute) launch_shade_h<true>(c, a, compact, sort, st);
      else launch_shade_h<false>(c, a, compact, sort, st);
      HIP_TRY(hipGetLastError());
      if (compact || sort) {
        // survivors' offsets + the next bounce's path count; with the hand-off also the candidate-list
        // offsets per tile + the next bounce's candidate count (a second workgroup)
        const ScanJob j0{c->tile_counts, c->tile_off, sort ? c->nkeys : 1, c->counts + depth + 1};
        const ScanJob j1{c->tile_ccounts, c->tile_coff, 1, c->ccount + depth + 1};
        hipLaunchKernelGGL(k_scan, dim3(prep_next ? 2 : 1), dim3(SCAN_TB), 0, st, j0, j1, c->counts, depth, c->ntiles);
        HIP_TRY(hipGetLastError());
        const int nxt = c->cur ^ 1;
        ScatterPrep sp{prep_next ? 1 : 0, c->prep, c->cray, c->hits, c->cand, c->tile_coff};
        if (sort)
          hipLaunchKernelGGL(k_scatter<true>, dim3(c->ntiles), dim3(TILE), 0, st, c->buf[c->cur], c->buf[nxt],
                             c->tile_off, c->counts, depth, c->ntiles, compact ? 1 : 0, sp);
        else
          hipLaunchKernelGGL(k_scatter<false>, dim3(c->ntiles), dim3(TILE), 0, st, c->buf[c->cur], c->buf[nxt],
                             c->tile_off, c->counts, depth, c->ntiles, compact ? 1 : 0, sp);
        HIP_TRY(hipGetLastError());
        c->cur = nxt;
      } else {
        // no compaction, no sort: the live range stays the whole image
        HIP_TRY(hipMemcpyAsync(c->counts + depth + 1, c->counts + depth, sizeof(int), hipMemcpyDeviceToDevice, st));
      }
    }
    if (nfused) {  // the batch's fused iterations in one launch
      const dim3 g(fused_grid, nfused), bl(SHADE_TB);
      if (fused_hyb && fused_stage) hipLaunchKernelGGL((k_shade_fused_b<true, true>), g, bl, 0, st, sbatch);
      else if (fused_hyb) hipLaunchKernelGGL((k_shade_fused_b<true, false>), g, bl, 0, st, sbatch);
      else if (fused_stage) hipLaunchKernelGGL((k_shade_fused_b<false, true>), g, bl, 0, st, sbatch);
      else hipLaunchKernelGGL((k_shade_fused_b<false, false>), g, bl, 0, st, sbatch);
      HIP_TRY(hipGetLastError());
    }
    if (c0->sync_debug) {
      HIP_TRY(hipStreamSynchronize(st));
      fprintf(stderr, "[kdpt] shade depth %d done\n", depth);
    }
    if (stop_depth == depth) return KDPT_OK;
    prep_ready = prep_next;
  }
  if (!compact) {
    for (int b = 0; b < nb; b++) {
      kdpt_ctx* c = cs[b];
      hipLaunchKernelGGL(k_final_gather, dim3((c->npix + 255) / 256), dim3(256), 0, st, c->buf[c->cur], c->counts,
                         c->cap, c->image);
      HIP_TRY(hipGetLastError());
    }
  }
  return KDPT_OK;
}

int launch_iteration(kdpt_ctx* c, int iter, int stop_depth, bool count) {
  int rc = join_accum(c);
  if (rc) return rc;
  return launch_batch(&c, &iter, 1, c->stream, stop_depth, count, c->rec_ev ? c->rec_ev : &c->bounce_ev);
}

}  // namespace

// ---------------------------------------------------------------------------
// Multi-GPU: samples per pixel sharded across GPUs (the reference renders one GPU's
// iterations in pathtrace(), src/pathtrace.cu:2405-2635).  Frame f covers global iterations f * spp + 1 ..
// (f + 1) * spp; rank r of N renders those with (iteration - 1 - f * spp) % N == r, in order, into its frame
// buffer, and one reduce (sum, to rank 0) per frame combines them -- the path's only exchange step.  Every
// iteration-dependent behaviour (RNG seeds, iteration 2's sort, cacherays) uses the global numbers.
//
// The reduce is RCCL's (ncclReduce over xGMI, one communicator rank per context; multi-process:
// kdpt_comm_init, one process per GPU) or, inside one process (kdpt_render_sharded), either RCCL
// (ncclCommInitAll) or a peer-copy reduce on device 0 that adds the ranks' frames in rank order (also usable
// with several contexts on one device, which RCCL refuses).  RCCL is loaded at run time (dlopen): the library
// has no link-time dependency on it, and a process that already holds it (torch) shares that copy.  Each
// context queues its frames' reduces and rank 0's image adds on a reduce stream of its own, which waits for
// the frame's last add (the batch streams' add chain), so frames stay in flight: frame f + 1's iterations run
// while frame f is reduced.
// ---------------------------------------------------------------------------
namespace {

struct Rccl {
  ncclResult_t (*getUniqueId)(ncclUniqueId*);
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*);
  ncclResult_t (*commDestroy)(ncclComm_t);
  ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*groupStart)();
  ncclResult_t (*groupEnd)();
  const char* (*errorString)(ncclResult_t);
};

const Rccl* rccl() {
  static std::once_flag once;
  static Rccl r{};
  static bool ok = false;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.getUniqueId = (decltype(r.getUniqueId))dlsym(h, "ncclGetUniqueId");
    r.commInitRank = (decltype(r.commInitRank))dlsym(h, "ncclCommInitRank");
    r.commInitAll = (decltype(r.commInitAll))dlsym(h, "ncclCommInitAll");
    r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
    r.reduce = (decltype(r.reduce))dlsym(h, "ncclReduce");
    r.groupStart = (decltype(r.groupStart))dlsym(h, "ncclGroupStart");
    r.groupEnd = (decltype(r.groupEnd))dlsym(h, "ncclGroupEnd");
    r.errorString = (decltype(r.errorString))dlsym(h, "ncclGetErrorString");
    ok = r.getUniqueId && r.commInitRank && r.commInitAll && r.commDestroy && r.reduce && r.groupStart &&
         r.groupEnd && r.errorString;
  });
  return ok ? &r : nullptr;
}

#define RCCL_TRY(R, x)                                                                 \
  do {                                                                                 \
    const ncclResult_t e_ = (x);                                                       \
    if (e_ != ncclSuccess) return fail(KDPT_ERR_HIP, std::string("rccl: ") + (R)->errorString(e_)); \
  } while (0)

// frame image = a + b + ... (rank order), the copy-reduce's sum
struct FrameParts {
  const float* p[8];
  int n;
};
__global__ void k_sum_frames(float* __restrict__ out, FrameParts parts, int n3) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n3) return;
  float v = parts.p[0][i];
  for (int k = 1; k < parts.n; k++) v += parts.p[k][i];
  out[i] = v;
}

// Diagnostic ("reduce_spin_us" knob): one wave that spins for `ticks` of the device's constant-rate clock on the
// reduce stream ahead of a frame's reduce -- what an ncclReduce waiting for a slower peer looks like to this
// GPU's queues (tools/reduce_spin_probe.py).
__global__ void k_spin(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

int reduce_spin(kdpt_ctx* c, hipStream_t st) {
  if (!(c->reduce_spin_us > 0)) return KDPT_OK;
  const unsigned long long ticks = (unsigned long long)(c->reduce_spin_us * c->wall_khz / 1000.0);
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, ticks);
  HIP_TRY(hipGetLastError());
  return KDPT_OK;
}

void release_comm(kdpt_ctx* c) {
  const Rccl* R = c->comm && c->owns_comm ? rccl() : nullptr;
  if (R) (void)R->commDestroy((ncclComm_t)c->comm);
  c->comm = nullptr;
  c->owns_comm = false;
}

void unregister_host(kdpt_ctx* c) {
  for (void* p : c->host_reg) (void)hipHostUnregister(p);
  c->host_reg.clear();
}

int frame_buffers(kdpt_ctx* c) {
  const size_t n3 = 3 * (size_t)c->npix;
  if (!c->reduce_stream) {
    int rc = create_stream(c, &c->reduce_stream);
    if (rc) return rc;
  }
  for (int k = 0; k < 2; k++) {
    if (!c->frame_buf[k]) {
      int rc = dalloc(c, &c->frame_buf[k], n3);
      if (rc) return rc;
      HIP_TRY(hipEventCreateWithFlags(&c->frame_ev[k], hipEventDisableTiming));
      HIP_TRY(hipEventRecord(c->frame_ev[k], c->stream));
    }
  }
  if (!c->frame_sum && c->rank == 0) return dalloc(c, &c->frame_sum, n3);
  return KDPT_OK;
}

// A pageable host `out` is pinned in place for the frames' copies (hipHostRegister), so they run as queued
// instead of staging synchronously at every frame's enqueue (which would serialise frame f + 1's enqueue behind
// frame f's reduce); device memory, already pinned memory and failed registrations are left as they are.
void pin_host_out(kdpt_ctx* c, void* p, size_t bytes) {
  if (!p || !bytes) return;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type != hipMemoryTypeUnregistered) return;
  (void)hipGetLastError();
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess) c->host_reg.push_back(p);
  else (void)hipGetLastError();
}

// Iterations of frame f for rank r of n: first, stride n, count.
void frame_share(int f, int spp, int n, int r, int* first, int* count) {
  *first = f * spp + 1 + r;
  *count = r < spp ? (spp - r + n - 1) / n : 0;
}

// Queue frame f's share of this rank into frame_buf[f & 1] (zeroed first, after its previous reduce), and make
// the reduce stream wait for it: the share's last add (c->acc_last), or, for a rank with no iterations in the
// frame, the zeroing itself, done on the reduce stream (which already follows the previous reduce).
int enqueue_frame(kdpt_ctx* c, int f, int spp, int pipeline, int batch) {
  int rc = frame_buffers(c);
  if (rc) return rc;
  float* fb = c->frame_buf[f & 1];
  int first, count;
  frame_share(f, spp, c->nranks, c->rank, &first, &count);
  if (count > 0) {
    if ((rc = enqueue_iterations(c, first, count, c->nranks, pipeline, batch, fb, c->frame_ev[f & 1]))) return rc;
    HIP_TRY(hipStreamWaitEvent(c->reduce_stream, c->acc_last, 0));
  } else {
    HIP_TRY(hipMemsetAsync(fb, 0, sizeof(float) * 3 * (size_t)c->npix, c->reduce_stream));
  }
  return KDPT_OK;
}

// Rank 0, after its frame image is in `sum`: add it into the context's image and copy it out.
int finish_frame(kdpt_ctx* c, const float* sum, float* out, int k, hipStream_t st) {
  const int n3 = 3 * c->npix;
  PartialImages parts{};
  parts.p[0] = sum;
  parts.nb = 1;
  hipLaunchKernelGGL(k_accumulate_batch, dim3((n3 + 255) / 256), dim3(256), 0, st, c->image, parts, n3);
  HIP_TRY(hipGetLastError());
  if (out) HIP_TRY(hipMemcpyAsync(out + (size_t)k * n3, sum, sizeof(float) * n3, hipMemcpyDefault, st));
  return KDPT_OK;
}

int check_frames_args(kdpt_ctx* c, int first_frame, int frames, int spp) {
  if (!c || first_frame < 0 || frames < 0 || spp < 1) return fail(KDPT_ERR_ARG, "bad arguments");
  if (c->parent) return fail(KDPT_ERR_ARG, "not a top-level context");
  return KDPT_OK;
}

}  // namespace

int kdpt_comm_library(char* path, int len) {
  if (!path || len < 1) return fail(KDPT_ERR_ARG, "bad arguments");
  const Rccl* R = rccl();
  if (!R) return fail(KDPT_ERR_UNSUPPORTED, "librccl.so.1 not found");
  // the file that actually provides ncclReduce (in a torch process: torch's own librccl, if loaded first)
  Dl_info info{};
  const char* f = dladdr(reinterpret_cast<void*>(R->reduce), &info) && info.dli_fname ? info.dli_fname : "?";
  snprintf(path, (size_t)len, "%s", f);
  return KDPT_OK;
}

int kdpt_comm_unique_id(unsigned char* id) {
  if (!id) return fail(KDPT_ERR_ARG, "null id");
  const Rccl* R = rccl();
  if (!R) return fail(KDPT_ERR_UNSUPPORTED, "librccl.so.1 not found");
  static_assert(sizeof(ncclUniqueId) == KDPT_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  RCCL_TRY(R, R->getUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return KDPT_OK;
}

int kdpt_comm_init(kdpt_ctx* c, int nranks, int rank, const unsigned char* id) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks) return fail(KDPT_ERR_ARG, "bad arguments");
  if (c->parent) return fail(KDPT_ERR_ARG, "not a top-level context");
  HIP_TRY(hipSetDevice(c->device));
  int rc = kdpt_synchronize(c);
  if (rc) return rc;
  release_comm(c);
  const Rccl* R = rccl();
  c->nranks = nranks;
  c->rank = rank;
  c->external_reduce = nranks > 1 && !id;
  // (one rank with an id gets a communicator too: kdpt_render_frames then runs the same ncclReduce per frame
  // as on N GPUs, so one GPU exercises the multi-GPU path end to end)
  if (id) {
    if (!R) return fail(KDPT_ERR_UNSUPPORTED, "librccl.so.1 not found");
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclComm_t comm;
    RCCL_TRY(R, R->commInitRank(&comm, nranks, u, rank));
    c->comm = comm;
    c->owns_comm = true;
  }
  return KDPT_OK;
}

int kdpt_render_frames(kdpt_ctx* c, int first_frame, int frames, int spp, int pipeline, int batch, float* out) {
  int rc = check_frames_args(c, first_frame, frames, spp);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  const Rccl* R = c->comm ? rccl() : nullptr;
  if (c->nranks > 1 && !R && !c->external_reduce) return fail(KDPT_ERR_ARG, "kdpt_comm_init first");
  const size_t n3 = 3 * (size_t)c->npix;
  if (c->rank == 0 || c->external_reduce) pin_host_out(c, out, sizeof(float) * n3 * (size_t)frames);
  for (int k = 0; k < frames; k++) {
    const int f = first_frame + k;
    if ((rc = enqueue_frame(c, f, spp, pipeline, batch))) return rc;
    float* fb = c->frame_buf[f & 1];
    // the frame's reduce and image add run on the reduce stream once its adds are done (enqueue_frame), while
    // the batch streams go on with the next frame's (other buffer)
    const hipStream_t rs = c->reduce_stream;
    if ((rc = reduce_spin(c, rs))) return rc;
    const float* sum = fb;
    if (c->external_reduce) {  // the caller reduces: every rank's share goes out as it is
      if (out) HIP_TRY(hipMemcpyAsync(out + (size_t)k * n3, fb, sizeof(float) * n3, hipMemcpyDefault, rs));
    } else {
      if (R) {
        RCCL_TRY(R, R->reduce(fb, c->rank == 0 ? c->frame_sum : nullptr, n3, ncclFloat32, ncclSum, 0,
                              (ncclComm_t)c->comm, rs));
        sum = c->frame_sum;
      }
      if (c->rank == 0 && (rc = finish_frame(c, sum, out, k, rs))) return rc;
    }
    HIP_TRY(hipEventRecord(c->frame_ev[f & 1], rs));
    // (entry points that read or write the image, and adds into it, follow the last reduce: join_accum)
    c->img_last = c->frame_ev[f & 1];
  }
  return KDPT_OK;
}

int kdpt_render_sharded(const kdpt_scene* scene, const kdpt_options* opt, int ndev, const int* devices,
                        int first_frame, int frames, int spp, int pipeline, int batch, int reduce, float* out) {
  if (!scene || ndev < 1 || ndev > 8 || !devices || first_frame < 0 || frames < 0 || spp < 1 ||
      (reduce != KDPT_REDUCE_RCCL && reduce != KDPT_REDUCE_COPY))
    return fail(KDPT_ERR_ARG, "bad arguments");
  kdpt_options o;
  if (opt) o = *opt;
  else kdpt_default_options(&o);
  o.external_image = nullptr;
  std::vector<kdpt_ctx*> cs(ndev, nullptr);
  // every event this call records across devices (destroyed once the contexts' streams are drained)
  std::vector<std::pair<int, hipEvent_t>> xev;
  auto cleanup = [&](int rc) {
    for (auto c : cs)
      if (c) kdpt_destroy(c);  // (drains its streams, releases its communicator)
    for (auto& de : xev) {
      (void)hipSetDevice(de.first);
      (void)hipEventDestroy(de.second);
    }
    return rc;
  };
  int rc;
  for (int i = 0; i < ndev; i++) {
    if ((rc = kdpt_create(scene, &o, devices[i], &cs[i]))) return cleanup(rc);
    cs[i]->nranks = ndev;
    cs[i]->rank = i;
  }
  const Rccl* R = nullptr;
  if (reduce == KDPT_REDUCE_RCCL) {
    R = rccl();
    if (!R) return cleanup(fail(KDPT_ERR_UNSUPPORTED, "librccl.so.1 not found"));
    std::vector<ncclComm_t> comms(ndev);
    const ncclResult_t e = R->commInitAll(comms.data(), ndev, devices);
    if (e != ncclSuccess) return cleanup(fail(KDPT_ERR_HIP, std::string("rccl: ") + R->errorString(e)));
    for (int i = 0; i < ndev; i++) {
      cs[i]->comm = comms[i];
      cs[i]->owns_comm = true;
    }
  }
  kdpt_ctx* c0 = cs[0];
  const int n3 = 3 * c0->npix;
  std::vector<float*> staged(ndev, nullptr);  // copy-reduce: the other ranks' frames on device 0
  if (reduce == KDPT_REDUCE_COPY)
    for (int i = 1; i < ndev; i++)
      if ((rc = dalloc(c0, &staged[i], (size_t)n3))) return cleanup(rc);
  // a pageable host `out` pinned for the call (released by the final kdpt_synchronize of c0)
  pin_host_out(c0, out, sizeof(float) * (size_t)n3 * (size_t)frames);
  auto xevent = [&](int dev, hipStream_t st, hipEvent_t* e) {
    if (hipSetDevice(dev) != hipSuccess || hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(*e, st) != hipSuccess)
      return false;
    xev.push_back({dev, *e});
    return true;
  };
  for (int k = 0; k < frames; k++) {
    const int f = first_frame + k;
    // each rank queues its share on its batch streams; its reduce stream waits for the share (as in
    // kdpt_render_frames), so frame f + 1's adds never queue behind frame f's reduce
    std::vector<hipEvent_t> share_done(ndev, nullptr);  // each rank's last add of the frame (copy reduce)
    for (int i = 0; i < ndev; i++) {
      kdpt_ctx* ci = cs[i];
      if (hipSetDevice(ci->device) != hipSuccess) return cleanup(fail(KDPT_ERR_HIP, "hipSetDevice"));
      if ((rc = enqueue_frame(ci, f, spp, pipeline, batch))) return cleanup(rc);
      if ((rc = reduce_spin(ci, ci->reduce_stream))) return cleanup(rc);
      // (recorded on the rank's reduce stream, which already waits for the share)
      if (!xevent(ci->device, ci->reduce_stream, &share_done[i])) return cleanup(fail(KDPT_ERR_HIP, "frame events"));
    }
    if (hipSetDevice(c0->device) != hipSuccess) return cleanup(fail(KDPT_ERR_HIP, "hipSetDevice"));
    if ((rc = frame_buffers(c0))) return cleanup(rc);
    if (reduce == KDPT_REDUCE_RCCL) {
      R->groupStart();
      ncclResult_t e = ncclSuccess;
      for (int i = 0; i < ndev && e == ncclSuccess; i++)
        e = R->reduce(cs[i]->frame_buf[f & 1], i == 0 ? c0->frame_sum : nullptr, (size_t)n3, ncclFloat32, ncclSum,
                      0, (ncclComm_t)cs[i]->comm, cs[i]->reduce_stream);
      const ncclResult_t e2 = R->groupEnd();
      if (e != ncclSuccess || e2 != ncclSuccess)
        return cleanup(fail(KDPT_ERR_HIP, std::string("rccl: ") + R->errorString(e != ncclSuccess ? e : e2)));
    } else {
      // device 0's reduce stream waits for every rank's share and copies the others' over (peer copies: xGMI
      // between GPUs), then adds them in rank order
      FrameParts parts{};
      parts.n = ndev;
      parts.p[0] = c0->frame_buf[f & 1];
      for (int i = 1; i < ndev; i++) {
        kdpt_ctx* ci = cs[i];
        if (hipSetDevice(c0->device) != hipSuccess ||
            hipStreamWaitEvent(c0->reduce_stream, share_done[i], 0) != hipSuccess ||
            hipMemcpyPeerAsync(staged[i], c0->device, ci->frame_buf[f & 1], ci->device, sizeof(float) * (size_t)n3,
                               c0->reduce_stream) != hipSuccess)
          return cleanup(fail(KDPT_ERR_HIP, "copy reduce"));
        parts.p[i] = staged[i];
      }
      hipLaunchKernelGGL(k_sum_frames, dim3((n3 + 255) / 256), dim3(256), 0, c0->reduce_stream, c0->frame_sum, parts, n3);
      if (hipGetLastError() != hipSuccess) return cleanup(fail(KDPT_ERR_HIP, "k_sum_frames"));
      // the other ranks' frame_buf[f & 1] may be reused (frame f + 2) once these copies are done
      hipEvent_t done;
      if (!xevent(c0->device, c0->reduce_stream, &done)) return cleanup(fail(KDPT_ERR_HIP, "copy reduce"));
      for (int i = 1; i < ndev; i++)
        if (hipSetDevice(cs[i]->device) != hipSuccess || hipStreamWaitEvent(cs[i]->reduce_stream, done, 0) != hipSuccess)
          return cleanup(fail(KDPT_ERR_HIP, "copy reduce"));
    }
    if (hipSetDevice(c0->device) != hipSuccess) return cleanup(fail(KDPT_ERR_HIP, "hipSetDevice"));
    if ((rc = finish_frame(c0, c0->frame_sum, out, k, c0->reduce_stream))) return cleanup(rc);
    for (int i = 0; i < ndev; i++) {
      if (hipSetDevice(cs[i]->device) != hipSuccess ||
          hipEventRecord(cs[i]->frame_ev[f & 1], cs[i]->reduce_stream) != hipSuccess)
        return cleanup(fail(KDPT_ERR_HIP, "hipEventRecord"));
    }
  }
  for (int i = 0; i < ndev; i++)
    if ((rc = kdpt_synchronize(cs[i]))) return cleanup(rc);
  return cleanup(KDPT_OK);
}
