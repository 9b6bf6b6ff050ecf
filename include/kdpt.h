/*
 * kdpt.h -- C-ABI drop-in boundary of the MI355X (gfx950) KD-tree path tracer.
 *
 * Replaces the reference's device entry points (src/pathtrace.h:6-21):
 *   pathtraceInit(Scene*, bool enablekd)   -> kdpt_create
 *   pathtrace(uchar4* pbo, int frame, int iter, ...13 flags)
 *                                          -> kdpt_trace_iteration (+ kdpt_read_image,
 *                                             kdpt_write_pbo for the uchar4 preview)
 *   pathtraceFree(Scene*, bool enablekd)   -> kdpt_destroy
 * Plain POD in, host pointers in, no HIP/torch types.  Every entry point returns
 * an int status (KDPT_OK == 0) instead of exit(1) (src/pathtrace.cu:42-60);
 * kdpt_last_error() gives the message.  One context per device; a context is
 * not re-entrant (like the reference's file-static device globals,
 * src/pathtrace.cu:92-98).
 *
 * The structs keep the reference's byte layouts so the
 * arrays the reference's host code builds (Scene::newNodesBare,
 * Scene::newTrianglesBare, Scene::geoms, Scene::materials) pass through as is.
 */
#ifndef KDPT_H
#define KDPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KDPT_OK 0
#define KDPT_ERR_ARG -1
#define KDPT_ERR_HIP -2
#define KDPT_ERR_UNSUPPORTED -3
#define KDPT_ERR_IO -4

/* struct Geom, src/sceneStructs.h:22-31 (236 bytes, glm::mat4 column-major) */
typedef struct kdpt_geom {
    int type; /* enum GeomType: 0 SPHERE, 1 CUBE */
    int materialid;
    float translation[3];
    float rotation[3];
    float scale[3];
    float transform[16];
    float inverseTransform[16];
    float invTranspose[16];
} kdpt_geom;

/* struct Material, src/sceneStructs.h:33-44 (56 bytes) */
typedef struct kdpt_material {
    float color[3];
    float specular_exponent;
    float specular_color[3];
    float hasReflective;
    float hasRefractive;
    float indexOfRefraction;
    float emittance;
    float transmittance[3];
} kdpt_material;

/* struct Camera, src/sceneStructs.h:46-55 (84 bytes) */
typedef struct kdpt_camera {
    int resolution[2];
    float position[3];
    float lookAt[3];
    float view[3];
    float up[3];
    float right[3];
    float fov[2];
    float pixelLength[2];
} kdpt_camera;

/* KDN::NodeBare, src/KDnode.h:64-82 (64 bytes) */
typedef struct kdpt_node_bare {
    int axis;
    float splitPos;
    float mins[3];
    float maxs[3];
    int ID;
    int parentID;
    int leftID;
    int rightID;
    int triIdStart;
    int triIdSize;
    float tmin;
    float tmax;
} kdpt_node_bare;

/* KDN::TriBare, src/KDnode.h:51-62 (76 bytes) */
typedef struct kdpt_tri_bare {
    float x1, x2, x3, y1, y2, y3, z1, z2, z3;
    float nx1, nx2, nx3, ny1, ny2, ny3, nz1, nz2, nz3;
    int mtlIdx;
} kdpt_tri_bare;

/* struct PathSegment (+ Ray), src/sceneStructs.h:15-20,65-71 (56 bytes) */
typedef struct kdpt_path_segment {
    float origin[3];
    float direction[3];
    uint8_t isinside;
    uint8_t pad_[3];
    float sdepth;
    float color[3];
    int pixelIndex;
    int remainingBounces;
    int materialIdHit;
} kdpt_path_segment;

/* struct ShadeableIntersection, src/sceneStructs.h:81-85 (20 bytes) */
typedef struct kdpt_shadeable_intersection {
    float t;
    float surfaceNormal[3];
    int materialId;
} kdpt_shadeable_intersection;

/* Everything pathtraceInit reads from Scene (src/pathtrace.cu:201-272). */
typedef struct kdpt_scene {
    kdpt_camera camera;        /* hst_scene->state.camera (after runCuda's camera update) */
    int traceDepth;            /* hst_scene->state.traceDepth */
    const kdpt_geom *geoms;
    int num_geoms;
    const kdpt_material *materials;
    int num_materials;
    int has_obj;               /* hst_scene->hasObj */
    const kdpt_node_bare *nodes; /* hst_scene->newNodesBare (ID order) */
    int num_nodes;
    const kdpt_tri_bare *tris; /* hst_scene->newTrianglesBare */
    int num_tris;
    const int *obj_materialOffsets; /* one per OBJ shape */
    int num_shapes;
    /* enable_kd = 0 only (brute force, pathTraceOneBounce src/pathtrace.cu:402-628): the raw OBJ arrays
       pathtraceInit uploads in that mode (src/pathtrace.cu:225-257), as Scene::loadObj builds them
       (src/scene.cpp:603-712).  Ignored when enable_kd = 1. */
    const float *obj_verts;      /* attrib.vertices: 3 floats per vertex index */
    int num_obj_verts;           /* floats */
    const float *obj_norms;      /* attrib.normals, read at 3*vertex_index like the reference */
    int num_obj_norms;           /* floats */
    const int *obj_polyoffsets;  /* per shape: number of vertex indices (3 per triangle) */
    const int *obj_polysidxflat; /* vertex indices, shape after shape */
    int polyidxcount;
    const float *obj_bboxes;     /* Scene::obj_bboxes; shape i's box is read at [i .. i+5] (use_bbox) */
    int num_bbox_floats;
} kdpt_scene;

/* The flags of pathtrace() with src/main.cpp:35-60 defaults (kdpt_default_options). */
typedef struct kdpt_options {
    float focal_length;  /* dofDistance, 6 */
    float dof_angle;     /* dofAngle, 0 */
    float softness;      /* 0 */
    int cacherays;       /* 0: regenerate camera rays every iteration */
    int antialias;       /* 1 */
    int enable_sss;      /* 0 */
    int testing_mode;    /* 0: 1 = also time the intersect kernel per bounce (TESTINGMODE) */
    int compaction;      /* 1 */
    int enable_kd;       /* 1; 0 = brute force over the OBJ arrays (pathTraceOneBounce) */
    int viz_kd;          /* 0; 1 = KD node boxes drawn as boxes (pathTraceOneBounceKDbareBoxes) */
    int use_bbox;        /* 0; brute force only: each shape's bbox test first (src/pathtrace.cu:497-513) */
    int short_stack;     /* 1: traverseKDbareShortHybrid, 0: traverseKDbare */
    int bounce_cap;      /* 8 == `depth > 7` (src/pathtrace.cu:2608); 16 for the stress config */
    int block_size;      /* 0 = default (256) */
    float *external_image; /* optional device float[3*W*H] to accumulate into (e.g. an RCCL buffer) */
} kdpt_options;

typedef struct kdpt_stats {
    long long segments;          /* sum over bounces of paths launched into the intersect kernel */
    long long seg_per_bounce[32];
    int bounces;                 /* bounces launched in the last iteration */
    int iterations;              /* iterations traced since create/reset */
    float ms_last_iteration;     /* hipEvent time of the last kdpt_trace_iteration (gen .. last gather) */
    float ms_intersect;          /* testing_mode: sum of intersect-kernel time, last iteration */
    long long total_segments;    /* since create/reset */
    double intersect_ms_total;   /* testing_mode: intersect-kernel time summed over launches since reset */
    long long intersect_launches_total; /* ... and the number of those launches */
    double intersect_device_ms_total;   /* intersect launches on the device clock (first block start to
                                           last block end), summed since reset -- unlike the events,
                                           not inflated by queueing when iterations overlap */
    long long intersect_device_launches_total;
    float intersect_grid_share;  /* fraction of the persistent intersect grid one launch used in the last
                                    kdpt_trace_iterations (1 for one-at-a-time tracing) */
    long long total_trace_rays;  /* since create/reset: rays handed to the KD traversal kernel (k_trace), i.e.
                                    the segments whose ray meets the KD root box */
    double create_ms;            /* host wall time of kdpt_create (uploads, cluster build, masks, kernel setup) */
    double mask_build_ms;        /* ... of which the masked cull's direction masks (built on the device; 0: none) */
} kdpt_stats;

typedef struct kdpt_ctx kdpt_ctx;

void kdpt_default_options(kdpt_options *opt);

/* pathtraceInit: allocate + upload (geoms, materials, nodes, triangles, offsets). */
int kdpt_create(const kdpt_scene *scene, const kdpt_options *opt, int device, kdpt_ctx **out);
/* pathtrace(pbo, frame, iter, ...): one iteration (1 sample per pixel); iter is 1-based and
 * seeds the RNG.  Synchronous on return, like the reference. */
int kdpt_trace_iteration(kdpt_ctx *ctx, int frame, int iter);
/* Iterations first_iter + k*stride (k < count), in batches of `batch` (<= 16) that share each bounce's
 * intersect launch, with `pipeline` batches in flight at once (each on its own stream and buffers).
 * Partial images are added into the image in iteration order, so the result is bit-identical to
 * calling kdpt_trace_iteration for each.  Returns after enqueueing; follow with kdpt_synchronize.
 * Stats: iterations, total_segments and the intersect totals. */
int kdpt_trace_iterations(kdpt_ctx *ctx, int frame, int first_iter, int count, int stride, int pipeline,
                          int batch);
/* As kdpt_trace_iteration but returns after enqueueing (no host sync, no stats). */
int kdpt_trace_iteration_async(kdpt_ctx *ctx, int frame, int iter);
int kdpt_synchronize(kdpt_ctx *ctx);
/* The float3 accumulation image (sum over iterations, not averaged): 3*W*H floats. */
int kdpt_read_image(kdpt_ctx *ctx, float *rgb);
/* sendImageToPBO (src/pathtrace.cu:69-89) into uchar4[W*H] (x,y,z,w bytes).  `rgba` may be device memory
 * (the reference's GL-mapped PBO: written by the kernel directly) or host memory (copied out through a
 * staging buffer the context keeps).  Synchronous. */
int kdpt_write_pbo(kdpt_ctx *ctx, int iter, uint8_t *rgba);
int kdpt_reset(kdpt_ctx *ctx);

/* ---- Headless output (saveImage, src/main.cpp:1087-1108 + image::savePNG/saveHDR, src/image.cpp:22-45) ---- */
/* The bytes savePNG encodes: x-flipped, image / samples, glm::clamp(0, 1) * 255.f, (unsigned char). */
int kdpt_save_rgb8(kdpt_ctx *ctx, float samples, uint8_t *rgb);
/* image::savePNG / image::saveHDR of the current image (stb_image_write's encoders, restated). */
int kdpt_save_png(kdpt_ctx *ctx, const char *path, float samples);
int kdpt_save_hdr(kdpt_ctx *ctx, const char *path, float samples);
/* The encoders alone (host; no device needed).  *out is malloc'd: release with kdpt_free. */
int kdpt_png_encode(const uint8_t *rgb, int w, int h, uint8_t **out, size_t *len);
int kdpt_write_png(const char *path, const uint8_t *rgb, int w, int h);
int kdpt_hdr_encode(const float *rgb, int w, int h, uint8_t **out, size_t *len);
int kdpt_write_hdr(const char *path, const float *rgb, int w, int h);
void kdpt_free(void *p);
int kdpt_get_stats(kdpt_ctx *ctx, kdpt_stats *st);
/* pathtrace()'s per-call flags without a new context: focal_length, dof_angle, softness, cacherays,
 * antialias, enable_sss, testing_mode, compaction and short_stack take effect from the next iteration
 * (the accumulation image is kept).  enable_kd, viz_kd, use_bbox, bounce_cap, block_size and
 * external_image must equal the context's (KDPT_ERR_UNSUPPORTED otherwise: they decide what
 * kdpt_create uploads and allocates). */
int kdpt_set_options(kdpt_ctx *ctx, const kdpt_options *opt);
/* Explicit A/B and diagnostic knobs (the library reads no environment variables; a context created
 * without this call always runs the tested default route).  Names: "shade_fused" (1; 0 = k_shade +
 * k_scan + k_scatter), "early_walk" (16) / "early_leaf" (1) (node-phase hand-over thresholds),
 * "chunk_width0..2" (16, 64, 64), "trace_grid_frac" (grid share of every intersect launch, (0, 1]),
 * "tree_global" (0; 1 = KD tree read from HBM/L2 instead of LDS), "profile_batches" (0; 1 = counting intersect kernel for kdpt_wave_profile, 2 = also its
 * per-ray node-step histogram),
 * "shade_batch" (1; 0 = one k_shade_fused launch per iteration instead of one per batch), "gen_geoms" (1;
 * 0 = camera rays and bounce 0's k_geoms as two launches instead of one k_gen_geoms_b),
 * "tree_format" (0 = best fit; 16 / 32 = only that LDS record size), "super_cull" (1; 0 = no two-level
 * super-cluster route), "cluster_slab" (1; 0 = no normal slab in the second cull level), "cluster_obb" (1;
 * 0 = the second level tests the axis-aligned box and the normal slab only, not the oriented box),
 * "super_slab" (1; 0 = the first level tests the super-clusters' boxes only, not their slabs),
 * "flat_obb" (1; 0 = the one-level cluster cull tests the clusters' axis-aligned boxes only, not also
 * their oriented boxes),
 * "cluster_cull" (1; 0 = no cluster / chunk cull at all: every big-leaf cluster is swept, exact by
 * construction), "cull_margin" (0 = the scene's; > 0 overrides the cull's margin coefficient, no masks),
 * "cull_exact" (1; 0 = for meshes of large triangles the margin-only cull instead of the masked exact one, not
 * exact), "cull_mask_n" (the direction masks' cube-map cells per face edge, 1 .. 512; default: the finest of
 * 256 / 128 / 64 ... within 640 MB), "cull_fast_k" (the masked cull's box coefficient, default 1e-3; the masks
 * are rebuilt for it), "reduce_spin_us" (0; > 0: a device spin of that many
 * microseconds on the reduce stream before every frame's reduce, emulating an ncclReduce that waits for a slower
 * peer -- a diagnostic of the frame pipeline; ctx = NULL sets it for contexts created later, e.g. the ones
 * kdpt_render_sharded creates), "sync_debug" (0).  ctx = NULL only (process defaults of the contexts created afterwards):
 * "cluster_chord" (-1: normal cones of chord 0.02 before the Morton runs for meshes whose cull margin is
 * rigorous, Morton runs only otherwise; 0: Morton runs only; > 0: cones of that chord for every mesh -- the
 * cluster layout, same bits), "cu_mask_streams" (1: the context's streams are created with a mask of every CU,
 * each on a hardware queue of its own; 0: plain non-blocking streams, which HIP multiplexes onto
 * GPU_MAX_HW_QUEUES in-order queues).  KDPT_ERR_ARG for an unknown name.  Drops the pipeline slots
 * (they are remade). */
int kdpt_set_tuning(kdpt_ctx *ctx, const char *name, double value);
/* The intersect kernel's configuration: tree source (0 HBM 64-byte records, 1 HBM 32-byte, 2 LDS 32-byte,
 * 3 LDS 16-byte derived-box records + cluster boxes, 4 LDS 16-byte records with cluster boxes in HBM,
 * 5 LDS 16-byte records + super-cluster records (half-precision boxes rounded outward; cluster boxes and
 * normal slabs in HBM, culled in two levels)), workgroup size, persistent grid (workgroups of the full grid)
 * and dynamic LDS bytes per workgroup. */
int kdpt_trace_config(kdpt_ctx *ctx, int *tree_mode, int *block, int *grid, long long *lds_bytes);
/* The big-leaf cluster cull (and the brute-force chunk cull): the margin coefficient in use, the scene's
 * rigorous coefficient, and exact = 1 when the one in use is >= the rigorous one -- the cull then never
 * drops a cluster holding a triangle that passes glm's u/v tests, for any ray ("Cluster cull").
 * For meshes whose triangles are too large for a rigorous margin that still culls (dragon_5), the box levels
 * use a fast coefficient and per-cluster direction masks decide the missed pairs' near-parallel triangles
 * one by one (the masked cull): exact = 1 as well.  exact = 0 after tuning "cull_exact" = 0 or a fixed
 * "cull_margin", and for the brute-force route (enable_kd = 0) of such meshes, whose 64-triangle chunk boxes are
 * culled at the box coefficient (1e-3) without masks: the cull is then conservative except for rays nearly
 * coplanar with a triangle. */
int kdpt_cull_margin(kdpt_ctx *ctx, float *margin, double *rigorous, int *exact);
/* The masked cull's danger masks as the device built them (bucket-major: cell b * num_clusters + c, 6 mask_n^2
 * buckets).  *mask_n = 0 when the scene has none (its cull is exact without them).  masks may be NULL (sizes
 * only); otherwise 6 mask_n^2 num_clusters entries.  For parity tests against the host builder
 * (kdpt_clusters.h build_dir_masks). */
int kdpt_cull_masks(kdpt_ctx *ctx, int *mask_n, int *num_clusters, unsigned long long *masks);

/* ---- Multi-GPU: samples per pixel sharded across GPUs ----
 * Frame f covers global iterations f*spp + 1 .. (f+1)*spp (the RNG seeds, iteration 2's sort and cacherays
 * use these numbers); rank r of N renders those with (iteration - 1 - f*spp) % N == r, in order, into a frame
 * buffer, and one reduce (float sum, to rank 0) per frame over xGMI combines them.  Rank 0 adds each frame
 * into its context's image (kdpt_read_image, kdpt_save_png) and copies it to `out` when given.  With one
 * rank, one frame and a zero image, the image equals kdpt_trace_iterations(first, spp, stride 1) bit for bit;
 * with N ranks it equals the rank partial sums added in the reduce's order.  The calls queue their work and
 * return (kdpt_synchronize waits); frame f + 1 renders while frame f is reduced.  RCCL (librccl.so.1) is
 * loaded at run time; KDPT_ERR_UNSUPPORTED when it is absent.
 * Replaces the reference's single-GPU pathtrace() loop (src/pathtrace.cu:2405-2635, src/main.cpp runCuda). */
#define KDPT_COMM_ID_BYTES 128
#define KDPT_REDUCE_RCCL 0  /* ncclReduce (one communicator rank per context) */
#define KDPT_REDUCE_COPY 1  /* in-process: peer copies to the first device, added in rank order */
/* One process per GPU: rank 0 makes the id, the caller hands it to every rank (any channel), and each rank
 * joins with its context (collective: every rank must call it).  An id is single-use: every communicator (every
 * kdpt_comm_init round over the ranks) needs a fresh kdpt_comm_unique_id -- reusing one makes RCCL fail
 * ("remote process exited or there was a network error").  id = NULL with nranks > 1: no
 * communicator; kdpt_render_frames then copies every rank's frame shares to its `out` and the caller reduces
 * them (e.g. over gloo when ranks share a GPU, which RCCL refuses); the image is left alone. */
int kdpt_comm_unique_id(unsigned char *id);
/* id given: a communicator for any nranks >= 1 (one rank runs the same per-frame ncclReduce as N). */
int kdpt_comm_init(kdpt_ctx *ctx, int nranks, int rank, const unsigned char *id);
/* The path of the RCCL library whose ncclReduce the calls use (dladdr; in a torch process torch's copy when
 * it was loaded first).  KDPT_ERR_UNSUPPORTED when no librccl.so.1 can be loaded. */
int kdpt_comm_library(char *path, int len);
/* This rank's share of frames first_frame .. first_frame + frames - 1 (every rank calls it with the same
 * arguments); out: rank 0, frames * 3*W*H floats, device or host memory, or NULL. */
int kdpt_render_frames(kdpt_ctx *ctx, int first_frame, int frames, int spp, int pipeline, int batch, float *out);
/* (a pageable host `out` is pinned for the copies -- hipHostRegister -- until kdpt_synchronize; it must stay
 * allocated until kdpt_synchronize returns, and two contexts must not render into one `out` range at once) */
/* One process, one context per device (devices[0..ndev), <= 8; a device may repeat with KDPT_REDUCE_COPY):
 * renders the frames, waits, and frees everything.  out (host or device 0 memory, frames * 3*W*H floats, or
 * NULL) receives each frame's reduced image. */
int kdpt_render_sharded(const kdpt_scene *scene, const kdpt_options *opt, int ndev, const int *devices,
                        int first_frame, int frames, int spp, int pipeline, int batch, int reduce, float *out);
int kdpt_destroy(kdpt_ctx *ctx);
const char *kdpt_last_error(void);

/* Device pointer of the accumulation image (for an in-place RCCL reduce). */
int kdpt_image_device_ptr(kdpt_ctx *ctx, void **dptr);
/* Debug / parity: run iteration `iter` through bounce `stop_depth` (0-based) and copy the
 * live PathSegment array (reference layout) to host `out` (>= W*H entries). */
int kdpt_debug_paths(kdpt_ctx *ctx, int iter, int stop_depth, kdpt_path_segment *out, int *npaths);
/* Roofline counters: one extra, untimed iteration that also counts AABB tests, triangle
 * tests and triangle hits (aabb_tri_hit[3]); the image is not touched.  Afterwards kdpt_get_stats
 * reports that iteration's segments and seg_per_bounce. */
int kdpt_count_iteration(kdpt_ctx *ctx, int iter, unsigned long long *aabb_tri_hit);
/* Of the last kdpt_count_iteration: the AABB tests done before the intersect kernel (the root-box test of
 * the rays that miss the KD root, made by k_geoms / the previous bounce's shading pass) and the number of
 * ray segments handed to the intersect kernel (aabb_prep_cand[2]). */
int kdpt_count_split(kdpt_ctx *ctx, unsigned long long *aabb_prep_cand);
/* Diagnostic: cycle profile of the intersect kernel during the last kdpt_count_iteration.
 * Copies up to n values -- node trips, node cycles, big-leaf sweeps, big-leaf cycles,
 * small-leaf phases, small-leaf rounds, small-leaf cycles, recombination cycles, setup
 * cycles, analytic-geometry cycles, post cycles, node lane-steps, big leaves swept, their
 * clusters, clusters tested with a u/v pass, ... with several, small-leaf (ray, triangle) pairs,
 * node-trip lanes waiting on a leaf, ... finished, cycles after the ray queue ran dry, finished
 * node-trip lanes then (each summed over waves), waves, wave cycles, aabb, tri, hit, then a 64-bin
 * histogram of intersect-wave lifetimes
 * (10 us bins), a 64-bin histogram of node steps per ray (bins of 4), and node steps summed / rays counted
 * by the ray's chord through the KD root box (8 bins, eighths of its diagonal) -- and returns how many exist. */
int kdpt_wave_profile(kdpt_ctx *ctx, unsigned long long *out, int n);
/* Device-math known answers: sinf/cosf/pow-5 Fresnel/u01 evaluated by the gfx950 code. */
int kdpt_selftest_math(const float *x, int n, float *sin_out, float *cos_out);
int kdpt_selftest_rng(const int *iter_idx_depth, int n, int k, float *u_out);
/* The first k uniform draws (n x k) of thrust::default_random_engine + uniform_real_distribution<float>
 * as the device restates them, per input: mode 0 makeSeededRandomEngine(iter, index, depth) of int
 * triples (src/pathtrace.cu:62-66), 1 the camera jitter's engine(utilhash(iter)) (src/pathtrace.cu:334),
 * 2 engine(seed) of raw uint32 seeds.  Pinned to rocThrust by tests/golden/ref_pins.json. */
int kdpt_selftest_rng_draws(int mode, const uint32_t *in, int n, int k, float *out);
int kdpt_selftest_fresnel(const float *cosines, int n, float ior, float *f_out);
/* The glm pieces on the path (kdpt_device.h glm_kat, vendored glm 0.9.6.3 restated): fn 0
 * intersectRayTriangle (15 floats in -> {passed, bary.xyz}; `out` holds sentinels on entry, kept where
 * glm leaves bary unwritten), 1 normalize (3 -> 3), 2 reflect (6 -> 3), 3 refract (7 -> 3),
 * 4 glm::rotate(quat, vec3) (7 -> 3).  Run on the device. */
int kdpt_selftest_glm(int fn, const float *in, int n, float *out);
/* The scatter's glibc calls as restated for gfx950 (src/interactions.h:67-83,214): fn 0 acosf(x),
 * 1 sin((double)x), 2 cos((double)x); results as doubles. */
int kdpt_selftest_libm(int fn, const float *x, int n, double *out);
/* Order-independent digest of fn over the float bit patterns first .. first+count-1 (count <= 2^32):
 * sum mod 2^64 of splitmix64(result bits ^ splitmix64(input bits)); the oracle's orc_libm_digest
 * computes the same with the host glibc. */
int kdpt_selftest_libm_digest(int fn, uint32_t first, unsigned long long count, unsigned long long *digest);

/* ---- Host scene building (C++ restatement of the reference's host code) ---- */
typedef struct kdpt_scene_data kdpt_scene_data;

/* Scene text (src/scene.cpp:7-271) + optional OBJ (src/scene.cpp:579-968, tinyobjloader)
 * + the runCuda camera (src/main.cpp:1059-1073,1111-1129).  Overrides <= 0 keep the file
 * values; a resolution override recomputes pixelLength with the loadCamera formula. */
int kdpt_scene_load(const char *scene_path, const char *obj_path, int res_w, int res_h, int depth,
                    kdpt_scene_data **out);

/* kdpt_scene_load with the KD tree built on GPU `device` (byte-identical; see kdpt_scene_build_device). */
int kdpt_scene_load_device(const char *scene_path, const char *obj_path, int res_w, int res_h, int depth,
                           int device, kdpt_scene_data **out);

/* The same from already-parsed values (what the parsers produce; fixtures use this). */
typedef struct kdpt_scene_desc {
    int res[2];
    float fovy;
    int iterations;
    int traceDepth;
    float eye[3], lookAt[3], up[3];
    int num_materials;
    const kdpt_material *materials;
    int num_geoms;
    const int *geom_type;
    const int *geom_material;
    const float *geom_trs;          /* per geom: translation[3], rotation[3], scale[3] */
    int ntri;                       /* 0: no OBJ */
    const float *verts9, *norms9;   /* per triangle, vertex-index-gathered normals */
    const int *shape_of_tri;
    int num_shapes;
    const kdpt_material *shape_materials;
    int kd_max_depth;               /* 0 = 13, the reference's split(13) */
} kdpt_scene_desc;
int kdpt_scene_build(const kdpt_scene_desc *desc, kdpt_scene_data **out);
/* The same, with the KD tree built on GPU `device` (csrc/kd_build.hip: level by level, breadth first, then
 * pre-order IDs) instead of the host recursion; the arrays are byte-identical to kdpt_scene_build's
 * (KDnode::split src/KDnode.cpp:151-249, Scene::loadObj src/scene.cpp:866-968). */
int kdpt_scene_build_device(const kdpt_scene_desc *desc, int device, kdpt_scene_data **out);
/* Wall time of the GPU KD build of a kdpt_scene_build_device scene (0 for a host build). */
int kdpt_scene_kd_build_ms(const kdpt_scene_data *sd, double *ms);
/* The GPU KD build alone over a triangle soup (9 vertex + 9 normal floats and an mtlIdx per triangle, the
 * reference's Triangle order): NodeBare[] in ID order and TriBare[] in leaf order, malloc'd (kdpt_free). */
int kdpt_build_kd_device(const float *verts9, const float *norms9, const int *mtl, int ntri, int maxdepth,
                         int device, kdpt_node_bare **nodes, int *nnodes, kdpt_tri_bare **tris, int *ntris,
                         double *ms);
/* View of the built scene as the C-ABI struct (pointers owned by the scene data). */
int kdpt_scene_view(const kdpt_scene_data *sd, kdpt_scene *out);
int kdpt_scene_free(kdpt_scene_data *sd);

#ifdef __cplusplus
}
#endif
#endif /* KDPT_H */
