/*
 * kdpt_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of reddeupenn/kdtreePathTracerOptimization's host scene
 * builder and its per-sample path-tracing bounce, used as the oracle that the
 * MI355X HIP path is checked against.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - KD builder: rnd/houdini/data -> rnd/houdini/dataout byte-exact KAT
 *     (the reference's only committed known answer), plus byte equality with
 *     oracle/_ref (the reference's own KDnode.cpp/KDtree.cpp/tiny_obj_loader.cpp
 *     compiled from /root/reference by oracle/ref/Makefile).
 *   - Render path: segment counts and image sums the survey measured by running
 *     the reference's own kernels host-side (SURVEY.md section 8(c) anchor table).
 *
 * All structs below keep the reference's byte layout.
 */
#ifndef KDPT_ORACLE_H
#define KDPT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/sceneStructs.h:22-31 */
typedef struct {
    int type; /* 0 = SPHERE, 1 = CUBE (enum GeomType) */
    int materialid;
    float translation[3];
    float rotation[3];
    float scale[3];
    float transform[16];        /* column-major glm::mat4 */
    float inverseTransform[16];
    float invTranspose[16];
} orc_geom;

/* src/sceneStructs.h:33-44 */
typedef struct {
    float color[3];
    float spec_exponent;
    float spec_color[3];
    float hasReflective;
    float hasRefractive;
    float indexOfRefraction;
    float emittance;
    float transmittance[3];
} orc_material;

/* src/sceneStructs.h:46-55 */
typedef struct {
    int resolution[2];
    float position[3];
    float lookAt[3];
    float view[3];
    float up[3];
    float right[3];
    float fov[2];
    float pixelLength[2];
} orc_camera;

/* src/KDnode.h:64-82 */
typedef struct {
    int axis;
    float splitPos;
    float mins[3];
    float maxs[3];
    int ID, parentID, leftID, rightID;
    int triIdStart, triIdSize;
    float tmin, tmax;
} orc_node;

/* src/KDnode.h:51-62 */
typedef struct {
    float x1, x2, x3, y1, y2, y3, z1, z2, z3;
    float nx1, nx2, nx3, ny1, ny2, ny3, nz1, nz2, nz3;
    int mtlIdx;
} orc_tri;

/* src/sceneStructs.h:15-20,65-71 */
typedef struct {
    float origin[3];
    float direction[3];
    uint8_t isinside;
    uint8_t pad_[3];
    float sdepth;
    float color[3];
    int pixelIndex;
    int remainingBounces;
    int materialIdHit;
} orc_path;

/* src/sceneStructs.h:81-85 */
typedef struct {
    float t;
    float surfaceNormal[3];
    int materialId;
} orc_isect;

typedef struct {
    orc_camera camera;
    int iterations;
    int traceDepth;
    int num_geoms, num_materials;
    orc_geom *geoms;
    orc_material *materials;
    int has_obj;
    int num_shapes;
    int *obj_materialOffsets;
    int num_nodes, num_tris;
    orc_node *nodes;
    orc_tri *tris;
    /* enable_kd == false (pathTraceOneBounce): the raw OBJ arrays, src/scene.cpp:603-712 */
    int polyidxcount;
    float *obj_verts, *obj_norms;
    int *obj_polysidxflat, *obj_polyoffsets;
    float *obj_bboxes;
    int num_bbox_floats;
} orc_scene;

/* Flags of pathtrace() (src/pathtrace.h:6-21, defaults src/main.cpp:35-60). */
typedef struct {
    float focalLength;   /* dofDistance = 6 */
    float dofAngle;      /* 0 */
    int cacherays;       /* 0 */
    int antialias;       /* 1 */
    float softness;      /* 0 */
    int enableSss;       /* 0 */
    int compaction;      /* 1 */
    int shortstack;      /* 1 */
    int bounce_cap;      /* 8 == the reference's hard-coded `depth > 7` (src/pathtrace.cu:2608) */
    int enable_kd;       /* 1; 0 = brute-force pathTraceOneBounce (src/pathtrace.cu:402-628) */
    int usebbox;         /* 0; brute force only: per-shape bbox test first */
    int vizkd;           /* 0; 1 = pathTraceOneBounceKDbareBoxes (KD node boxes drawn as boxes) */
} orc_opts;

typedef struct {
    long long segments;   /* sum over bounces of paths launched into the intersect kernel */
    long long aabb_tests; /* intersectAABBarrays calls */
    long long tri_tests;  /* glm::intersectRayTriangle calls */
    long long tri_hits;   /* intersectRayTriangle returned true */
    int bounces;          /* bounces executed in the last iteration */
    long long seg_per_bounce[32];
} orc_stats;

/* A parsed-but-unbuilt scene: exactly the values the reference's parsers
 * produce (scene text: src/scene.cpp:118-271; OBJ: tinyobjloader) before any
 * matrix, camera or KD work.  Fixtures under tests/golden/ store this form. */
typedef struct {
    int res[2];
    float fovy;
    int iterations;
    int traceDepth;
    float eye[3], lookAt[3], up[3];
    int num_materials;
    const orc_material *materials;
    int num_geoms;
    const int *geom_type;      /* per geom: 0 sphere, 1 cube */
    const int *geom_material;  /* per geom */
    const float *geom_trs;     /* per geom: translation[3], rotation[3], scale[3] */
    int ntri;                  /* 0: no OBJ */
    const float *verts9, *norms9;
    const int *shape_of_tri;
    int num_shapes;
    const orc_material *shape_materials;
} orc_scene_desc;

void orc_default_opts(orc_opts *o);

/* Build matrices (src/utilities.cpp:256-263, glm inverse/inverseTranspose),
 * the loadCamera/runCuda camera and the KD tree (split(13)) from a desc. */
int orc_build_scene(const orc_scene_desc *d, orc_scene *out);

/* Parse scene text (+ optional OBJ) into a desc; arrays are malloc'd and must
 * be released with orc_free_desc. */
int orc_parse_scene(const char *scene_path, const char *obj_path, orc_scene_desc *d);
void orc_free_desc(orc_scene_desc *d);

/* Scene text (src/scene.cpp:7-271) + optional OBJ (src/scene.cpp:579-968) +
 * the runCuda camera (src/main.cpp:1059-1073,1111-1129).  res_w/res_h/depth
 * overrides <= 0 keep the file values; a resolution override recomputes
 * pixelLength with the loadCamera formula (src/scene.cpp:216-223). */
int orc_load_scene(const char *scene_path, const char *obj_path, int res_w, int res_h,
                   int depth, orc_scene *out);
void orc_free_scene(orc_scene *s);

/* KD-tree known-answer: KDtree(path) + updateBbox + split(maxdepth) + writeKDtoFile
 * (src/KDtree.cpp:35-135, src/KDnode.cpp:112-249). Writes the pre-order bbox dump. */
int orc_kd_kat(const char *tri_file, int maxdepth, const char *out_path);

/* Build + flatten a KD tree from a triangle soup (9 vertex + 9 normal floats and
 * an mtlIdx per triangle), exactly as Scene::loadObj does (src/scene.cpp:866-968). */
int orc_build_kd(const float *verts9, const float *norms9, const int *mtl, int ntri,
                 int maxdepth, orc_node **nodes, int *nnodes, orc_tri **tris, int *ntris);
void orc_free(void *p);

/* Parse an OBJ (+ its mtllib) with tinyobjloader's semantics and emit the
 * scene-side arrays Scene::loadObj builds: per-triangle vertices/normals
 * (normals gathered by VERTEX index, src/scene.cpp:545-567), shape index, and
 * per-shape materials (src/scene.cpp:716-822). */
int orc_load_obj(const char *obj_path, float **verts9, float **norms9, int **shape_of_tri,
                 int *ntri, orc_material **mats, int *nshapes);

/* Render iterations [iter_first, iter_first+iter_count) (1-based iter, the RNG
 * seed) accumulating into image (3*W*H floats, caller-zeroed), exactly like
 * repeated pathtrace() calls (src/pathtrace.cu:2405-2635).  nthreads<=0: all. */
int orc_render(const orc_scene *s, const orc_opts *o, int iter_first, int iter_count,
               float *image, orc_stats *stats, int nthreads);

/* Debug: run iteration `iter` through bounce `stop_depth` (0-based) and copy the
 * path array (after compaction/sort of that bounce) to out (>= W*H entries). */
int orc_paths_after(const orc_scene *s, const orc_opts *o, int iter, int stop_depth,
                    orc_path *out, int *npaths);

/* One ray through the geoms + KD traversal of pathTraceOneBounceKDbare (no scatter).
 * out[0]=t_min out[1]=hit_geom_index out[2..4]=intersect point out[5..7]=normal
 * out[8]=obj_intersect out[9]=objMaterialIdx out[10..12]=aabb/tri/hit tests out[13]=leaves visited (size > 0). */
int orc_trace_ray(const orc_scene *s, const float *origin, const float *direction, int hybrid, double *out);

/* saveImage + image::savePNG's bytes (src/main.cpp:1087-1108, src/image.cpp:22-35); lin may be NULL. */
void orc_save_image(const float *image, int W, int H, float samples, unsigned char *rgb, float *lin);

/* Device-math known answers shared with the HIP tests. */
unsigned int orc_utilhash(unsigned int a);
float orc_u01_sequence(int iter, int index, int depth, int k); /* k-th uniform */
float orc_sinf(float x);  /* the libm call the reference makes (glibc) */
float orc_cosf(float x);
void orc_sincos_array(const float *x, int n, float *s, float *c);
/* u01 draws: for each (iter, index, depth) triple, the k-th uniform of makeSeededRandomEngine */
void orc_u01_array(const int *iid, int n, int k, float *u);
/* first k draws per input, n x k: mode 0 seeded triples, 1 camera engine(utilhash(iter)), 2 raw seeds */
void orc_rng_draws(int mode, const unsigned int *in, int n, int k, float *out);
/* glibc acosf(x) (fn 0), sin((double)x) (1), cos((double)x) (2), as doubles */
void orc_libm_array(int fn, const float *x, int n, double *out);
/* order-independent digest of fn over the float bit patterns first .. first+count-1:
   sum of splitmix64(result bits ^ splitmix64(input bits)) (kdpt_selftest_libm_digest computes the same) */
uint64_t orc_libm_digest(int fn, uint32_t first, uint64_t count);
/* glm known answers (kdpt_selftest_glm's numbering): 0 intersectRayTriangle, 1 normalize, 2 reflect,
 * 3 refract, 4 glm::rotate(quat, vec3); out[1..3] of fn 0 hold sentinels on entry */
void orc_glm_array(int fn, const float *in, int n, float *out);
/* Geom matrices: transform, inverse, invTranspose (48 floats) per translation/rotation/scale triple */
void orc_geom_matrices(const float *trs, int n, float *out);
/* getFresnelVal with dot(N,-I) == cosines[i] */
void orc_fresnel_array(const float *cosines, int n, float ior, float *f);

#ifdef __cplusplus
}
#endif
#endif
