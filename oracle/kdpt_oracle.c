/*
 * kdpt_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU oracle (parity checker).
 *
 * A plain-C restatement of reddeupenn/kdtreePathTracerOptimization's
 *   - scene text parser          src/scene.cpp:7-271, src/utilities.cpp:256-303
 *   - tinyobjloader OBJ/MTL parse src/tiny_obj_loader.cpp:160-276,425-1156
 *     (tinyobjloader is MIT, Copyright (c) 2012-2016 Syoyo Fujita and many contributors;
 *     THIRD_PARTY_NOTICES.md)
 *   - KD build + flatten         src/KDnode.cpp:112-249, src/scene.cpp:275-968
 *   - runCuda camera             src/main.cpp:1059-1073,1111-1129
 *   - the per-sample bounce      src/pathtrace.cu:315-397 (camera rays),
 *                                1023-1235 (short-stack hybrid KD traversal),
 *                                881-1020 (standard KD traversal),
 *                                1571-1734 (intersect + scatter kernel),
 *                                2304-2399 (shade / gather), 2405-2635 (driver)
 *   - device math                src/intersections.h, src/interactions.h and the
 *                                vendored glm 0.9.6.3 functions they call
 *   - thrust minstd_rand + uniform_real_distribution<float> (rocThrust 7.2's
 *     restatement: /opt/rocm/include/thrust/random/detail/ *.inl)
 *
 * Compiled with -ffp-contract=off (no FMA contraction) and without
 * -ffast-math so that every float/double operation is the single IEEE
 * operation the reference source spells.  libm calls (sinf/cosf/tanf/atanf/
 * acosf/pow/ldexp) are the system glibc's, as the reference's host build does.
 *
 * Documented definitions of the reference's undefined behaviour (SURVEY.md 5,
 * 8(a) a5): visited-bitmap writes to nodeIDs[-1] go to a sink slot that is read
 * back by the "skip other side" line; the bitmap is sized numNodes+1 (no 4000
 * cap); unqualified min/max in intersectAABBarrays are std::min/std::max.
 *
 * Nothing in the product (kdtreepathtraceroptimization_amd/) links this file.
 */
#define _GNU_SOURCE
#include "kdpt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* src/utilities.h:9-12 */
#define PI_F 3.1415926535897932384626422832795028841971f
#define TWO_PI_F 6.2831853071795864769252867665590057683943f
#define SQRT_OF_ONE_THIRD_F 0.5773502691896257645091487805019574556476f

/* ------------------------------------------------------------------ */
/* glm 0.9.6.3 vec3 / mat4 arithmetic, operation order preserved        */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { v4 c[4]; } m4; /* column major, c[col] */

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float vget(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline void vset(v3 *v, int i, float f) { if (i == 0) v->x = f; else if (i == 1) v->y = f; else v->z = f; }
/* glm detail/func_geometric.inl compute_dot<tvec3>: tmp = x*y; tmp.x+tmp.y+tmp.z */
static inline float vdot(v3 a, v3 b) {
    float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return tx + ty + tz;
}
/* glm cross */
static inline v3 vcross(v3 x, v3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* glm normalize = x * inversesqrt(dot(x,x)), inversesqrt = 1/sqrt */
static inline v3 vnormalize(v3 x) { float inv = 1.0f / sqrtf(vdot(x, x)); return vscale(x, inv); }
static inline float vlength(v3 v) { return sqrtf(vdot(v, v)); }
static inline float vdistance(v3 p0, v3 p1) { return vlength(vsub(p1, p0)); }
static inline v4 v4add(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline v4 v4sub(v4 a, v4 b) { return V4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline v4 v4mul(v4 a, v4 b) { return V4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static inline v4 v4scale(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline v4 v4div(v4 a, float s) { return V4(a.x / s, a.y / s, a.z / s, a.w / s); }
static inline float m4get(const m4 *m, int c, int r) { const float *p = &m->c[c].x; return p[r]; }
static inline void m4set(m4 *m, int c, int r, float f) { float *p = &m->c[c].x; p[r] = f; }

static m4 m4identity(void) {
    m4 m;
    m.c[0] = V4(1, 0, 0, 0); m.c[1] = V4(0, 1, 0, 0); m.c[2] = V4(0, 0, 1, 0); m.c[3] = V4(0, 0, 0, 1);
    return m;
}
/* glm detail/type_mat4x4.inl:592-638 -- (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
static inline v4 m4mulv(const m4 *m, v4 v) {
    v4 add0 = v4add(v4scale(m->c[0], v.x), v4scale(m->c[1], v.y));
    v4 add1 = v4add(v4scale(m->c[2], v.z), v4scale(m->c[3], v.w));
    return v4add(add0, add1);
}
static inline v3 multiplyMV(const m4 *m, v4 v) { v4 r = m4mulv(m, v); return V3(r.x, r.y, r.z); }
/* glm detail/type_mat4x4.inl:686-703 */
static m4 m4mul(const m4 *a, const m4 *b) {
    m4 r;
    for (int i = 0; i < 4; i++) {
        v4 t = v4add(v4add(v4add(v4scale(a->c[0], b->c[i].x), v4scale(a->c[1], b->c[i].y)),
                           v4scale(a->c[2], b->c[i].z)),
                     v4scale(a->c[3], b->c[i].w));
        r.c[i] = t;
    }
    return r;
}
/* glm gtc/matrix_transform.inl translate */
static m4 m4translate(const m4 *m, v3 v) {
    m4 r = *m;
    r.c[3] = v4add(v4add(v4add(v4scale(m->c[0], v.x), v4scale(m->c[1], v.y)), v4scale(m->c[2], v.z)), m->c[3]);
    return r;
}
/* glm gtc/matrix_transform.inl rotate (cos/sin of a float angle -> cosf/sinf) */
static m4 m4rotate(const m4 *m, float angle, v3 v) {
    float a = angle, c = cosf(a), s = sinf(a);
    v3 axis = vnormalize(v);
    v3 temp = vscale(axis, 1.0f - c); /* (T(1) - c) * axis */
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
    m4 r;
    for (int i = 0; i < 3; i++)
        r.c[i] = v4add(v4add(v4scale(m->c[0], R[i][0]), v4scale(m->c[1], R[i][1])), v4scale(m->c[2], R[i][2]));
    r.c[3] = m->c[3];
    return r;
}
static m4 m4scalev(const m4 *m, v3 v) {
    m4 r;
    r.c[0] = v4scale(m->c[0], v.x); r.c[1] = v4scale(m->c[1], v.y); r.c[2] = v4scale(m->c[2], v.z); r.c[3] = m->c[3];
    return r;
}
/* glm detail/type_mat4x4.inl:37-92 compute_inverse */
static m4 m4inverse(const m4 *mm) {
#define M(c, r) m4get(mm, c, r)
    float Coef00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float Coef02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float Coef03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float Coef04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float Coef06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float Coef07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float Coef08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float Coef10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float Coef11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float Coef12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float Coef14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float Coef15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float Coef16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float Coef18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float Coef19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float Coef20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float Coef22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float Coef23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    v4 Fac0 = V4(Coef00, Coef00, Coef02, Coef03);
    v4 Fac1 = V4(Coef04, Coef04, Coef06, Coef07);
    v4 Fac2 = V4(Coef08, Coef08, Coef10, Coef11);
    v4 Fac3 = V4(Coef12, Coef12, Coef14, Coef15);
    v4 Fac4 = V4(Coef16, Coef16, Coef18, Coef19);
    v4 Fac5 = V4(Coef20, Coef20, Coef22, Coef23);
    v4 Vec0 = V4(M(1, 0), M(0, 0), M(0, 0), M(0, 0));
    v4 Vec1 = V4(M(1, 1), M(0, 1), M(0, 1), M(0, 1));
    v4 Vec2 = V4(M(1, 2), M(0, 2), M(0, 2), M(0, 2));
    v4 Vec3 = V4(M(1, 3), M(0, 3), M(0, 3), M(0, 3));
    v4 Inv0 = v4add(v4sub(v4mul(Vec1, Fac0), v4mul(Vec2, Fac1)), v4mul(Vec3, Fac2));
    v4 Inv1 = v4add(v4sub(v4mul(Vec0, Fac0), v4mul(Vec2, Fac3)), v4mul(Vec3, Fac4));
    v4 Inv2 = v4add(v4sub(v4mul(Vec0, Fac1), v4mul(Vec1, Fac3)), v4mul(Vec3, Fac5));
    v4 Inv3 = v4add(v4sub(v4mul(Vec0, Fac2), v4mul(Vec1, Fac4)), v4mul(Vec2, Fac5));
    v4 SignA = V4(+1, -1, +1, -1), SignB = V4(-1, +1, -1, +1);
    m4 Inverse;
    Inverse.c[0] = v4mul(Inv0, SignA); Inverse.c[1] = v4mul(Inv1, SignB);
    Inverse.c[2] = v4mul(Inv2, SignA); Inverse.c[3] = v4mul(Inv3, SignB);
    v4 Row0 = V4(Inverse.c[0].x, Inverse.c[1].x, Inverse.c[2].x, Inverse.c[3].x);
    v4 Dot0 = v4mul(mm->c[0], Row0);
    float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
    float OneOverDeterminant = 1.0f / Dot1;
    m4 r;
    for (int i = 0; i < 4; i++) r.c[i] = v4scale(Inverse.c[i], OneOverDeterminant);
    return r;
#undef M
}
/* glm gtc/matrix_inverse.inl:95-147 inverseTranspose */
static m4 m4inverseTranspose(const m4 *mm) {
#define M(c, r) m4get(mm, c, r)
    float S00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float S01 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float S02 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float S03 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float S04 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float S05 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float S06 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float S07 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float S08 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float S09 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float S10 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float S11 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float S12 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float S13 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float S14 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float S15 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float S16 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float S17 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float S18 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    m4 I;
    m4set(&I, 0, 0, +(M(1, 1) * S00 - M(1, 2) * S01 + M(1, 3) * S02));
    m4set(&I, 0, 1, -(M(1, 0) * S00 - M(1, 2) * S03 + M(1, 3) * S04));
    m4set(&I, 0, 2, +(M(1, 0) * S01 - M(1, 1) * S03 + M(1, 3) * S05));
    m4set(&I, 0, 3, -(M(1, 0) * S02 - M(1, 1) * S04 + M(1, 2) * S05));
    m4set(&I, 1, 0, -(M(0, 1) * S00 - M(0, 2) * S01 + M(0, 3) * S02));
    m4set(&I, 1, 1, +(M(0, 0) * S00 - M(0, 2) * S03 + M(0, 3) * S04));
    m4set(&I, 1, 2, -(M(0, 0) * S01 - M(0, 1) * S03 + M(0, 3) * S05));
    m4set(&I, 1, 3, +(M(0, 0) * S02 - M(0, 1) * S04 + M(0, 2) * S05));
    m4set(&I, 2, 0, +(M(0, 1) * S06 - M(0, 2) * S07 + M(0, 3) * S08));
    m4set(&I, 2, 1, -(M(0, 0) * S06 - M(0, 2) * S09 + M(0, 3) * S10));
    m4set(&I, 2, 2, +(M(0, 0) * S11 - M(0, 1) * S09 + M(0, 3) * S12));
    m4set(&I, 2, 3, -(M(0, 0) * S08 - M(0, 1) * S10 + M(0, 2) * S12));
    m4set(&I, 3, 0, -(M(0, 1) * S13 - M(0, 2) * S14 + M(0, 3) * S15));
    m4set(&I, 3, 1, +(M(0, 0) * S13 - M(0, 2) * S16 + M(0, 3) * S17));
    m4set(&I, 3, 2, -(M(0, 0) * S14 - M(0, 1) * S16 + M(0, 3) * S18));
    m4set(&I, 3, 3, +(M(0, 0) * S15 - M(0, 1) * S17 + M(0, 2) * S18));
    float Determinant = +M(0, 0) * m4get(&I, 0, 0) + M(0, 1) * m4get(&I, 0, 1) + M(0, 2) * m4get(&I, 0, 2) +
                        M(0, 3) * m4get(&I, 0, 3);
    for (int i = 0; i < 4; i++) I.c[i] = v4div(I.c[i], Determinant);
    return I;
#undef M
}
/* src/utilities.cpp:256-263 */
static m4 buildTransformationMatrix(v3 translation, v3 rotation, v3 scale) {
    m4 id = m4identity();
    m4 translationMat = m4translate(&id, translation);
    m4 rotationMat = m4rotate(&id, rotation.x * (float)PI_F / 180.0f, V3(1, 0, 0));
    m4 r2 = m4rotate(&id, rotation.y * (float)PI_F / 180.0f, V3(0, 1, 0));
    rotationMat = m4mul(&rotationMat, &r2);
    m4 r3 = m4rotate(&id, rotation.z * (float)PI_F / 180.0f, V3(0, 0, 1));
    rotationMat = m4mul(&rotationMat, &r3);
    m4 scaleMat = m4scalev(&id, scale);
    m4 tr = m4mul(&translationMat, &rotationMat);
    return m4mul(&tr, &scaleMat);
}

/* ------------------------------------------------------------------ */
/* RNG: utilhash (src/intersections.h:15-23), thrust minstd_rand,        */
/* uniform_real_distribution<float>(0,1), makeSeededRandomEngine        */
/* (src/pathtrace.cu:62-66)                                             */
/* ------------------------------------------------------------------ */
unsigned int orc_utilhash(unsigned int a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}
typedef struct { unsigned int x; } rng_t;
static inline rng_t rng_seed(unsigned int s) {
    rng_t r;
    r.x = s % 2147483647u;
    if (r.x == 0u) r.x = 1u; /* linear_congruential_engine::seed: c%m==0 && s%m==0 -> 1 */
    return r;
}
static inline unsigned int rng_next(rng_t *r) {
    r->x = (unsigned int)(((unsigned long long)r->x * 48271ull) % 2147483647ull);
    return r->x;
}
static inline float u01(rng_t *r) {
    float result = (float)(rng_next(r) - 1u); /* urng() - min, min = 1 */
    result /= (1.0f + (float)(2147483646u - 1u));
    return (result * (1.0f - 0.0f)) + 0.0f;
}
static inline rng_t makeSeededRandomEngine(int iter, int index, int depth) {
    unsigned int a = 0x80000000u | ((unsigned int)depth << 22) | (unsigned int)iter;
    int h = (int)(orc_utilhash(a) ^ orc_utilhash((unsigned int)index));
    return rng_seed((unsigned int)h);
}
float orc_u01_sequence(int iter, int index, int depth, int k) {
    rng_t r = makeSeededRandomEngine(iter, index, depth);
    float u = 0;
    for (int i = 0; i <= k; i++) u = u01(&r);
    return u;
}
float orc_sinf(float x) { return sinf(x); }
float orc_cosf(float x) { return cosf(x); }
void orc_sincos_array(const float *x, int n, float *s, float *c) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) { s[i] = sinf(x[i]); c[i] = cosf(x[i]); }
}
/* glibc acosf / sin / cos as the reference's soft-lobe and fake-SSS scatter calls them
   (src/interactions.h:67-83,214): fn 0 acosf(x), 1 sin((double)x), 2 cos((double)x). */
static uint64_t libm_bits(int fn, float x) {
    if (fn == 0) { float r = acosf(x); uint32_t u; memcpy(&u, &r, 4); return u; }
    double r = fn == 1 ? sin((double)x) : cos((double)x);
    uint64_t u;
    memcpy(&u, &r, 8);
    return u;
}
static uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
void orc_libm_array(int fn, const float *x, int n, double *out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
        uint64_t b = libm_bits(fn, x[i]);
        if (fn == 0) { float r; uint32_t u = (uint32_t)b; memcpy(&r, &u, 4); out[i] = r; }
        else memcpy(&out[i], &b, 8);
    }
}
uint64_t orc_libm_digest(int fn, uint32_t first, uint64_t count) {
    uint64_t acc = 0;
#pragma omp parallel for reduction(+ : acc) schedule(static, 1 << 16)
    for (int64_t k = 0; k < (int64_t)count; k++) {
        uint32_t xb = (uint32_t)(first + (uint64_t)k);
        float x;
        memcpy(&x, &xb, 4);
        acc += splitmix64(libm_bits(fn, x) ^ splitmix64(xb));
    }
    return acc;
}
void orc_u01_array(const int *iid, int n, int k, float *u) {
    for (int i = 0; i < n; i++) u[i] = orc_u01_sequence(iid[3 * i], iid[3 * i + 1], iid[3 * i + 2], k);
}
/* The first k draws of an engine per input, laid out n x k (the layout of oracle/ref/thrust_rng):
   mode 0 makeSeededRandomEngine(iter, index, depth) from int triples (src/pathtrace.cu:62-66),
   mode 1 the camera jitter's engine(utilhash(iter)) (src/pathtrace.cu:334), mode 2 engine(raw seed). */
void orc_rng_draws(int mode, const unsigned int *in, int n, int k, float *out) {
    for (int i = 0; i < n; i++) {
        rng_t r = mode == 0 ? makeSeededRandomEngine((int)in[3 * i], (int)in[3 * i + 1], (int)in[3 * i + 2])
                : mode == 1 ? rng_seed(orc_utilhash(in[i])) : rng_seed(in[i]);
        for (int j = 0; j < k; j++) out[(size_t)i * k + j] = u01(&r);
    }
}

/* ------------------------------------------------------------------ */
/* Intersections (src/intersections.h)                                  */
/* ------------------------------------------------------------------ */
typedef struct { v3 origin, direction; int isinside; float sdepth; } ray_t;

static inline v3 getPointOnRay(ray_t r, float t) { /* :30-32 */
    return vadd(r.origin, vscale(vnormalize(r.direction), t - .0001f));
}
static inline float glm_min(float x, float y) { return x < y ? x : y; }
static inline float glm_max(float x, float y) { return x > y ? x : y; }
static inline float std_min(float a, float b) { return (b < a) ? b : a; }
static inline float std_max(float a, float b) { return (a < b) ? b : a; }

static inline m4 geom_m4(const float *f) { m4 m; memcpy(&m, f, sizeof m); return m; }

/* :107-149 */
static float boxIntersectionTest(const orc_geom *box, ray_t r, v3 *ip, v3 *nrm, int *outside) {
    m4 inv = geom_m4(box->inverseTransform), tr = geom_m4(box->transform);
    ray_t q;
    q.origin = multiplyMV(&inv, V4(r.origin.x, r.origin.y, r.origin.z, 1.0f));
    q.direction = vnormalize(multiplyMV(&inv, V4(r.direction.x, r.direction.y, r.direction.z, 0.0f)));
    float tmin = -1e38f, tmax = 1e38f;
    v3 tmin_n = V3(0, 0, 0), tmax_n = V3(0, 0, 0);
    for (int xyz = 0; xyz < 3; ++xyz) {
        float qd = vget(q.direction, xyz);
        float t1 = (-0.5f - vget(q.origin, xyz)) / qd;
        float t2 = (+0.5f - vget(q.origin, xyz)) / qd;
        float ta = glm_min(t1, t2);
        float tb = glm_max(t1, t2);
        v3 n = V3(0, 0, 0);
        vset(&n, xyz, t2 < t1 ? +1.0f : -1.0f);
        if (ta > 0 && ta > tmin) { tmin = ta; tmin_n = n; }
        if (tb < tmax) { tmax = tb; tmax_n = n; }
    }
    if (tmax >= tmin && tmax > 0) {
        *outside = 1;
        if (tmin <= 0) { tmin = tmax; tmin_n = tmax_n; *outside = 0; }
        v3 p = getPointOnRay(q, tmin);
        *ip = multiplyMV(&tr, V4(p.x, p.y, p.z, 1.0f));
        *nrm = vnormalize(multiplyMV(&tr, V4(tmin_n.x, tmin_n.y, tmin_n.z, 0.0f)));
        return vlength(vsub(r.origin, *ip));
    }
    return -1;
}
/* :161-203 */
static float sphereIntersectionTest(const orc_geom *sphere, ray_t r, v3 *ip, v3 *nrm, int *outside) {
    m4 inv = geom_m4(sphere->inverseTransform), tr = geom_m4(sphere->transform),
       it = geom_m4(sphere->invTranspose);
    float radius = .5f;
    v3 ro = multiplyMV(&inv, V4(r.origin.x, r.origin.y, r.origin.z, 1.0f));
    v3 rd = vnormalize(multiplyMV(&inv, V4(r.direction.x, r.direction.y, r.direction.z, 0.0f)));
    ray_t rt; rt.origin = ro; rt.direction = rd; rt.isinside = 0; rt.sdepth = 0;
    float vDotDirection = vdot(rt.origin, rt.direction);
    float radicand = vDotDirection * vDotDirection - (vdot(rt.origin, rt.origin) - radius * radius);
    if (radicand < 0) return -1;
    float squareRoot = sqrtf(radicand);
    float firstTerm = -vDotDirection;
    float t1 = firstTerm + squareRoot, t2 = firstTerm - squareRoot;
    float t = 0;
    if (t1 < 0 && t2 < 0) return -1;
    else if (t1 > 0 && t2 > 0) { t = std_min(t1, t2); *outside = 1; }
    else { t = std_max(t1, t2); *outside = 0; }
    v3 os = getPointOnRay(rt, t);
    *ip = multiplyMV(&tr, V4(os.x, os.y, os.z, 1.f));
    *nrm = vnormalize(multiplyMV(&it, V4(os.x, os.y, os.z, 0.f)));
    if (!*outside) *nrm = vneg(*nrm);
    return vlength(vsub(r.origin, *ip));
}
/* :253-286 */
static inline int intersectAABBarrays(ray_t r, const float *mins, const float *maxs, float *dist) {
    v3 invdir = V3(1.0f / r.direction.x, 1.0f / r.direction.y, 1.0f / r.direction.z);
    float v1 = (mins[0] - r.origin.x) * invdir.x;
    float v2 = (maxs[0] - r.origin.x) * invdir.x;
    float v3_ = (mins[1] - r.origin.y) * invdir.y;
    float v4_ = (maxs[1] - r.origin.y) * invdir.y;
    float v5 = (mins[2] - r.origin.z) * invdir.z;
    float v6 = (maxs[2] - r.origin.z) * invdir.z;
    float dmin = std_max(std_max(std_min(v1, v2), std_min(v3_, v4_)), std_min(v5, v6));
    float dmax = std_min(std_min(std_max(v1, v2), std_max(v3_, v4_)), std_max(v5, v6));
    if (dmax < 0) { *dist = dmax; return 0; }
    if (dmin > dmax) { *dist = dmax; return 0; }
    *dist = dmin;
    return 1;
}
/* glm gtx/intersect.inl:37-74 (single sided, bary written before early exits) */
static inline int intersectRayTriangle(v3 orig, v3 dir, v3 v0, v3 v1, v3 v2, v3 *bary) {
    v3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    v3 p = vcross(dir, e2);
    float a = vdot(e1, p);
    if (a < FLT_EPSILON) return 0;
    float f = 1.0f / a;
    v3 s = vsub(orig, v0);
    bary->x = f * vdot(s, p);
    if (bary->x < 0.0f) return 0;
    if (bary->x > 1.0f) return 0;
    v3 q = vcross(s, e1);
    bary->y = f * vdot(dir, q);
    if (bary->y < 0.0f) return 0;
    if (bary->y + bary->x > 1.0f) return 0;
    bary->z = f * vdot(e2, q);
    return bary->z >= 0.0f;
}

/* ------------------------------------------------------------------ */
/* Interactions (src/interactions.h)                                    */
/* ------------------------------------------------------------------ */
static v3 calculateRandomDirectionInHemisphere(v3 normal, rng_t *rng) { /* :9-41 */
    float up = sqrtf(u01(rng));
    float over = sqrtf(1 - up * up);
    float around = u01(rng) * TWO_PI_F;
    v3 dnn;
    if (fabsf(normal.x) < SQRT_OF_ONE_THIRD_F) dnn = V3(1, 0, 0);
    else if (fabsf(normal.y) < SQRT_OF_ONE_THIRD_F) dnn = V3(0, 1, 0);
    else dnn = V3(0, 0, 1);
    v3 p1 = vnormalize(vcross(normal, dnn));
    v3 p2 = vnormalize(vcross(normal, p1));
    float ca = cosf(around), sa = sinf(around);
    /* up * normal + cos(around) * over * p1 + sin(around) * over * p2 */
    v3 t0 = vscale(normal, up);
    v3 t1 = vscale(p1, ca * over);
    v3 t2 = vscale(p2, sa * over);
    return vadd(vadd(t0, t1), t2);
}
static v3 rotateVector(v3 n1, v3 axis, float angle) { /* :44-65 */
    axis = vnormalize(axis);
    float u = axis.x, v = axis.y, w = axis.z, x = n1.x, y = n1.y, z = n1.z;
    float ca = cosf(angle), sa = sinf(angle);
    float d = -u * x - v * y - w * z;
    return V3((-u * d) * (1 - ca) + x * ca + (-w * y + v * z) * sa,
              (-v * d) * (1 - ca) + y * ca + (w * x - u * z) * sa,
              (-w * d) * (1 - ca) + z * ca + (-v * x + u * y) * sa);
}
static v3 randSphericalVec(float angle, rng_t *rng) { /* :67-83 */
    double theta = 2 * PI_F * u01(rng);
    double phi = acosf((angle * PI_F * u01(rng) - 1.0f));
    v3 V = V3((float)(cos(theta) * sin(phi)), (float)(sin(theta) * sin(phi)), (float)cos(phi));
    return vnormalize(V);
}
static float getFresnelVal(v3 I, v3 N, float ior) { /* :127-133 */
    float rr = (1.0f - ior) / (1.0f + ior);
    float R0 = rr * rr; /* glm::pow(float, 2.0f) -> pow(x, 2) folds to x*x */
    double F = (double)R0 + (double)(1.0f - R0) * pow((double)(1.0f - vdot(N, vneg(I))), 5.0);
    return (float)F;
}
void orc_fresnel_array(const float *cosines, int n, float ior, float *f) {
    /* getFresnelVal(I, N, ior) with N = (0,0,1) and I chosen so dot(N,-I) == cosines[i] exactly */
    for (int i = 0; i < n; i++) f[i] = getFresnelVal(V3(0.0f, 0.0f, -cosines[i]), V3(0.0f, 0.0f, 1.0f), ior);
}
static v3 glm_reflect(v3 I, v3 N) { return vsub(I, vscale(vscale(N, vdot(N, I)), 2.0f)); }
static v3 glm_refract(v3 I, v3 N, float eta) {
    float dv = vdot(N, I);
    float k = 1.0f - eta * eta * (1.0f - dv * dv);
    v3 r = vsub(vscale(I, eta), vscale(N, eta * dv + sqrtf(k)));
    return vscale(r, (float)(k >= 0.0f));
}
static v3 soft_lobe(v3 dir, rng_t *rng) {
    v3 v = randSphericalVec(0.02f, rng);
    float angle = acosf(vdot(V3(0.0f, 0.0f, -1.0f), dir));
    v3 axis = vnormalize(vcross(V3(0.0f, 0.0f, -1.0f), dir));
    return rotateVector(v, axis, angle);
}
/* :195-358 */
static void scatterRay(ray_t *ray, v3 intersect, v3 normal, const orc_material *m, rng_t *rng, float softness) {
    if (m->transmittance[0] > 0.0f || m->transmittance[1] > 0.0f || m->transmittance[2] > 0.0f) {
        float randval = u01(rng);
        if (randval < 0.5f && !ray->isinside) {
            v3 v = randSphericalVec(0.0001f, rng);
            float angle = acosf(vdot(V3(0.0f, 0.0f, -1.0f), ray->direction));
            v3 axis = vnormalize(vcross(V3(0.0f, 0.0f, -1.0f), ray->direction));
            ray->direction = rotateVector(v, axis, angle);
            ray->origin = vadd(ray->origin, vscale(ray->direction, 0.0001f));
            ray->sdepth = vdistance(ray->origin, intersect);
            ray->isinside = 1;
        } else {
            ray->direction = calculateRandomDirectionInHemisphere(normal, rng);
            ray->origin = vadd(intersect, vscale(normal, 0.00001f));
            ray->sdepth = 0.0f;
        }
    } else if (m->hasRefractive != 0.0f) {
        float randval = u01(rng);
        ray->direction = vnormalize(ray->direction);
        normal = vnormalize(normal);
        float fresn = getFresnelVal(ray->direction, normal, m->indexOfRefraction);
        if (randval < 1.0f - fresn) {
            float ior = m->indexOfRefraction;
            if (!ray->isinside) ior = 1.0f / m->indexOfRefraction;
            double dd = (double)vdot(normal, ray->direction);
            float angle = (float)(1.0f - ((double)ior * (double)ior) * (1.0f - dd * dd));
            if (angle < 0.0f) {
                float val = u01(rng);
                if (val < m->hasReflective) {
                    ray->direction = glm_reflect(ray->direction, normal);
                    if (softness > 0.0f) ray->direction = soft_lobe(ray->direction, rng);
                    ray->origin = vadd(intersect, vscale(normal, 0.00001f));
                } else {
                    ray->direction = calculateRandomDirectionInHemisphere(normal, rng);
                    ray->origin = vadd(intersect, vscale(normal, 0.00001f));
                }
            } else {
                float val = u01(rng);
                if (val < m->hasRefractive) {
                    ray->direction = glm_refract(ray->direction, normal, ior);
                    if (softness > 0.0f) ray->direction = soft_lobe(ray->direction, rng);
                    ray->origin = vsub(intersect, vscale(normal, 0.001f));
                    ray->isinside = !ray->isinside;
                } else {
                    ray->direction = calculateRandomDirectionInHemisphere(normal, rng);
                    ray->origin = vadd(intersect, vscale(normal, 0.00001f));
                }
            }
        } else {
            ray->direction = glm_reflect(ray->direction, normal);
            ray->origin = vadd(intersect, vscale(normal, 0.00001f));
            ray->isinside = 0;
        }
    } else if (m->hasReflective != 0.0f) {
        float randval = u01(rng);
        if (randval < m->hasReflective) {
            ray->direction = glm_reflect(ray->direction, normal);
            if (softness > 0.0f) ray->direction = soft_lobe(ray->direction, rng);
            ray->origin = vadd(intersect, vscale(normal, 0.0001f));
            ray->isinside = 0;
        } else {
            ray->direction = calculateRandomDirectionInHemisphere(normal, rng);
            ray->origin = vadd(intersect, vscale(normal, 0.00001f));
        }
    } else {
        ray->direction = calculateRandomDirectionInHemisphere(normal, rng);
        ray->origin = vadd(intersect, vscale(normal, 0.00001f));
        ray->isinside = 0;
    }
}

/* ------------------------------------------------------------------ */
/* KD traversals (src/pathtrace.cu:881-1020 and 1023-1235)               */
/* ------------------------------------------------------------------ */
typedef struct {
    long long aabb, tri, hit, leaves;
} counters_t;

typedef struct {
    float t_min;
    int hit_geom_index;
    v3 intersect_point, normal;
    int obj_intersect;
    int objMaterialIdx;
} hitrec_t;

/* visited[] holds numNodes+1 flags; index id+1, slot 0 is the nodeIDs[-1] sink. */
static void traverseKD(const orc_scene *s, ray_t ray, v3 *bary, hitrec_t *h, unsigned char *visited,
                       int hybrid, int material_size, counters_t *cnt) {
    const orc_node *nodes = s->nodes;
    const orc_tri *tris = s->tris;
    int numNodes = s->num_nodes;
    if (numNodes == 0) return;
    memset(visited, 0, (size_t)numNodes + 1);
#define VIS(id) visited[(id) + 1]
    int currID = 0;
    for (int i = 0; i < numNodes; i++)
        if (nodes[i].parentID == -1) { currID = nodes[i].ID; break; }
    int hitGeom = 0;
    float dist = -1.0f;
    bary->z = FLT_MAX;
    const float hit_eps = hybrid ? 0.0001f : 0.00001f;
    while (1) {
        if (currID == -1) break;
        const orc_node *node = &nodes[currID];
        if (!hitGeom && node->parentID == -1 && VIS(node->ID)) break;
        hitGeom = intersectAABBarrays(ray, node->mins, node->maxs, &dist);
        cnt->aabb++;
        if (VIS(currID)) {
            VIS(node->ID) = 1; VIS(node->leftID) = 1; VIS(node->rightID) = 1;
            currID = node->parentID;
            continue;
        } else if (!hitGeom && node->parentID == -1) {
            break;
        }
        if (!hitGeom || dist > bary->z) {
            VIS(node->ID) = 1; VIS(node->leftID) = 1; VIS(node->rightID) = 1;
            currID = node->parentID;
            continue;
        }
        int leftFirst = hybrid ? (vget(ray.direction, node->axis) > 0.0f) : 1;
        int firstID = leftFirst ? node->leftID : node->rightID;
        int secondID = leftFirst ? node->rightID : node->leftID;
        if (firstID != -1 && !VIS(firstID)) { currID = firstID; continue; }
        if (secondID != -1 && !VIS(secondID)) { currID = secondID; continue; }
        if (VIS(node->ID)) { currID = node->parentID; continue; }
        VIS(node->ID) = 1;
        int size = node->triIdSize;
        if (size > 0) cnt->leaves++;
        if (size > 0) {
            int start = node->triIdStart, end = start + size;
            for (int i = start; i < end; i++) {
                const orc_tri *T = &tris[i];
                v3 v1 = V3(T->x1, T->y1, T->z1), v2 = V3(T->x2, T->y2, T->z2), v3_ = V3(T->x3, T->y3, T->z3);
                cnt->tri++;
                int intersected = intersectRayTriangle(ray.origin, ray.direction, v1, v2, v3_, bary);
                if (!intersected) continue;
                cnt->hit++;
                if (hybrid) {
                    /* "skip other side": nodeIDs[nodes[nodeIDs[parentID]].(right|left)ID] = true */
                    int b = VIS(node->parentID) ? 1 : 0;
                    int target = -1;
                    if (b < numNodes) target = leftFirst ? nodes[b].rightID : nodes[b].leftID;
                    VIS(target) = 1;
                }
                v3 n1 = V3(T->nx1, T->ny1, T->nz1), n2 = V3(T->nx2, T->ny2, T->nz2), n3 = V3(T->nx3, T->ny3, T->nz3);
                h->objMaterialIdx = T->mtlIdx + material_size - 1;
                v3 hit = vadd(ray.origin, vscale(ray.direction, bary->z));
                float w0 = 1 - bary->x - bary->y;
                v3 norm = vnormalize(vadd(vadd(vscale(n1, w0), vscale(n2, bary->x)), vscale(n3, bary->y)));
                hit = vadd(hit, vscale(norm, hit_eps));
                float t = vdistance(ray.origin, hit);
                if (t > 0.0f && h->t_min > t) {
                    h->t_min = t;
                    h->hit_geom_index = s->obj_materialOffsets[T->mtlIdx];
                    h->intersect_point = hit;
                    h->normal = norm;
                    h->obj_intersect = 1;
                }
            }
        }
    }
#undef VIS
}

/* intersectBbox, src/interactions.h:136-165 (min/max as in intersectAABBarrays) */
static inline float intersectBbox(v3 origin, v3 direction, v3 mn, v3 mx) {
    v3 invdir = V3(1.0f / direction.x, 1.0f / direction.y, 1.0f / direction.z);
    float v1 = (mn.x - origin.x) * invdir.x;
    float v2 = (mx.x - origin.x) * invdir.x;
    float v3_ = (mn.y - origin.y) * invdir.y;
    float v4_ = (mx.y - origin.y) * invdir.y;
    float v5 = (mn.z - origin.z) * invdir.z;
    float v6 = (mx.z - origin.z) * invdir.z;
    float dmin = std_max(std_max(std_min(v1, v2), std_min(v3_, v4_)), std_min(v5, v6));
    float dmax = std_min(std_min(std_max(v1, v2), std_max(v3_, v4_)), std_max(v5, v6));
    if (dmax < 0) return dmax;
    if (dmin > dmax) return dmax;
    return dmin;
}

/* The polygon loop of pathTraceOneBounce (enable_kd == false), src/pathtrace.cu:485-576: every
 * triangle of every OBJ shape in file order, optionally behind the shape's bbox test.  Kept as the
 * reference spells it: the bbox is read at obj_polysbboxes[i .. i+5] (shape index, not 6*i), the
 * double +-0.01 margin is rounded to float by glm::vec3's converting constructor, `iterator` only
 * advances for shapes whose bbox test passed, and objMaterialIdx ends as the LAST shape's offset. */
static void bruteForceObj(const orc_scene *s, ray_t ray, int usebbox, hitrec_t *h, counters_t *cnt) {
    int iterator = 0;
    int objMaterialIdx = -1;
    const float *bb = s->obj_bboxes;
    for (int i = 0; i < s->num_shapes; i++) {
        objMaterialIdx = s->obj_materialOffsets[i];
        float T;
        if (usebbox) {
            v3 mn = V3((float)((double)bb[i] - 0.01), (float)((double)bb[i + 1] - 0.01), (float)((double)bb[i + 2] - 0.01));
            v3 mx = V3((float)((double)bb[i + 3] + 0.01), (float)((double)bb[i + 4] + 0.01), (float)((double)bb[i + 5] + 0.01));
            T = intersectBbox(ray.origin, ray.direction, mn, mx);
        } else {
            T = 0;
        }
        if (T > -1.0f) {
            for (int j = iterator; j < iterator + s->obj_polyoffsets[i]; j += 3) {
                int p1 = 3 * s->obj_polysidxflat[j], p2 = 3 * s->obj_polysidxflat[j + 1], p3 = 3 * s->obj_polysidxflat[j + 2];
                const float *V = s->obj_verts, *N = s->obj_norms;
                v3 v1 = V3(V[p1], V[p1 + 1], V[p1 + 2]), v2 = V3(V[p2], V[p2 + 1], V[p2 + 2]), v3_ = V3(V[p3], V[p3 + 1], V[p3 + 2]);
                v3 n1 = V3(N[p1], N[p1 + 1], N[p1 + 2]), n2 = V3(N[p2], N[p2 + 1], N[p2 + 2]), n3 = V3(N[p3], N[p3 + 1], N[p3 + 2]);
                v3 bary = V3(0.0f, 0.0f, 0.0f);
                cnt->tri++;
                int intersected = intersectRayTriangle(ray.origin, ray.direction, v1, v2, v3_, &bary);
                if (!intersected) continue;
                cnt->hit++;
                v3 hit = vadd(ray.origin, vscale(ray.direction, bary.z));
                float w0 = 1 - bary.x - bary.y;
                v3 norm = vnormalize(vadd(vadd(vscale(n1, w0), vscale(n2, bary.x)), vscale(n3, bary.y)));
                hit = vadd(hit, vscale(norm, 0.0001f));
                float t = vdistance(ray.origin, hit);
                if (t > 0.0f && h->t_min > t) {
                    h->t_min = t;
                    h->hit_geom_index = s->obj_materialOffsets[i];
                    h->intersect_point = hit;
                    h->normal = norm;
                    h->obj_intersect = 1;
                }
            }
            iterator += s->obj_polyoffsets[i];
        }
    }
    h->objMaterialIdx = objMaterialIdx;
}

/* ------------------------------------------------------------------ */
/* Kernels as host loops                                                */
/* ------------------------------------------------------------------ */
static inline ray_t path_ray(const orc_path *p) {
    ray_t r;
    r.origin = V3(p->origin[0], p->origin[1], p->origin[2]);
    r.direction = V3(p->direction[0], p->direction[1], p->direction[2]);
    r.isinside = p->isinside;
    r.sdepth = p->sdepth;
    return r;
}
static inline void path_set_ray(orc_path *p, ray_t r) {
    p->origin[0] = r.origin.x; p->origin[1] = r.origin.y; p->origin[2] = r.origin.z;
    p->direction[0] = r.direction.x; p->direction[1] = r.direction.y; p->direction[2] = r.direction.z;
    p->isinside = (uint8_t)(r.isinside != 0);
    p->sdepth = r.sdepth;
}

/* src/pathtrace.cu:315-397 */
static void generateRayFromCamera(const orc_camera *cam, int iter, int traceDepth, orc_path *paths,
                                  float focalLength, float dofAngle, int antialias) {
    /* The RNG is seeded by utilhash(iter) only: every pixel draws the same numbers. */
    int W = cam->resolution[0], H = cam->resolution[1];
    v3 view = V3(cam->view[0], cam->view[1], cam->view[2]);
    v3 right = V3(cam->right[0], cam->right[1], cam->right[2]);
    v3 upv = V3(cam->up[0], cam->up[1], cam->up[2]);
    v3 pos = V3(cam->position[0], cam->position[1], cam->position[2]);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            int index = x + (y * W);
            orc_path *seg = &paths[index];
            ray_t ray;
            ray.origin = pos;
            ray.isinside = 0;
            ray.sdepth = seg->sdepth;
            seg->color[0] = 1.0f; seg->color[1] = 1.0f; seg->color[2] = 1.0f;
            /* cam.right * cam.pixelLength.x * (...): (vec * float) * float, left to right */
            v3 a = vscale(vscale(right, cam->pixelLength[0]), ((float)x - (float)W * 0.5f));
            v3 b = vscale(vscale(upv, cam->pixelLength[1]), ((float)y - (float)H * 0.5f));
            ray.direction = vnormalize(vsub(vsub(view, a), b));
            rng_t rng = rng_seed(orc_utilhash((unsigned int)iter));
            if (antialias) {
                float jitterscale = (float)0.002;
                float j0 = u01(&rng), j1 = u01(&rng), j2 = u01(&rng);
                v3 v3a = vnormalize(V3(j0, j1, j2));
                ray.direction = vadd(ray.direction, vscale(v3a, jitterscale));
                ray.direction = vnormalize(ray.direction);
            }
            float u = cosf(PI_F * u01(&rng));
            float u2 = u * u;
            float sq = sqrtf(1 - u2);
            float theta = 2 * PI_F * u01(&rng);
            v3 vv = vnormalize(V3(sq * cosf(theta), sq * sinf(theta), u));
            (void)u01(&rng); /* R1 */
            (void)u01(&rng); /* R2 */
            float randangle = u01(&rng) * PI_F * dofAngle;
            float qw = cosf(randangle / 2.0f);
            float sh = sinf(randangle / 2.0f);
            v3 qv = V3(vv.x * sh, vv.y * sh, vv.z * sh);
            /* glm quat * vec3 (gtc/quaternion.inl): v + ((uv * w) + uuv) * 2 */
            v3 uv = vcross(qv, ray.direction);
            v3 uuv = vcross(qv, uv);
            v3 randrot = vadd(ray.direction, vscale(vadd(vscale(uv, qw), uuv), 2.0f));
            ray.origin = vsub(vadd(ray.origin, vscale(ray.direction, focalLength)), vscale(randrot, focalLength));
            ray.direction = vnormalize(randrot);
            path_set_ray(seg, ray);
            seg->pixelIndex = index;
            seg->remainingBounces = traceDepth;
        }
    }
}

/* boxIntersectionTestBox's transform (src/intersections.h:51-63): the node box as a unit cube scaled by
 * maxs - mins and moved to (mins + maxs) * 0.5 (a double product, converted to float by glm::mat4's
 * constructor), with glm::inverse; the rest of that function is boxIntersectionTest's. */
static orc_geom node_box_geom(const orc_node *n) {
    orc_geom g;
    memset(&g, 0, sizeof g);
    g.type = 1;
    m4 t = m4identity();
    m4set(&t, 0, 0, n->maxs[0] - n->mins[0]);
    m4set(&t, 1, 1, n->maxs[1] - n->mins[1]);
    m4set(&t, 2, 2, n->maxs[2] - n->mins[2]);
    m4set(&t, 3, 0, (float)((double)(n->mins[0] + n->maxs[0]) * 0.5));
    m4set(&t, 3, 1, (float)((double)(n->mins[1] + n->maxs[1]) * 0.5));
    m4set(&t, 3, 2, (float)((double)(n->mins[2] + n->maxs[2]) * 0.5));
    m4 inv = m4inverse(&t);
    memcpy(g.transform, &t, 64);
    memcpy(g.inverseTransform, &inv, 64);
    return g;
}

/* The node loop of pathTraceOneBounceKDbareBoxes (vizkd, src/pathtrace.cu:1813-1831): every KD node's box
 * as a box; a winning box reports material_size - 1 and hit_geom_index = geoms_size. */
static void vizNodes(const orc_scene *s, const orc_geom *boxes, ray_t ray, hitrec_t *h) {
    int outside = 1;
    v3 tmp_i, tmp_n;
    for (int i = 0; i < s->num_nodes; i++) {
        float t = boxIntersectionTest(&boxes[i], ray, &tmp_i, &tmp_n, &outside);
        if (t > 0.0f && h->t_min > t) {
            h->t_min = t;
            h->hit_geom_index = s->num_geoms;
            h->intersect_point = tmp_i;
            h->normal = tmp_n;
            h->obj_intersect = 1;
            h->objMaterialIdx = s->num_materials - 1;
        }
    }
}

/* src/pathtrace.cu:1571-1734 */
static void traceOneBounce(const orc_scene *s, const orc_opts *o, int depth, int iter, int num_paths,
                           orc_path *paths, orc_isect *isects, counters_t *tot) {
    orc_geom *boxes = NULL;
    if (o->vizkd && s->has_obj) {
        boxes = (orc_geom *)malloc(sizeof(orc_geom) * (size_t)(s->num_nodes > 0 ? s->num_nodes : 1));
        for (int k = 0; k < s->num_nodes; k++) boxes[k] = node_box_geom(&s->nodes[k]);
    }
    long long ca = 0, ct = 0, ch = 0;
    int nmat = s->num_materials;
#pragma omp parallel reduction(+ : ca, ct, ch)
    {
        unsigned char *visited = (unsigned char *)malloc((size_t)s->num_nodes + 1);
        counters_t cnt = {0, 0, 0, 0};
#pragma omp for schedule(dynamic, 256)
        for (int path_index = 0; path_index < num_paths; path_index++) {
            orc_path *P = &paths[path_index];
            if (!(P->remainingBounces > 0)) continue;
            ray_t ray = path_ray(P);
            hitrec_t h;
            h.t_min = FLT_MAX; h.hit_geom_index = -1; h.obj_intersect = 0; h.objMaterialIdx = -1;
            h.intersect_point = V3(0, 0, 0); h.normal = V3(0, 0, 0);
            v3 tmp_i = V3(0, 0, 0), tmp_n = V3(0, 0, 0);
            int outside = 1;
            float t = 0;
            for (int i = 0; i < s->num_geoms; i++) {
                const orc_geom *g = &s->geoms[i];
                if (g->type == 1) t = boxIntersectionTest(g, ray, &tmp_i, &tmp_n, &outside);
                else if (g->type == 0) t = sphereIntersectionTest(g, ray, &tmp_i, &tmp_n, &outside);
                if (t > 0.0f && h.t_min > t) {
                    h.t_min = t; h.hit_geom_index = i; h.intersect_point = tmp_i; h.normal = tmp_n;
                }
            }
            v3 bary = V3(0, 0, 0);
            if (s->has_obj) {
                if (!o->enable_kd) bruteForceObj(s, ray, o->usebbox, &h, &cnt);
                else if (o->vizkd) vizNodes(s, boxes, ray, &h);
                else traverseKD(s, ray, &bary, &h, visited, o->shortstack, nmat, &cnt);
            }
            orc_isect *I = &isects[path_index];
            if (h.hit_geom_index == -1) {
                I->t = -1.0f;
            } else {
                rng_t rng = makeSeededRandomEngine(iter, path_index, depth);
                const orc_material *m;
                int mid;
                if (h.obj_intersect) mid = h.objMaterialIdx;
                else mid = s->geoms[h.hit_geom_index].materialid;
                m = &s->materials[mid];
                P->materialIdHit = mid;
                ray_t r2 = path_ray(P);
                scatterRay(&r2, h.intersect_point, h.normal, m, &rng, o->softness);
                path_set_ray(P, r2);
                I->t = h.t_min;
                I->materialId = mid;
                I->surfaceNormal[0] = h.normal.x; I->surfaceNormal[1] = h.normal.y; I->surfaceNormal[2] = h.normal.z;
            }
        }
        ca += cnt.aabb; ct += cnt.tri; ch += cnt.hit;
        free(visited);
    }
    tot->aabb += ca; tot->tri += ct; tot->hit += ch;
    free(boxes);
}

int orc_trace_ray(const orc_scene *s, const float *origin, const float *direction, int hybrid, double *out) {
    unsigned char *visited = (unsigned char *)malloc((size_t)s->num_nodes + 1);
    counters_t cnt = {0, 0, 0, 0};
    ray_t ray;
    ray.origin = V3(origin[0], origin[1], origin[2]);
    ray.direction = V3(direction[0], direction[1], direction[2]);
    ray.isinside = 0; ray.sdepth = 0;
    hitrec_t h;
    h.t_min = FLT_MAX; h.hit_geom_index = -1; h.obj_intersect = 0; h.objMaterialIdx = -1;
    h.intersect_point = V3(0, 0, 0); h.normal = V3(0, 0, 0);
    v3 tmp_i = V3(0, 0, 0), tmp_n = V3(0, 0, 0);
    int outside = 1;
    float t = 0;
    for (int i = 0; i < s->num_geoms; i++) {
        const orc_geom *g = &s->geoms[i];
        if (g->type == 1) t = boxIntersectionTest(g, ray, &tmp_i, &tmp_n, &outside);
        else if (g->type == 0) t = sphereIntersectionTest(g, ray, &tmp_i, &tmp_n, &outside);
        if (t > 0.0f && h.t_min > t) { h.t_min = t; h.hit_geom_index = i; h.intersect_point = tmp_i; h.normal = tmp_n; }
    }
    v3 bary = V3(0, 0, 0);
    if (s->has_obj) traverseKD(s, ray, &bary, &h, visited, hybrid, s->num_materials, &cnt);
    out[0] = h.t_min; out[1] = h.hit_geom_index;
    out[2] = h.intersect_point.x; out[3] = h.intersect_point.y; out[4] = h.intersect_point.z;
    out[5] = h.normal.x; out[6] = h.normal.y; out[7] = h.normal.z;
    out[8] = h.obj_intersect; out[9] = h.objMaterialIdx;
    out[10] = (double)cnt.aabb; out[11] = (double)cnt.tri; out[12] = (double)cnt.hit; out[13] = (double)cnt.leaves;
    free(visited);
    return 0;
}

/* src/pathtrace.cu:2304-2369 */
static void shadeMaterial(const orc_scene *s, const orc_opts *o, int num_paths, const orc_isect *isects,
                          orc_path *paths) {
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < num_paths; idx++) {
        orc_path *P = &paths[idx];
        if (!(P->remainingBounces > 0)) continue;
        const orc_isect *I = &isects[idx];
        if (I->t > 0.0f) {
            const orc_material *m = &s->materials[I->materialId];
            v3 c = V3(m->color[0], m->color[1], m->color[2]);
            v3 col = V3(P->color[0], P->color[1], P->color[2]);
            v3 spec = V3(m->spec_color[0], m->spec_color[1], m->spec_color[2]);
            if (m->emittance > 0.0f) {
                col = vmul(col, vscale(c, m->emittance));
                P->remainingBounces = 0;
            } else {
                if (o->enableSss && (m->transmittance[0] > 0.0f || m->transmittance[1] > 0.0f ||
                                     m->transmittance[2] > 0.0f)) {
                    float scenescale = 1.0f;
                    float sss = (double)(scenescale * P->sdepth) > 1.0 ? 1.0f : P->sdepth;
                    sss = (double)(1.0f - sss) < 0.0 ? 0.0f : sss;
                    sss = (float)((double)sss * (double)sss);
                    v3 tr = V3(m->transmittance[0], m->transmittance[1], m->transmittance[2]);
                    col = vmul(col, vadd(vadd(vscale(c, 1.0f), vscale(spec, m->hasRefractive)), vscale(tr, sss)));
                } else if (m->hasRefractive > 0.0f) {
                    col = vmul(col, vadd(vscale(c, 1.0f), vscale(spec, m->hasRefractive)));
                } else if (m->hasReflective > 0.0f) {
                    col = vmul(col, vadd(vscale(c, 1.0f), vscale(spec, m->hasReflective)));
                } else {
                    col = vmul(col, vscale(c, 1.0f));
                }
                P->remainingBounces--;
            }
            P->color[0] = col.x; P->color[1] = col.y; P->color[2] = col.z;
        } else {
            P->color[0] = 0.0f; P->color[1] = 0.0f; P->color[2] = 0.0f;
            P->remainingBounces = 0;
        }
    }
}

static int cmp_paths_stable_key(const void *a, const void *b) { (void)a; (void)b; return 0; }

/* One pathtrace() iteration.  stop_depth >= 0: return after that bounce. */
static int run_iteration(const orc_scene *s, const orc_opts *o, int iter, orc_path *paths, orc_path *tmp,
                         orc_isect *isects, float *image, orc_stats *st, int stop_depth, int *npaths_out) {
    const orc_camera *cam = &s->camera;
    int W = cam->resolution[0], H = cam->resolution[1];
    int pixelcount = W * H;
    /* cacherays (src/pathtrace.cu:2448-2456): camera rays of iteration 1 are reused; the
       bounce RNG still uses the real iter */
    generateRayFromCamera(cam, o->cacherays ? 1 : iter, s->traceDepth, paths, o->focalLength, o->dofAngle,
                          o->antialias);
    int depth = 0;
    int num_paths = pixelcount;
    counters_t cnt = {0, 0, 0, 0};
    int complete = 0;
    int cap = o->bounce_cap > 0 ? o->bounce_cap : 8;
    st->bounces = 0;
    while (!complete) {
        memset(isects, 0, sizeof(orc_isect) * (size_t)pixelcount);
        st->segments += num_paths;
        if (depth < 32) st->seg_per_bounce[depth] += num_paths;
        traceOneBounce(s, o, depth, iter, num_paths, paths, isects, &cnt);
        depth++;
        st->bounces = depth;
        shadeMaterial(s, o, num_paths, isects, paths);
        if (o->compaction) {
            /* partialGather: one path per pixel, so the adds never collide */
#pragma omp parallel for schedule(static)
            for (int i = 0; i < num_paths; i++) {
                if (paths[i].remainingBounces == 0) {
                    int px = paths[i].pixelIndex;
                    image[3 * px + 0] += paths[i].color[0];
                    image[3 * px + 1] += paths[i].color[1];
                    image[3 * px + 2] += paths[i].color[2];
                }
            }
            /* thrust::remove_if(is_zero_bounce) -- stable */
            int n = 0;
            for (int i = 0; i < num_paths; i++)
                if (paths[i].remainingBounces != 0) paths[n++] = paths[i];
            num_paths = n;
        }
        if (iter == 2) {
            /* thrust::sort(paths) by materialIdHit: merge sort for user types (stable) */
            int maxk = 0;
            for (int i = 0; i < num_paths; i++) if (paths[i].materialIdHit > maxk) maxk = paths[i].materialIdHit;
            int mink = 0;
            for (int i = 0; i < num_paths; i++) if (paths[i].materialIdHit < mink) mink = paths[i].materialIdHit;
            int nk = maxk - mink + 2;
            long long *cntk = (long long *)calloc((size_t)nk, sizeof(long long));
            for (int i = 0; i < num_paths; i++) cntk[paths[i].materialIdHit - mink + 1]++;
            for (int k = 1; k < nk; k++) cntk[k] += cntk[k - 1];
            for (int i = 0; i < num_paths; i++) tmp[cntk[paths[i].materialIdHit - mink]++] = paths[i];
            memcpy(paths, tmp, sizeof(orc_path) * (size_t)num_paths);
            free(cntk);
            (void)cmp_paths_stable_key;
        }
        if (stop_depth >= 0 && depth - 1 == stop_depth) {
            if (npaths_out) *npaths_out = num_paths;
            st->aabb_tests += cnt.aabb; st->tri_tests += cnt.tri; st->tri_hits += cnt.hit;
            return 0;
        }
        if (num_paths <= 0 || depth > cap - 1) complete = 1;
    }
    if (!o->compaction) {
        /* finalGather (src/pathtrace.cu:2373-2383), including its index = paths[index].pixelIndex quirk */
        for (int index = 0; index < num_paths; index++) {
            int j = paths[index].pixelIndex;
            const orc_path *p = &paths[j];
            int px = p->pixelIndex;
            image[3 * px + 0] += p->color[0];
            image[3 * px + 1] += p->color[1];
            image[3 * px + 2] += p->color[2];
        }
    }
    st->aabb_tests += cnt.aabb; st->tri_tests += cnt.tri; st->tri_hits += cnt.hit;
    if (npaths_out) *npaths_out = num_paths;
    return 0;
}

void orc_default_opts(orc_opts *o) {
    o->focalLength = 6.0f;
    o->dofAngle = 0.0f;
    o->cacherays = 0;
    o->antialias = 1;
    o->softness = 0.0f;
    o->enableSss = 0;
    o->compaction = 1;
    o->shortstack = 1;
    o->bounce_cap = 8;
    o->enable_kd = 1;
    o->usebbox = 0;
    o->vizkd = 0;
}

int orc_render(const orc_scene *s, const orc_opts *o, int iter_first, int iter_count, float *image,
               orc_stats *stats, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int pixelcount = s->camera.resolution[0] * s->camera.resolution[1];
    orc_path *paths = (orc_path *)calloc((size_t)pixelcount, sizeof(orc_path));
    orc_path *tmp = (orc_path *)calloc((size_t)pixelcount, sizeof(orc_path));
    orc_isect *isects = (orc_isect *)calloc((size_t)pixelcount, sizeof(orc_isect));
    if (!paths || !tmp || !isects) { free(paths); free(tmp); free(isects); return -1; }
    orc_stats local;
    memset(&local, 0, sizeof local);
    for (int it = iter_first; it < iter_first + iter_count; it++)
        run_iteration(s, o, it, paths, tmp, isects, image, &local, -1, NULL);
    if (stats) *stats = local;
    free(paths); free(tmp); free(isects);
    return 0;
}

int orc_paths_after(const orc_scene *s, const orc_opts *o, int iter, int stop_depth, orc_path *out, int *npaths) {
    int pixelcount = s->camera.resolution[0] * s->camera.resolution[1];
    orc_path *tmp = (orc_path *)calloc((size_t)pixelcount, sizeof(orc_path));
    orc_isect *isects = (orc_isect *)calloc((size_t)pixelcount, sizeof(orc_isect));
    float *image = (float *)calloc((size_t)pixelcount * 3, sizeof(float));
    orc_stats st;
    memset(&st, 0, sizeof st);
    memset(out, 0, sizeof(orc_path) * (size_t)pixelcount);
    run_iteration(s, o, iter, out, tmp, isects, image, &st, stop_depth, npaths);
    free(tmp); free(isects); free(image);
    return 0;
}

/* ------------------------------------------------------------------ */
/* KD build (src/KDnode.cpp, src/KDtree.cpp) and flatten (src/scene.cpp) */
/* ------------------------------------------------------------------ */
typedef struct {
    float x1, x2, x3, y1, y2, y3, z1, z2, z3;
    float nx1, nx2, nx3, ny1, ny2, ny3, nz1, nz2, nz3;
    float center[3], mins[3], maxs[3];
    int mtlIdx;
} ktri;

typedef struct { float mins[3], maxs[3], center[3], size[3]; } kbbox;

typedef struct knode {
    int axis;
    float splitPos;
    struct knode *parent, *left, *right;
    kbbox bbox;
    ktri **tris;
    int ntris;
    int ID, parentID, leftID, rightID, triIdStart, triIdSize;
} knode;

typedef struct { int currentID; } kctx;

static void ktri_bounds(ktri *t) { /* KDnode.h:209-225 */
    t->center[0] = (float)((double)(t->x1 + t->x2 + t->x3) / 3.0);
    t->center[1] = (float)((double)(t->y1 + t->y2 + t->y3) / 3.0);
    t->center[2] = (float)((double)(t->z1 + t->z2 + t->z3) / 3.0);
    t->mins[0] = t->x1 < t->x2 ? (t->x1 < t->x3 ? t->x1 : t->x3) : (t->x2 < t->x3 ? t->x2 : t->x3);
    t->mins[1] = t->y1 < t->y2 ? (t->y1 < t->y3 ? t->y1 : t->y3) : (t->y2 < t->y3 ? t->y2 : t->y3);
    t->mins[2] = t->z1 < t->z2 ? (t->z1 < t->z3 ? t->z1 : t->z3) : (t->z2 < t->z3 ? t->z2 : t->z3);
    t->maxs[0] = t->x1 > t->x2 ? (t->x1 > t->x3 ? t->x1 : t->x3) : (t->x2 > t->x3 ? t->x2 : t->x3);
    t->maxs[1] = t->y1 > t->y2 ? (t->y1 > t->y3 ? t->y1 : t->y3) : (t->y2 > t->y3 ? t->y2 : t->y3);
    t->maxs[2] = t->z1 > t->z2 ? (t->z1 > t->z3 ? t->z1 : t->z3) : (t->z2 > t->z3 ? t->z2 : t->z3);
}
static void bb_updateSize(kbbox *b) {
    for (int i = 0; i < 3; i++) b->size[i] = b->mins[i] < b->maxs[i] ? b->maxs[i] - b->mins[i] : b->mins[i] - b->maxs[i];
}
static void bb_updateCentroid(kbbox *b) { /* KDnode.h:273-279 */
    for (int i = 0; i < 3; i++) b->center[i] = (float)((double)(b->mins[i] + b->maxs[i]) / 2.0);
    bb_updateSize(b);
}
static void bb_setBoundsTri(kbbox *b, const ktri *t) { /* KDnode.h:260-271 */
    for (int i = 0; i < 3; i++) { b->mins[i] = t->mins[i]; b->maxs[i] = t->maxs[i]; }
    bb_updateCentroid(b);
    bb_updateSize(b);
}
static void bb_setBounds6(kbbox *b, const float *mn, const float *mx) { /* KDnode.h:281-288 */
    for (int i = 0; i < 3; i++) { b->mins[i] = mn[i]; b->maxs[i] = mx[i]; }
    bb_updateCentroid(b);
}
static void knode_merge(knode *n, const kbbox *b) { /* KDnode.cpp:99-110 */
    for (int i = 0; i < 3; i++) {
        n->bbox.mins[i] = n->bbox.mins[i] > b->mins[i] ? b->mins[i] : n->bbox.mins[i];
        n->bbox.maxs[i] = n->bbox.maxs[i] < b->maxs[i] ? b->maxs[i] : n->bbox.maxs[i];
    }
    bb_updateCentroid(&n->bbox);
}
static kbbox knode_updateBbox(knode *n) { /* KDnode.cpp:112-149 */
    if (n->ntris > 0) bb_setBoundsTri(&n->bbox, n->tris[0]);
    for (int i = 1; i < n->ntris; i++) {
        kbbox b;
        bb_setBoundsTri(&b, n->tris[i]);
        knode_merge(n, &b);
    }
    if (n->left) { kbbox b = knode_updateBbox(n->left); knode_merge(n, &b); }
    if (n->right) { kbbox b = knode_updateBbox(n->right); knode_merge(n, &b); }
    float pad = (float)0.001;
    for (int i = 0; i < 3; i++) { n->bbox.mins[i] -= pad; n->bbox.maxs[i] += pad; }
    return n->bbox;
}
static knode *knode_new(void) { /* KDnode.cpp:4-19 (+ BoundingBox() setBounds(0)) */
    knode *n = (knode *)calloc(1, sizeof(knode));
    n->axis = 0; n->splitPos = 0.0f; n->ID = 0;
    n->parentID = -1; n->leftID = -1; n->rightID = -1; n->triIdStart = -1; n->triIdSize = -1;
    return n;
}
static knode *knode_from_tris(ktri **t, int size, int axis) { /* KDnode.cpp:57-77 */
    knode *n = knode_new();
    n->tris = (ktri **)malloc(sizeof(ktri *) * (size_t)(size > 0 ? size : 1));
    memcpy(n->tris, t, sizeof(ktri *) * (size_t)size);
    n->ntris = size;
    n->axis = axis;
    knode_updateBbox(n);
    return n;
}
static int knode_level(const knode *n) {
    int l = 0;
    while (n->parent) { l++; n = n->parent; }
    return l;
}
static void knode_split(kctx *ctx, knode *self, int maxdepth) { /* KDnode.cpp:151-249 */
    int num = self->ntris;
    if (num == 0) {
        if (self->left) knode_split(ctx, self->left, maxdepth);
        if (self->right) knode_split(ctx, self->right, maxdepth);
        return;
    }
    if (num <= 2) return;
    int level = knode_level(self);
    if (level > maxdepth) return;
    level = level % 3;
    ktri **L = (ktri **)malloc(sizeof(ktri *) * (size_t)num);
    ktri **R = (ktri **)malloc(sizeof(ktri *) * (size_t)num);
    int nl = 0, nr = 0;
    double c = (double)self->bbox.center[level];
    for (int i = 0; i < num; i++) {
        if ((double)self->tris[i]->mins[level] < c + 0.0001) L[nl++] = self->tris[i];
        if ((double)self->tris[i]->maxs[level] >= c - 0.0001) R[nr++] = self->tris[i];
    }
    if (nl == num || nr == num) { free(L); free(R); return; }
    if (nl != 0) {
        if (self->left == NULL) {
            self->left = knode_from_tris(L, nl, (level + 1) % 3);
            ctx->currentID++;
            self->left->ID = ctx->currentID;
            self->left->parentID = self->ID;
            self->leftID = ctx->currentID;
            self->left->parent = self;
        }
        bb_setBounds6(&self->left->bbox, self->bbox.mins, self->bbox.maxs);
        self->left->bbox.maxs[level] = self->bbox.center[level];
        bb_updateCentroid(&self->left->bbox);
        bb_updateSize(&self->left->bbox);
        self->left->splitPos = self->bbox.maxs[level];
        knode_split(ctx, self->left, maxdepth);
    }
    if (nr != 0) {
        if (self->right == NULL) {
            self->right = knode_from_tris(R, nr, (level + 1) % 3);
            ctx->currentID++;
            self->right->ID = ctx->currentID;
            self->right->parentID = self->ID;
            self->rightID = ctx->currentID;
            self->right->parent = self;
        }
        bb_setBounds6(&self->right->bbox, self->bbox.mins, self->bbox.maxs);
        self->right->bbox.mins[level] = self->bbox.center[level];
        bb_updateCentroid(&self->right->bbox);
        bb_updateSize(&self->right->bbox);
        self->right->splitPos = self->bbox.mins[level];
        knode_split(ctx, self->right, maxdepth);
    }
    free(L); free(R);
    self->ntris = 0; /* triangles.erase(...) */
}
static void knode_free(knode *n) {
    if (!n) return;
    knode_free(n->left); knode_free(n->right);
    free(n->tris); free(n);
}
static int knode_count(const knode *n) { return n ? 1 + knode_count(n->left) + knode_count(n->right) : 0; }
static void knode_preorder(knode *n, knode **out, int *k) {
    if (!n) return;
    out[(*k)++] = n;
    knode_preorder(n->left, out, k);
    knode_preorder(n->right, out, k);
}
static void fprint_g(FILE *f, float v) { fprintf(f, "%g", (double)v); }
static void kd_print(knode *n, FILE *f) { /* KDtree.cpp:100-110 (ostream << float == %g) */
    if (!n) return;
    for (int i = 0; i < 3; i++) { fprint_g(f, n->bbox.mins[i]); fputc(' ', f); }
    for (int i = 0; i < 3; i++) { fprint_g(f, n->bbox.maxs[i]); fputc(i < 2 ? ' ' : '\n', f); }
    kd_print(n->left, f);
    kd_print(n->right, f);
}

int orc_kd_kat(const char *tri_file, int maxdepth, const char *out_path) {
    FILE *f = fopen(tri_file, "rb");
    if (!f) return -1;
    /* KDtree::getTrianglesFromFile: nine getline+atof per triangle */
    size_t cap = 1024, n = 0;
    float *vals = (float *)malloc(cap * sizeof(float));
    char line[4096];
    int lines_ok = 1;
    while (lines_ok) {
        if (!fgets(line, sizeof line, f)) break;
        float tv[9];
        tv[0] = (float)atof(line);
        for (int k = 1; k < 9; k++) {
            if (!fgets(line, sizeof line, f)) line[0] = 0;
            tv[k] = (float)atof(line);
        }
        if (n + 9 > cap) { cap *= 2; vals = (float *)realloc(vals, cap * sizeof(float)); }
        memcpy(vals + n, tv, sizeof tv);
        n += 9;
    }
    fclose(f);
    int ntri = (int)(n / 9);
    ktri *T = (ktri *)calloc((size_t)(ntri > 0 ? ntri : 1), sizeof(ktri));
    ktri **P = (ktri **)malloc(sizeof(ktri *) * (size_t)(ntri > 0 ? ntri : 1));
    for (int i = 0; i < ntri; i++) {
        float *v = vals + 9 * i;
        T[i].x1 = v[0]; T[i].y1 = v[1]; T[i].z1 = v[2];
        T[i].x2 = v[3]; T[i].y2 = v[4]; T[i].z2 = v[5];
        T[i].x3 = v[6]; T[i].y3 = v[7]; T[i].z3 = v[8];
        T[i].mtlIdx = -1;
        ktri_bounds(&T[i]);
        P[i] = &T[i];
    }
    kctx ctx = {0};
    knode *root = knode_new();
    root->tris = P; root->ntris = ntri;
    knode_updateBbox(root);
    knode_split(&ctx, root, maxdepth);
    FILE *o = fopen(out_path, "wb");
    if (!o) return -2;
    kd_print(root, o);
    fclose(o);
    knode_free(root);
    free(T); free(vals);
    return 0;
}

int orc_build_kd(const float *verts9, const float *norms9, const int *mtl, int ntri, int maxdepth,
                 orc_node **nodes_out, int *nnodes, orc_tri **tris_out, int *ntris_out) {
    ktri *T = (ktri *)calloc((size_t)(ntri > 0 ? ntri : 1), sizeof(ktri));
    ktri **P = (ktri **)malloc(sizeof(ktri *) * (size_t)(ntri > 0 ? ntri : 1));
    for (int i = 0; i < ntri; i++) {
        const float *v = verts9 + 9 * (size_t)i, *nn = norms9 + 9 * (size_t)i;
        /* Triangle(X1,Y1,Z1, X2,Y2,Z2, X3,Y3,Z3, NX1,...) KDnode.h:140-159 */
        T[i].x1 = v[0]; T[i].y1 = v[1]; T[i].z1 = v[2];
        T[i].x2 = v[3]; T[i].y2 = v[4]; T[i].z2 = v[5];
        T[i].x3 = v[6]; T[i].y3 = v[7]; T[i].z3 = v[8];
        T[i].nx1 = nn[0]; T[i].ny1 = nn[1]; T[i].nz1 = nn[2];
        T[i].nx2 = nn[3]; T[i].ny2 = nn[4]; T[i].nz2 = nn[5];
        T[i].nx3 = nn[6]; T[i].ny3 = nn[7]; T[i].nz3 = nn[8];
        T[i].mtlIdx = mtl[i];
        ktri_bounds(&T[i]);
        P[i] = &T[i];
    }
    kctx ctx = {0};
    knode *root = knode_new();
    root->tris = P; root->ntris = ntri;
    knode_updateBbox(root);
    knode_split(&ctx, root, maxdepth);
    int nn = knode_count(root);
    knode **order = (knode **)malloc(sizeof(knode *) * (size_t)nn);
    int k = 0;
    knode_preorder(root, order, &k); /* pre-order == ID order (IDs are assigned pre-order) */
    /* cacheTriangles_ (src/scene.cpp:409-459) */
    long long total = 0;
    for (int i = 0; i < nn; i++) total += order[i]->ntris;
    orc_tri *tris = (orc_tri *)calloc((size_t)(total > 0 ? total : 1), sizeof(orc_tri));
    int tc = 0;
    for (int i = 0; i < nn; i++) {
        knode *nd = order[i];
        if (nd->ntris > 0) {
            nd->triIdStart = tc;
            nd->triIdSize = nd->ntris;
            for (int j = 0; j < nd->ntris; j++) {
                const ktri *t = nd->tris[j];
                orc_tri *o = &tris[tc++];
                o->x1 = t->x1; o->x2 = t->x2; o->x3 = t->x3;
                o->y1 = t->y1; o->y2 = t->y2; o->y3 = t->y3;
                o->z1 = t->z1; o->z2 = t->z2; o->z3 = t->z3;
                o->nx1 = t->nx1; o->nx2 = t->nx2; o->nx3 = t->nx3;
                o->ny1 = t->ny1; o->ny2 = t->ny2; o->ny3 = t->ny3;
                o->nz1 = t->nz1; o->nz2 = t->nz2; o->nz3 = t->nz3;
                o->mtlIdx = t->mtlIdx;
            }
        }
    }
    /* cacheNodesBare (src/scene.cpp:905-932), nodes sorted by ID */
    orc_node *nodes = (orc_node *)calloc((size_t)nn, sizeof(orc_node));
    for (int i = 0; i < nn; i++) {
        knode *nd = order[i];
        orc_node *o = &nodes[nd->ID];
        o->axis = nd->axis;
        o->ID = nd->ID; o->parentID = nd->parentID; o->leftID = nd->leftID; o->rightID = nd->rightID;
        for (int a = 0; a < 3; a++) { o->mins[a] = nd->bbox.mins[a]; o->maxs[a] = nd->bbox.maxs[a]; }
        o->triIdSize = nd->triIdSize; o->triIdStart = nd->triIdStart;
        o->splitPos = nd->splitPos;
        o->tmin = 0.0f; o->tmax = 0.0f;
    }
    free(order);
    knode_free(root);
    free(T);
    *nodes_out = nodes; *nnodes = nn; *tris_out = tris; *ntris_out = tc;
    return 0;
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------ */
/* Text readers                                                          */
/* ------------------------------------------------------------------ */
typedef struct { char *buf; size_t len, pos; int eof; } lreader;

static int lr_open(lreader *r, const char *path) {
    memset(r, 0, sizeof *r);
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    r->buf = (char *)malloc((size_t)n + 1);
    r->len = fread(r->buf, 1, (size_t)n, f);
    r->buf[r->len] = 0;
    fclose(f);
    return 0;
}
/* utilityCore::safeGetline (src/utilities.cpp:273-303) */
static size_t lr_getline(lreader *r, char *out, size_t cap) {
    size_t n = 0;
    for (;;) {
        if (r->pos >= r->len) { if (n == 0) r->eof = 1; break; }
        char c = r->buf[r->pos++];
        if (c == '\n') break;
        if (c == '\r') { if (r->pos < r->len && r->buf[r->pos] == '\n') r->pos++; break; }
        if (n + 1 < cap) out[n++] = c;
    }
    out[n] = 0;
    return n;
}
#define MAXTOK 16
static int tokenize(char *line, char **tok) { /* istream_iterator<string>: whitespace split */
    int n = 0;
    char *p = line;
    while (*p && n < MAXTOK) {
        while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\v' || *p == '\f' || *p == '\r') p++;
        if (!*p) break;
        tok[n++] = p;
        while (*p && !(*p == ' ' || *p == '\t' || *p == '\n' || *p == '\v' || *p == '\f' || *p == '\r')) p++;
        if (*p) *p++ = 0;
    }
    return n;
}

/* tinyobjloader tryParseDouble (src/tiny_obj_loader.cpp:160-266) */
#define IS_DIGIT(x) ((unsigned int)((x) - '0') < (unsigned int)(10))
static int tryParseDouble(const char *s, const char *s_end, double *result) {
    if (s >= s_end) return 0;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char *curr = s;
    int read = 0;
    int end_not_reached = 0;
    if (*curr == '+' || *curr == '-') { sign = *curr; curr++; }
    else if (IS_DIGIT(*curr)) { }
    else return 0;
    end_not_reached = (curr != s_end);
    while (end_not_reached && IS_DIGIT(*curr)) {
        mantissa *= 10;
        mantissa += (int)(*curr - 0x30);
        curr++; read++;
        end_not_reached = (curr != s_end);
    }
    if (read == 0) return 0;
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            mantissa += (int)(*curr - 0x30) * pow(10.0, -read);
            read++; curr++;
            end_not_reached = (curr != s_end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = (curr != s_end);
        if (end_not_reached && (*curr == '+' || *curr == '-')) { exp_sign = *curr; curr++; }
        else if (IS_DIGIT(*curr)) { }
        else return 0;
        read = 0;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            exponent *= 10;
            exponent += (int)(*curr - 0x30);
            curr++; read++;
            end_not_reached = (curr != s_end);
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return 0;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * ldexp(mantissa * pow(5.0, exponent), exponent);
    return 1;
}
static float parseFloatTok(const char **token, double def) { /* :268-276 */
    (*token) += strspn(*token, " \t");
    const char *end = (*token) + strcspn(*token, " \t\r");
    double val = def;
    tryParseDouble(*token, end, &val);
    float f = (float)val;
    *token = end;
    return f;
}
static int fixIndex(int idx, int n) { if (idx > 0) return idx - 1; if (idx == 0) return 0; return n + idx; }

typedef struct {
    char name[256];
    float ambient[3], diffuse[3], specular[3], transmittance[3];
    float ior;
    int illum;
} tmat;

static void tmat_init(tmat *m) { memset(m, 0, sizeof *m); m->ior = 1.f; }

typedef struct { tmat *v; int n, cap; } tmatvec;
static void tmv_push(tmatvec *mv, const tmat *m) {
    if (mv->n == mv->cap) { mv->cap = mv->cap ? 2 * mv->cap : 4; mv->v = (tmat *)realloc(mv->v, sizeof(tmat) * (size_t)mv->cap); }
    mv->v[mv->n++] = *m;
}
static void trim_line(char *line) {
    size_t L = strlen(line);
    /* trailing whitespace trim (LoadMtl only), then \n, \r */
    while (L > 0 && (line[L - 1] == ' ' || line[L - 1] == '\t')) line[--L] = 0;
}
static void load_mtl(const char *path, tmatvec *mv, char names[][256], int *nnames) {
    tmat m;
    tmat_init(&m);
    lreader r;
    int ok = lr_open(&r, path) == 0;
    char line[8192];
    while (ok && r.pos < r.len) {
        lr_getline(&r, line, sizeof line);
        trim_line(line);
        size_t L = strlen(line);
        if (L > 0 && line[L - 1] == '\n') line[--L] = 0;
        if (L > 0 && line[L - 1] == '\r') line[--L] = 0;
        if (L == 0) continue;
        const char *token = line + strspn(line, " \t");
        if (token[0] == 0 || token[0] == '#') continue;
#define ISSP(c) ((c) == ' ' || (c) == '\t')
        if (strncmp(token, "newmtl", 6) == 0 && ISSP(token[6])) {
            if (m.name[0]) { tmv_push(mv, &m); }
            tmat_init(&m);
            sscanf(token + 7, "%255s", m.name);
            continue;
        }
        if (token[0] == 'K' && token[1] == 'a' && ISSP(token[2])) {
            token += 2; for (int i = 0; i < 3; i++) m.ambient[i] = parseFloatTok(&token, 0.0); continue;
        }
        if (token[0] == 'K' && token[1] == 'd' && ISSP(token[2])) {
            token += 2; for (int i = 0; i < 3; i++) m.diffuse[i] = parseFloatTok(&token, 0.0); continue;
        }
        if (token[0] == 'K' && token[1] == 's' && ISSP(token[2])) {
            token += 2; for (int i = 0; i < 3; i++) m.specular[i] = parseFloatTok(&token, 0.0); continue;
        }
        if ((token[0] == 'K' && token[1] == 't' && ISSP(token[2])) || (token[0] == 'T' && token[1] == 'f' && ISSP(token[2]))) {
            token += 2; for (int i = 0; i < 3; i++) m.transmittance[i] = parseFloatTok(&token, 0.0); continue;
        }
        if (token[0] == 'N' && token[1] == 'i' && ISSP(token[2])) { token += 2; m.ior = parseFloatTok(&token, 0.0); continue; }
        if (strncmp(token, "illum", 5) == 0 && ISSP(token[5])) {
            token += 6; token += strspn(token, " \t"); m.illum = atoi(token); continue;
        }
#undef ISSP
    }
    tmv_push(mv, &m); /* "flush last material" always pushes */
    (void)names; (void)nnames;
    free(r.buf);
}

typedef struct { int *idx; int n, cap; } ivec;
static void iv_push(ivec *v, int x) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 64; v->idx = (int *)realloc(v->idx, sizeof(int) * (size_t)v->cap); }
    v->idx[v->n++] = x;
}
typedef struct { float *f; size_t n, cap; } fvec;
static void fv_push(fvec *v, float x) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->f = (float *)realloc(v->f, sizeof(float) * v->cap); }
    v->f[v->n++] = x;
}

/* exportFaceGroupToShape (src/tiny_obj_loader.cpp:425-486): triangle fan into the shape */
static int flush_facegroup(ivec *fg_v, ivec *fg_sz, ivec *shape_idx) {
    int had = fg_sz->n > 0;
    int off = 0;
    for (int fi = 0; fi < fg_sz->n; fi++) {
        int np = fg_sz->idx[fi];
        int i0 = fg_v->idx[off], i1 = -1, i2 = np > 1 ? fg_v->idx[off + 1] : -1;
        for (int kk = 2; kk < np; kk++) {
            i1 = i2; i2 = fg_v->idx[off + kk];
            iv_push(shape_idx, i0); iv_push(shape_idx, i1); iv_push(shape_idx, i2);
        }
        off += np;
    }
    fg_v->n = 0; fg_sz->n = 0;
    return had;
}

int orc_load_obj(const char *obj_path, float **verts9_out, float **norms9_out, int **shape_of_tri, int *ntri_out,
                 orc_material **mats_out, int *nshapes_out) {
    lreader r;
    if (lr_open(&r, obj_path) != 0) return -1;
    char base[4096];
    {
        const char *p1 = strrchr(obj_path, '/'), *p2 = strrchr(obj_path, '\\');
        const char *p = p1 > p2 ? p1 : p2;
        size_t bl = p ? (size_t)(p - obj_path + 1) : 0;
        memcpy(base, obj_path, bl);
        base[bl] = 0;
    }
    fvec v = {0}, vn = {0}, vt = {0};
    tmatvec mats = {0};
    /* faceGroup: flat list of vertex indices per face, with face sizes */
    ivec fg_v = {0}, fg_sz = {0};
    /* current shape (vertex indices of triangulated faces) and finished shapes */
    ivec shape_idx = {0};
    ivec all_idx = {0}, shape_len = {0};
    int cur_material = -1;
    int mapid[4096];
    for (int q = 0; q < 4096; q++) mapid[q] = q;
    char line[65536];
    while (r.pos < r.len) {
        lr_getline(&r, line, sizeof line);
        size_t L = strlen(line);
        if (L > 0 && line[L - 1] == '\n') line[--L] = 0;
        if (L > 0 && line[L - 1] == '\r') line[--L] = 0;
        if (L == 0) continue;
        const char *token = line + strspn(line, " \t");
        if (token[0] == 0 || token[0] == '#') continue;
#define ISSP(c) ((c) == ' ' || (c) == '\t')
#define ISNL(c) ((c) == '\r' || (c) == '\n' || (c) == '\0')
        if (token[0] == 'v' && ISSP(token[1])) {
            token += 2;
            for (int i = 0; i < 3; i++) fv_push(&v, parseFloatTok(&token, 0.0));
            continue;
        }
        if (token[0] == 'v' && token[1] == 'n' && ISSP(token[2])) {
            token += 3;
            for (int i = 0; i < 3; i++) fv_push(&vn, parseFloatTok(&token, 0.0));
            continue;
        }
        if (token[0] == 'v' && token[1] == 't' && ISSP(token[2])) {
            token += 3;
            for (int i = 0; i < 2; i++) fv_push(&vt, parseFloatTok(&token, 0.0));
            continue;
        }
        if (token[0] == 'f' && ISSP(token[1])) {
            token += 2;
            token += strspn(token, " \t");
            int cnt = 0;
            while (!ISNL(token[0])) {
                int vi = fixIndex(atoi(token), (int)(v.n / 3));
                token += strcspn(token, "/ \t\r");
                if (token[0] == '/') {
                    token++;
                    if (token[0] == '/') { token++; token += strcspn(token, "/ \t\r"); }
                    else {
                        token += strcspn(token, "/ \t\r");
                        if (token[0] == '/') { token++; token += strcspn(token, "/ \t\r"); }
                    }
                }
                iv_push(&fg_v, vi);
                cnt++;
                token += strspn(token, " \t\r");
            }
            iv_push(&fg_sz, cnt);
            continue;
        }
        int is_usemtl = (strncmp(token, "usemtl", 6) == 0 && ISSP(token[6]));
        int is_g = (token[0] == 'g' && ISSP(token[1]));
        int is_o = (token[0] == 'o' && ISSP(token[1]));
        if (is_usemtl) {
            /* src/tiny_obj_loader.cpp:977-1002: flush into the CURRENT shape only when the id changes */
            char nm[4096] = {0};
            sscanf(token + 7, "%4095s", nm);
            int newid = -1;
            for (int q = 0; q < mats.n; q++)
                if (strcmp(mats.v[q].name, nm) == 0) { newid = mapid[q]; break; }
            if (newid != cur_material) {
                flush_facegroup(&fg_v, &fg_sz, &shape_idx);
                cur_material = newid;
            }
            continue;
        }
        if (is_g || is_o) {
            /* src/tiny_obj_loader.cpp:1031-1089: flush, push the shape only if the group had faces */
            int had = flush_facegroup(&fg_v, &fg_sz, &shape_idx);
            if (had) {
                for (int q = 0; q < shape_idx.n; q++) iv_push(&all_idx, shape_idx.idx[q]);
                iv_push(&shape_len, shape_idx.n);
            }
            shape_idx.n = 0;
            continue;
        }
        if (strncmp(token, "mtllib", 6) == 0 && ISSP(token[6])) {
            char nm[4096];
            if (sscanf(token + 7, "%4095s", nm) == 1) {
                char path[8192];
                snprintf(path, sizeof path, "%s%s", base, nm);
                load_mtl(path, &mats, NULL, NULL);
            }
            continue;
        }
#undef ISSP
#undef ISNL
    }
    {   /* final flush (src/tiny_obj_loader.cpp:1140-1144) */
        int had = flush_facegroup(&fg_v, &fg_sz, &shape_idx);
        if (had) {
            for (int q = 0; q < shape_idx.n; q++) iv_push(&all_idx, shape_idx.idx[q]);
            iv_push(&shape_len, shape_idx.n);
        }
    }
    /* Scene::getTrianglesFromScene_ (src/scene.cpp:531-577): normals gathered by VERTEX index */
    int ntri = all_idx.n / 3;
    float *V9 = (float *)malloc(sizeof(float) * 9 * (size_t)(ntri > 0 ? ntri : 1));
    float *N9 = (float *)malloc(sizeof(float) * 9 * (size_t)(ntri > 0 ? ntri : 1));
    int *S = (int *)malloc(sizeof(int) * (size_t)(ntri > 0 ? ntri : 1));
    int t = 0, pos = 0;
    for (int sh = 0; sh < shape_len.n; sh++) {
        for (int j = pos; j < pos + shape_len.idx[sh]; j += 3) {
            for (int c = 0; c < 3; c++) {
                size_t p = 3 * (size_t)all_idx.idx[j + c];
                for (int a = 0; a < 3; a++) {
                    V9[9 * t + 3 * c + a] = (p + a < v.n) ? v.f[p + a] : 0.0f;
                    N9[9 * t + 3 * c + a] = (p + a < vn.n) ? vn.f[p + a] : 0.0f;
                }
            }
            S[t] = sh;
            t++;
        }
        pos += shape_len.idx[sh];
    }
    /* per-shape materials (src/scene.cpp:716-822) */
    int nsh = shape_len.n;
    orc_material *M = (orc_material *)calloc((size_t)(nsh > 0 ? nsh : 1), sizeof(orc_material));
    for (int i = 0; i < nsh; i++) {
        orc_material *om = &M[i];
        if (mats.n > i) {
            const tmat *tm = &mats.v[i];
            for (int c = 0; c < 3; c++) om->color[c] = tm->ambient[c] > tm->diffuse[c] ? tm->ambient[c] : tm->diffuse[c];
            if (tm->illum <= 2) {
                om->spec_exponent = 0.0f; om->hasReflective = 0.0f; om->hasRefractive = 0.0f; om->indexOfRefraction = 0.0f;
            } else if (tm->illum == 3) {
                om->spec_exponent = 1.0f;
                for (int c = 0; c < 3; c++) om->spec_color[c] = tm->specular[c];
                om->hasReflective = 1.0f; om->hasRefractive = 0.0f; om->indexOfRefraction = 0.0f;
            } else {
                om->spec_exponent = 1.0f;
                for (int c = 0; c < 3; c++) om->spec_color[c] = tm->specular[c];
                om->hasReflective = 1.0f; om->hasRefractive = 1.0f; om->indexOfRefraction = tm->ior;
            }
            for (int c = 0; c < 3; c++) om->transmittance[c] = tm->transmittance[c];
        } else {
            for (int c = 0; c < 3; c++) om->color[c] = 1.0f;
            /* objmesh->materials[i].transmittance is read out of bounds here in the reference; zero */
        }
        om->emittance = 0.0f;
    }
    *verts9_out = V9; *norms9_out = N9; *shape_of_tri = S; *ntri_out = ntri;
    *mats_out = M; *nshapes_out = nsh;
    free(v.f); free(vn.f); free(vt.f); free(mats.v); free(fg_v.idx); free(fg_sz.idx);
    free(shape_idx.idx); free(all_idx.idx); free(shape_len.idx); free(r.buf);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Scene (src/scene.cpp) + runCuda camera (src/main.cpp)                  */
/* ------------------------------------------------------------------ */
int orc_parse_scene(const char *scene_path, const char *obj_path, orc_scene_desc *d) {
    memset(d, 0, sizeof *d);
    lreader r;
    if (lr_open(&r, scene_path) != 0) return -1;
    int gcap = 16, mcap = 16, ng = 0, nm = 0;
    orc_material *mats = (orc_material *)calloc((size_t)mcap, sizeof(orc_material));
    int *gtype = (int *)calloc((size_t)gcap, sizeof(int));
    int *gmat = (int *)calloc((size_t)gcap, sizeof(int));
    float *gtrs = (float *)calloc((size_t)gcap * 9, sizeof(float));
    char line[8192], work[8192];
    char *tok[MAXTOK];
    while (!r.eof) {
        lr_getline(&r, line, sizeof line);
        if (!line[0]) continue;
        strcpy(work, line);
        int nt = tokenize(work, tok);
        if (nt == 0) continue;
        if (strcmp(tok[0], "MATERIAL") == 0 && nt > 1) {
            /* Scene::loadMaterial src/scene.cpp:236-271 */
            int id = atoi(tok[1]);
            if (id != nm) continue;
            orc_material m;
            memset(&m, 0, sizeof m);
            for (int i = 0; i < 7; i++) {
                lr_getline(&r, line, sizeof line);
                strcpy(work, line);
                int n2 = tokenize(work, tok);
                if (n2 == 0) continue;
                if (strcmp(tok[0], "RGB") == 0 && n2 >= 4) { for (int c = 0; c < 3; c++) m.color[c] = (float)atof(tok[1 + c]); }
                else if (strcmp(tok[0], "SPECEX") == 0 && n2 >= 2) m.spec_exponent = (float)atof(tok[1]);
                else if (strcmp(tok[0], "SPECRGB") == 0 && n2 >= 4) { for (int c = 0; c < 3; c++) m.spec_color[c] = (float)atof(tok[1 + c]); }
                else if (strcmp(tok[0], "REFL") == 0 && n2 >= 2) m.hasReflective = (float)atof(tok[1]);
                else if (strcmp(tok[0], "REFR") == 0 && n2 >= 2) m.hasRefractive = (float)atof(tok[1]);
                else if (strcmp(tok[0], "REFRIOR") == 0 && n2 >= 2) m.indexOfRefraction = (float)atof(tok[1]);
                else if (strcmp(tok[0], "EMITTANCE") == 0 && n2 >= 2) m.emittance = (float)atof(tok[1]);
            }
            if (nm == mcap) { mcap *= 2; mats = (orc_material *)realloc(mats, sizeof(orc_material) * (size_t)mcap); }
            mats[nm++] = m;
        } else if (strcmp(tok[0], "OBJECT") == 0 && nt > 1) {
            /* Scene::loadGeom src/scene.cpp:118-173 */
            int id = atoi(tok[1]);
            if (id != ng) continue;
            int type = -1, matid = 0;
            lr_getline(&r, line, sizeof line);
            if (line[0] && !r.eof) {
                if (strcmp(line, "sphere") == 0) type = 0;
                else if (strcmp(line, "cube") == 0) type = 1;
            }
            lr_getline(&r, line, sizeof line);
            if (line[0] && !r.eof) {
                strcpy(work, line);
                int n2 = tokenize(work, tok);
                if (n2 > 1) matid = atoi(tok[1]);
            }
            float trs[9] = {0};
            lr_getline(&r, line, sizeof line);
            while (line[0] && !r.eof) {
                strcpy(work, line);
                int n2 = tokenize(work, tok);
                if (n2 >= 4) {
                    float vv[3] = {(float)atof(tok[1]), (float)atof(tok[2]), (float)atof(tok[3])};
                    if (strcmp(tok[0], "TRANS") == 0) memcpy(trs, vv, 12);
                    else if (strcmp(tok[0], "ROTAT") == 0) memcpy(trs + 3, vv, 12);
                    else if (strcmp(tok[0], "SCALE") == 0) memcpy(trs + 6, vv, 12);
                }
                lr_getline(&r, line, sizeof line);
            }
            if (ng == gcap) {
                gcap *= 2;
                gtype = (int *)realloc(gtype, sizeof(int) * (size_t)gcap);
                gmat = (int *)realloc(gmat, sizeof(int) * (size_t)gcap);
                gtrs = (float *)realloc(gtrs, sizeof(float) * 9 * (size_t)gcap);
            }
            gtype[ng] = type; gmat[ng] = matid; memcpy(gtrs + 9 * ng, trs, sizeof trs);
            ng++;
        } else if (strcmp(tok[0], "CAMERA") == 0) {
            /* Scene::loadCamera src/scene.cpp:175-234 */
            for (int i = 0; i < 5; i++) {
                lr_getline(&r, line, sizeof line);
                strcpy(work, line);
                int n2 = tokenize(work, tok);
                if (n2 == 0) continue;
                if (strcmp(tok[0], "RES") == 0 && n2 >= 3) { d->res[0] = atoi(tok[1]); d->res[1] = atoi(tok[2]); }
                else if (strcmp(tok[0], "FOVY") == 0 && n2 >= 2) d->fovy = (float)atof(tok[1]);
                else if (strcmp(tok[0], "ITERATIONS") == 0 && n2 >= 2) d->iterations = atoi(tok[1]);
                else if (strcmp(tok[0], "DEPTH") == 0 && n2 >= 2) d->traceDepth = atoi(tok[1]);
            }
            lr_getline(&r, line, sizeof line);
            while (line[0] && !r.eof) {
                strcpy(work, line);
                int n2 = tokenize(work, tok);
                if (n2 >= 4) {
                    float vv[3] = {(float)atof(tok[1]), (float)atof(tok[2]), (float)atof(tok[3])};
                    if (strcmp(tok[0], "EYE") == 0) memcpy(d->eye, vv, 12);
                    else if (strcmp(tok[0], "LOOKAT") == 0) memcpy(d->lookAt, vv, 12);
                    else if (strcmp(tok[0], "UP") == 0) memcpy(d->up, vv, 12);
                }
                lr_getline(&r, line, sizeof line);
            }
        }
    }
    free(r.buf);
    d->num_materials = nm; d->materials = mats;
    d->num_geoms = ng; d->geom_type = gtype; d->geom_material = gmat; d->geom_trs = gtrs;
    if (obj_path && obj_path[0]) {
        float *V9, *N9;
        int *S, ntri, nsh;
        orc_material *M;
        if (orc_load_obj(obj_path, &V9, &N9, &S, &ntri, &M, &nsh) != 0) return -2;
        d->ntri = ntri; d->verts9 = V9; d->norms9 = N9; d->shape_of_tri = S;
        d->num_shapes = nsh; d->shape_materials = M;
    }
    return 0;
}

void orc_free_desc(orc_scene_desc *d) {
    free((void *)d->materials); free((void *)d->geom_type); free((void *)d->geom_material); free((void *)d->geom_trs);
    free((void *)d->verts9); free((void *)d->norms9); free((void *)d->shape_of_tri); free((void *)d->shape_materials);
    memset(d, 0, sizeof *d);
}

/* The raw OBJ arrays Scene::loadObj keeps for the brute-force kernel (src/scene.cpp:603-712), from
 * the per-triangle soup: vertex index 3*t+k holds triangle t's k-th vertex (and its vertex-index-
 * gathered normal), so every value the kernel reads is the one the reference reads.  Shapes are the
 * runs of shape_of_tri.  The bboxes follow the reference's loop: first vertex of each triangle only,
 * max initialised to 0, stored at [iterator .. iterator+5] (in-bounds here: the buffer is sized for it). */
static void obj_arrays(const orc_scene_desc *d, orc_scene *out) {
    int nt = d->ntri, nsh = d->num_shapes;
    out->polyidxcount = 3 * nt;
    out->obj_verts = (float *)malloc(sizeof(float) * 9 * (size_t)nt);
    out->obj_norms = (float *)malloc(sizeof(float) * 9 * (size_t)nt);
    memcpy(out->obj_verts, d->verts9, sizeof(float) * 9 * (size_t)nt);
    memcpy(out->obj_norms, d->norms9, sizeof(float) * 9 * (size_t)nt);
    out->obj_polysidxflat = (int *)malloc(sizeof(int) * 3 * (size_t)nt);
    for (int j = 0; j < 3 * nt; j++) out->obj_polysidxflat[j] = j;
    out->obj_polyoffsets = (int *)calloc((size_t)(nsh > 0 ? nsh : 1), sizeof(int));
    for (int t = 0; t < nt; t++) {
        int sh = d->shape_of_tri[t];
        if (sh >= 0 && sh < nsh) out->obj_polyoffsets[sh] += 3;
    }
    int nb = 6 * nsh, it = 0;
    for (int i = 0; i < nsh; i++) { if (it + 6 > nb) nb = it + 6; it += out->obj_polyoffsets[i]; }
    if (nsh + 5 > nb) nb = nsh + 5;
    out->num_bbox_floats = nb;
    out->obj_bboxes = (float *)calloc((size_t)nb, sizeof(float));
    int iterator = 0;
    for (int i = 0; i < nsh; i++) {
        float minx = FLT_MAX, maxx = 0.0f, miny = FLT_MAX, maxy = 0.0f, minz = FLT_MAX, maxz = 0.0f;
        for (int j = iterator; j < iterator + out->obj_polyoffsets[i]; j += 3) {
            const float *v = out->obj_verts + 3 * out->obj_polysidxflat[j];
            if (v[0] < minx) minx = v[0];
            if (v[0] > maxx) maxx = v[0];
            if (v[1] < miny) miny = v[1];
            if (v[1] > maxy) maxy = v[1];
            if (v[2] < minz) minz = v[2];
            if (v[2] > maxz) maxz = v[2];
        }
        float *b = out->obj_bboxes + iterator;
        b[0] = minx; b[1] = miny; b[2] = minz; b[3] = maxx; b[4] = maxy; b[5] = maxz;
        iterator += out->obj_polyoffsets[i];
    }
}

int orc_build_scene(const orc_scene_desc *d, orc_scene *out) {
    memset(out, 0, sizeof *out);
    orc_camera *cam = &out->camera;
    out->iterations = d->iterations;
    out->traceDepth = d->traceDepth;
    int nm = d->num_materials + (d->ntri > 0 ? d->num_shapes : 0);
    out->materials = (orc_material *)calloc((size_t)(nm > 0 ? nm : 1), sizeof(orc_material));
    memcpy(out->materials, d->materials, sizeof(orc_material) * (size_t)d->num_materials);
    out->num_materials = d->num_materials;
    out->geoms = (orc_geom *)calloc((size_t)(d->num_geoms > 0 ? d->num_geoms : 1), sizeof(orc_geom));
    out->num_geoms = d->num_geoms;
    for (int i = 0; i < d->num_geoms; i++) {
        orc_geom *g = &out->geoms[i];
        g->type = d->geom_type[i];
        g->materialid = d->geom_material[i];
        const float *trs = d->geom_trs + 9 * i;
        memcpy(g->translation, trs, 12); memcpy(g->rotation, trs + 3, 12); memcpy(g->scale, trs + 6, 12);
        m4 tr = buildTransformationMatrix(V3(trs[0], trs[1], trs[2]), V3(trs[3], trs[4], trs[5]), V3(trs[6], trs[7], trs[8]));
        m4 inv = m4inverse(&tr);
        m4 it = m4inverseTranspose(&tr);
        memcpy(g->transform, &tr, 64); memcpy(g->inverseTransform, &inv, 64); memcpy(g->invTranspose, &it, 64);
    }
    cam->resolution[0] = d->res[0]; cam->resolution[1] = d->res[1];
    memcpy(cam->position, d->eye, 12); memcpy(cam->lookAt, d->lookAt, 12); memcpy(cam->up, d->up, 12);
    float fovy = d->fovy;
    {   /* loadCamera fov / pixelLength / view (src/scene.cpp:215-225) */
        float yscaled = tanf(fovy * (PI_F / 180.0f));
        float xscaled = (yscaled * (float)cam->resolution[0]) / (float)cam->resolution[1];
        float fovx = (atanf(xscaled) * 180.0f) / PI_F;
        cam->fov[0] = fovx; cam->fov[1] = fovy;
        cam->pixelLength[0] = 2 * xscaled / (float)cam->resolution[0];
        cam->pixelLength[1] = 2 * yscaled / (float)cam->resolution[1];
        v3 view = vnormalize(vsub(V3(d->lookAt[0], d->lookAt[1], d->lookAt[2]), V3(d->eye[0], d->eye[1], d->eye[2])));
        memcpy(cam->view, &view, 12);
    }
    {   /* main(): phi/theta/zoom (src/main.cpp:1059-1073) then runCuda (src/main.cpp:1111-1129) */
        v3 view = V3(cam->view[0], cam->view[1], cam->view[2]);
        v3 pos = V3(cam->position[0], cam->position[1], cam->position[2]);
        v3 look = V3(cam->lookAt[0], cam->lookAt[1], cam->lookAt[2]);
        v3 viewXZ = V3(view.x, 0.0f, view.z), viewZY = V3(0.0f, view.y, view.z);
        float phi = acosf(vdot(vnormalize(viewXZ), V3(0, 0, -1)));
        float theta = acosf(vdot(vnormalize(viewZY), V3(0, 1, 0)));
        float zoom = vlength(vsub(pos, look));
        v3 camoffset = V3(0, 0, 0);
        v3 cp;
        cp.x = zoom * sinf(phi) * sinf(theta) + camoffset.x;
        cp.y = zoom * cosf(theta) + camoffset.y;
        cp.z = zoom * cosf(phi) * sinf(theta) + camoffset.z;
        v3 nv = vneg(vnormalize(cp));
        v3 rr = vcross(nv, V3(0, 1, 0));
        v3 nu = vcross(rr, nv);
        memcpy(cam->view, &nv, 12); memcpy(cam->up, &nu, 12); memcpy(cam->right, &rr, 12);
        cp = vadd(cp, vadd(look, camoffset));
        memcpy(cam->position, &cp, 12);
    }
    if (d->ntri > 0) {
        int nsh = d->num_shapes;
        out->num_shapes = nsh;
        out->obj_materialOffsets = (int *)calloc((size_t)(nsh > 0 ? nsh : 1), sizeof(int));
        for (int i = 0; i < nsh; i++) {
            out->obj_materialOffsets[i] = out->num_materials;
            out->materials[out->num_materials++] = d->shape_materials[i];
        }
        orc_build_kd(d->verts9, d->norms9, d->shape_of_tri, d->ntri, 13, &out->nodes, &out->num_nodes, &out->tris,
                     &out->num_tris);
        out->has_obj = 1;
        obj_arrays(d, out);
    }
    return 0;
}

int orc_load_scene(const char *scene_path, const char *obj_path, int res_w, int res_h, int depth, orc_scene *out) {
    orc_scene_desc d;
    int rc = orc_parse_scene(scene_path, obj_path, &d);
    if (rc) { orc_free_desc(&d); return rc; }
    if (res_w > 0 && res_h > 0) { d.res[0] = res_w; d.res[1] = res_h; }
    if (depth > 0) d.traceDepth = depth;
    rc = orc_build_scene(&d, out);
    orc_free_desc(&d);
    return rc;
}

void orc_free_scene(orc_scene *s) {
    free(s->geoms); free(s->materials); free(s->obj_materialOffsets); free(s->nodes); free(s->tris);
    free(s->obj_verts); free(s->obj_norms); free(s->obj_polysidxflat); free(s->obj_polyoffsets); free(s->obj_bboxes);
    memset(s, 0, sizeof *s);
}

/* saveImage (src/main.cpp:1087-1108) + image::savePNG's byte conversion (src/image.cpp:22-35):
 * img.setPixel(width-1-x, y, pix / samples); glm::clamp(p, 0, 1) * 255.f; (unsigned char).
 * lin (optional) receives the flipped, divided floats (what image::saveHDR writes). */
void orc_save_image(const float *image, int W, int H, float samples, unsigned char *rgb, float *lin) {
    for (int x = 0; x < W; x++)
        for (int y = 0; y < H; y++) {
            int src = 3 * (x + y * W), dst = 3 * ((W - 1 - x) + y * W);
            for (int k = 0; k < 3; k++) {
                float v = image[src + k] / samples;
                if (lin) lin[dst + k] = v;
                float mx = v > 0.0f ? v : 0.0f;       /* glm::max(x, y) = x > y ? x : y */
                float cl = mx < 1.0f ? mx : 1.0f;     /* glm::min(x, y) = x < y ? x : y */
                if (rgb) rgb[dst + k] = (unsigned char)(cl * 255.f);
            }
        }
}

/* Known answers of the glm pieces (vendored glm 0.9.6.3; kdpt_selftest_glm's numbering):
 * fn 0 intersectRayTriangle (o, d, v0, v1, v2 -> passed, bary.xyz; out[1..3] hold the caller's
 * sentinels, kept where glm does not write), 1 normalize, 2 reflect, 3 refract, 4 glm::rotate(quat, v). */
void orc_glm_array(int fn, const float *in, int n, float *out) {
    const int ni = fn == 0 ? 15 : fn == 1 ? 3 : fn == 2 ? 6 : 7, no = fn == 0 ? 4 : 3;
    for (int i = 0; i < n; i++) {
        const float *a = in + (size_t)ni * i;
        float *o = out + (size_t)no * i;
        v3 r = V3(0.0f, 0.0f, 0.0f);
        if (fn == 0) {
            v3 bary = V3(o[1], o[2], o[3]);
            int hit = intersectRayTriangle(V3(a[0], a[1], a[2]), V3(a[3], a[4], a[5]), V3(a[6], a[7], a[8]),
                                           V3(a[9], a[10], a[11]), V3(a[12], a[13], a[14]), &bary);
            o[0] = hit ? 1.0f : 0.0f;
            o[1] = bary.x; o[2] = bary.y; o[3] = bary.z;
            continue;
        } else if (fn == 1) {
            r = vnormalize(V3(a[0], a[1], a[2]));
        } else if (fn == 2) {
            r = glm_reflect(V3(a[0], a[1], a[2]), V3(a[3], a[4], a[5]));
        } else if (fn == 3) {
            r = glm_refract(V3(a[0], a[1], a[2]), V3(a[3], a[4], a[5]), a[6]);
        } else if (fn == 4) { /* q * v, gtc/quaternion.inl:319-326 */
            v3 q = V3(a[1], a[2], a[3]), v = V3(a[4], a[5], a[6]);
            v3 uv = vcross(q, v), uuv = vcross(q, uv);
            r = vadd(v, vscale(vadd(vscale(uv, a[0]), uuv), 2.0f));
        }
        o[0] = r.x; o[1] = r.y; o[2] = r.z;
    }
}

/* Geom matrices (src/scene.cpp:165-168): buildTransformationMatrix (src/utilities.cpp:65-72),
 * glm::inverse, glm::inverseTranspose of n translation/rotation/scale triples -> 48 floats each. */
void orc_geom_matrices(const float *trs, int n, float *out) {
    for (int i = 0; i < n; i++) {
        const float *t = trs + 9 * (size_t)i;
        m4 tr = buildTransformationMatrix(V3(t[0], t[1], t[2]), V3(t[3], t[4], t[5]), V3(t[6], t[7], t[8]));
        m4 inv = m4inverse(&tr), it = m4inverseTranspose(&tr);
        memcpy(out + 48 * (size_t)i, &tr, 64);
        memcpy(out + 48 * (size_t)i + 16, &inv, 64);
        memcpy(out + 48 * (size_t)i + 32, &it, 64);
    }
}
