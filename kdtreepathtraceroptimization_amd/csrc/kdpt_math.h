// kdpt_math.h -- float/double arithmetic of the reference hot path, restated so
// that gfx950 and x86 evaluate the SAME IEEE operations in the SAME order.
//
// Compiled with -ffp-contract=off (never fuse) and without fast-math, so a
// correctly-rounded v_div/v_sqrt sequence is used for `/` and sqrtf.  Every
// function cites the reference (or vendored glm 0.9.6.3 / rocThrust) code it
// follows.  Transcendentals the reference gets from glibc are restated
// bit-exactly (kdpt_sinf/kdpt_cosf: glibc 2.35 sysdeps/ieee754/flt-32
// s_sinf.c/s_cosf.c FMA variant -- verified over every |x| < 119 float).
//
// The glibc restatements below follow GNU C Library 2.35 (LGPL-2.1-or-later; e_acosf.c also under
// Sun Microsystems' fdlibm notice): see THIRD_PARTY_NOTICES.md at the repository root.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define KDPT_HD __host__ __device__ inline
#define KDPT_HDI __host__ __device__ inline __attribute__((always_inline))
#else
#define KDPT_HDI static inline
#define KDPT_HD static inline
#include <math.h>
// host-only builds (tests/native differential harness): HIP's vector types
struct float4 { float x, y, z, w; };
struct int4 { int x, y, z, w; };
struct int2 { int x, y; };
struct ulonglong2 { unsigned long long x, y; };
static inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }
static inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }
static inline int2 make_int2(int x, int y) { return int2{x, y}; }
#endif

namespace kdpt {

// src/utilities.h:9-12
constexpr float PI_F = 3.1415926535897932384626422832795028841971f;
constexpr float TWO_PI_F = 6.2831853071795864769252867665590057683943f;
constexpr float SQRT_OF_ONE_THIRD_F = 0.5773502691896257645091487805019574556476f;
constexpr float FLT_EPS = 1.19209290e-07f;   // std::numeric_limits<float>::epsilon()
constexpr float FLT_MAXV = 3.40282347e+38f;
constexpr float FLT_INFV = __builtin_inff();

struct f3 {
  float x, y, z;
};
struct f4 {
  float x, y, z, w;
};

KDPT_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
KDPT_HD f3 add(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
KDPT_HD f3 sub(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
KDPT_HD f3 mul(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
KDPT_HD f3 scl(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
KDPT_HD f3 neg(f3 a) { return mk3(-a.x, -a.y, -a.z); }
KDPT_HD float comp(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
// glm compute_dot<tvec3>: tmp = x*y; (tmp.x + tmp.y) + tmp.z
KDPT_HD float dot(f3 a, f3 b) {
  float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return tx + ty + tz;
}
// glm cross (detail/func_geometric.inl)
KDPT_HD f3 cross(f3 x, f3 y) {
  return mk3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// glm normalize = x * inversesqrt(dot(x,x)); inversesqrt(x) = 1 / sqrt(x)
KDPT_HD f3 normalize(f3 x) {
  float inv = 1.0f / sqrtf(dot(x, x));
  return scl(x, inv);
}
KDPT_HD float length(f3 v) { return sqrtf(dot(v, v)); }
KDPT_HD float distance(f3 p0, f3 p1) { return length(sub(p1, p0)); }
// glm reflect / refract (detail/func_geometric.inl)
KDPT_HD f3 reflect(f3 I, f3 N) { return sub(I, scl(scl(N, dot(N, I)), 2.0f)); }
KDPT_HD f3 refract(f3 I, f3 N, float eta) {
  float dv = dot(N, I);
  float k = 1.0f - eta * eta * (1.0f - dv * dv);
  f3 r = sub(scl(I, eta), scl(N, eta * dv + sqrtf(k)));
  return scl(r, (float)(k >= 0.0f));
}
// glm::rotate(quat, vec3) = quat * vec3 (gtx/quaternion.inl:153-160, gtc/quaternion.inl:319-326):
// v + ((uv * w) + uuv) * 2 with uv = cross(q.xyz, v), uuv = cross(q.xyz, uv)
KDPT_HD f3 quat_rotate(float w, f3 q, f3 v) {
  const f3 uv = cross(q, v);
  const f3 uuv = cross(q, uv);
  return add(v, scl(add(scl(uv, w), uuv), 2.0f));
}
// glm::min/max (detail/func_common.inl:409-435) and std::min/max
KDPT_HD float glm_min(float x, float y) { return x < y ? x : y; }
KDPT_HD float glm_max(float x, float y) { return x > y ? x : y; }
KDPT_HD float std_min(float a, float b) { return (b < a) ? b : a; }
KDPT_HD float std_max(float a, float b) { return (a < b) ? b : a; }

// ---- mat4 (column major, glm detail/type_mat4x4.inl) ----
struct m4 {
  f4 c[4];
};
KDPT_HD f4 add4(f4 a, f4 b) { return f4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
KDPT_HD f4 sub4(f4 a, f4 b) { return f4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
KDPT_HD f4 mul4(f4 a, f4 b) { return f4{a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
KDPT_HD f4 scl4(f4 a, float s) { return f4{a.x * s, a.y * s, a.z * s, a.w * s}; }
// operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)   (type_mat4x4.inl:592-638)
KDPT_HD f3 mulMV(const float* m, f4 v) {
  f4 c0{m[0], m[1], m[2], m[3]}, c1{m[4], m[5], m[6], m[7]};
  f4 c2{m[8], m[9], m[10], m[11]}, c3{m[12], m[13], m[14], m[15]};
  f4 a0 = add4(scl4(c0, v.x), scl4(c1, v.y));
  f4 a1 = add4(scl4(c2, v.z), scl4(c3, v.w));
  f4 r = add4(a0, a1);
  return mk3(r.x, r.y, r.z);
}

// ---- glibc sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, s_sincosf.h,
//      sincosf_data.c), x86_64 FMA ifunc variant: GCC fuses every a + b*c. ----
KDPT_HD uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
KDPT_HD float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
KDPT_HD int fbits(float f) { return (int)f2u(f); }
KDPT_HD float ibits(int i) { return u2f((uint32_t)i); }
KDPT_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }
KDPT_HD double dfma(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return fma(a, b, c);
#endif
}
// __sincosf_table[2] (sincosf_data.c): the two entries differ only in the sign of
// the cosine polynomial c0..c4, so entry k is passed as cs = +1.0 / -1.0 (exact).
KDPT_HD float sinf_poly(double x, double x2, double cs, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = dfma(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
    double x7 = x3 * x2;
    double s = dfma(x3, -0x1.555545995a603p-3, x);
    return (float)dfma(x7, s1, s);
  } else {
    double x4 = x2 * x2;
    double c2 = dfma(x2, cs * 0x1.99343027bf8c3p-16, cs * -0x1.6c087e89a359dp-10);
    double c1 = dfma(x2, cs * -0x1.ffffffd0c621cp-2, cs * 0x1p0);
    double x6 = x4 * x2;
    double c = dfma(x4, cs * 0x1.55553e1068f19p-5, c1);
    return (float)dfma(x6, c2, c);
  }
}
KDPT_HD double quadrant_sign(int q) { return (q == 1 || q == 2) ? -1.0 : 1.0; }  // sign[4] = {1,-1,-1,1}
KDPT_HD double reduce_fast(double x, int* np) {
  double r = x * 0x1.45F306DC9C883p+23;  // hpi_inv (2/PI * 2^24, !TOINT_INTRINSICS)
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return dfma(-(double)n, 0x1.921FB54442D18p0, x);  // x - n * hpi, fused in the FMA build
}
// 4/PI in 8-bit steps (glibc __inv_pio4); bits of 2/PI = 0.A2F9836E4E441529FC2757D1F534DDC0DB6295993C439041
KDPT_HD uint32_t inv_pio4(int i) {
  const uint64_t w0 = 0xA2F9836E4E441529ull, w1 = 0xFC2757D1F534DDC0ull, w2 = 0xDB6295993C439041ull;
  // entry i = bytes [i-3 .. i] of the 24-byte string (zero-extended on the left)
  uint32_t r = 0;
  for (int b = i - 3; b <= i; b++) {
    uint32_t byte = 0;
    if (b >= 0) {
      uint64_t w = b < 8 ? w0 : (b < 16 ? w1 : w2);
      int sh = 56 - 8 * (b & 7);
      byte = (uint32_t)((w >> sh) & 0xff);
    }
    r = (r << 8) | byte;
  }
  return r;
}
KDPT_HD double reduce_large(uint32_t xi, int* np) {
  const int base = (xi >> 26) & 15;
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = xi * inv_pio4(base);
  res1 = (uint64_t)xi * inv_pio4(base + 4);
  res2 = (uint64_t)xi * inv_pio4(base + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;  // pi63
}
KDPT_HD float kdpt_sinf(float y) {
  double x = y, s;
  int n;
  const float pio4f = (float)0x1.921FB54442D18p-1;
  if (abstop12(y) < abstop12(pio4f)) {
    s = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return sinf_poly(x, s, 1.0, 0);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, &n);
    s = quadrant_sign(n & 3);
    return sinf_poly(x * s, x * x, (n & 2) ? -1.0 : 1.0, n);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    uint32_t xi = f2u(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    s = quadrant_sign((n + sign) & 3);
    return sinf_poly(x * s, x * x, ((n + sign) & 2) ? -1.0 : 1.0, n);
  }
  return (y - y) / (y - y);
}
KDPT_HD float kdpt_cosf(float y) {
  double x = y, s;
  int n;
  const float pio4f = (float)0x1.921FB54442D18p-1;
  if (abstop12(y) < abstop12(pio4f)) {
    double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x2, 1.0, 1);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, &n);
    s = quadrant_sign(n & 3);
    return sinf_poly(x * s, x * x, (n & 2) ? -1.0 : 1.0, n ^ 1);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    uint32_t xi = f2u(y);
    int sign = xi >> 31;
    x = reduce_large(xi, &n);
    s = quadrant_sign((n + sign) & 3);
    return sinf_poly(x * s, x * x, ((n + sign) & 2) ? -1.0 : 1.0, n ^ 1);
  }
  return (y - y) / (y - y);
}

// pow(double x, 5.0) as glibc's correctly-rounded-in-practice pow computes it:
// x is a float value, so x*x is exact; x^4 and x^5 are carried double-double.
KDPT_HD double pow5(double x) {
  double x2 = x * x;
  double x4 = x2 * x2;
  double x4e = dfma(x2, x2, -x4);
  double x5 = x4 * x;
  double x5e = dfma(x4, x, -x5) + x4e * x;
  return x5 + x5e;
}

// ---- glibc 2.35 acosf (sysdeps/ieee754/flt-32/e_acosf.c, the fdlibm float version; the
//      libm.so.6 code is plain SSE single precision, no FMA variant).  Constants are the
//      fdlibm words.  Used by randSphericalVec / the soft lobe / fake SSS (src/interactions.h:73,
//      214, 266-...).  |x| > 1 (possible when a normalised direction's z rounds above 1): glibc's
//      wrapper returns the quiet NaN 0x7fc00000 (__kernel_standard_f, acosf domain error); a NaN
//      input comes back quietened.
KDPT_HDI float kdpt_acosf(float x) {
  const float one = 1.0f, pi = u2f(0x40490fdau), pio2_hi = u2f(0x3fc90fdau), pio2_lo = u2f(0x33a22168u);
  const float pS0 = u2f(0x3e2aaaabu), pS1 = u2f(0xbea6b090u), pS2 = u2f(0x3e4e0aa8u), pS3 = u2f(0xbd241146u),
              pS4 = u2f(0x3a4f7f04u), pS5 = u2f(0x3811ef08u);
  const float qS1 = u2f(0xc019d139u), qS2 = u2f(0x4001572du), qS3 = u2f(0xbf303361u), qS4 = u2f(0x3d9dc62eu);
  const int32_t hx = (int32_t)f2u(x);
  const int32_t ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) {  // |x| == 1
    if (hx > 0) return 0.0f;
    return pi + 2.0f * pio2_lo;
  } else if (ix > 0x7f800000) {
    return u2f((uint32_t)hx | 0x00400000u);  // NaN in: (x - x) / (x - x), the input quietened
  } else if (ix > 0x3f800000) {
    return u2f(0x7fc00000u);  // |x| > 1: the wrapper's domain-error NaN
  }
  if (ix < 0x3f000000) {  // |x| < 0.5
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    float z = x * x;
    float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    float r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {  // x < -0.5
    float z = (one + x) * 0.5f;
    float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    float s = sqrtf(z);
    float r = p / q;
    float w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  } else {  // x > 0.5
    float z = (one - x) * 0.5f;
    float s = sqrtf(z);
    float df = u2f(f2u(s) & 0xfffff000u);
    float c = (z - df * df) / (s + df);
    float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    float r = p / q;
    float w = r * s + c;
    return 2.0f * (df + w);
  }
}

// ---- glibc 2.35 double sin / cos (sysdeps/ieee754/dbl-64/s_sin.c: do_sin, do_cos,
//      reduce_sincos, TAYLOR_SIN; constants usncs.h), as the x86_64 FMA ifunc variant
//      (__sin_fma / __cos_fma, built with -mfma -mavx2) evaluates it: the products GCC fused
//      into vfmadd/vfnmadd/vfmsub are the dfma() calls below, everything else is a single
//      IEEE double op.  Read off the libm.so.6 machine code; checked against glibc on every
//      float argument below 8 (tests/test_libm_restated.py).  Arguments |x| >= 105414350
//      (glibc's __branred path) are outside the reference's use (theta < 2 pi, phi <= pi) and
//      return NaN here.
}  // namespace kdpt
#include "glibc_sincostab.h"
namespace kdpt {
// The table lives in constant memory on the device (a constexpr array indexed at run time would be
// copied into every lane's scratch) and as a plain array on the host.
#if defined(__HIPCC__) || defined(__HIP__)
static __device__ __constant__ double GLIBC_SINCOSTAB_DEV[KDPT_GLIBC_SINCOSTAB_N] = {KDPT_GLIBC_SINCOSTAB_INIT};
#endif
static const double GLIBC_SINCOSTAB_HOST[KDPT_GLIBC_SINCOSTAB_N] = {KDPT_GLIBC_SINCOSTAB_INIT};
KDPT_HD const double* glibc_sincostab() {
#if defined(__HIP_DEVICE_COMPILE__)
  return GLIBC_SINCOSTAB_DEV;
#else
  return GLIBC_SINCOSTAB_HOST;
#endif
}
KDPT_HD uint64_t d2u(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}
KDPT_HD double u2d(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return d;
}
KDPT_HD double dabs(double x) { return u2d(d2u(x) & 0x7fffffffffffffffull); }
KDPT_HD double dcopysign(double m, double s) {
  return u2d((d2u(m) & 0x7fffffffffffffffull) | (d2u(s) & 0x8000000000000000ull));
}
namespace glibc_sin {
constexpr double sn3 = -0x1.5555555555515p-3, sn5 = 0x1.11110e829872fp-7;
constexpr double cs2 = 0x1.0p-1, cs4 = -0x1.5555555555535p-5, cs6 = 0x1.6c16bedd9e239p-10;
constexpr double s1 = -0x1.5555555555555p-3, s2 = 0x1.1111111110ecep-7, s3 = -0x1.a01a019db08b8p-13,
                 s4 = 0x1.71de27b9a7ed9p-19, s5 = -0x1.addffc2fcdf59p-26;
constexpr double big = 0x1.8p45, hp0 = 0x1.921fb54442d18p0, hp1 = 0x1.1a62633145c07p-54;
constexpr double mp1 = 0x1.921fb58p0, mp2 = -0x1.dde973cp-27, pp3 = -0x1.cb3b398p-55,
                 pp4 = -0x1.d747f23e32ed7p-83, hpinv = 0x1.45f306dc9c883p-1, toint = 0x1.8p52;
}  // namespace glibc_sin
// TAYLOR_SIN(xx, a, da): a + (xx * (P(xx) * a - 0.5 * da) + da), P = s1 + xx*(s2 + ...)
KDPT_HDI double glibc_taylor_sin(double xx, double a, double da) {
  using namespace glibc_sin;
  double p = dfma(xx, dfma(xx, dfma(xx, dfma(xx, s5, s4), s3), s2), s1);
  double t = dfma(xx, dfma(p, a, -(0.5 * da)), da);
  return a + t;
}
KDPT_HDI double glibc_do_sin(double x, double dx) {
  using namespace glibc_sin;
  const double xold = x;
  if (dabs(x) < 0.126) return glibc_taylor_sin(x * x, x, dx);
  if (x <= 0) dx = -dx;
  const double ax = dabs(x);
  const double u = big + ax;
  const int k = (int)(uint32_t)d2u(u) << 2;
  x = ax - (u - big);
  const double xx = x * x;
  const double s = x + dfma(x * xx, dfma(xx, sn5, sn3), dx);
  const double c = dfma(x, dx, xx * dfma(xx, dfma(xx, cs6, cs4), cs2));
  const double* tab = glibc_sincostab();
  const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
  const double cor = dfma(s, cs, dfma(-c, sn, dfma(s, ccs, ssn)));
  return dcopysign(sn + cor, xold);
}
KDPT_HDI double glibc_do_cos(double x, double dx) {
  using namespace glibc_sin;
  if (x < 0) dx = -dx;
  const double ax = dabs(x);
  const double u = big + ax;
  const int k = (int)(uint32_t)d2u(u) << 2;
  x = (ax - (u - big)) + dx;
  const double xx = x * x;
  const double s = dfma(x * xx, dfma(xx, sn5, sn3), x);
  const double c = xx * dfma(xx, dfma(xx, cs6, cs4), cs2);
  const double* tab = glibc_sincostab();
  const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
  const double cor = dfma(-s, sn, dfma(-c, cs, dfma(-s, ssn, ccs)));
  return cs + cor;
}
// reduce_sincos: x = n * pi/2 + (a + da), |x| < 105414350; returns n & 3
KDPT_HDI int glibc_reduce_sincos(double x, double* a, double* da) {
  using namespace glibc_sin;
  const double t = dfma(x, hpinv, toint);
  const double xn = t - toint;
  const int n = (int)(d2u(t) & 3u);
  double y = dfma(-xn, mp1, x);
  y = dfma(-xn, mp2, y);
  const double t2 = dfma(-xn, pp3, y);
  double db = dfma(-pp3, xn, y - t2);
  const double b = dfma(-xn, pp4, t2);
  db = db + dfma(-xn, pp4, t2 - b);
  *a = b;
  *da = db;
  return n;
}
KDPT_HDI double glibc_do_sincos(double a, double da, int n) {
  double r = (n & 1) ? glibc_do_cos(a, da) : glibc_do_sin(a, da);
  return (n & 2) ? -r : r;
}
KDPT_HDI double kdpt_sin(double x) {
  using namespace glibc_sin;
  const uint32_t k = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e500000u) return x;
  if (k < 0x3feb6000u) return glibc_do_sin(x, 0.0);
  if (k < 0x400368fdu) return dcopysign(glibc_do_cos(hp0 - dabs(x), hp1), x);
  if (k < 0x419921fbu) {
    double a, da;
    int n = glibc_reduce_sincos(x, &a, &da);
    return glibc_do_sincos(a, da, n);
  }
  return u2d(0x7ff8000000000000ull);
}
KDPT_HDI double kdpt_cos(double x) {
  using namespace glibc_sin;
  const uint32_t k = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
  if (k < 0x3e400000u) return 1.0;
  if (k < 0x3feb6000u) return glibc_do_cos(x, 0.0);
  if (k < 0x400368fdu) {
    const double y = hp0 - dabs(x);
    const double a = y + hp1;
    const double da = (y - a) + hp1;
    return glibc_do_sin(a, da);
  }
  if (k < 0x419921fbu) {
    double a, da;
    int n = glibc_reduce_sincos(x, &a, &da);
    return glibc_do_sincos(a, da, n + 1);
  }
  return u2d(0x7ff8000000000000ull);
}

// ---- RNG: utilhash (src/intersections.h:15-23), thrust minstd_rand (a=48271,
//      m=2^31-1) and uniform_real_distribution<float>(0,1) ----
KDPT_HD uint32_t utilhash(uint32_t a) {
  a = (a + 0x7ed55d16u) + (a << 12);
  a = (a ^ 0xc761c23cu) ^ (a >> 19);
  a = (a + 0x165667b1u) + (a << 5);
  a = (a + 0xd3a2646cu) ^ (a << 9);
  a = (a + 0xfd7046c5u) + (a << 3);
  a = (a ^ 0xb55a4f09u) ^ (a >> 16);
  return a;
}
struct Rng {
  uint32_t x;
};
KDPT_HD Rng rng_seed(uint32_t s) {
  Rng r;
  r.x = s % 2147483647u;
  if (r.x == 0u) r.x = 1u;
  return r;
}
KDPT_HD float u01(Rng& r) {
  r.x = (uint32_t)(((uint64_t)r.x * 48271ull) % 2147483647ull);
  float result = (float)(r.x - 1u);
  result /= (1.0f + (float)(2147483646u - 1u));
  return (result * (1.0f - 0.0f)) + 0.0f;
}
// makeSeededRandomEngine (src/pathtrace.cu:62-66)
KDPT_HD Rng seeded_rng(int iter, int index, int depth) {
  uint32_t a = 0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter;
  int h = (int)(utilhash(a) ^ utilhash((uint32_t)index));
  return rng_seed((uint32_t)h);
}

}  // namespace kdpt
