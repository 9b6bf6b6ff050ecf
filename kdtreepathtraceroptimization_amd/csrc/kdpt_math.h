// kdpt_math.h -- float/double arithmetic of the reference hot path, restated so
// that gfx950 and x86 evaluate the SAME IEEE operations in the SAME order.
//
// Compiled with -ffp-contract=off (never fuse) and without fast-math, so a
// correctly-rounded v_div/v_sqrt sequence is used for `/` and sqrtf.  Every
// function cites the reference (or vendored glm 0.9.6.3 / rocThrust) code it
// follows.  Transcendentals the reference gets from glibc are restated
// bit-exactly (kdpt_sinf/kdpt_cosf: glibc 2.35 sysdeps/ieee754/flt-32
// s_sinf.c/s_cosf.c FMA variant -- verified over every |x| < 119 float).
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define KDPT_HD __host__ __device__ inline
#else
#define KDPT_HD static inline
#include <math.h>
// host-only builds (tests/native differential harness): HIP's vector types
struct float4 { float x, y, z, w; };
struct int4 { int x, y, z, w; };
struct int2 { int x, y; };
static inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }
static inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }
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
