// ref_pins_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Driver linked against the reference's OWN image writer, utilities and vendored glm
// (src/image.cpp + src/stb.cpp + src/utilities.cpp compiled in place from /root/reference by
// oracle/ref/Makefile, output in oracle/_ref/).  It produces the known answers that pin the
// product's restatements where the reference's code compiles here without stand-ins:
//   img  W H IN.f32 BASE     image(W,H) + setPixel per pixel + savePNG(BASE) + saveHDR(BASE)
//                            (src/image.cpp:7-45; stb_image_write via src/stb.cpp)
//   geom N IN.f32 OUT.f32    per translation/rotation/scale triple: buildTransformationMatrix
//                            (src/utilities.cpp:65-72), glm::inverse, glm::inverseTranspose -- the
//                            three Geom matrices Scene::loadGeom stores (src/scene.cpp:165-168)
//   glm  FN N IN.f32 OUT.f32 the vendored glm on the path: 0 intersectRayTriangle (gtx/intersect.inl:
//                            37-74; OUT is read first: its bary slots are the sentinels glm leaves
//                            unwritten), 1 normalize, 2 reflect, 3 refract, 4 glm::rotate(quat, vec3)
//                            (src/pathtrace.cu:389)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_inverse.hpp>
#include <glm/gtx/intersect.hpp>
#include <glm/gtx/quaternion.hpp>

#include "image.h"
#include "utilities.h"

static std::vector<float> read_f32(const char* path, size_t n) {
  std::vector<float> v(n);
  FILE* f = fopen(path, "rb");
  if (!f || fread(v.data(), sizeof(float), n, f) != n) {
    fprintf(stderr, "cannot read %zu floats from %s\n", n, path);
    exit(3);
  }
  fclose(f);
  return v;
}

static void write_f32(const char* path, const std::vector<float>& v) {
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(v.data(), sizeof(float), v.size(), f) != v.size()) {
    fprintf(stderr, "cannot write %s\n", path);
    exit(3);
  }
  fclose(f);
}

int main(int argc, char** argv) {
  const std::string cmd = argc > 1 ? argv[1] : "";
  if (cmd == "img" && argc == 6) {
    const int w = atoi(argv[2]), h = atoi(argv[3]);
    std::vector<float> px = read_f32(argv[4], 3 * (size_t)w * h);
    image img(w, h);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        const float* p = &px[3 * ((size_t)y * w + x)];
        img.setPixel(x, y, glm::vec3(p[0], p[1], p[2]));
      }
    img.savePNG(argv[5]);
    img.saveHDR(argv[5]);
    return 0;
  }
  if (cmd == "geom" && argc == 5) {
    const size_t n = (size_t)atol(argv[2]);
    std::vector<float> in = read_f32(argv[3], 9 * n), out(48 * n);
    for (size_t i = 0; i < n; i++) {
      const float* t = &in[9 * i];
      const glm::mat4 T = utilityCore::buildTransformationMatrix(glm::vec3(t[0], t[1], t[2]),
                                                                 glm::vec3(t[3], t[4], t[5]),
                                                                 glm::vec3(t[6], t[7], t[8]));
      const glm::mat4 I = glm::inverse(T), IT = glm::inverseTranspose(T);
      memcpy(&out[48 * i], &T[0][0], 64);
      memcpy(&out[48 * i + 16], &I[0][0], 64);
      memcpy(&out[48 * i + 32], &IT[0][0], 64);
    }
    write_f32(argv[4], out);
    return 0;
  }
  if (cmd == "glm" && argc == 6) {
    const int fn = atoi(argv[2]);
    const size_t n = (size_t)atol(argv[3]);
    const int ni = fn == 0 ? 15 : fn == 1 ? 3 : fn == 2 ? 6 : 7, no = fn == 0 ? 4 : 3;
    if (fn < 0 || fn > 4) return 2;
    std::vector<float> in = read_f32(argv[4], ni * n), out = read_f32(argv[5], no * n);
    for (size_t i = 0; i < n; i++) {
      const float* a = &in[ni * i];
      float* o = &out[no * i];
      glm::vec3 r(0.0f);
      if (fn == 0) {
        glm::vec3 bary(o[1], o[2], o[3]);
        const bool hit = glm::intersectRayTriangle(glm::vec3(a[0], a[1], a[2]), glm::vec3(a[3], a[4], a[5]),
                                                   glm::vec3(a[6], a[7], a[8]), glm::vec3(a[9], a[10], a[11]),
                                                   glm::vec3(a[12], a[13], a[14]), bary);
        o[0] = hit ? 1.0f : 0.0f;
        o[1] = bary.x;
        o[2] = bary.y;
        o[3] = bary.z;
        continue;
      }
      if (fn == 1) r = glm::normalize(glm::vec3(a[0], a[1], a[2]));
      if (fn == 2) r = glm::reflect(glm::vec3(a[0], a[1], a[2]), glm::vec3(a[3], a[4], a[5]));
      if (fn == 3) r = glm::refract(glm::vec3(a[0], a[1], a[2]), glm::vec3(a[3], a[4], a[5]), a[6]);
      if (fn == 4) {
        glm::quat q;
        q.w = a[0];
        q.x = a[1];
        q.y = a[2];
        q.z = a[3];
        r = glm::rotate(q, glm::vec3(a[4], a[5], a[6]));
      }
      o[0] = r.x;
      o[1] = r.y;
      o[2] = r.z;
    }
    write_f32(argv[5], out);
    return 0;
  }
  fprintf(stderr, "usage: %s img W H IN.f32 BASE | geom N IN.f32 OUT.f32 | glm FN N IN.f32 OUT.f32\n", argv[0]);
  return 2;
}
