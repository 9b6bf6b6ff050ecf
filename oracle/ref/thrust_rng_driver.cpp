// thrust_rng_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Known answers for the reference's random numbers from the third party's own implementation.
// The reference draws every random number from thrust::default_random_engine (minstd_rand) through
// thrust::uniform_real_distribution<float>(0, 1):
//   - makeSeededRandomEngine(iter, index, depth)   src/pathtrace.cu:62-66 (scatter, src/interactions.h:
//     12,70,207,232,314)
//   - the camera jitter's engine seeded by utilhash(iter)   src/pathtrace.cu:334-335
// Thrust is a dependency the reference does not vendor (it comes with the CUDA toolkit).  The image has
// rocThrust (/opt/rocm/include/thrust, THRUST_VERSION 200805), whose random engines are the same
// published algorithm; this driver is compiled host-only against it (oracle/ref/Makefile, target
// thrust_rng) and nothing of the product or the oracle is linked in.  utilhash (src/intersections.h:15-23)
// is restated here: intersections.h includes sceneStructs.h -> <cuda_runtime.h>, which is absent.
//
//   thrust_rng seeded N IN.i32 K OUT.f32   IN = N (iter, index, depth) int32 triples; OUT = N x K draws
//                                          of makeSeededRandomEngine(iter, index, depth)
//   thrust_rng camera N IN.i32 K OUT.f32   IN = N iters; OUT = N x K draws of engine(utilhash(iter))
//   thrust_rng raw    N IN.u32 K OUT.f32   IN = N raw seeds; OUT = N x K draws of engine(seed)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <thrust/random.h>

static unsigned int utilhash(unsigned int a) {  // src/intersections.h:15-23
  a = (a + 0x7ed55d16) + (a << 12);
  a = (a ^ 0xc761c23c) ^ (a >> 19);
  a = (a + 0x165667b1) + (a << 5);
  a = (a + 0xd3a2646c) ^ (a << 9);
  a = (a + 0xfd7046c5) + (a << 3);
  a = (a ^ 0xb55a4f09) ^ (a >> 16);
  return a;
}

static thrust::default_random_engine seeded(int iter, int index, int depth) {  // src/pathtrace.cu:63-66
  int h = utilhash((1u << 31) | (depth << 22) | iter) ^ utilhash(index);
  return thrust::default_random_engine(h);
}

template <class T>
static std::vector<T> read_all(const char* path, size_t n) {
  std::vector<T> v(n);
  FILE* f = fopen(path, "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "cannot read %zu items from %s\n", n, path);
    exit(3);
  }
  fclose(f);
  return v;
}

static void draw(thrust::default_random_engine rng, int k, float* out) {
  thrust::uniform_real_distribution<float> u01(0, 1);
  for (int j = 0; j < k; j++) out[j] = u01(rng);
}

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s seeded|camera|raw N IN K OUT\n", argv[0]);
    return 2;
  }
  const char* mode = argv[1];
  const size_t n = (size_t)atol(argv[2]);
  const int k = atoi(argv[4]);
  std::vector<float> out(n * (size_t)k);
  if (!strcmp(mode, "seeded")) {
    std::vector<int> in = read_all<int>(argv[3], 3 * n);
    for (size_t i = 0; i < n; i++) draw(seeded(in[3 * i], in[3 * i + 1], in[3 * i + 2]), k, &out[i * k]);
  } else if (!strcmp(mode, "camera")) {
    std::vector<int> in = read_all<int>(argv[3], n);
    for (size_t i = 0; i < n; i++) draw(thrust::default_random_engine(utilhash(in[i])), k, &out[i * k]);
  } else if (!strcmp(mode, "raw")) {
    std::vector<unsigned int> in = read_all<unsigned int>(argv[3], n);
    for (size_t i = 0; i < n; i++) draw(thrust::default_random_engine(in[i]), k, &out[i * k]);
  } else {
    return 2;
  }
  FILE* f = fopen(argv[5], "wb");
  if (!f || fwrite(out.data(), sizeof(float), out.size(), f) != out.size()) return 3;
  fclose(f);
  return 0;
}
