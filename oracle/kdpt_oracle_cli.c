/*
 * kdpt_oracle_cli.c -- TEST INFRASTRUCTURE ONLY: command-line front end of the
 * oracle (fixture generation, CPU baseline timing).  Not part of the product.
 *
 *   kdpt_oracle render SCENE OBJ|- W H DEPTH ITERS [FIRST] [--bare] [--nocompact]
 *                      [--threads N] [--out IMAGE.f32]
 *   kdpt_oracle kat TRIFILE MAXDEPTH OUT
 */
#include "kdpt_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    if (argc >= 5 && strcmp(argv[1], "kat") == 0)
        return orc_kd_kat(argv[2], atoi(argv[3]), argv[4]);
    if (argc < 8 || strcmp(argv[1], "render") != 0) {
        fprintf(stderr, "usage: %s render SCENE OBJ|- W H DEPTH ITERS [FIRST] [--bare] [--nocompact] "
                        "[--threads N] [--out F]\n       %s kat TRIFILE MAXDEPTH OUT\n", argv[0], argv[0]);
        return 2;
    }
    const char *scene = argv[2];
    const char *obj = strcmp(argv[3], "-") == 0 ? NULL : argv[3];
    int W = atoi(argv[4]), H = atoi(argv[5]), depth = atoi(argv[6]), iters = atoi(argv[7]);
    int first = 1, threads = 0;
    const char *out = NULL;
    orc_opts o;
    orc_default_opts(&o);
    for (int i = 8; i < argc; i++) {
        if (strcmp(argv[i], "--bare") == 0) o.shortstack = 0;
        else if (strcmp(argv[i], "--nocompact") == 0) o.compaction = 0;
        else if (strcmp(argv[i], "--threads") == 0 && i + 1 < argc) threads = atoi(argv[++i]);
        else if (strcmp(argv[i], "--out") == 0 && i + 1 < argc) out = argv[++i];
        else first = atoi(argv[i]);
    }
    orc_scene s;
    double t0 = now_s();
    int rc = orc_load_scene(scene, obj, W, H, depth, &s);
    if (rc) { fprintf(stderr, "load failed %d\n", rc); return 1; }
    double t1 = now_s();
    size_t npx = (size_t)s.camera.resolution[0] * s.camera.resolution[1];
    float *img = (float *)calloc(npx * 3, sizeof(float));
    orc_stats st;
    orc_render(&s, &o, first, iters, img, &st, threads);
    double t2 = now_s();
    /* imgsum as the survey defines it: per-pixel float (r+g+b) accumulated in double */
    double sum = 0;
    for (size_t i = 0; i < npx; i++) sum += (double)(img[3 * i] + img[3 * i + 1] + img[3 * i + 2]);
    printf("{\"nodes\": %d, \"tris\": %d, \"segments\": %lld, \"imgsum\": %.6f, \"aabb\": %lld, \"tri\": %lld, "
           "\"hits\": %lld, \"load_s\": %.3f, \"render_s\": %.3f, \"mseg_per_s\": %.4f}\n",
           s.num_nodes, s.num_tris, st.segments, sum, st.aabb_tests, st.tri_tests, st.tri_hits, t1 - t0, t2 - t1,
           st.segments / (t2 - t1) / 1e6);
    if (out) {
        FILE *f = fopen(out, "wb");
        fwrite(img, sizeof(float), npx * 3, f);
        fclose(f);
    }
    free(img);
    orc_free_scene(&s);
    return 0;
}
