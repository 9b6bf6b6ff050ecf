// ref_kd_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Driver linked against the reference's OWN KD builder and OBJ loader sources
// (compiled in place from /root/reference/src by oracle/ref/Makefile, output in
// oracle/_ref/).  It reproduces the two host paths that pin the oracle and the
// product's host builder byte-for-byte:
//   kat  TRIFILE MAXDEPTH OUT   KDtree(path) -> updateBbox -> split -> writeKDtoFile
//                               (the disabled -t mode, src/main.cpp:739-1010)
//   obj  OBJ NODES.bin TRIS.bin tinyobj::LoadObj -> getTrianglesFromScene_ ->
//                               KDtree -> updateBbox -> split(13) -> flatten
//                               (src/scene.cpp:531-577, 866-968)
// Scene::loadObj itself cannot be compiled here (scene.h pulls cuda_runtime.h
// through sceneStructs.h), so its glue -- a few loops -- is restated below with
// the reference line numbers it follows.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "KDnode.h"
#include "KDtree.h"
#include "tiny_obj_loader.h"

static void preorder(KDN::KDnode *n, std::vector<KDN::KDnode *> &out) {  // getKDnodes_ :275-283
    if (!n) return;
    out.push_back(n);
    preorder(n->left, out);
    preorder(n->right, out);
}

int main(int argc, char **argv) {
    if (argc == 5 && std::string(argv[1]) == "kat") {
        KDtree *t = new KDtree(argv[2]);
        t->rootNode->updateBbox();
        t->split(atoi(argv[3]));
        t->writeKDtoFile(t->rootNode, argv[4]);
        return 0;
    }
    if (argc != 5 || std::string(argv[1]) != "obj") {
        fprintf(stderr, "usage: %s kat TRIFILE MAXDEPTH OUT | obj OBJ NODES.bin TRIS.bin\n", argv[0]);
        return 2;
    }
    std::string path = argv[2];
    std::string base = path.substr(0, path.find_last_of("/\\") + 1);
    tinyobj::attrib_t attrib;
    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> materials;
    std::string err;
    if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &err, path.c_str(), base.c_str(), true)) return 1;
    // Scene::getTrianglesFromScene_ (src/scene.cpp:531-577): normals by VERTEX index
    std::vector<KDN::Triangle *> tris;
    for (size_t i = 0; i < shapes.size(); i++) {
        const std::vector<tinyobj::index_t> &ix = shapes[i].mesh.indices;
        for (size_t j = 0; j + 2 < ix.size(); j += 3) {
            int p1 = 3 * ix[j].vertex_index, p2 = 3 * ix[j + 1].vertex_index, p3 = 3 * ix[j + 2].vertex_index;
            const std::vector<float> &v = attrib.vertices, &n = attrib.normals;
            KDN::Triangle *t = new KDN::Triangle(v[p1], v[p1 + 1], v[p1 + 2], v[p2], v[p2 + 1], v[p2 + 2],
                                                 v[p3], v[p3 + 1], v[p3 + 2], n[p1], n[p1 + 1], n[p1 + 2],
                                                 n[p2], n[p2 + 1], n[p2 + 2], n[p3], n[p3 + 1], n[p3 + 2]);
            t->mtlIdx = (int)i;
            tris.push_back(t);
        }
    }
    KDtree *kdt = new KDtree(tris);  // src/scene.cpp:868-872
    kdt->rootNode->updateBbox();
    kdt->split(13);
    std::vector<KDN::KDnode *> nodes;
    preorder(kdt->rootNode, nodes);
    std::sort(nodes.begin(), nodes.end(),
              [](const KDN::KDnode *a, const KDN::KDnode *b) { return a->ID < b->ID; });
    // cacheTriangles_ (src/scene.cpp:409-459) + cacheTrianglesBare (:934-968)
    std::vector<KDN::TriBare> tb;
    int tc = 0;
    for (size_t i = 0; i < nodes.size(); i++) {
        int nt = (int)nodes[i]->triangles.size();
        if (nt > 0) {
            nodes[i]->triIdStart = tc;
            nodes[i]->triIdSize = nt;
            tc += nt;
            for (int j = 0; j < nt; j++) {
                const KDN::Triangle &T = *nodes[i]->triangles[j];
                KDN::TriBare b;
                b.x1 = T.x1; b.x2 = T.x2; b.x3 = T.x3; b.y1 = T.y1; b.y2 = T.y2; b.y3 = T.y3;
                b.z1 = T.z1; b.z2 = T.z2; b.z3 = T.z3;
                b.nx1 = T.nx1; b.nx2 = T.nx2; b.nx3 = T.nx3; b.ny1 = T.ny1; b.ny2 = T.ny2; b.ny3 = T.ny3;
                b.nz1 = T.nz1; b.nz2 = T.nz2; b.nz3 = T.nz3;
                b.mtlIdx = T.mtlIdx;
                tb.push_back(b);
            }
        }
    }
    // cacheNodesBare (src/scene.cpp:905-932)
    std::vector<KDN::NodeBare> nb(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) {
        const KDN::KDnode &n = *nodes[i];
        KDN::NodeBare &o = nb[i];
        memset(&o, 0, sizeof o);
        o.axis = n.axis; o.ID = n.ID; o.parentID = n.parentID; o.leftID = n.leftID; o.rightID = n.rightID;
        for (int a = 0; a < 3; a++) { o.mins[a] = n.bbox.mins[a]; o.maxs[a] = n.bbox.maxs[a]; }
        o.triIdSize = n.triIdSize; o.triIdStart = n.triIdStart; o.splitPos = n.splitPos;
        o.tmin = 0.0f; o.tmax = 0.0f;
    }
    FILE *f = fopen(argv[3], "wb");
    fwrite(nb.data(), sizeof(KDN::NodeBare), nb.size(), f);
    fclose(f);
    f = fopen(argv[4], "wb");
    fwrite(tb.data(), sizeof(KDN::TriBare), tb.size(), f);
    fclose(f);
    printf("{\"nodes\": %zu, \"tris\": %zu}\n", nb.size(), tb.size());
    return 0;
}
