// shim_test.cpp -- drives the reference-shaped bridge (miro_shim.h) the way the
// reference's scene scripts do (src/assignment2.h:440-524, Cornell box): a
// TriangleMesh of 16-B Vector3s, one Object per triangle (makeMeshObjs), a
// Lambert material, a PointLight, Scene::preCalc, Scene::raytraceImage and
// Scene::trace.  The mesh comes from a binary file (int32 nv, nn, nt; float
// verts[3nv], normals[3nn]; uint32 vidx[3nt], nidx[3nt]), written by
// tests/test_shim.py, which checks the outputs against the CPU oracle.
//   shim_test mesh.bin W H out.rgb8 [rays.bin hits.bin] [device ...]
// rays.bin: int32 n, float o[3n], d[3n], tmax[n]; hits.bin: per ray float t, a, b,
// int32 object index (-1 = miss) -- first from Scene::trace one ray at a time,
// then the same rays again through Scene::traceBatch (the two must agree).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "miro_shim.h"

using namespace miro;

template <typename T>
static bool read_n(FILE* f, T* p, size_t n) { return fread(p, sizeof(T), n, f) == n; }

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s mesh.bin W H out.rgb8 [rays.bin hits.bin] [device ...]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    int32_t hdr[3];
    if (!f || !read_n(f, hdr, 3)) { fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }
    const int nv = hdr[0], nn = hdr[1], nt = hdr[2];
    std::vector<float> v(3 * (size_t)nv), n(3 * (size_t)nn);
    std::vector<uint32_t> vi(3 * (size_t)nt), ni(3 * (size_t)nt);
    if (!read_n(f, v.data(), v.size()) || !read_n(f, n.data(), n.size()) || !read_n(f, vi.data(), vi.size()) ||
        !read_n(f, ni.data(), ni.size())) { fprintf(stderr, "short mesh file\n"); return 2; }
    fclose(f);
    std::vector<Vector3> verts(nv), norms(nn);
    for (int i = 0; i < nv; i++) verts[i] = Vector3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
    for (int i = 0; i < nn; i++) norms[i] = Vector3(n[3 * i], n[3 * i + 1], n[3 * i + 2]);
    TriangleMesh mesh;
    mesh.m_vertices = verts.data();
    mesh.m_normals = norms.data();
    mesh.m_vertexIndices = reinterpret_cast<TupleI3*>(vi.data());
    mesh.m_normalIndices = reinterpret_cast<TupleI3*>(ni.data());
    mesh.m_numTris = (uint32_t)nt;

    Scene scene;                                   // config C1 (miro/scenes.py)
    Lambert mat(Vector3(1.f));
    std::vector<Object*> objs;
    for (int i = 0; i < nt; i++) {                  // makeMeshObjs: one Object per triangle
        objs.push_back(new Object(&mat, &mesh, (uint32_t)i));
        scene.addObject(objs.back());
    }
    PointLight light;
    light.m_position = Vector3(2.75f, 5.0f, -2.75f);
    light.m_power = 40.f;
    scene.addLight(&light);
    scene.setBGColor(Vector3(0.f, 0.f, 0.2f));
    int argi = 5;
    const char *rays_path = nullptr, *hits_path = nullptr;
    if (argc >= 7) { rays_path = argv[5]; hits_path = argv[6]; argi = 7; }
    for (; argi < argc; argi++) scene.m_devices.push_back(atoi(argv[argi]));
    int rc = scene.preCalc();
    if (rc) { fprintf(stderr, "preCalc: %d %s\n", rc, mrt_last_error()); return 1; }
    Camera cam;
    cam.m_eye = Vector3(2.75f, 2.75f, 5.0f);
    cam.m_lookAt = Vector3(2.75f, 2.75f, 0.0f);
    cam.m_up = Vector3(0.f, 1.f, 0.f);
    cam.m_fov = 55.f;
    Image img;
    img.resize(atoi(argv[2]), atoi(argv[3]));
    if ((rc = scene.raytraceImage(&cam, &img))) { fprintf(stderr, "raytraceImage: %d %s\n", rc, mrt_last_error()); return 1; }
    FILE* o = fopen(argv[4], "wb");
    fwrite(img.m_pixels.data(), 3, img.m_pixels.size(), o);
    fclose(o);
    if (rays_path) {
        FILE* rf = fopen(rays_path, "rb");
        int32_t nr = 0;
        if (!rf || !read_n(rf, &nr, 1)) { fprintf(stderr, "cannot read %s\n", rays_path); return 2; }
        std::vector<float> ro(3 * (size_t)nr), rd(3 * (size_t)nr), tm(nr);
        if (!read_n(rf, ro.data(), ro.size()) || !read_n(rf, rd.data(), rd.size()) || !read_n(rf, tm.data(), tm.size())) {
            fprintf(stderr, "short rays file\n"); return 2;
        }
        fclose(rf);
        std::vector<Ray> rays(nr);
        std::vector<HitInfo> one(nr), batch(nr);
        for (int i = 0; i < nr; i++) {
            for (int k = 0; k < 3; k++) { rays[i].o[k] = ro[3 * i + k]; rays[i].d[k] = rd[3 * i + k]; }
            one[i].t = batch[i].t = tm[i];
        }
        for (int i = 0; i < nr; i++) scene.trace(0, one[i], rays[i]);   // Scene::trace, ray at a time
        if ((rc = scene.traceBatch(rays.data(), batch.data(), nr))) { fprintf(stderr, "traceBatch: %d\n", rc); return 1; }
        FILE* hf = fopen(hits_path, "wb");
        for (int i = 0; i < nr; i++) {
            const HitInfo& h = one[i];
            const HitInfo& g = batch[i];
            if ((h.obj != g.obj) || (h.obj && (h.t != g.t || h.a != g.a || h.b != g.b))) {
                fprintf(stderr, "trace / traceBatch disagree at ray %d\n", i);
                return 1;
            }
            const int32_t idx = h.obj ? (int32_t)(std::find(objs.begin(), objs.end(), h.obj) - objs.begin()) : -1;
            float tab[3] = {h.t, h.a, h.b};
            fwrite(tab, 4, 3, hf);
            fwrite(&idx, 4, 1, hf);
        }
        fclose(hf);
    }
    for (Object* p : objs) delete p;
    printf("shim_test OK: %dx%d frame, %d objects\n", img.m_width, img.m_height, nt);
    return 0;
}
