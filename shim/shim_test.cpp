// shim_test.cpp -- drives the reference-shaped bridge (miro_shim.h) the way the
// reference's scene scripts do (src/assignment2.h:440-524, Cornell box): a
// TriangleMesh of 16-B Vector3s, one Object per triangle (makeMeshObjs), a
// Lambert material, a PointLight, Scene::preCalc, Scene::raytraceImage and
// Scene::trace.  The mesh comes from a binary file (int32 nv, nn, nt; float
// verts[3nv], normals[3nn]; uint32 vidx[3nt], nidx[3nt]), written by
// tests/test_shim.py, which checks the outputs against the CPU oracle.
//   shim_test mesh.bin W H out.rgb8 [rays.bin hits.bin] [device ...]
//   shim_test c5 spec.txt W H out.rgb8 out.rgbf out.hits rays.bin rayhits.bin (run_c5)
// rays.bin: int32 n, float o[3n], d[3n], tmax[n]; hits.bin: per ray float t, a, b,
// int32 object index (-1 = miss) -- first from Scene::trace one ray at a time,
// then the same rays again through Scene::traceBatch (the two must agree).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "miro_shim.h"

using namespace miro;

template <typename T>
static bool read_n(FILE* f, T* p, size_t n) { return fread(p, sizeof(T), n, f) == n; }

// Config C5 through the bridge: two proxy BVHs (ProxyObject::setupProxy),
// instances alternating between them, the floor triangle, a DomeLight and the
// environment map from one HDR texture.  spec.txt (written by tests/test_shim.py):
//   obj PATH (x2) / hdr PATH / camera ex ey ez lx ly lz ux uy uz fov /
//   material kd0 kd1 kd2 specExp specAmt / bg r g b / dome power samples noise /
//   env exposure / instance m00 .. m33 (one line per instance)
// Outputs: rgb8 bytes, float RGB, per-pixel hits (t, a, b, global id, instance),
// and for rays.bin the Scene::trace hits in the same record format.
struct HitRec {
    float t, a, b;
    int32_t id, inst;
};
static int run_c5(int argc, char** argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s c5 spec.txt W H out.rgb8 out.rgbf out.hits rays.bin rayhits.bin\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[2], "r");
    if (!f) { fprintf(stderr, "cannot read %s\n", argv[2]); return 2; }
    std::vector<std::string> objs_path;
    std::string hdr;
    Camera cam;
    Blinn mat;
    Vector3 bg;
    DomeLight dome;
    float exposure = 1.f;
    std::vector<Matrix4x4> inst;
    char key[64], path[4096];
    while (fscanf(f, "%63s", key) == 1) {
        std::string k(key);
        if (k == "obj" && fscanf(f, "%4095s", path) == 1) objs_path.push_back(path);
        else if (k == "hdr" && fscanf(f, "%4095s", path) == 1) hdr = path;
        else if (k == "camera") {
            float v[10];
            for (float& x : v) if (fscanf(f, "%f", &x) != 1) return 2;
            cam.m_eye = Vector3(v[0], v[1], v[2]); cam.m_lookAt = Vector3(v[3], v[4], v[5]);
            cam.m_up = Vector3(v[6], v[7], v[8]); cam.m_fov = v[9];
        } else if (k == "material") {
            float v[5];
            for (float& x : v) if (fscanf(f, "%f", &x) != 1) return 2;
            mat.m_kd = Vector3(v[0], v[1], v[2]); mat.m_specExp = v[3]; mat.m_specAmt = v[4];
        } else if (k == "bg") {
            float v[3];
            for (float& x : v) if (fscanf(f, "%f", &x) != 1) return 2;
            bg = Vector3(v[0], v[1], v[2]);
        } else if (k == "dome") {
            float p, n;
            int s;
            if (fscanf(f, "%f %d %f", &p, &s, &n) != 3) return 2;
            dome.setPower(p); dome.setSamples(s); dome.setNoiseThreshold(n);
        } else if (k == "env") {
            if (fscanf(f, "%f", &exposure) != 1) return 2;
        } else if (k == "instance") {
            Matrix4x4 M;
            for (int r = 0; r < 4; r++)
                for (int c = 0; c < 4; c++) if (fscanf(f, "%f", &M.m[r][c]) != 1) return 2;
            inst.push_back(M);
        } else { fprintf(stderr, "bad spec key %s\n", key); return 2; }
    }
    fclose(f);
    if (objs_path.size() != 2 || hdr.empty() || inst.empty()) { fprintf(stderr, "incomplete spec\n"); return 2; }
    TriangleMesh protos[2];
    Objects pobjs[2];
    BVH bvh[2];
    for (int k = 0; k < 2; k++) {
        if (!protos[k].load(objs_path[k].c_str())) { fprintf(stderr, "load %s: %s\n", objs_path[k].c_str(), mrt_last_error()); return 1; }
        ProxyObject::setupProxy(&protos[k], &mat, &pobjs[k], &bvh[k]);
    }
    Scene scene;
    std::vector<Object*> mine;
    for (size_t i = 0; i < inst.size(); i++) {
        mine.push_back(new ProxyObject(&pobjs[i % 2], &bvh[i % 2], inst[i]));
        scene.addObject(mine.back());
    }
    TriangleMesh floor;   // src/assignment2.h:110-124 floor triangle (miro/scenes.py)
    floor.createSingleTriangle();
    floor.setV1(Vector3(-100, 0, -100)); floor.setV2(Vector3(0, 0, 100)); floor.setV3(Vector3(100, 0, -100));
    floor.setN1(Vector3(0, 1, 0)); floor.setN2(Vector3(0, 1, 0)); floor.setN3(Vector3(0, 1, 0));
    mine.push_back(new Object(&mat, &floor, 0));
    scene.addObject(mine.back());
    RawImage img;
    if (!img.loadImage(hdr.c_str())) { fprintf(stderr, "image %s: %s\n", hdr.c_str(), mrt_last_error()); return 1; }
    Texture tex(&img);
    dome.setTexture(&tex);
    scene.addLight(&dome);
    scene.setEnvMap(&tex);
    scene.setEnvExposure(exposure);
    scene.setBGColor(bg);
    scene.m_keepFrame = true;
    int rc = scene.preCalc();
    if (rc) { fprintf(stderr, "preCalc: %d %s\n", rc, mrt_last_error()); return 1; }
    Image im;
    im.resize(atoi(argv[3]), atoi(argv[4]));
    if ((rc = scene.raytraceImage(&cam, &im))) { fprintf(stderr, "raytraceImage: %d %s\n", rc, mrt_last_error()); return 1; }
    // global hit id of a HitInfo: world objects by index, then each instance's
    // BLAS objects (the proxy's Objects) after the world objects
    std::vector<int32_t> base(inst.size());
    int32_t run = (int32_t)mine.size();
    for (size_t i = 0; i < inst.size(); i++) { base[i] = run; run += (int32_t)pobjs[i % 2].size(); }
    auto rec = [&](const HitInfo& h, bool hit) {
        HitRec r{h.t, h.a, h.b, -1, -1};
        if (!hit || !h.obj) return r;
        if (h.m_proxy) {
            const Objects& os = *h.m_proxy->m_objects;
            r.id = base[(size_t)h.m_instance] + (int32_t)(std::find(os.begin(), os.end(), h.obj) - os.begin());
            r.inst = h.m_instance;
            if (mine[(size_t)h.m_instance] != h.m_proxy) r.id = -2;   // m_proxy must be the instance's ProxyObject
        } else {
            r.id = (int32_t)(std::find(mine.begin(), mine.end(), h.obj) - mine.begin());
        }
        return r;
    };
    FILE* o = fopen(argv[5], "wb");
    fwrite(im.m_pixels.data(), 3, im.m_pixels.size(), o);
    fclose(o);
    o = fopen(argv[6], "wb");
    fwrite(scene.m_lastRGB.data(), 4, scene.m_lastRGB.size(), o);
    fclose(o);
    o = fopen(argv[7], "wb");
    for (const HitInfo& h : scene.m_lastHits) { const HitRec r = rec(h, h.obj != nullptr); fwrite(&r, sizeof r, 1, o); }
    fclose(o);
    FILE* rf = fopen(argv[8], "rb");
    int32_t nr = 0;
    if (!rf || !read_n(rf, &nr, 1)) { fprintf(stderr, "cannot read %s\n", argv[8]); return 2; }
    std::vector<float> ro(3 * (size_t)nr), rd(3 * (size_t)nr), tm(nr);
    if (!read_n(rf, ro.data(), ro.size()) || !read_n(rf, rd.data(), rd.size()) || !read_n(rf, tm.data(), tm.size())) return 2;
    fclose(rf);
    std::vector<Ray> rays(nr);
    std::vector<HitInfo> one(nr), batch(nr);
    for (int i = 0; i < nr; i++) {
        for (int k = 0; k < 3; k++) { rays[i].o[k] = ro[3 * i + k]; rays[i].d[k] = rd[3 * i + k]; }
        one[i].t = batch[i].t = tm[i];
    }
    std::vector<char> hit(nr);
    for (int i = 0; i < nr; i++) hit[i] = scene.trace(0, one[i], rays[i]);   // Scene::trace, ray at a time
    if ((rc = scene.traceBatch(rays.data(), batch.data(), nr))) { fprintf(stderr, "traceBatch: %d\n", rc); return 1; }
    o = fopen(argv[9], "wb");
    for (int i = 0; i < nr; i++) {
        const HitRec a = rec(one[i], hit[i]), b = rec(batch[i], batch[i].obj != nullptr);
        if (memcmp(&a, &b, sizeof a)) { fprintf(stderr, "trace / traceBatch disagree at ray %d\n", i); return 1; }
        fwrite(&a, sizeof a, 1, o);
    }
    fclose(o);
    printf("shim_test c5 OK: %dx%d frame, %zu instances, %d rays\n", im.m_width, im.m_height, inst.size(), nr);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::string(argv[1]) == "c5") return run_c5(argc, argv);
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
