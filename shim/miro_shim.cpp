// miro_shim.cpp -- Scene::preCalc / raytraceImage / trace of the reference
// (src/Scene.cpp:62-217,295-298) implemented on the libmrt C-ABI.
#include "miro_shim.h"

#include <string.h>

#include <algorithm>
#include <map>

namespace miro {

Scene::~Scene() {
    if (m_gpu) mrt_scene_destroy(m_gpu);
}

static void f3(float* out, const Vector3& v) {
    out[0] = v.x;
    out[1] = v.y;
    out[2] = v.z;
}

// Material as data (mrt_material + the Blinn setters); -1 for an unknown type.
static int add_material(mrt_scene* s, const Material* m) {
    mrt_material mm;
    memset(&mm, 0, sizeof mm);
    if (const Lambert* l = dynamic_cast<const Lambert*>(m)) {
        mm.type = MRT_LAMBERT;
        f3(mm.kd, l->m_kd);
        f3(mm.ka, l->m_ka);
        mm.ks[0] = mm.ks[1] = mm.ks[2] = 1.f;
        mm.spec_exp = 1.f;
        return mrt_scene_add_material(s, &mm);
    }
    const Blinn* b = dynamic_cast<const Blinn*>(m);
    if (!b) return MRT_ERR_INVALID;
    mm.type = MRT_BLINN;
    f3(mm.kd, b->m_kd);
    f3(mm.ka, b->m_ka);
    f3(mm.ks, b->m_ks);
    mm.spec_exp = b->m_specExp;
    mm.spec_amt = b->m_specAmt;
    f3(mm.le, b->m_Le);
    mm.emitted = b->m_lightEmitted;
    int id = mrt_scene_add_material(s, &mm);
    if (id < 0) return id;
    int rc;
    // m_ior[1] is the one Blinn::shade reads (src/Blinn.cpp:183)
    if ((rc = mrt_scene_set_material_optics(s, id, b->m_reflectAmt, b->m_refractAmt, b->m_ior[1])) ||
        (rc = mrt_scene_set_material_gloss(s, id, b->m_specGloss)) ||
        (rc = mrt_scene_set_material_translucency(s, id, b->m_translucency)) ||
        (rc = mrt_scene_set_material_sample_env(s, id, b->m_sampleEnv ? 1 : 0)))
        return rc;
    if (b->m_disperse && (rc = mrt_scene_set_material_dispersion(s, id, 1, b->m_ior))) return rc;
    return id;
}

static int add_light(mrt_scene* s, const Light* l) {
    mrt_light ml;
    memset(&ml, 0, sizeof ml);
    ml.power = l->m_power;
    ml.samples = l->m_numSamples;
    ml.noise_threshold = l->m_noiseThreshold;
    ml.cast_shadows = l->m_castShadows ? 1 : 0;
    ml.texture = -1;
    if (const PointLight* p = dynamic_cast<const PointLight*>(l)) {
        ml.type = MRT_POINT_LIGHT;
        f3(ml.pos, p->m_position);
    } else if (const RectangleLight* r = dynamic_cast<const RectangleLight*>(l)) {
        ml.type = MRT_RECT_LIGHT;
        f3(ml.v1, r->m_v1);
        f3(ml.v2, r->m_v2);
        f3(ml.v3, r->m_v3);
    } else {
        return MRT_ERR_INVALID;
    }
    return mrt_scene_add_light(s, &ml);
}

// Scene::preCalc.  The objects are walked in order; every maximal run of
// consecutive Objects of one mesh and one material becomes one mrt mesh whose
// triangles are those objects' triangles in object order, so the C-ABI's global
// hit id of a triangle is its index in m_objects (HitInfo::obj below).  The mesh
// arrays go over as they are: 16-B Vector3s (stride 4), TupleI3 index triples.
int Scene::preCalc() {
    if (m_gpu) mrt_scene_destroy(m_gpu);
    m_gpu = mrt_scene_create();
    if (!m_gpu) return MRT_ERR_INVALID;
    std::map<const Material*, int> mats;
    int rc;
    for (size_t i = 0; i < m_objects.size();) {
        const Object* o = m_objects[i];
        const TriangleMesh* mesh = o->m_mesh;
        if (!mesh || !o->m_material) return MRT_ERR_INVALID;
        size_t j = i;
        std::vector<uint32_t> vidx, nidx;
        while (j < m_objects.size() && m_objects[j]->m_mesh == mesh && m_objects[j]->m_material == o->m_material) {
            const uint32_t t = m_objects[j]->m_index;
            if (t >= mesh->m_numTris) return MRT_ERR_INVALID;
            const TupleI3 v = mesh->m_vertexIndices[t], n = mesh->m_normalIndices[t];
            vidx.insert(vidx.end(), {v.x, v.y, v.z});
            nidx.insert(nidx.end(), {n.x, n.y, n.z});
            j++;
        }
        // the reference's TriangleMesh keeps no vertex / normal counts: the
        // arrays are as long as the largest index any triangle uses
        uint32_t nv = 0, nn = 0;
        for (uint32_t t = 0; t < mesh->m_numTris; t++) {
            const TupleI3 v = mesh->m_vertexIndices[t], n = mesh->m_normalIndices[t];
            nv = std::max({nv, v.x + 1, v.y + 1, v.z + 1});
            nn = std::max({nn, n.x + 1, n.y + 1, n.z + 1});
        }
        auto it = mats.find(o->m_material);
        if (it == mats.end()) {
            const int id = add_material(m_gpu, o->m_material);
            if (id < 0) return id;
            it = mats.emplace(o->m_material, id).first;
        }
        mrt_mesh mm;
        memset(&mm, 0, sizeof mm);
        mm.verts = &mesh->m_vertices[0].x;
        mm.normals = &mesh->m_normals[0].x;
        mm.vidx = vidx.data();
        mm.nidx = nidx.data();
        mm.nv = (int32_t)nv;
        mm.nn = (int32_t)nn;
        mm.nt = (int32_t)(vidx.size() / 3);
        mm.vert_stride = mm.normal_stride = 4;   // sizeof(Vector3) / sizeof(float)
        if ((rc = mrt_scene_add_mesh(m_gpu, &mm, it->second)) < 0) return rc;
        i = j;
    }
    for (const Light* l : m_lights)
        if ((rc = add_light(m_gpu, l)) < 0) return rc;
    float bg[3];
    f3(bg, m_BGColor);
    if ((rc = mrt_scene_set_background(m_gpu, bg)) || (rc = mrt_scene_set_num_paths(m_gpu, m_numPaths)) ||
        (rc = mrt_scene_set_subdivs(m_gpu, m_minSubdivs, m_maxSubdivs, m_noiseThreshold)) ||
        (rc = mrt_scene_set_path_trace(m_gpu, m_pathTrace ? 1 : 0, m_maxBounces, 0)))
        return rc;
    return mrt_scene_build_bvh(m_gpu);
}

// Scene::raytraceImage(Camera*, Image*): the whole frame on the GPU, then the
// tone-mapped 8-bit pixels (Image::setPixel -> Map) into the caller's Image.
int Scene::raytraceImage(Camera* cam, Image* img) {
    if (!m_gpu || !cam || !img || img->m_width <= 0 || img->m_height <= 0) return MRT_ERR_INVALID;
    mrt_camera c;
    f3(c.eye, cam->m_eye);
    f3(c.look_at, cam->m_lookAt);
    f3(c.up, cam->m_up);
    c.fov_deg = cam->m_fov;
    c.aperture = cam->m_aperture;
    c.focus_plane = cam->m_focusPlane;
    c.shutter_speed = cam->m_shutterSpeed;
    mrt_render_opts o;
    memset(&o, 0, sizeof o);
    o.width = img->m_width;
    o.height = img->m_height;
    o.want_rgb8 = 1;
    o.devices = m_devices.empty() ? nullptr : m_devices.data();
    o.n_devices = (int32_t)m_devices.size();
    if (!m_devices.empty()) o.device = m_devices[0];
    const size_t px = (size_t)img->m_width * img->m_height;
    std::vector<float> rgb(px * 3);
    static_assert(sizeof(Image::Pixel) == 3, "Image::Pixel is packed rgb");
    return mrt_render(m_gpu, &c, &o, rgb.data(), reinterpret_cast<uint8_t*>(img->m_pixels.data()), nullptr);
}

int Scene::traceBatch(const Ray* rays, HitInfo* hits, size_t n, float tMin) const {
    if (!m_gpu || (n && (!rays || !hits))) return MRT_ERR_INVALID;
    std::vector<float> o(3 * n), d(3 * n), tmin(n, tMin), tmax(n);
    for (size_t i = 0; i < n; i++) {
        memcpy(&o[3 * i], rays[i].o, 12);
        memcpy(&d[3 * i], rays[i].d, 12);
        tmax[i] = hits[i].t;   // HitInfo::t is tMax on entry (src/BVH.cpp:1112-1178)
    }
    std::vector<mrt_hit> out(n);
    const int rc = mrt_trace(m_gpu, o.data(), d.data(), tmin.data(), tmax.data(), n, 0, out.data());
    if (rc) return rc;
    for (size_t i = 0; i < n; i++) {
        if (out[i].prim < 0) continue;
        HitInfo& h = hits[i];
        h.t = out[i].t;
        h.a = out[i].a;
        h.b = out[i].b;
        h.m_instance = out[i].inst;
        // world hit ids are object indices (preCalc keeps object order)
        h.obj = out[i].inst < 0 && (size_t)out[i].prim < m_objects.size() ? m_objects[out[i].prim] : nullptr;
    }
    return MRT_OK;
}

bool Scene::trace(unsigned int, HitInfo& hitInfo, const Ray& ray, float tMin) const {
    HitInfo h = hitInfo;
    h.obj = nullptr;
    if (traceBatch(&ray, &h, 1, tMin) != MRT_OK || !h.obj) return false;
    hitInfo = h;
    return true;
}

}  // namespace miro
