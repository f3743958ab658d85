// miro_shim.cpp -- Scene::preCalc / raytraceImage / trace of the reference
// (src/Scene.cpp:62-217,295-298) implemented on the libmrt C-ABI, with the
// scene objects of the reference's final scenes: ProxyObject instances of
// shared BVHs, MBObjects, DomeLight image-based lighting, environment maps and
// material texture maps.
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

// ------------------------------------------------------------------ assets
bool TriangleMesh::load(const char* file, const Matrix4x4& ctm) {
    mrt_scene* s = mrt_scene_create();
    if (!s) return false;
    mrt_material mm;
    memset(&mm, 0, sizeof mm);
    mm.kd[0] = mm.kd[1] = mm.kd[2] = 1.f;
    const int mat = mrt_scene_add_material(s, &mm);
    const int id = mat < 0 ? mat : mrt_scene_add_obj(s, file, &ctm.m[0][0], mat);
    int32_t nv = 0, nn = 0, nt = 0, ntex = 0;
    bool ok = id >= 0 && mrt_scene_mesh_info(s, id, &nv, &nn, &nt) == MRT_OK;
    std::vector<float> v, n;
    std::vector<uint32_t> vi, ni, ti;
    std::vector<float> uv;
    if (ok) {
        v.resize(3 * (size_t)nv);
        n.resize(3 * (size_t)nn);
        vi.resize(3 * (size_t)nt);
        ni.resize(3 * (size_t)nt);
        ok = mrt_scene_mesh_export(s, id, v.data(), n.data(), vi.data(), ni.data()) == MRT_OK &&
             mrt_scene_mesh_texcoords(s, id, &ntex, nullptr, nullptr) == MRT_OK;
    }
    if (ok && ntex > 0) {
        uv.resize(2 * (size_t)ntex);
        ti.resize(3 * (size_t)nt);
        ok = mrt_scene_mesh_texcoords(s, id, &ntex, uv.data(), ti.data()) == MRT_OK;
    }
    mrt_scene_destroy(s);
    if (!ok) return false;
    m_vstore.resize((size_t)nv);
    m_nstore.resize((size_t)nn);
    for (int32_t i = 0; i < nv; i++) m_vstore[i] = Vector3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
    for (int32_t i = 0; i < nn; i++) m_nstore[i] = Vector3(n[3 * i], n[3 * i + 1], n[3 * i + 2]);
    m_vistore.resize((size_t)nt);
    m_nistore.resize((size_t)nt);
    memcpy(m_vistore.data(), vi.data(), vi.size() * 4);
    memcpy(m_nistore.data(), ni.data(), ni.size() * 4);
    m_vertices = m_vstore.data();
    m_normals = m_nstore.data();
    m_vertexIndices = m_vistore.data();
    m_normalIndices = m_nistore.data();
    m_numTris = (uint32_t)nt;
    if (ntex > 0) {
        m_tstore.resize((size_t)ntex);
        for (int32_t i = 0; i < ntex; i++) m_tstore[i] = VectorR2{uv[2 * i], uv[2 * i + 1]};
        m_tistore.resize((size_t)nt);
        memcpy(m_tistore.data(), ti.data(), ti.size() * 4);
        m_texCoords = m_tstore.data();
        m_texCoordIndices = m_tistore.data();
    }
    return true;
}

void TriangleMesh::createSingleTriangle() {
    m_vstore.assign(3, Vector3(0.f));
    m_nstore.assign(3, Vector3(0.f));
    m_vistore.assign(1, TupleI3{0, 1, 2});
    m_nistore.assign(1, TupleI3{0, 1, 2});
    m_vertices = m_vstore.data();
    m_normals = m_nstore.data();
    m_vertexIndices = m_vistore.data();
    m_normalIndices = m_nistore.data();
    m_numTris = 1;
}

bool RawImage::loadImage(const char* filename) {
    int32_t w = 0, h = 0, type = 0;
    if (mrt_image_info(filename, &w, &h, &type) != MRT_OK) return false;
    const int ch = type == MRT_TEX_GRAY ? 1 : type == MRT_TEX_RGBA ? 4 : 3;
    m_store.assign((size_t)w * h * ch, 0.f);
    if (mrt_image_load(filename, m_store.data(), w, h) != MRT_OK) return false;
    m_rawData = m_store.data();
    m_width = w;
    m_height = h;
    m_imageType = type == MRT_TEX_HDR ? HDR : type == MRT_TEX_GRAY ? GRAYSCALE : type == MRT_TEX_RGBA ? RGBA : RGB;
    return true;
}

void ProxyObject::setupProxy(TriangleMesh* mesh, const Material* mat, Objects* m, BVH* b) {
    TriangleMesh* meshes[1] = {mesh};
    const Material* mats[1] = {mat};
    setupMultiProxy(meshes, 1, mats, m, b);
}

void ProxyObject::setupMultiProxy(TriangleMesh* mesh[], int numObjs, const Material* mat[], Objects* m, BVH* b) {
    for (int j = 0; j < numObjs; j++) {
        const int n = (int)mesh[j]->m_numTris;
        Object* t = new Object[n];
        for (int i = n - 1; i >= 0; i--) {
            t[i].setMesh(mesh[j]);
            t[i].setIndex((uint32_t)i);
            t[i].setMaterial(mat[j]);
            m->push_back(&t[i]);
        }
    }
    b->build(m);
}

// ------------------------------------------------------------------ scene build
namespace {
struct Builder {
    mrt_scene* s;
    std::map<const Material*, int> mats;
    std::map<const Texture*, int> texs;
    std::map<const BVH*, std::pair<int, int32_t>> blas;   // BLAS id, objects

    int texture(const Texture* t) {
        if (!t) return -1;
        auto it = texs.find(t);
        if (it != texs.end()) return it->second;
        const RawImage* im = t->m_image;
        if (!im || !im->m_rawData || im->m_width <= 0 || im->m_height <= 0) return MRT_ERR_INVALID;
        const int type = im->m_imageType == HDR ? MRT_TEX_HDR : im->m_imageType == GRAYSCALE ? MRT_TEX_GRAY
                         : im->m_imageType == RGBA ? MRT_TEX_RGBA : MRT_TEX_RGB;
        const int id = mrt_scene_add_texture_typed(s, im->m_rawData, im->m_width, im->m_height, type);
        if (id >= 0) texs.emplace(t, id);
        return id;
    }

    // Material as data (mrt_material + the Blinn setters + the maps)
    int material(const Material* m) {
        auto it = mats.find(m);
        if (it != mats.end()) return it->second;
        mrt_material mm;
        memset(&mm, 0, sizeof mm);
        int id;
        if (const Lambert* l = dynamic_cast<const Lambert*>(m)) {
            mm.type = MRT_LAMBERT;
            f3(mm.kd, l->m_kd);
            f3(mm.ka, l->m_ka);
            mm.ks[0] = mm.ks[1] = mm.ks[2] = 1.f;
            mm.spec_exp = 1.f;
            if ((id = mrt_scene_add_material(s, &mm)) < 0) return id;
        } else if (const Blinn* b = dynamic_cast<const Blinn*>(m)) {
            mm.type = MRT_BLINN;
            f3(mm.kd, b->m_kd);
            f3(mm.ka, b->m_ka);
            f3(mm.ks, b->m_ks);
            mm.spec_exp = b->m_specExp;
            mm.spec_amt = b->m_specAmt;
            f3(mm.le, b->m_Le);
            mm.emitted = b->m_lightEmitted;
            if ((id = mrt_scene_add_material(s, &mm)) < 0) return id;
            int rc;
            // m_ior[1] is the one Blinn::shade reads (src/Blinn.cpp:183)
            if ((rc = mrt_scene_set_material_optics(s, id, b->m_reflectAmt, b->m_refractAmt, b->m_ior[1])) ||
                (rc = mrt_scene_set_material_gloss(s, id, b->m_specGloss)))
                return rc;
            if (b->m_disperse && (rc = mrt_scene_set_material_dispersion(s, id, 1, b->m_ior))) return rc;
        } else {
            return MRT_ERR_INVALID;
        }
        int rc;
        if ((rc = mrt_scene_set_material_translucency(s, id, m->m_translucency)) ||
            (rc = mrt_scene_set_material_sample_env(s, id, m->m_sampleEnv ? 1 : 0)))
            return rc;
        // Material maps, in mrt order: colour, normal, specular, reflect, refract, alpha
        const Texture* mp[6] = {m->m_colorMap, m->m_normalMap, m->m_specularMap, m->m_reflectMap, m->m_refractMap,
                                m->m_alphaMap};
        int32_t ids[6];
        bool any = false;
        for (int k = 0; k < 6; k++) {
            if ((ids[k] = texture(mp[k])) < -1) return ids[k];
            any |= ids[k] >= 0;
        }
        if (any && (rc = mrt_scene_set_material_maps(s, id, ids))) return rc;
        if (m->m_envMap) {   // Material::setEnvMap / m_envExposure (src/Material.h:19,41-42)
            const int t = texture(m->m_envMap);
            if (t < 0) return t;
            if ((rc = mrt_scene_set_material_env_map(s, id, t, m->m_envExposure))) return rc;
        }
        mats.emplace(m, id);
        return id;
    }

    // One mrt mesh from triangles tris (in order) of `mesh` with `mat`; the
    // reference's TriangleMesh keeps no vertex / normal / texcoord counts, so the
    // arrays are as long as the largest index any of the mesh's triangles uses.
    int mesh(const TriangleMesh* mesh, const Material* mat, const std::vector<uint32_t>& tris,
             const TriangleMesh* mesh_t2) {
        const int mid = material(mat);
        if (mid < 0) return mid;
        std::vector<uint32_t> vidx, nidx, tidx;
        for (uint32_t t : tris) {
            if (t >= mesh->m_numTris) return MRT_ERR_INVALID;
            const TupleI3 v = mesh->m_vertexIndices[t], n = mesh->m_normalIndices[t];
            vidx.insert(vidx.end(), {v.x, v.y, v.z});
            nidx.insert(nidx.end(), {n.x, n.y, n.z});
            if (mesh->m_texCoordIndices) {
                const TupleI3 x = mesh->m_texCoordIndices[t];
                tidx.insert(tidx.end(), {x.x, x.y, x.z});
            }
        }
        uint32_t nv = 0, nn = 0, ntex = 0;
        for (uint32_t t = 0; t < mesh->m_numTris; t++) {
            const TupleI3 v = mesh->m_vertexIndices[t], n = mesh->m_normalIndices[t];
            nv = std::max({nv, v.x + 1, v.y + 1, v.z + 1});
            nn = std::max({nn, n.x + 1, n.y + 1, n.z + 1});
            if (mesh->m_texCoordIndices) {
                const TupleI3 x = mesh->m_texCoordIndices[t];
                ntex = std::max({ntex, x.x + 1, x.y + 1, x.z + 1});
            }
        }
        mrt_mesh mm;
        memset(&mm, 0, sizeof mm);
        mm.verts = &mesh->m_vertices[0].x;
        mm.normals = &mesh->m_normals[0].x;
        mm.vidx = vidx.data();
        mm.nidx = nidx.data();
        mm.nv = (int32_t)nv;
        mm.nn = (int32_t)nn;
        mm.nt = (int32_t)tris.size();
        mm.vert_stride = mm.normal_stride = 4;   // sizeof(Vector3) / sizeof(float)
        const int id = mrt_scene_add_mesh(s, &mm, mid);
        if (id < 0) return id;
        int rc;
        if (mesh->m_texCoords && ntex > 0) {
            std::vector<float> uv(2 * (size_t)ntex);
            for (uint32_t i = 0; i < ntex; i++) { uv[2 * i] = mesh->m_texCoords[i].x; uv[2 * i + 1] = mesh->m_texCoords[i].y; }
            if ((rc = mrt_scene_mesh_set_texcoords(s, id, uv.data(), (int32_t)ntex, tidx.data()))) return rc;
        }
        if (mesh_t2) {   // MBObject: the time-1 positions of the same vertices
            std::vector<float> v2(3 * (size_t)nv);
            for (uint32_t i = 0; i < nv; i++) {
                v2[3 * i] = mesh_t2->m_vertices[i].x;
                v2[3 * i + 1] = mesh_t2->m_vertices[i].y;
                v2[3 * i + 2] = mesh_t2->m_vertices[i].z;
            }
            if ((rc = mrt_scene_set_mesh_motion(s, id, v2.data()))) return rc;
        }
        return id;
    }

    // A proxy's shared BVH (built once for all its instances): its Objects must
    // be whole meshes, each mesh's triangles last to first, as setupProxy /
    // setupMultiProxy create them; mrt_scene_make_blas restates that order.
    int bvh(const BVH* b, int32_t& n_objects) {
        auto it = blas.find(b);
        if (it != blas.end()) { n_objects = it->second.second; return it->second.first; }
        if (!b || !b->m_objects) return MRT_ERR_INVALID;
        const Objects& os = *b->m_objects;
        std::vector<int32_t> ids;
        for (size_t i = 0; i < os.size();) {
            const Object* o = os[i];
            if (!o->m_mesh || !o->m_material || dynamic_cast<const ProxyObject*>(o) || dynamic_cast<const MBObject*>(o))
                return MRT_ERR_INVALID;
            const uint32_t n = o->m_mesh->m_numTris;
            if (n == 0 || i + n > os.size()) return MRT_ERR_INVALID;
            std::vector<uint32_t> tris(n);
            for (uint32_t k = 0; k < n; k++) {
                const Object* q = os[i + k];
                if (q->m_mesh != o->m_mesh || q->m_material != o->m_material || q->m_index != n - 1 - k)
                    return MRT_ERR_INVALID;
                tris[k] = k;   // the whole mesh in its own order; make_blas walks it last to first
            }
            const int id = mesh(o->m_mesh, o->m_material, tris, nullptr);
            if (id < 0) return id;
            ids.push_back(id);
            i += n;
        }
        const int id = mrt_scene_make_blas(s, ids.data(), (int32_t)ids.size());
        if (id < 0) return id;
        n_objects = (int32_t)os.size();
        blas.emplace(b, std::make_pair(id, n_objects));
        return id;
    }
};
}  // namespace

// Scene::preCalc.  The objects are walked in order, so the C-ABI's world hit id
// of an object is its index in m_objects: every maximal run of consecutive
// triangle Objects of one mesh and one material (MBObjects: also one time-1
// mesh) becomes one mrt mesh whose triangles are those objects' triangles in
// object order; a ProxyObject becomes one instance of its BVH's BLAS (built on
// its first instance; the BLAS meshes leave the world list).  The mesh arrays
// go over as they are: 16-B Vector3s (stride 4), TupleI3 index triples.
int Scene::preCalc() {
    if (m_gpu) mrt_scene_destroy(m_gpu);
    m_gpu = mrt_scene_create();
    if (!m_gpu) return MRT_ERR_INVALID;
    m_instProxy.clear();
    m_instBase.clear();
    Builder B{m_gpu, {}, {}, {}};
    int rc;
    int32_t blas_objects = 0;
    for (size_t i = 0; i < m_objects.size();) {
        Object* o = m_objects[i];
        if (ProxyObject* p = dynamic_cast<ProxyObject*>(o)) {
            int32_t n = 0;
            const int b = B.bvh(p->m_BVH, n);
            if (b < 0) return b;
            if ((rc = mrt_scene_add_instance(m_gpu, b, &p->m_transform.m[0][0])) < 0) return rc;
            m_instProxy.push_back(p);
            m_instBase.push_back(blas_objects);
            blas_objects += n;
            i++;
            continue;
        }
        const MBObject* mb = dynamic_cast<const MBObject*>(o);
        const TriangleMesh* mesh = o->m_mesh;
        if (!mesh || !o->m_material) return MRT_ERR_INVALID;
        size_t j = i;
        std::vector<uint32_t> tris;
        while (j < m_objects.size()) {
            const Object* q = m_objects[j];
            const MBObject* qmb = dynamic_cast<const MBObject*>(q);
            if (dynamic_cast<const ProxyObject*>(q) || q->m_mesh != mesh || q->m_material != o->m_material ||
                (qmb != nullptr) != (mb != nullptr) || (mb && qmb->m_mesh_t2 != mb->m_mesh_t2))
                break;
            tris.push_back(q->m_index);
            j++;
        }
        if ((rc = B.mesh(mesh, o->m_material, tris, mb ? mb->m_mesh_t2 : nullptr)) < 0) return rc;
        i = j;
    }
    for (const Light* l : m_lights) {
        mrt_light ml;
        memset(&ml, 0, sizeof ml);
        ml.power = l->m_power;
        ml.samples = l->m_numSamples;
        ml.noise_threshold = l->m_noiseThreshold;
        ml.cast_shadows = l->m_castShadows ? 1 : 0;
        ml.transparent_shadows = l->m_fastShadows ? 0 : 1;
        ml.texture = -1;
        if (const PointLight* p = dynamic_cast<const PointLight*>(l)) {
            ml.type = MRT_POINT_LIGHT;
            f3(ml.pos, p->m_position);
        } else if (const RectangleLight* r = dynamic_cast<const RectangleLight*>(l)) {
            ml.type = MRT_RECT_LIGHT;
            f3(ml.v1, r->m_v1);
            f3(ml.v2, r->m_v2);
            f3(ml.v3, r->m_v3);
        } else if (const DomeLight* d = dynamic_cast<const DomeLight*>(l)) {
            ml.type = MRT_DOME_LIGHT;
            ml.power = d->m_Gain;   // DomeLight::setPower sets m_Gain (src/DomeLight.h:53)
            if ((ml.texture = B.texture(d->m_lightMap)) < 0) return MRT_ERR_INVALID;
        } else {
            return MRT_ERR_INVALID;
        }
        if ((rc = mrt_scene_add_light(m_gpu, &ml)) < 0) return rc;
    }
    if (m_envMap) {   // Scene::setEnvMap / setEnvExposure (src/Scene.h:23-24)
        const int t = B.texture(m_envMap);
        if (t < 0) return MRT_ERR_INVALID;
        if ((rc = mrt_scene_set_env_map(m_gpu, t, m_envExposure))) return rc;
    }
    float bg[3];
    f3(bg, m_BGColor);
    if ((rc = mrt_scene_set_background(m_gpu, bg)) || (rc = mrt_scene_set_num_paths(m_gpu, m_numPaths)) ||
        (rc = mrt_scene_set_subdivs(m_gpu, m_minSubdivs, m_maxSubdivs, m_noiseThreshold)) ||
        (rc = mrt_scene_set_path_trace(m_gpu, m_pathTrace ? 1 : 0, m_maxBounces, 0)))
        return rc;
    if ((rc = mrt_scene_build_bvh(m_gpu))) return rc;
    mrt_bvh_info info;
    if ((rc = mrt_scene_bvh_info(m_gpu, &info))) return rc;
    for (int32_t& b : m_instBase) b += info.prims;   // BLAS object ids follow the world objects
    return MRT_OK;
}

// HitInfo of a C-ABI hit record: world ids are object indices (preCalc keeps
// object order); an instance hit is the proxy's Object (BLAS object order =
// the proxy's Objects, ProxyObject::intersect sets obj and m_proxy,
// src/ProxyObject.cpp:76-95).
void Scene::to_hit(const mrt_hit& r, HitInfo& h) const {
    h.t = r.t;
    h.a = r.a;
    h.b = r.b;
    h.m_instance = r.inst;
    h.m_proxy = nullptr;
    h.obj = nullptr;
    if (r.prim < 0) return;
    if (r.inst >= 0 && (size_t)r.inst < m_instProxy.size()) {
        ProxyObject* p = m_instProxy[(size_t)r.inst];
        const int32_t k = r.prim - m_instBase[(size_t)r.inst];
        h.m_proxy = p;
        if (p->m_objects && k >= 0 && (size_t)k < p->m_objects->size()) h.obj = (*p->m_objects)[(size_t)k];
    } else if ((size_t)r.prim < m_objects.size()) {
        h.obj = m_objects[(size_t)r.prim];
    }
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
    std::vector<mrt_hit> hits(m_keepFrame ? px : 0);
    static_assert(sizeof(Image::Pixel) == 3, "Image::Pixel is packed rgb");
    const int rc = mrt_render(m_gpu, &c, &o, rgb.data(), reinterpret_cast<uint8_t*>(img->m_pixels.data()),
                              m_keepFrame ? hits.data() : nullptr);
    if (rc == MRT_OK && m_keepFrame) {
        m_lastRGB.swap(rgb);
        m_lastHits.resize(px);
        for (size_t i = 0; i < px; i++) to_hit(hits[i], m_lastHits[i]);
    }
    return rc;
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
    for (size_t i = 0; i < n; i++)
        if (out[i].prim >= 0) to_hit(out[i], hits[i]);
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
