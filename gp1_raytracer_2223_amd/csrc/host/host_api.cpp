// host_api.cpp — extern "C" wrappers of the host scene model (include/rtx_host.h).
#include <dlfcn.h>

#include <cstring>
#include <new>
#include <string>

#include "rtx_host.h"
#include "scene.h"

// Default asset directory: <dir of librtx_host.so>/../assets (the in-tree package layout).
static std::string default_asset_dir() {
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&default_asset_dir), &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t slash = p.rfind('/');
        if (slash != std::string::npos) return p.substr(0, slash) + "/../assets";
    }
    return "assets";
}

struct rtx_host_scene {
    std::unique_ptr<rtx::Scene> scene;
};

static void set_err(char* err, size_t len, const std::string& msg) {
    if (err && len) {
        std::strncpy(err, msg.c_str(), len - 1);
        err[len - 1] = 0;
    }
}

extern "C" int rtx_host_scene_create(const char* name, const char* asset_dir, rtx_host_scene** out, char* err,
                                     size_t err_len) {
    if (!name || !out) return RTX_E_INVALID;
    *out = nullptr;
    try {
        auto s = rtx::MakeScene(name, (asset_dir && *asset_dir) ? asset_dir : default_asset_dir());
        if (!s) { set_err(err, err_len, std::string("unknown scene: ") + name); return RTX_E_INVALID; }
        if (!s->Initialize()) { set_err(err, err_len, s->Error()); return RTX_E_UNSUPPORTED; }
        auto* h = new rtx_host_scene;
        h->scene = std::move(s);
        *out = h;
        return RTX_OK;
    } catch (const std::bad_alloc&) {
        set_err(err, err_len, "out of memory");
        return RTX_E_NOMEM;
    } catch (const std::exception& e) {
        set_err(err, err_len, e.what());
        return RTX_E_INVALID;
    }
}

extern "C" void rtx_host_scene_destroy(rtx_host_scene* s) { delete s; }

extern "C" int rtx_host_scene_update(rtx_host_scene* s, float total_time) {
    if (!s) return RTX_E_INVALID;
    s->scene->Update(total_time);
    return RTX_OK;
}

extern "C" int rtx_host_scene_copy_state(rtx_host_scene* dst, const rtx_host_scene* src) {
    if (!dst || !src) return RTX_E_INVALID;
    return dst->scene->CopyStateFrom(*src->scene) ? RTX_OK : RTX_E_INVALID;
}

extern "C" int rtx_host_scene_view(rtx_host_scene* s, rtx_scene* out_scene, rtx_camera* out_camera) {
    if (!s) return RTX_E_INVALID;
    rtx::Camera& cam = s->scene->GetCamera();
    cam.CalculateCameraToWorld();   // Renderer.cpp:40
    if (out_scene) *out_scene = s->scene->View();
    if (out_camera) *out_camera = cam.View();
    return RTX_OK;
}

extern "C" int rtx_host_scene_animated(const rtx_host_scene* s) {
    if (!s) return RTX_E_INVALID;
    return s->scene->Animated() ? 1 : 0;
}

extern "C" int rtx_host_scene_spinning(rtx_host_scene* s, int32_t* mesh_ids, uint32_t capacity) {
    if (!s) return RTX_E_INVALID;
    const auto spin = s->scene->Spinning();
    for (size_t i = 0; i < spin.size() && i < capacity && mesh_ids; ++i) {
        int32_t id = -1;
        for (size_t k = 0; k < s->scene->m_Meshes.size(); ++k)
            if (s->scene->m_Meshes[k].get() == spin[i]) id = static_cast<int32_t>(k);
        mesh_ids[i] = id;
    }
    return static_cast<int>(spin.size());
}

extern "C" int rtx_host_scene_mesh_source(rtx_host_scene* s, uint32_t mesh, rtx_mesh_source* out) {
    if (!s || !out || mesh >= s->scene->m_Meshes.size()) return RTX_E_INVALID;
    const rtx::TriangleMesh& m = *s->scene->m_Meshes[mesh];
    if (m.normals.size() * 3 < m.indices.size()) return RTX_E_INVALID;
    out->positions = m.positions.empty() ? nullptr : &m.positions[0].x;
    out->n_positions = static_cast<uint32_t>(m.positions.size());
    out->normals = m.normals.empty() ? nullptr : &m.normals[0].x;
    out->indices = m.indices.empty() ? nullptr : m.indices.data();
    out->n_indices = static_cast<uint32_t>(m.indices.size());
    return RTX_OK;
}

extern "C" int rtx_host_scene_transforms(rtx_host_scene* s, float total_time, float* out, uint32_t capacity) {
    if (!s || (!out && capacity)) return RTX_E_INVALID;
    const float yaw = rtx::Scene::SpinYaw(total_time);
    uint32_t i = 0;
    for (rtx::TriangleMesh* m : s->scene->Spinning()) {
        m->RotateY(yaw);   // every turning mesh turns; only the first `capacity` are written
        if (i < capacity) {
            const rtx::Mat4 f = m->scaleTransform * m->rotationTransform * m->translationTransform;   // DataTypes.h:213
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) out[16 * i + 4 * r + c] = f.d[r].at(c);
        }
        ++i;
    }
    return static_cast<int>(i);
}

extern "C" int rtx_host_camera_set(rtx_host_scene* s, const float origin[3], float fov_degrees, float pitch,
                                   float yaw) {
    if (!s || !origin) return RTX_E_INVALID;
    rtx::Camera& cam = s->scene->GetCamera();
    cam.origin = {origin[0], origin[1], origin[2]};
    cam.SetCameraFOV(fov_degrees);
    cam.totalPitch = pitch;
    cam.totalYaw = yaw;
    cam.CalculateForwardVector();
    cam.CalculateCameraToWorld();
    return RTX_OK;
}

extern "C" int rtx_host_parse_obj(const char* path, float* positions, uint32_t* n_positions, float* normals,
                                  int32_t* indices, uint32_t* n_indices, uint32_t cap_pos, uint32_t cap_idx) {
    if (!path || !n_positions || !n_indices) return RTX_E_INVALID;
    std::vector<rtx::Vec3> p, n;
    std::vector<int32_t> idx;
    try {
        if (!rtx::ParseOBJ(path, p, n, idx)) return RTX_E_INVALID;
    } catch (const std::exception&) {
        return RTX_E_INVALID;
    }
    *n_positions = static_cast<uint32_t>(p.size());
    *n_indices = static_cast<uint32_t>(idx.size());
    if (positions && p.size() <= cap_pos)
        for (size_t k = 0; k < p.size(); ++k) { positions[3 * k] = p[k].x; positions[3 * k + 1] = p[k].y; positions[3 * k + 2] = p[k].z; }
    if (normals && n.size() * 3 <= static_cast<size_t>(cap_idx))
        for (size_t k = 0; k < n.size(); ++k) { normals[3 * k] = n[k].x; normals[3 * k + 1] = n[k].y; normals[3 * k + 2] = n[k].z; }
    if (indices && idx.size() <= cap_idx) std::memcpy(indices, idx.data(), idx.size() * 4);
    return RTX_OK;
}

extern "C" int rtx_host_obj_to_asset(const char* obj_path, const char* asset_path) {
    if (!obj_path || !asset_path) return RTX_E_INVALID;
    std::vector<rtx::Vec3> p, n;
    std::vector<int32_t> idx;
    try {
        if (!rtx::ParseOBJ(obj_path, p, n, idx)) return RTX_E_INVALID;
    } catch (const std::exception&) {
        return RTX_E_INVALID;
    }
    return rtx::SaveMeshAsset(asset_path, p, idx) ? RTX_OK : RTX_E_INVALID;
}
