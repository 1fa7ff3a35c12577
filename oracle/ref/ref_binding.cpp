// ref_binding.cpp — TEST INFRASTRUCTURE ONLY: INTEGRATION.md §2's reference-side binding,
// compiled against the reference's OWN types (/root/reference/source, built in place by
// oracle/ref/Makefile, nothing copied) and linked with the product's librtx_hip.so.
//
// 1. The static_asserts below pin the C-ABI records (include/rtx.h) to the reference's structs
//    byte for byte: the binding hands the reference's std::vector<Sphere/Plane/Light> and
//    BVHNode arrays to rtx_upload_scene by reinterpret_cast (DataTypes.h:13-54, 528-536).
// 2. main(): Scene_W4_BunnyScene::Initialize() (Scene.cpp:402-430; cwd must hold
//    Resources/lowpoly_bunny2.obj), then Renderer::Render as the binding would replace it
//    (Renderer.cpp:34-98): flatten the Scene, rtx_create / rtx_upload_scene / rtx_render on the
//    GPU, and write the uint32 frame (raw, row-major) to <out>.  tests/test_gpu_binding.py
//    compares it with the reference's frame (tests/golden/config_W4_Bunny_1920x1080.npz).
//
//   ref_binding <W> <H> <out> [scene: W4_Bunny | W4_Reference | W4_Optional | W3]
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

// Binding-only access to the Scene's and the Materials' members ("a friend
// or two getters are the only changes there"); access specifiers do not change layout.
#define protected public
#define private public
#include "Scene.h"
#include "Material.h"
#undef private
#undef protected

#include "rtx.h"

using namespace dae;

// ---- 1. the records the binding casts: same size, same field offsets, same enum values
static_assert(sizeof(Vector3) == 3 * sizeof(float), "Vector3 must be three packed floats");
static_assert(sizeof(ColorRGB) == 3 * sizeof(float), "ColorRGB must be three packed floats");
static_assert(sizeof(Sphere) == sizeof(rtx_sphere), "dae::Sphere vs rtx_sphere");
static_assert(offsetof(Sphere, origin) == offsetof(rtx_sphere, origin), "Sphere::origin");
static_assert(offsetof(Sphere, radius) == offsetof(rtx_sphere, radius), "Sphere::radius");
static_assert(offsetof(Sphere, materialIndex) == offsetof(rtx_sphere, material), "Sphere::materialIndex");
static_assert(sizeof(Plane) == sizeof(rtx_plane), "dae::Plane vs rtx_plane");
static_assert(offsetof(Plane, origin) == offsetof(rtx_plane, origin), "Plane::origin");
static_assert(offsetof(Plane, normal) == offsetof(rtx_plane, normal), "Plane::normal");
static_assert(offsetof(Plane, materialIndex) == offsetof(rtx_plane, material), "Plane::materialIndex");
static_assert(sizeof(BVHNode) == sizeof(rtx_bvh_node), "dae::BVHNode vs rtx_bvh_node");
static_assert(offsetof(BVHNode, minAABB) == offsetof(rtx_bvh_node, min), "BVHNode::minAABB");
static_assert(offsetof(BVHNode, maxAABB) == offsetof(rtx_bvh_node, max), "BVHNode::maxAABB");
static_assert(offsetof(BVHNode, firstIdx) == offsetof(rtx_bvh_node, first_idx), "BVHNode::firstIdx");
static_assert(offsetof(BVHNode, idxCount) == offsetof(rtx_bvh_node, idx_count), "BVHNode::idxCount");
static_assert(offsetof(BVHNode, leftNode) == offsetof(rtx_bvh_node, left_node), "BVHNode::leftNode");
static_assert(sizeof(Light) == sizeof(rtx_light), "dae::Light vs rtx_light");
static_assert(offsetof(Light, origin) == offsetof(rtx_light, origin), "Light::origin");
static_assert(offsetof(Light, direction) == offsetof(rtx_light, direction), "Light::direction");
static_assert(offsetof(Light, color) == offsetof(rtx_light, color), "Light::color");
static_assert(offsetof(Light, intensity) == offsetof(rtx_light, intensity), "Light::intensity");
static_assert(offsetof(Light, type) == offsetof(rtx_light, type), "Light::type");
static_assert(sizeof(LightType) == sizeof(int32_t), "LightType is an int");
static_assert(static_cast<int>(LightType::Point) == RTX_LIGHT_POINT &&
              static_cast<int>(LightType::Directional) == RTX_LIGHT_DIRECTIONAL, "light types");
static_assert(static_cast<int>(TriangleCullMode::FrontFaceCulling) == RTX_CULL_FRONT &&
              static_cast<int>(TriangleCullMode::BackFaceCulling) == RTX_CULL_BACK &&
              static_cast<int>(TriangleCullMode::NoCulling) == RTX_CULL_NONE, "cull modes");

// ---- 2. the binding
static rtx_material Flatten(Material* m) {
    rtx_material r{};
    if (auto* a = dynamic_cast<Material_SolidColor*>(m)) {
        r.kind = RTX_MAT_SOLID_COLOR;
        r.color[0] = a->m_Color.r; r.color[1] = a->m_Color.g; r.color[2] = a->m_Color.b;
    } else if (auto* b = dynamic_cast<Material_Lambert*>(m)) {
        r.kind = RTX_MAT_LAMBERT;
        r.color[0] = b->m_DiffuseColor.r; r.color[1] = b->m_DiffuseColor.g; r.color[2] = b->m_DiffuseColor.b;
        r.kd = b->m_DiffuseReflectance;
    } else if (auto* c = dynamic_cast<Material_LambertPhong*>(m)) {
        r.kind = RTX_MAT_LAMBERT_PHONG;
        r.color[0] = c->m_DiffuseColor.r; r.color[1] = c->m_DiffuseColor.g; r.color[2] = c->m_DiffuseColor.b;
        r.kd = c->m_DiffuseReflectance;
        r.ks = c->m_SpecularReflectance;
        r.exponent = c->m_PhongExponent;
    } else if (auto* d = dynamic_cast<Material_CookTorrence*>(m)) {
        r.kind = RTX_MAT_COOK_TORRANCE;
        r.color[0] = d->m_Albedo.r; r.color[1] = d->m_Albedo.g; r.color[2] = d->m_Albedo.b;
        r.metalness = d->m_Metalness;
        r.roughness = d->m_Roughness;
    }
    return r;
}

// Renderer::Render(Scene*) with the parallel_for body replaced by the C-ABI call
static int RenderThroughAbi(rtx_ctx* ctx, Scene* pScene, int W, int H, uint32_t* pixels) {
    Camera& camera = pScene->GetCamera();
    camera.CalculateCameraToWorld();
    std::vector<rtx_mesh> meshes;
    for (const TriangleMesh& m : pScene->m_TriangleMeshGeometries)
        meshes.push_back({&m.transformedPositions[0].x, static_cast<uint32_t>(m.transformedPositions.size()),
                          m.indices.data(), static_cast<uint32_t>(m.indices.size()), &m.transformedNormals[0].x,
                          reinterpret_cast<const rtx_bvh_node*>(m.pBVHNodes), m.nodesUsed,
                          static_cast<int32_t>(m.cullMode), m.materialIndex, {0, 0, 0}});
    std::vector<rtx_material> mats;
    for (Material* pm : pScene->GetMaterials()) mats.push_back(Flatten(pm));
    const auto& sph = pScene->GetSphereGeometries();
    const auto& pl = pScene->GetPlaneGeometries();
    const auto& li = pScene->GetLights();
    const rtx_scene s{reinterpret_cast<const rtx_sphere*>(sph.data()), static_cast<uint32_t>(sph.size()),
                      reinterpret_cast<const rtx_plane*>(pl.data()), static_cast<uint32_t>(pl.size()),
                      meshes.data(), static_cast<uint32_t>(meshes.size()),
                      reinterpret_cast<const rtx_light*>(li.data()), static_cast<uint32_t>(li.size()),
                      mats.data(), static_cast<uint32_t>(mats.size())};
    int rc = rtx_upload_scene(ctx, &s);
    if (rc != RTX_OK) return rc;
    const rtx_camera cam{{camera.origin.x, camera.origin.y, camera.origin.z},
                         {camera.right.x, camera.right.y, camera.right.z},
                         {camera.up.x, camera.up.y, camera.up.z},
                         {camera.forward.x, camera.forward.y, camera.forward.z},
                         camera.fov};
    // SDL_MapRGB on an XRGB8888 window surface (Renderer.cpp:178-181)
    const rtx_render_params p{static_cast<uint32_t>(W), static_cast<uint32_t>(H), RTX_MODE_COMBINED, 1,
                              {16, 8, 0, 0}, 0, 0, 1};
    return rtx_render(ctx, &cam, &p, pixels, nullptr);   // blocking, like the parallel_for
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: ref_binding <W> <H> <out> [W4_Bunny|W4_Reference|W4_Optional|W3]\n");
        return 2;
    }
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]);
    const std::string which = argc > 4 ? argv[4] : "W4_Bunny";
    Scene* pScene = nullptr;
    if (which == "W4_Bunny") pScene = new Scene_W4_BunnyScene();
    else if (which == "W4_Reference") pScene = new Scene_W4_ReferenceScene();
    else if (which == "W4_Optional") pScene = new Scene_W4_OptionalScene();
    else if (which == "W3") pScene = new Scene_W3();
    else { std::fprintf(stderr, "unknown scene %s\n", which.c_str()); return 2; }
    pScene->Initialize();
    rtx_ctx* ctx = nullptr;
    if (rtx_create(&ctx, 0) != RTX_OK) {
        std::fprintf(stderr, "rtx_create: %s\n", rtx_last_error(nullptr));
        return 1;
    }
    std::vector<uint32_t> px(static_cast<size_t>(W) * H);
    const int rc = RenderThroughAbi(ctx, pScene, W, H, px.data());
    if (rc != RTX_OK) {
        std::fprintf(stderr, "render: %d %s\n", rc, rtx_last_error(ctx));
        return 1;
    }
    FILE* f = std::fopen(argv[3], "wb");
    if (!f || std::fwrite(px.data(), 4, px.size(), f) != px.size()) return 1;
    std::fclose(f);
    rtx_destroy(ctx);
    delete pScene;
    std::printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d}\n", which.c_str(), W, H);
    return 0;
}
