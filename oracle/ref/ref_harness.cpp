// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Drives the UNMODIFIED reference sources (compiled in place from
// /root/reference/source by oracle/ref/Makefile; nothing is copied) to produce the
// golden fixtures under tests/golden/ and the "reference" CPU baseline.
//
// What is built from the reference: Vector3.cpp, Vector4.cpp, Matrix.cpp, Scene.cpp and
// the header-only GeometryUtils / LightUtils / Material / BRDF / TriangleMesh+BVH code.
// What is NOT built: Renderer.cpp (needs Microsoft PPL <ppl.h> and an SDL window
// surface, neither exists in this image), Timer.cpp and main.cpp (SDL runtime).  The
// ~40-line per-pixel body Renderer::RenderPixel (source/Renderer.cpp:100-182) is
// therefore restated below, line for line in the reference's own types, and calls the
// reference's Scene::GetClosestHit / Scene::DoesHit / LightUtils / Material::Shade.
// concurrency::parallel_for (Renderer.cpp:81-85) becomes a std::thread pool pulling
// 1024-pixel chunks from an atomic counter (PPL's parallel_for is work-stealing).
//
// Subcommands (all binary outputs use the RTXB container read by tests/golden/rtxb.py):
//   scene  <name> <t|-1> <out>                      flattened scene after Initialize (+Update(t))
//   scene  <name> <t1,t2,...> <out>                 ... after a sequence of Updates (the BVH
//                                                   permutation carries over between builds)
//   render <name> <t|-1> <W> <H> <mode> <shadows> <threads> <out>
//   bench  <name> <t|-1> <W> <H> <threads> <frames> [mode shadows]   -> one JSON line
//   obj    <path> <out>                             Utils::ParseOBJ result
//   prims  <seed> <n> <out>                         primitive known-answer vectors
// Scenes are constructed with cwd = the directory holding Resources/*.obj.

#include <algorithm>
#include <cctype>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

// Harness-only access to the reference's protected/private members (scene arrays,
// material parameters).  Access specifiers do not change object layout here.
#define protected public
#define private public
#include "Scene.h"
#include "Material.h"
#include "Utils.h"
#undef private
#undef protected

using namespace dae;

// ----------------------------------------------------------------------------------
// RTXB container: repeated { u32 name_len, name, u32 dtype, u64 nbytes, bytes }.
// dtype: 0 = f32, 1 = i32, 2 = u32, 3 = u8.
struct Writer {
    FILE* f{};
    explicit Writer(const char* path) {
        f = std::fopen(path, "wb");
        if (!f) { std::perror(path); std::exit(2); }
        std::fwrite("RTXB", 1, 4, f);
    }
    ~Writer() { if (f) std::fclose(f); }
    void put(const std::string& name, uint32_t dtype, const void* p, uint64_t n) {
        uint32_t nl = static_cast<uint32_t>(name.size());
        std::fwrite(&nl, 4, 1, f);
        std::fwrite(name.data(), 1, nl, f);
        std::fwrite(&dtype, 4, 1, f);
        std::fwrite(&n, 8, 1, f);
        if (n) std::fwrite(p, 1, n, f);
    }
    void f32(const std::string& n, const std::vector<float>& v) { put(n, 0, v.data(), v.size() * 4); }
    void i32(const std::string& n, const std::vector<int32_t>& v) { put(n, 1, v.data(), v.size() * 4); }
    void u32(const std::string& n, const std::vector<uint32_t>& v) { put(n, 2, v.data(), v.size() * 4); }
    void u8(const std::string& n, const std::vector<uint8_t>& v) { put(n, 3, v.data(), v.size()); }
};

static void push3(std::vector<float>& v, const Vector3& a) { v.push_back(a.x); v.push_back(a.y); v.push_back(a.z); }

// ----------------------------------------------------------------------------------
// Scenes.  The reference catalogue (Scene.cpp:163-474) plus the two synthetic configs
// of SURVEY.md §8(d), built with the reference's own Add*/ParseOBJ/BVH code.

// Synthetic 100k-triangle height field: 250 x 200 quads over
// x in [-3,3], z in [-1,3], y = 0.3 + 0.5*u with u = (mt19937(42)() >> 8) * 2^-24 per
// vertex (row-major, z outer).  Two triangles per quad, normals +y.  Bunny-scene
// planes, lights and materials.
class Scene_Synthetic100k final : public Scene {
public:
    void Initialize() override {
        sceneName = "Synthetic 100k";
        m_Camera.origin = {0.f, 3.f, -9.f};
        m_Camera.SetCameraFOV(45.f);
        const auto matLambert_GrayBlue = AddMaterial(new Material_Lambert({0.49f, 0.57f, 0.57f}, 1.f));
        const auto matLambert_White = AddMaterial(new Material_Lambert(colors::White, 1.f));
        m_pMesh = AddTriangleMesh(TriangleCullMode::BackFaceCulling, matLambert_White);
        const int NX = 250, NZ = 200;
        std::mt19937 rng(42);
        for (int j = 0; j <= NZ; ++j) {
            for (int i = 0; i <= NX; ++i) {
                const float u = static_cast<float>(rng() >> 8) * (1.0f / 16777216.0f);
                const float x = -3.0f + (6.0f * static_cast<float>(i)) / 250.0f;
                const float z = -1.0f + (4.0f * static_cast<float>(j)) / 200.0f;
                const float y = 0.3f + 0.5f * u;
                m_pMesh->positions.push_back({x, y, z});
            }
        }
        for (int j = 0; j < NZ; ++j) {
            for (int i = 0; i < NX; ++i) {
                const int v00 = j * (NX + 1) + i, v10 = v00 + 1;
                const int v01 = v00 + (NX + 1), v11 = v01 + 1;
                const int tri[6] = {v00, v01, v10, v10, v01, v11};
                for (int k = 0; k < 6; ++k) m_pMesh->indices.push_back(tri[k]);
            }
        }
        m_pMesh->CalculateNormals();
        m_pMesh->pBVHNodes = new BVHNode[m_pMesh->indices.size()];
        m_pMesh->UpdateAABB();
        m_pMesh->UpdateTransforms();

        AddPlane({0.f, 0.f, 10.f}, {0.f, 0.f, -1.f}, matLambert_GrayBlue);
        AddPlane({0.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, matLambert_GrayBlue);
        AddPlane({0.f, 10.f, 0.f}, {0.f, -1.f, 0.f}, matLambert_GrayBlue);
        AddPlane({5.f, 0.f, 0.f}, {-1.f, 0.f, 0.f}, matLambert_GrayBlue);
        AddPlane({-5.f, 0.f, 0.f}, {1.f, 0.f, 0.f}, matLambert_GrayBlue);

        AddPointLight({0.f, 5.f, 5.f}, 50.f, ColorRGB{1.f, 0.61f, 0.45f});
        AddPointLight({-2.5f, 5.f, -5.f}, 70.f, ColorRGB{1.f, 0.8f, 0.45f});
        AddPointLight({2.5f, 2.5f, -5.f}, 50.f, ColorRGB{0.34f, 0.47f, 0.68f});
    }
    TriangleMesh* m_pMesh{nullptr};
};

// The 5 extra lights of the "Bunny + 8 lights" config.
static void add_extra_lights(Scene* s) {
    const ColorRGB trio[3] = {ColorRGB{1.f, 0.61f, 0.45f}, ColorRGB{1.f, 0.8f, 0.45f},
                              ColorRGB{0.34f, 0.47f, 0.68f}};
    for (int k = 0; k < 5; ++k) {
        const float theta = PI_2 * static_cast<float>(k) / 5.f;
        const float x = 3.5f * cosf(theta);
        const float z = 3.5f * sinf(theta) - 2.f;
        s->AddPointLight({x, 5.5f, z}, 40.f, trio[k % 3]);
    }
}

// Scene file (gp1_raytracer_2223_amd/csrc/host/scene.cpp, "scene files"): the same
// grammar built with the REFERENCE's own classes and builders, so file-defined scenes
// are pinned against the reference like the catalogue scenes.
class Scene_File final : public Scene {
public:
    explicit Scene_File(std::string path) : m_Path(std::move(path)) {}
    void Initialize() override {
        std::ifstream in(m_Path);
        if (!in) { std::fprintf(stderr, "cannot open %s\n", m_Path.c_str()); std::exit(2); }
        std::string line;
        while (std::getline(in, line)) {
            const size_t hash = line.find('#');
            if (hash != std::string::npos) line.resize(hash);
            std::vector<std::string> t;
            size_t i = 0;
            while (i < line.size()) {
                while (i < line.size() && std::isspace(static_cast<unsigned char>(line[i]))) ++i;
                size_t j = i;
                while (j < line.size() && !std::isspace(static_cast<unsigned char>(line[j]))) ++j;
                if (j > i) t.push_back(line.substr(i, j - i));
                i = j;
            }
            if (t.empty()) continue;
            if (!Directive(t)) { std::fprintf(stderr, "bad directive in %s: %s\n", m_Path.c_str(), line.c_str()); std::exit(2); }
        }
    }
    std::vector<TriangleMesh*> m_Spin;

private:
    static float F(const std::string& s) { return std::strtof(s.c_str(), nullptr); }
    bool Directive(const std::vector<std::string>& t) {
        const std::string& d = t[0];
        if (d == "camera" && t.size() == 5) {
            m_Camera.origin = {F(t[1]), F(t[2]), F(t[3])};
            m_Camera.SetCameraFOV(F(t[4]));
            return true;
        }
        if (d == "material" && t.size() >= 2) {
            const ColorRGB c = t.size() >= 5 ? ColorRGB{F(t[2]), F(t[3]), F(t[4])} : ColorRGB{};
            if (t[1] == "solid" && t.size() == 5) { AddMaterial(new Material_SolidColor(c)); return true; }
            if (t[1] == "lambert" && t.size() == 6) { AddMaterial(new Material_Lambert(c, F(t[5]))); return true; }
            if (t[1] == "lambert_phong" && t.size() == 8) {
                AddMaterial(new Material_LambertPhong(c, F(t[5]), F(t[6]), F(t[7])));
                return true;
            }
            if (t[1] == "cook_torrance" && t.size() == 7) {
                AddMaterial(new Material_CookTorrence(c, F(t[5]), F(t[6])));
                return true;
            }
            return false;
        }
        if (d == "sphere" && t.size() == 6) {
            AddSphere({F(t[1]), F(t[2]), F(t[3])}, F(t[4]), static_cast<unsigned char>(std::atoi(t[5].c_str())));
            return true;
        }
        if (d == "plane" && t.size() == 8) {
            AddPlane({F(t[1]), F(t[2]), F(t[3])}, {F(t[4]), F(t[5]), F(t[6])},
                     static_cast<unsigned char>(std::atoi(t[7].c_str())));
            return true;
        }
        if (d == "light" && t.size() == 9) {
            const Vector3 v{F(t[2]), F(t[3]), F(t[4])};
            const ColorRGB c{F(t[6]), F(t[7]), F(t[8])};
            if (t[1] == "point") { AddPointLight(v, F(t[5]), c); return true; }
            if (t[1] == "directional") { AddDirectionalLight(v, F(t[5]), c); return true; }
            return false;
        }
        if (d == "mesh" && t.size() >= 4) {
            TriangleCullMode cull;
            if (t[3] == "front") cull = TriangleCullMode::FrontFaceCulling;
            else if (t[3] == "back") cull = TriangleCullMode::BackFaceCulling;
            else if (t[3] == "none") cull = TriangleCullMode::NoCulling;
            else return false;
            TriangleMesh* m = AddTriangleMesh(cull, static_cast<unsigned char>(std::atoi(t[2].c_str())));
            Utils::ParseOBJ("Resources/" + t[1] + ".obj", m->positions, m->normals, m->indices);
            bool spin = false;
            for (size_t i = 4; i < t.size();) {
                if (t[i] == "scale" && i + 3 < t.size()) { m->Scale({F(t[i + 1]), F(t[i + 2]), F(t[i + 3])}); i += 4; }
                else if (t[i] == "translate" && i + 3 < t.size()) { m->Translate({F(t[i + 1]), F(t[i + 2]), F(t[i + 3])}); i += 4; }
                else if (t[i] == "spin") { spin = true; ++i; }
                else return false;
            }
            m->pBVHNodes = new BVHNode[m->indices.size()];
            m->UpdateAABB();
            m->UpdateTransforms();
            if (spin) m_Spin.push_back(m);
            return true;
        }
        return false;
    }
    std::string m_Path;
};

static std::unique_ptr<Scene> make_scene(const std::string& name) {
    if (name.rfind("file:", 0) == 0) {
        auto f = std::make_unique<Scene_File>(name.substr(5));
        f->Initialize();
        return f;
    }
    std::unique_ptr<Scene> s;
    if (name == "W1") s = std::make_unique<Scene_W1>();
    else if (name == "W2") s = std::make_unique<Scene_W2>();
    else if (name == "W3") s = std::make_unique<Scene_W3>();
    else if (name == "W3_Test") s = std::make_unique<Scene_W3_TestScene>();
    else if (name == "W4_Reference") s = std::make_unique<Scene_W4_ReferenceScene>();
    else if (name == "W4_Bunny" || name == "Bunny8Lights") s = std::make_unique<Scene_W4_BunnyScene>();
    else if (name == "W4_Optional") s = std::make_unique<Scene_W4_OptionalScene>();
    else if (name == "Synthetic100k") s = std::make_unique<Scene_Synthetic100k>();
    else { std::fprintf(stderr, "unknown scene %s\n", name.c_str()); std::exit(2); }
    s->Initialize();
    if (name == "Bunny8Lights") add_extra_lights(s.get());
    return s;
}

static void apply_update(Scene* s, const std::string& name, float t);
// Scene_W4_*::Update without the SDL-driven camera part (Scene.cpp:391-400, 431-437,
// 468-474): yaw = (cos(t)+1)/2 * 2pi applied to every animated mesh.
static void apply_time(Scene* s, const std::string& name, float t) {
    if (t < 0.f) return;
    apply_update(s, name, t);
}
static void apply_time(Scene* s, const std::string& name, const char* times) {
    // "t" or a comma-separated sequence "t1,t2,...": one Update per entry, in order
    std::string list(times);
    size_t pos = 0;
    for (;;) {
        const size_t comma = list.find(',', pos);
        apply_time(s, name, std::stof(list.substr(pos, comma - pos)));
        if (comma == std::string::npos) break;
        pos = comma + 1;
    }
}
static void apply_update(Scene* s, const std::string& name, float t) {
    const auto yawAngle{(cosf(t) + 1.f) / 2.f * PI_2};
    if (name.rfind("file:", 0) == 0) {
        for (const auto m : static_cast<Scene_File*>(s)->m_Spin) { m->RotateY(yawAngle); m->UpdateTransforms(); }
        return;
    }
    if (name == "W4_Reference") {
        auto* r = static_cast<Scene_W4_ReferenceScene*>(s);
        for (const auto m : r->m_Meshes) { m->RotateY(yawAngle); m->UpdateTransforms(); }
    } else if (name == "W4_Bunny" || name == "Bunny8Lights") {
        auto* b = static_cast<Scene_W4_BunnyScene*>(s);
        b->m_pMesh->RotateY(yawAngle); b->m_pMesh->UpdateTransforms();
    } else if (name == "W4_Optional") {
        auto* o = static_cast<Scene_W4_OptionalScene*>(s);
        o->m_pMesh->RotateY(yawAngle); o->m_pMesh->UpdateTransforms();
    }
}

// ----------------------------------------------------------------------------------
// Renderer::RenderPixel restated (source/Renderer.cpp:100-182).  SDL_MapRGB for an
// XRGB8888 surface (Rshift 16, Gshift 8, Bshift 0, Amask 0).
struct RenderState {
    int width{}, height{};
    float aspect{};
    int mode{3};            // Renderer::LightingMode::Combined
    bool shadows{true};
};

static void render_pixel(const RenderState& rs, Scene* pScene, uint32_t pixelIndex, const Camera& camera,
                         const std::vector<Light>& lights, const std::vector<Material*>& materials,
                         uint32_t* outPixels, float* outRgb) {
    const int m_Width = rs.width, m_Height = rs.height;
    const float m_AspectRatio = rs.aspect;
    const int px = pixelIndex % m_Width;
    const int py = pixelIndex / m_Width;

    const float cx = (2.f * ((px + 0.5f) / m_Width) - 1) * m_AspectRatio * camera.fov;
    const float cy = (1.f - (2.f * (py + 0.5f) / m_Height)) * camera.fov;

    Vector3 viewDirection{camera.cameraToWorld.TransformVector(cx, cy, 1)};
    viewDirection.Normalize();
    const Ray viewRay{camera.origin, viewDirection};

    HitRecord closestHit{};
    pScene->GetClosestHit(viewRay, closestHit);

    float shadowFactor{1.f};
    ColorRGB finalColor{};

    if (closestHit.didHit) {
        const Vector3 originOffset{closestHit.origin + closestHit.normal * 0.0001f};
        for (const auto& light : lights) {
            Vector3 lightDirection{LightUtils::GetDirectionToLight(light, originOffset)};
            const float magnitude{lightDirection.Normalize()};
            if (rs.shadows) {
                const Ray shadowRay{originOffset, lightDirection, 0.0001f, magnitude};
                if (pScene->DoesHit(shadowRay)) {
                    shadowFactor *= 0.95f;
                    continue;
                }
            }
            switch (rs.mode) {
            case 3: {
                const float observedArea{std::max(Vector3::Dot(closestHit.normal, lightDirection), 0.f)};
                const ColorRGB radiance{LightUtils::GetRadiance(light, closestHit.origin)};
                const ColorRGB brdf{materials[closestHit.materialIndex]->Shade(closestHit, lightDirection, -viewDirection)};
                finalColor += observedArea * radiance * brdf;
                break;
            }
            case 0: {
                const float observedArea{std::max(Vector3::Dot(closestHit.normal, lightDirection), 0.f)};
                finalColor += ColorRGB{observedArea, observedArea, observedArea};
                break;
            }
            case 1: {
                finalColor += LightUtils::GetRadiance(light, closestHit.origin);
                break;
            }
            case 2: {
                finalColor += materials[closestHit.materialIndex]->Shade(closestHit, lightDirection, -viewDirection);
                break;
            }
            }
        }
        finalColor *= shadowFactor;
    }
    finalColor.MaxToOne();

    const uint8_t r = static_cast<uint8_t>(finalColor.r * 255);
    const uint8_t g = static_cast<uint8_t>(finalColor.g * 255);
    const uint8_t b = static_cast<uint8_t>(finalColor.b * 255);
    const size_t o = static_cast<size_t>(px) + static_cast<size_t>(py) * m_Width;
    outPixels[o] = (uint32_t(r) << 16) | (uint32_t(g) << 8) | uint32_t(b);
    if (outRgb) {
        outRgb[3 * o + 0] = finalColor.r;
        outRgb[3 * o + 1] = finalColor.g;
        outRgb[3 * o + 2] = finalColor.b;
    }
}

// concurrency::parallel_for stand-in for THIS harness: dynamic 1024-pixel chunks.
static void parallel_pixels(uint32_t n, int threads, const std::function<void(uint32_t)>& fn) {
    if (threads <= 1) { for (uint32_t i = 0; i < n; ++i) fn(i); return; }
    std::atomic<uint32_t> next{0};
    const uint32_t chunk = 1024;
    auto worker = [&]() {
        for (;;) {
            const uint32_t b = next.fetch_add(chunk);
            if (b >= n) break;
            const uint32_t e = std::min(n, b + chunk);
            for (uint32_t i = b; i < e; ++i) fn(i);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
}

// Renderer::Render (source/Renderer.cpp:34-98) minus SDL presentation.
static void render(Scene* pScene, const RenderState& rs, int threads, uint32_t* px, float* rgb) {
    Camera& camera = pScene->GetCamera();
    auto materials = pScene->GetMaterials();  // by value, as Scene.h:43 returns it
    auto& lights = pScene->GetLights();
    const uint32_t numPixels = rs.width * rs.height;
    camera.CalculateCameraToWorld();
    parallel_pixels(numPixels, threads, [&](uint32_t i) {
        render_pixel(rs, pScene, i, camera, lights, materials, px, rgb);
    });
}

static RenderState make_state(int W, int H, int mode, bool shadows) {
    RenderState rs;
    rs.width = W; rs.height = H;
    rs.aspect = W / static_cast<float>(H);   // Renderer.cpp:30
    rs.mode = mode; rs.shadows = shadows;
    return rs;
}

// ----------------------------------------------------------------------------------
static void dump_scene(Scene* s, const char* out) {
    Writer w(out);
    Camera& cam = s->GetCamera();
    cam.CalculateCameraToWorld();
    std::vector<float> camv;
    push3(camv, cam.origin); push3(camv, cam.right); push3(camv, cam.up); push3(camv, cam.forward);
    camv.push_back(cam.fov); camv.push_back(cam.fovAngle);
    w.f32("camera", camv);

    std::vector<float> sph; std::vector<uint8_t> sphm;
    for (auto& sp : s->m_SphereGeometries) { push3(sph, sp.origin); sph.push_back(sp.radius); sphm.push_back(sp.materialIndex); }
    w.f32("spheres", sph); w.u8("sphere_mat", sphm);

    std::vector<float> pl; std::vector<uint8_t> plm;
    for (auto& p : s->m_PlaneGeometries) { push3(pl, p.origin); push3(pl, p.normal); plm.push_back(p.materialIndex); }
    w.f32("planes", pl); w.u8("plane_mat", plm);

    std::vector<uint32_t> meshinfo;  // per mesh: cull, mat, nV, nI, nodesUsed
    int mi = 0;
    for (auto& m : s->m_TriangleMeshGeometries) {
        meshinfo.push_back(static_cast<uint32_t>(m.cullMode));
        meshinfo.push_back(m.materialIndex);
        meshinfo.push_back(static_cast<uint32_t>(m.transformedPositions.size()));
        meshinfo.push_back(static_cast<uint32_t>(m.indices.size()));
        meshinfo.push_back(m.nodesUsed);
        const std::string p = "mesh" + std::to_string(mi) + "_";
        std::vector<float> pos, tpos, nrm, tnrm, nodes_f;
        for (auto& v : m.positions) push3(pos, v);
        for (auto& v : m.transformedPositions) push3(tpos, v);
        for (auto& v : m.normals) push3(nrm, v);
        for (auto& v : m.transformedNormals) push3(tnrm, v);
        std::vector<uint32_t> nodes_u;
        for (unsigned k = 0; k < m.nodesUsed && m.pBVHNodes; ++k) {
            const BVHNode& n = m.pBVHNodes[k];
            push3(nodes_f, n.minAABB); push3(nodes_f, n.maxAABB);
            nodes_u.push_back(n.firstIdx); nodes_u.push_back(n.idxCount); nodes_u.push_back(n.leftNode);
        }
        std::vector<int32_t> idx(m.indices.begin(), m.indices.end());
        w.f32(p + "positions", pos); w.f32(p + "tpositions", tpos);
        w.f32(p + "normals", nrm); w.f32(p + "tnormals", tnrm);
        w.i32(p + "indices", idx);
        w.f32(p + "node_bounds", nodes_f); w.u32(p + "node_links", nodes_u);
        ++mi;
    }
    w.u32("meshes", meshinfo);

    std::vector<float> lf; std::vector<int32_t> lt;
    for (auto& l : s->m_Lights) {
        push3(lf, l.origin); push3(lf, l.direction);
        lf.push_back(l.color.r); lf.push_back(l.color.g); lf.push_back(l.color.b);
        lf.push_back(l.intensity);
        lt.push_back(static_cast<int32_t>(l.type));
    }
    w.f32("lights", lf); w.i32("light_type", lt);

    // materials: kind + 8 floats {r,g,b,kd,ks,exp,metal,rough}
    std::vector<int32_t> mk; std::vector<float> mf;
    for (auto* pm : s->m_Materials) {
        float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int kind = -1;
        if (auto* a = dynamic_cast<Material_SolidColor*>(pm)) {
            kind = 0; v[0] = a->m_Color.r; v[1] = a->m_Color.g; v[2] = a->m_Color.b;
        } else if (auto* b = dynamic_cast<Material_Lambert*>(pm)) {
            kind = 1; v[0] = b->m_DiffuseColor.r; v[1] = b->m_DiffuseColor.g; v[2] = b->m_DiffuseColor.b;
            v[3] = b->m_DiffuseReflectance;
        } else if (auto* c = dynamic_cast<Material_LambertPhong*>(pm)) {
            kind = 2; v[0] = c->m_DiffuseColor.r; v[1] = c->m_DiffuseColor.g; v[2] = c->m_DiffuseColor.b;
            v[3] = c->m_DiffuseReflectance; v[4] = c->m_SpecularReflectance; v[5] = c->m_PhongExponent;
        } else if (auto* d = dynamic_cast<Material_CookTorrence*>(pm)) {
            kind = 3; v[0] = d->m_Albedo.r; v[1] = d->m_Albedo.g; v[2] = d->m_Albedo.b;
            v[6] = d->m_Metalness; v[7] = d->m_Roughness;
        }
        mk.push_back(kind);
        for (float x : v) mf.push_back(x);
    }
    w.i32("material_kind", mk); w.f32("material_params", mf);
}

// ----------------------------------------------------------------------------------
// Primitive known-answer vectors through the reference's own GeometryUtils,
// LightUtils and BRDF functions (source/Utils.h, source/BRDFs.h).
static void dump_prims(uint32_t seed, int n, const char* out) {
    std::mt19937 rng(seed);
    auto U = [&](float a, float b) { return a + (b - a) * (static_cast<float>(rng() >> 8) * (1.0f / 16777216.0f)); };
    auto rv = [&](float a, float b) { return Vector3{U(a, b), U(a, b), U(a, b)}; };
    Writer w(out);
    std::vector<float> rays;          // origin(3), dir(3), min, max
    std::vector<float> sph, pl, tri;  // sphere(4), plane(6), triangle v0 v1 v2 n (12)
    std::vector<int32_t> cull;
    std::vector<float> res_s, res_p, res_t;  // hit?, t, origin(3), normal(3)  (closest form)
    std::vector<uint8_t> any_s, any_p, any_t, slab;
    std::vector<float> aabb;
    for (int i = 0; i < n; ++i) {
        Vector3 o = rv(-3.f, 3.f);
        Vector3 d = rv(-1.f, 1.f);
        if (i % 17 == 0) d.y = 0.f;         // exercise inf inverse direction
        d.Normalize();
        float mx = (i % 3 == 0) ? U(0.5f, 8.f) : FLT_MAX;
        Ray ray{o, d, 0.0001f, mx};
        push3(rays, o); push3(rays, d); rays.push_back(ray.min); rays.push_back(ray.max);

        Sphere s; s.origin = rv(-3.f, 3.f); s.radius = U(0.2f, 2.5f); s.materialIndex = 7;
        push3(sph, s.origin); sph.push_back(s.radius);
        HitRecord h{};
        bool hit = GeometryUtils::HitTest_Sphere(s, ray, h);
        res_s.push_back(hit ? 1.f : 0.f); res_s.push_back(h.t); push3(res_s, h.origin); push3(res_s, h.normal);
        any_s.push_back(GeometryUtils::HitTest_Sphere(s, ray) ? 1 : 0);

        Plane p; p.origin = rv(-3.f, 3.f); p.normal = rv(-1.f, 1.f).Normalized(); p.materialIndex = 3;
        if (i % 13 == 0) p.normal = Vector3{0.f, 1.f, 0.f};
        push3(pl, p.origin); push3(pl, p.normal);
        HitRecord hp{};
        hit = GeometryUtils::HitTest_Plane(p, ray, hp);
        res_p.push_back(hit ? 1.f : 0.f); res_p.push_back(hp.t); push3(res_p, hp.origin); push3(res_p, hp.normal);
        any_p.push_back(GeometryUtils::HitTest_Plane(p, ray) ? 1 : 0);

        // aim the triangle roughly at the ray so that a good fraction hit
        Vector3 c = o + d * U(0.5f, 5.f);
        Triangle t{c + rv(-1.f, 1.f), c + rv(-1.f, 1.f), c + rv(-1.f, 1.f)};
        t.cullMode = static_cast<TriangleCullMode>(i % 3);
        t.materialIndex = 5;
        push3(tri, t.v0); push3(tri, t.v1); push3(tri, t.v2); push3(tri, t.normal);
        cull.push_back(i % 3);
        HitRecord ht{};
        hit = GeometryUtils::HitTest_Triangle(t, ray, ht);
        res_t.push_back(hit ? 1.f : 0.f); res_t.push_back(ht.t); push3(res_t, ht.origin); push3(res_t, ht.normal);
        any_t.push_back(GeometryUtils::HitTest_Triangle(t, ray) ? 1 : 0);

        Vector3 bmin = c - Vector3{U(0.f, 1.f), U(0.f, 1.f), U(0.f, 1.f)};
        Vector3 bmax = c + Vector3{U(0.f, 1.f), U(0.f, 1.f), U(0.f, 1.f)};
        if (i % 11 == 0) { bmin.y = o.y; }  // (min - o) * inf = NaN path
        push3(aabb, bmin); push3(aabb, bmax);
        slab.push_back(GeometryUtils::SlabTest_BVH(bmin, bmax, ray) ? 1 : 0);
    }
    w.f32("rays", rays); w.f32("spheres", sph); w.f32("planes", pl); w.f32("triangles", tri);
    w.i32("tri_cull", cull);
    w.f32("sphere_hit", res_s); w.f32("plane_hit", res_p); w.f32("tri_hit", res_t);
    w.u8("sphere_any", any_s); w.u8("plane_any", any_p); w.u8("tri_any", any_t);
    w.f32("aabbs", aabb); w.u8("slab", slab);

    // BRDF / material shading vectors: n, l, v unit vectors + params -> Shade() results
    std::vector<float> shade_in, shade_out;
    std::vector<int32_t> shade_kind;
    for (int i = 0; i < n; ++i) {
        Vector3 nn = rv(-1.f, 1.f).Normalized();
        Vector3 l = rv(-1.f, 1.f).Normalized();
        Vector3 v = rv(-1.f, 1.f).Normalized();
        HitRecord hr{}; hr.normal = nn;
        ColorRGB col{U(0.f, 1.f), U(0.f, 1.f), U(0.f, 1.f)};
        const int kind = i % 4;
        float kd = U(0.f, 1.f), ks = U(0.f, 1.f), ex = U(1.f, 60.f), metal = (i % 8 < 4) ? 0.f : 1.f, rough = U(0.05f, 1.f);
        std::unique_ptr<Material> m;
        if (kind == 0) m.reset(new Material_SolidColor(col));
        else if (kind == 1) m.reset(new Material_Lambert(col, kd));
        else if (kind == 2) m.reset(new Material_LambertPhong(col, kd, ks, ex));
        else m.reset(new Material_CookTorrence(col, metal, rough));
        ColorRGB r = m->Shade(hr, l, v);
        shade_kind.push_back(kind);
        push3(shade_in, nn); push3(shade_in, l); push3(shade_in, v);
        shade_in.push_back(col.r); shade_in.push_back(col.g); shade_in.push_back(col.b);
        shade_in.push_back(kd); shade_in.push_back(ks); shade_in.push_back(ex);
        shade_in.push_back(metal); shade_in.push_back(rough);
        shade_out.push_back(r.r); shade_out.push_back(r.g); shade_out.push_back(r.b);
    }
    w.i32("shade_kind", shade_kind); w.f32("shade_in", shade_in); w.f32("shade_out", shade_out);
}

static void dump_obj(const char* path, const char* out) {
    std::vector<Vector3> positions, normals;
    std::vector<int> indices;
    const bool ok = Utils::ParseOBJ(path, positions, normals, indices);
    Writer w(out);
    std::vector<float> p, n;
    for (auto& v : positions) push3(p, v);
    for (auto& v : normals) push3(n, v);
    w.f32("positions", p); w.f32("normals", n);
    w.i32("indices", std::vector<int32_t>(indices.begin(), indices.end()));
    w.u8("ok", std::vector<uint8_t>{static_cast<uint8_t>(ok ? 1 : 0)});
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness scene|render|bench|obj|prims ...\n"); return 2; }
    const std::string cmd = argv[1];
    if (cmd == "scene" && argc == 5) {
        auto s = make_scene(argv[2]);
        apply_time(s.get(), argv[2], argv[3]);
        dump_scene(s.get(), argv[4]);
        return 0;
    }
    if (cmd == "render" && argc == 10) {
        auto s = make_scene(argv[2]);
        apply_time(s.get(), argv[2], argv[3]);
        const int W = std::atoi(argv[4]), H = std::atoi(argv[5]);
        RenderState rs = make_state(W, H, std::atoi(argv[6]), std::atoi(argv[7]) != 0);
        std::vector<uint32_t> px(static_cast<size_t>(W) * H);
        std::vector<float> rgb(static_cast<size_t>(W) * H * 3);
        render(s.get(), rs, std::atoi(argv[8]), px.data(), rgb.data());
        Writer w(argv[9]);
        w.u32("pixels", px); w.f32("rgb", rgb);
        w.u32("size", std::vector<uint32_t>{static_cast<uint32_t>(W), static_cast<uint32_t>(H)});
        return 0;
    }
    if (cmd == "bench" && (argc == 8 || argc == 10)) {
        auto s = make_scene(argv[2]);
        apply_time(s.get(), argv[2], argv[3]);
        const int W = std::atoi(argv[4]), H = std::atoi(argv[5]);
        const int threads = std::atoi(argv[6]), frames = std::atoi(argv[7]);
        const int mode = argc == 10 ? std::atoi(argv[8]) : 3;
        const bool sh = argc == 10 ? std::atoi(argv[9]) != 0 : true;
        RenderState rs = make_state(W, H, mode, sh);
        std::vector<uint32_t> px(static_cast<size_t>(W) * H);
        render(s.get(), rs, threads, px.data(), nullptr);  // warm-up
        std::vector<double> ts;
        for (int f = 0; f < frames; ++f) {
            auto t0 = std::chrono::steady_clock::now();
            render(s.get(), rs, threads, px.data(), nullptr);
            auto t1 = std::chrono::steady_clock::now();
            ts.push_back(std::chrono::duration<double>(t1 - t0).count());
        }
        std::vector<double> sorted = ts;
        std::sort(sorted.begin(), sorted.end());
        const double med = sorted[sorted.size() / 2];
        uint64_t h = 1469598103934665603ull;  // FNV-1a over the pixel bytes
        const uint8_t* b = reinterpret_cast<const uint8_t*>(px.data());
        for (size_t i = 0; i < px.size() * 4; ++i) { h ^= b[i]; h *= 1099511628211ull; }
        std::printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"threads\": %d, \"frames\": %d, "
                    "\"median_s\": %.6f, \"min_s\": %.6f, \"mpix_s\": %.4f, \"fnv\": \"%016llx\"}\n",
                    argv[2], W, H, threads, frames, med, sorted.front(), W * (double)H / med / 1e6,
                    (unsigned long long)h);
        return 0;
    }
    if (cmd == "obj" && argc == 4) { dump_obj(argv[2], argv[3]); return 0; }
    if (cmd == "prims" && argc == 5) { dump_prims(static_cast<uint32_t>(std::atoi(argv[2])), std::atoi(argv[3]), argv[4]); return 0; }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
