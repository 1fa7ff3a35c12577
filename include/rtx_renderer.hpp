// rtx_renderer.hpp — header-only C++ mirror of dae::Renderer (source/Renderer.h:17-61) on
// top of the C-ABI (rtx.h + rtx_host.h).  Same member names and state as the reference:
//
//   rtx::Renderer r(width, height);          // Renderer(SDL_Window*) — size of the surface
//   r.Render(scene);                         // Renderer::Render(Scene*) — fills r.Pixels()
//   r.CycleLightingMode(); r.ToggleShadows(); r.SaveBufferToImage("RayTracing_Buffer.bmp");
//
// `scene` is an rtx_host_scene (the C++ scene catalogue of librtx_host.so) or any
// caller-built rtx_scene + rtx_camera.  Errors throw std::runtime_error (the C-ABI below
// never throws).
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtx.h"
#include "rtx_host.h"

namespace rtx {

class Renderer {
public:
    enum class LightingMode { ObservedArea, Radiance, BRDF, Combined, Count };   // Renderer.h:40-48

    Renderer(int width, int height, int device = 0) : m_Width(width), m_Height(height) {
        if (rtx_create(&m_Ctx, device) != RTX_OK) throw std::runtime_error("rtx_create failed (no HIP device?)");
        m_Pixels.resize(static_cast<size_t>(width) * height);
    }
    ~Renderer() { rtx_destroy(m_Ctx); }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    // Upload only when the scene changed (after Initialize / Update), like the reference
    // which reads the Scene in place every frame.
    void Upload(const rtx_scene& scene) { Check(rtx_upload_scene(m_Ctx, &scene), "rtx_upload_scene"); }

    void Render(const rtx_camera& cam) {
        const rtx_render_params p = Params();
        Check(rtx_render(m_Ctx, &cam, &p, m_Pixels.data(), nullptr), "rtx_render");
    }

    void Render(rtx_host_scene* scene, bool upload = true) {
        rtx_scene s;
        rtx_camera cam;
        Check(rtx_host_scene_view(scene, &s, &cam), "rtx_host_scene_view");
        if (upload) Upload(s);
        Render(cam);
    }

    void CycleLightingMode() {                                                     // Renderer.cpp:189-193
        m_CurrentLightingMode = static_cast<LightingMode>((static_cast<int>(m_CurrentLightingMode) + 1) %
                                                          static_cast<int>(LightingMode::Count));
    }
    void ToggleShadows() { m_ShadowsEnabled = !m_ShadowsEnabled; }                // Renderer.h:34-36

    // SDL_SaveBMP of the XRGB8888 surface (Renderer.cpp:184-187): 32-bit BI_RGB, bottom-up.
    bool SaveBufferToImage(const std::string& path = "RayTracing_Buffer.bmp") const {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) return false;
        const uint32_t data = static_cast<uint32_t>(m_Pixels.size() * 4);
        const uint32_t hdr[13] = {0, 0, 54, 40, static_cast<uint32_t>(m_Width), static_cast<uint32_t>(m_Height),
                                  (32u << 16) | 1u, 0, data, 2835, 2835, 0, 0};
        const uint16_t bm = 0x4D42;
        const uint32_t size = 54 + data;
        bool ok = std::fwrite(&bm, 2, 1, f) == 1 && std::fwrite(&size, 4, 1, f) == 1 &&
                  std::fwrite(hdr + 1, 4, 12, f) == 12;
        for (int y = m_Height - 1; ok && y >= 0; --y)
            ok = std::fwrite(&m_Pixels[static_cast<size_t>(y) * m_Width], 4, m_Width, f) == static_cast<size_t>(m_Width);
        std::fclose(f);
        return ok;
    }

    const std::vector<uint32_t>& Pixels() const { return m_Pixels; }
    std::vector<uint32_t>& Pixels() { return m_Pixels; }
    int Width() const { return m_Width; }
    int Height() const { return m_Height; }
    rtx_ctx* Context() const { return m_Ctx; }
    LightingMode m_CurrentLightingMode{LightingMode::Combined};
    bool m_ShadowsEnabled{true};

    // The render parameters of the current state (Renderer::Render reads the same members).
    rtx_render_params Params() const {
        rtx_render_params p{};
        p.width = static_cast<uint32_t>(m_Width);
        p.height = static_cast<uint32_t>(m_Height);
        p.lighting_mode = static_cast<int32_t>(m_CurrentLightingMode);
        p.shadows_enabled = m_ShadowsEnabled ? 1 : 0;
        p.format = {16, 8, 0, 0};   // XRGB8888 window surface
        p.stripe_step = 1;
        return p;
    }
private:
    void Check(int rc, const char* what) const {
        if (rc != RTX_OK) throw std::runtime_error(std::string(what) + ": " + rtx_last_error(m_Ctx));
    }

    rtx_ctx* m_Ctx{};
    int m_Width, m_Height;
    std::vector<uint32_t> m_Pixels;
};

}  // namespace rtx
