// rtx_render — headless C++ host program (the reference's main.cpp frame loop without
// the SDL window): builds a catalogue scene with librtx_host.so, renders it through the
// C-ABI of librtx_hip.so and writes RayTracing_Buffer.bmp like the reference's X key.
//
//   rtx_render <scene> [width height] [--time T] [--mode 0..3] [--no-shadows]
//              [--frames N] [--out file.bmp] [--assets dir]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "rtx_renderer.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene> [width height] [--time T] [--mode M] [--no-shadows] [--frames N] "
                             "[--out f.bmp] [--assets dir]\n", argv[0]);
        return 2;
    }
    std::string scene = argv[1], out = "RayTracing_Buffer.bmp", assets;
    int W = 640, H = 480, mode = 3, frames = 1;
    float t = -1.f;
    bool shadows = true;
    int pos = 0;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--time" && i + 1 < argc) t = std::strtof(argv[++i], nullptr);
        else if (a == "--mode" && i + 1 < argc) mode = std::atoi(argv[++i]);
        else if (a == "--no-shadows") shadows = false;
        else if (a == "--frames" && i + 1 < argc) frames = std::atoi(argv[++i]);
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else if (a == "--assets" && i + 1 < argc) assets = argv[++i];
        else if (pos == 0) { W = std::atoi(argv[i]); ++pos; }
        else if (pos == 1) { H = std::atoi(argv[i]); ++pos; }
    }
    char err[512] = {0};
    rtx_host_scene* hs = nullptr;
    if (rtx_host_scene_create(scene.c_str(), assets.empty() ? nullptr : assets.c_str(), &hs, err, sizeof err) != RTX_OK) {
        std::fprintf(stderr, "scene %s: %s\n", scene.c_str(), err);
        return 1;
    }
    if (t >= 0.f) rtx_host_scene_update(hs, t);
    try {
        rtx::Renderer r(W, H);
        r.m_CurrentLightingMode = static_cast<rtx::Renderer::LightingMode>(mode);
        r.m_ShadowsEnabled = shadows;
        r.Render(hs, true);
        auto t0 = std::chrono::steady_clock::now();
        for (int f = 1; f < frames; ++f) r.Render(hs, false);
        auto t1 = std::chrono::steady_clock::now();
        if (frames > 1) {
            const double s = std::chrono::duration<double>(t1 - t0).count() / (frames - 1);
            std::printf("%s %dx%d: %.3f ms/frame incl. D2H, %.1f Mpix/s\n", scene.c_str(), W, H, s * 1e3,
                        W * (double)H / s / 1e6);
        }
        if (!r.SaveBufferToImage(out)) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); return 1; }
        std::printf("wrote %s\n", out.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        rtx_host_scene_destroy(hs);
        return 1;
    }
    rtx_host_scene_destroy(hs);
    return 0;
}
