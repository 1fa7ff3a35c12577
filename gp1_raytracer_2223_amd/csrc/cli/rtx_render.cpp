// rtx_render — headless C++ host program (the reference's main.cpp frame loop without
// the SDL window): builds a catalogue scene with librtx_host.so, renders it through the
// C-ABI of librtx_hip.so and writes RayTracing_Buffer.bmp like the reference's X key.
//
//   rtx_render <scene> [width height] [--time T] [--mode 0..3] [--no-shadows]
//              [--frames N] [--out file.bmp] [--assets dir] [--benchmark [windows]]
//
// --benchmark runs the reference's frame loop (main.cpp:86-100: Scene::Update with the
// timer's total time, Render into the host pixel buffer, Timer::Update) under its F6
// benchmark (Timer.cpp:44-131): `windows` one-second dFPS windows (default 10), then
// ">> HIGH/LOW/AVG" on stdout and benchmark.txt in the reference's format.  Animated
// scenes are re-uploaded after every Update; the per-stage means are printed as well.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <numeric>
#include <string>
#include <vector>

#include "rtx_renderer.hpp"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// Timer::StartBenchmark / Update FPS logic (Timer.cpp:44-131), same float arithmetic.
struct Benchmark {
    int frames;
    std::vector<float> dfps;
    float high = FLT_MIN, low = FLT_MAX, avg = 0.f;   // m_BenchmarkHigh = FLT_MIN as in the reference
    float fps_timer = 0.f;
    int fps_count = 0;
    explicit Benchmark(int n) : frames(n) {}
    bool Tick(float elapsed) {   // returns true when the last window closed
        fps_timer += elapsed;
        ++fps_count;
        if (fps_timer >= 1.0f) {
            const float d = fps_count / fps_timer;
            fps_count = 0;
            fps_timer = 0.f;
            dfps.push_back(d);
            low = std::min(low, d);
            high = std::max(high, d);
            if (static_cast<int>(dfps.size()) >= frames) {
                avg = std::accumulate(dfps.begin(), dfps.end(), 0.f) / float(frames);
                return true;
            }
        }
        return false;
    }
};

int run_benchmark(rtx::Renderer& r, rtx_host_scene* hs, int windows) {
    const bool animated = rtx_host_scene_animated(hs) == 1;
    Benchmark b(windows);
    std::cout << "**BENCHMARK STARTED**\n";
    double t_update = 0, t_upload = 0, t_render = 0;
    long frames = 0;
    const Clock::time_point start = Clock::now();
    Clock::time_point prev = start;
    rtx_scene s;
    rtx_camera cam;
    for (;;) {
        const Clock::time_point f0 = Clock::now();
        if (animated) rtx_host_scene_update(hs, static_cast<float>(secs(start, f0)));   // Scene::Update(pTimer)
        const Clock::time_point f1 = Clock::now();
        if (rtx_host_scene_view(hs, &s, &cam) != RTX_OK) return 1;
        if (animated || frames == 0) r.Upload(s);
        const Clock::time_point f2 = Clock::now();
        r.Render(cam);                                                                  // Renderer::Render
        const Clock::time_point f3 = Clock::now();
        t_update += secs(f0, f1);
        t_upload += secs(f1, f2);
        t_render += secs(f2, f3);
        ++frames;
        const float elapsed = static_cast<float>(secs(prev, f3));                      // Timer::Update
        prev = f3;
        if (b.Tick(elapsed)) break;
    }
    std::cout << "**BENCHMARK FINISHED**\n";
    std::cout << ">> HIGH = " << b.high << std::endl;
    std::cout << ">> LOW = " << b.low << std::endl;
    std::cout << ">> AVG = " << b.avg << std::endl;
    std::ofstream f("benchmark.txt");
    f << "FRAMES = " << b.dfps.size() << std::endl;
    f << "HIGH = " << b.high << std::endl;
    f << "LOW = " << b.low << std::endl;
    f << "AVG = " << b.avg << std::endl;
    std::printf("frames %ld%s: update %.3f ms, upload %.3f ms, render+D2H %.3f ms per frame\n", frames,
                animated ? " (animated)" : "", t_update / frames * 1e3, t_upload / frames * 1e3,
                t_render / frames * 1e3);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene> [width height] [--time T] [--mode M] [--no-shadows] [--frames N] "
                             "[--out f.bmp] [--assets dir] [--benchmark [windows]]\n", argv[0]);
        return 2;
    }
    std::string scene = argv[1], out = "RayTracing_Buffer.bmp", assets;
    int W = 640, H = 480, mode = 3, frames = 1, bench = 0;
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
        else if (a == "--benchmark") bench = (i + 1 < argc && std::atoi(argv[i + 1]) > 0) ? std::atoi(argv[++i]) : 10;
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
    int rc = 0;
    try {
        rtx::Renderer r(W, H);
        r.m_CurrentLightingMode = static_cast<rtx::Renderer::LightingMode>(mode);
        r.m_ShadowsEnabled = shadows;
        if (bench) {
            rc = run_benchmark(r, hs, bench);
        } else {
            r.Render(hs, true);
            auto t0 = Clock::now();
            for (int f = 1; f < frames; ++f) r.Render(hs, false);
            auto t1 = Clock::now();
            if (frames > 1) {
                const double s = secs(t0, t1) / (frames - 1);
                std::printf("%s %dx%d: %.3f ms/frame incl. D2H, %.1f Mpix/s\n", scene.c_str(), W, H, s * 1e3,
                            W * (double)H / s / 1e6);
            }
        }
        if (rc == 0 && !r.SaveBufferToImage(out)) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); rc = 1; }
        else if (rc == 0) std::printf("wrote %s\n", out.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        rc = 1;
    }
    rtx_host_scene_destroy(hs);
    return rc;
}
