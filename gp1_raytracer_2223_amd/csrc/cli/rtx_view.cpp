// rtx_view — the reference's window loop (source/main.cpp) on the HIP render path: poll events,
// Scene::Update, Renderer::Render into the window surface, present, the dFPS print, the screenshot
// and the F6 benchmark.  SDL2 is loaded at run time (dlopen of libSDL2-2.0.so.0): nothing links
// against it, so the program builds and runs where SDL2 is absent — it then says so and exits 0.
//
//   rtx_view [scene] [width height] [--assets dir] [--out file.bmp] [--keys K1,K2,...] [--frames N]
//
// The key handling is rtx_view_on_event (include/rtx_view.h, librtx_host.so): F2 shadows, F3 lighting
// mode, X screenshot of the next frame, F6 benchmark, acted on at key release like main.cpp:63-86.
// --keys runs the same loop headless (no SDL, no window): one scripted event per frame (X, F2, F3, F6,
// QUIT, or "-" for none), then frames until --frames (default: the events + 1), every frame rendered
// and its state printed — the loop's testable form.
//
// SDL2 ABI (2.0.x, 64-bit; declared here, no SDL header): the calls below, SDL_Surface {flags, format,
// w, h, pitch, pixels, ...}, SDL_PixelFormat {format, palette, BitsPerPixel, BytesPerPixel, pad[2],
// R/G/B/Amask, R/G/B/Aloss, R/G/B/Ashift, ...}, SDL_Event = 56 bytes with the type at 0 and, for a key
// event, the keysym's scancode at 16.
#include <dlfcn.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "benchmark.h"
#include "rtx.h"
#include "rtx_host.h"
#include "rtx_view.h"

namespace {

struct SdlPixelFormat {
    uint32_t format;
    void* palette;
    uint8_t bits, bytes, pad[2];
    uint32_t rmask, gmask, bmask, amask;
    uint8_t rloss, gloss, bloss, aloss;
    uint8_t rshift, gshift, bshift, ashift;
};
struct SdlSurface {
    uint32_t flags;
    SdlPixelFormat* format;
    int w, h, pitch;
    void* pixels;
};
struct SdlEvent {
    uint32_t type;
    uint8_t rest[52];
};
static_assert(sizeof(SdlEvent) == 56, "SDL_Event is 56 bytes");

constexpr uint32_t kSdlInitVideo = 0x20;
constexpr int kSdlWindowPosUndefined = 0x1FFF0000;

// the SDL2 entry points the loop calls, resolved with dlsym
struct Sdl {
    void* h = nullptr;
    int (*Init)(uint32_t) = nullptr;
    void (*Quit)() = nullptr;
    const char* (*GetError)() = nullptr;
    void* (*CreateWindow)(const char*, int, int, int, int, uint32_t) = nullptr;
    void (*DestroyWindow)(void*) = nullptr;
    SdlSurface* (*GetWindowSurface)(void*) = nullptr;
    int (*UpdateWindowSurface)(void*) = nullptr;
    int (*PollEvent)(SdlEvent*) = nullptr;
    int (*LockSurface)(SdlSurface*) = nullptr;
    void (*UnlockSurface)(SdlSurface*) = nullptr;

    bool Load(std::string& why) {
        for (const char* name : {"libSDL2-2.0.so.0", "libSDL2.so"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            why = "libSDL2-2.0.so.0 not found";
            return false;
        }
        bool ok = true;
        auto get = [&](auto& fn, const char* sym) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, sym));
            ok = ok && fn != nullptr;
        };
        get(Init, "SDL_Init");
        get(Quit, "SDL_Quit");
        get(GetError, "SDL_GetError");
        get(CreateWindow, "SDL_CreateWindow");
        get(DestroyWindow, "SDL_DestroyWindow");
        get(GetWindowSurface, "SDL_GetWindowSurface");
        get(UpdateWindowSurface, "SDL_UpdateWindowSurface");
        get(PollEvent, "SDL_PollEvent");
        get(LockSurface, "SDL_LockSurface");
        get(UnlockSurface, "SDL_UnlockSurface");
        if (!ok) why = "libSDL2 lacks an SDL2 entry point";
        return ok;
    }
    ~Sdl() {
        if (h) dlclose(h);
    }
};

// Timer (source/Timer.cpp): elapsed / total time, the always-running dFPS window and the benchmark
// capture that StartBenchmark arms (Timer.cpp:44-131)
struct Timer {
    using Clock = std::chrono::steady_clock;
    Clock::time_point base = Clock::now(), prev = base;
    float elapsed = 0.f, total = 0.f, fps_timer = 0.f, dfps = 0.f;
    int fps_count = 0;
    bool bench_active = false;
    rtx::Benchmark bench{10};
    void StartBenchmark(int frames = 10) {
        if (bench_active) {
            std::cout << "(Benchmark already running)";
            return;
        }
        bench_active = true;
        bench = rtx::Benchmark(frames);
        std::cout << "**BENCHMARK STARTED**\n";
    }
    void Update() {
        const Clock::time_point now = Clock::now();
        elapsed = std::max(0.f, std::chrono::duration<float>(now - prev).count());
        prev = now;
        total = std::chrono::duration<float>(now - base).count();
        fps_timer += elapsed;
        ++fps_count;
        if (fps_timer >= 1.0f) {
            dfps = fps_count / fps_timer;
            fps_count = 0;
            fps_timer = 0.f;
            if (bench_active) {   // the benchmark records the closed window's dFPS
                if (bench.Record(dfps)) {
                    bench_active = false;
                    rtx::WriteBenchmark(bench);
                }
            }
        }
    }
};

int usage(const char* argv0) {
    std::fprintf(stderr, "usage: %s [scene] [width height] [--assets dir] [--out file.bmp] [--keys X,F2,F3,F6,QUIT,-]"
                         " [--frames N]\n", argv0);
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    std::string scene = "W4_Reference", assets, out = "RayTracing_Buffer.bmp";   // main.cpp:44
    int W = 640, H = 480;                                                         // main.cpp:31-32
    std::vector<std::string> keys;
    bool headless = false;
    long frames = -1;
    int pos = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--assets" && i + 1 < argc) assets = argv[++i];
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else if (a == "--frames" && i + 1 < argc) frames = std::atol(argv[++i]);
        else if (a == "--keys" && i + 1 < argc) {
            headless = true;
            for (std::string k, all = argv[++i]; !all.empty();) {
                const size_t c = all.find(',');
                k = all.substr(0, c);
                keys.push_back(k);
                all = c == std::string::npos ? "" : all.substr(c + 1);
            }
        } else if (a.rfind("--", 0) == 0) return usage(argv[0]);
        else if (pos == 0 && !std::isdigit(static_cast<unsigned char>(a[0]))) { scene = a; }
        else if (pos == 0) { W = std::atoi(a.c_str()); ++pos; }
        else if (pos == 1) { H = std::atoi(a.c_str()); ++pos; }
    }
    if (W <= 0 || H <= 0) return usage(argv[0]);
    if (frames < 0) frames = static_cast<long>(keys.size()) + 1;

    // the presentation: SDL2 if present (nothing is linked against it), else nothing to show on
    Sdl sdl;
    void* window = nullptr;
    if (!headless) {
        std::string why;
        if (!sdl.Load(why)) {
            std::printf("rtx_view: %s: no window to present to (rtx_render renders headless, --keys runs this "
                        "loop without a window)\n", why.c_str());
            return 0;
        }
        if (sdl.Init(kSdlInitVideo) != 0) {
            std::printf("rtx_view: SDL_Init: %s\n", sdl.GetError());
            return 0;
        }
        window = sdl.CreateWindow("RayTracer - rtx_view (MI355X)", kSdlWindowPosUndefined, kSdlWindowPosUndefined, W,
                                  H, 0);
        if (!window) {
            std::printf("rtx_view: SDL_CreateWindow: %s\n", sdl.GetError());
            sdl.Quit();
            return 0;
        }
    }

    char err[512] = {0};
    rtx_host_scene* hs = nullptr;
    if (rtx_host_scene_create(scene.c_str(), assets.empty() ? nullptr : assets.c_str(), &hs, err, sizeof err) != RTX_OK) {
        std::fprintf(stderr, "scene %s: %s\n", scene.c_str(), err);
        if (window) { sdl.DestroyWindow(window); sdl.Quit(); }
        return 1;
    }
    rtx_ctx* ctx = nullptr;
    if (rtx_create(&ctx, 0) != RTX_OK) {
        std::fprintf(stderr, "rtx_create: %s\n", rtx_last_error(nullptr));
        rtx_host_scene_destroy(hs);
        if (window) { sdl.DestroyWindow(window); sdl.Quit(); }
        return 1;
    }
    const bool animated = rtx_host_scene_animated(hs) == 1;
    std::vector<uint32_t> px(static_cast<size_t>(W) * H);
    rtx_view_state st;
    rtx_view_init(&st);
    Timer timer;
    float print_timer = 0.f;
    int rc = 0;
    bool uploaded = false;
    for (long frame = 0; st.looping; ++frame) {
        // --------- input events (main.cpp:59-86)
        if (headless) {
            if (frame >= frames) break;
            if (frame < static_cast<long>(keys.size())) {
                const std::string& k = keys[frame];
                const int32_t code = k == "X" ? RTX_KEY_X : k == "F2" ? RTX_KEY_F2 : k == "F3" ? RTX_KEY_F3
                                   : k == "F6" ? RTX_KEY_F6 : -1;
                if (k == "QUIT") rtx_view_on_event(&st, RTX_EV_QUIT, 0);
                else if (code >= 0) rtx_view_on_event(&st, RTX_EV_KEYUP, code);
                if (!st.looping) break;
            }
        } else {
            SdlEvent e;
            while (sdl.PollEvent(&e)) {
                int32_t scancode = 0;
                std::memcpy(&scancode, e.rest + 12, 4);   // SDL_KeyboardEvent.keysym.scancode (offset 16)
                rtx_view_on_event(&st, e.type, scancode);
            }
            if (!st.looping) break;
        }
        if (st.start_benchmark) {
            st.start_benchmark = 0;
            timer.StartBenchmark();
        }
        // --------- Update (main.cpp:89): the W4 scenes turn their meshes and rebuild the BVH
        if (animated) rtx_host_scene_update(hs, timer.total);
        rtx_scene s;
        rtx_camera cam;
        rtx_host_scene_view(hs, &s, &cam);
        if ((animated || !uploaded) && rtx_upload_scene(ctx, &s) != RTX_OK) {
            std::fprintf(stderr, "rtx_upload_scene: %s\n", rtx_last_error(ctx));
            rc = 1;
            break;
        }
        uploaded = true;
        // --------- Render (main.cpp:92): straight into the window surface, in its pixel format
        SdlSurface* surf = window ? sdl.GetWindowSurface(window) : nullptr;
        rtx_pixel_format fmt{16, 8, 0, 0};
        if (surf) {
            if (!surf->format || surf->format->bytes != 4) {
                std::fprintf(stderr, "rtx_view: the window surface is not 32-bit\n");
                rc = 1;
                break;
            }
            fmt = {surf->format->rshift, surf->format->gshift, surf->format->bshift, surf->format->amask};
        }
        rtx_render_params p;
        rtx_view_params(&st, static_cast<uint32_t>(W), static_cast<uint32_t>(H), &fmt, &p);
        if (rtx_render(ctx, &cam, &p, px.data(), nullptr) != RTX_OK) {
            std::fprintf(stderr, "rtx_render: %s\n", rtx_last_error(ctx));
            rc = 1;
            break;
        }
        if (surf) {
            sdl.LockSurface(surf);
            for (int y = 0; y < H && y < surf->h; ++y)
                std::memcpy(static_cast<char*>(surf->pixels) + static_cast<size_t>(y) * surf->pitch,
                            px.data() + static_cast<size_t>(y) * W, 4 * static_cast<size_t>(std::min(W, surf->w)));
            sdl.UnlockSurface(surf);
            sdl.UpdateWindowSurface(window);   // Renderer.cpp:97
        }
        if (headless)
            std::printf("frame %ld: mode %d shadows %d\n", frame, st.lighting_mode, st.shadows_enabled);
        // --------- Timer (main.cpp:95-100)
        timer.Update();
        print_timer += timer.elapsed;
        if (print_timer >= 1.f) {
            print_timer = 0.f;
            std::cout << "dFPS: " << timer.dfps << std::endl;
        }
        // --------- screenshot after the full render (main.cpp:101-107)
        if (st.take_screenshot) {
            if (!rtx_view_save_bmp(out.c_str(), px.data(), static_cast<uint32_t>(W), static_cast<uint32_t>(H)))
                std::cout << "Screenshot saved!" << std::endl;
            else
                std::cout << "Something went wrong. Screenshot not saved!" << std::endl;
            st.take_screenshot = 0;
        }
    }
    rtx_destroy(ctx);
    rtx_host_scene_destroy(hs);
    if (window) {
        sdl.DestroyWindow(window);   // ShutDown (main.cpp:17-21)
        sdl.Quit();
    }
    return rc;
}
