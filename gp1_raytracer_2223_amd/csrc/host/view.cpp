// view.cpp — the reference frame loop's event switch and screenshot (include/rtx_view.h), pure host
// code shared by the SDL viewer (csrc/cli/rtx_view.cpp) and the tests.
#include <cstdio>
#include <cstring>

#include "rtx_view.h"

extern "C" void rtx_view_init(rtx_view_state* s) {
    if (!s) return;
    std::memset(s, 0, sizeof *s);
    s->lighting_mode = RTX_MODE_COMBINED;   // m_CurrentLightingMode{ LightingMode::Combined } (Renderer.h:49)
    s->shadows_enabled = 1;                 // m_ShadowsEnabled{ true } (Renderer.h:50)
    s->looping = 1;                         // isLooping (main.cpp:56)
}

// main.cpp:63-86: SDL_QUIT ends the loop; on SDL_KEYUP, X requests a screenshot of the next frame,
// F2 toggles shadows, F3 cycles the lighting mode, F6 starts the benchmark.  Key presses
// (SDL_KEYDOWN) and every other key do nothing.
extern "C" int rtx_view_on_event(rtx_view_state* s, uint32_t type, int32_t scancode) {
    if (!s) return 0;
    if (type == RTX_EV_QUIT) {
        const int changed = s->looping != 0;
        s->looping = 0;
        return changed;
    }
    if (type != RTX_EV_KEYUP) return 0;
    switch (scancode) {
    case RTX_KEY_X: s->take_screenshot = 1; return 1;
    case RTX_KEY_F2: s->shadows_enabled = !s->shadows_enabled; return 1;   // Renderer::ToggleShadows
    case RTX_KEY_F3:                                                       // Renderer::CycleLightingMode
        s->lighting_mode = (s->lighting_mode + 1) % RTX_MODE_COUNT;
        return 1;
    case RTX_KEY_F6: s->start_benchmark = 1; return 1;                     // Timer::StartBenchmark
    default: return 0;
    }
}

extern "C" void rtx_view_params(const rtx_view_state* s, uint32_t width, uint32_t height, const rtx_pixel_format* fmt,
                                rtx_render_params* out) {
    if (!s || !out) return;
    std::memset(out, 0, sizeof *out);
    out->width = width;
    out->height = height;
    out->lighting_mode = s->lighting_mode;
    out->shadows_enabled = s->shadows_enabled ? 1 : 0;
    if (fmt) out->format = *fmt;
    else out->format = rtx_pixel_format{16, 8, 0, 0};   // XRGB8888
    out->stripe_step = 1;
}

extern "C" int rtx_view_save_bmp(const char* path, const uint32_t* px, uint32_t w, uint32_t h) {
    if (!path || !px || w == 0 || h == 0 || w > 65536 || h > 65536) return -1;
    FILE* f = std::fopen(path, "wb");
    if (!f) return -1;
    const uint32_t data = w * h * 4u;
    unsigned char hdr[54] = {'B', 'M'};
    auto put32 = [&](int off, uint32_t v) {
        for (int k = 0; k < 4; ++k) hdr[off + k] = static_cast<unsigned char>(v >> (8 * k));
    };
    put32(2, 54u + data);   // bfSize
    put32(10, 54u);         // bfOffBits
    put32(14, 40u);         // biSize
    put32(18, w);           // biWidth
    put32(22, h);           // biHeight (> 0: bottom-up)
    put32(26, 1u | (32u << 16));   // biPlanes = 1, biBitCount = 32
    put32(30, 0u);          // BI_RGB
    put32(34, data);        // biSizeImage
    put32(38, 2835u);       // 72 dpi
    put32(42, 2835u);
    bool ok = std::fwrite(hdr, 1, sizeof hdr, f) == sizeof hdr;
    for (uint32_t y = h; ok && y-- > 0;)   // little-endian 32-bit words: B, G, R, X bytes
        ok = std::fwrite(px + static_cast<size_t>(y) * w, 4, w, f) == w;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? 0 : -1;
}
