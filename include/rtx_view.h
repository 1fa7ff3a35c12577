/*
 * rtx_view.h — the presentation side of the reference's frame loop (librtx_host.so, pure host
 * code: loads and runs without a GPU or SDL).
 *
 * The reference's main loop (source/main.cpp:57-113) polls SDL events, acts on key RELEASES only
 * (SDL_KEYUP) and keeps four bits of state: F2 toggles shadows (Renderer::ToggleShadows,
 * Renderer.h:34-36), F3 cycles the lighting mode in Renderer.h:40-48 order
 * (Renderer::CycleLightingMode, Renderer.cpp:189-193), X saves the next rendered frame as
 * RayTracing_Buffer.bmp (Renderer::SaveBufferToImage = SDL_SaveBMP of the window surface,
 * Renderer.cpp:184-187) and F6 starts the 10-window dFPS benchmark (Timer::StartBenchmark,
 * Timer.cpp:44-131); SDL_QUIT ends the loop.  `rtx_view_on_event` is that switch as a pure
 * function of (state, event), so the viewer (lib/rtx_view, csrc/cli/rtx_view.cpp: SDL2 loaded at
 * run time with dlopen) and the tests drive the same code.
 */
#ifndef RTX_VIEW_H_
#define RTX_VIEW_H_

#include <stdint.h>

#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* SDL2's event types and scancodes the loop reads (SDL_events.h / SDL_scancode.h values, SDL 2.0 ABI) */
enum {
    RTX_EV_QUIT = 0x100,     /* SDL_QUIT    */
    RTX_EV_KEYDOWN = 0x300,  /* SDL_KEYDOWN */
    RTX_EV_KEYUP = 0x301     /* SDL_KEYUP   */
};
enum {
    RTX_KEY_X = 27,          /* SDL_SCANCODE_X  */
    RTX_KEY_F2 = 59,         /* SDL_SCANCODE_F2 */
    RTX_KEY_F3 = 60,         /* SDL_SCANCODE_F3 */
    RTX_KEY_F6 = 63          /* SDL_SCANCODE_F6 */
};

/* The loop's state: the Renderer's m_CurrentLightingMode / m_ShadowsEnabled (Renderer.h:49-50) and
 * main.cpp's isLooping / takeScreenshot, plus a pending F6 (Timer::StartBenchmark). */
typedef struct rtx_view_state {
    int32_t lighting_mode;     /* RTX_MODE_*, starts Combined  */
    int32_t shadows_enabled;   /* starts 1                     */
    int32_t looping;           /* 0 after SDL_QUIT             */
    int32_t take_screenshot;   /* X released: save the next frame, then clear */
    int32_t start_benchmark;   /* F6 released: start the benchmark, then clear */
} rtx_view_state;

void rtx_view_init(rtx_view_state* s);
/* One polled event (main.cpp:63-86).  Returns 1 if it changed the state, 0 otherwise. */
int rtx_view_on_event(rtx_view_state* s, uint32_t event_type, int32_t scancode);
/* The render parameters of the state for a width x height surface whose pixel format is `fmt`
 * (SDL_MapRGB's shifts and alpha mask; NULL = XRGB8888): what Renderer::Render reads. */
void rtx_view_params(const rtx_view_state* s, uint32_t width, uint32_t height, const rtx_pixel_format* fmt,
                     rtx_render_params* out);
/* The screenshot (Renderer::SaveBufferToImage: SDL_SaveBMP of the window surface): the width x height
 * 32-bit surface (row-major pixels, pitch = width) as it is, in a 54-byte BITMAPFILEHEADER +
 * BITMAPINFOHEADER (BI_RGB, 32 bpp, 2835 px/m), rows bottom-up.  Returns 0 on success like SDL_SaveBMP
 * (which the reference's SaveBufferToImage returns as a bool: false = saved, main.cpp:101-106). */
int rtx_view_save_bmp(const char* path, const uint32_t* pixels, uint32_t width, uint32_t height);

#ifdef __cplusplus
}
#endif
#endif /* RTX_VIEW_H_ */
