"""The presentation side of the reference's frame loop (include/rtx_view.h, librtx_host.so; SURVEY
§8(f)3): the event switch of source/main.cpp:63-86 as a pure function, the render parameters it
gives Renderer::Render, the screenshot's bytes, and the viewer program's behaviour without SDL2.
CPU only: the viewer's GPU loop is tests/test_cli_gpu.py::test_viewer_keys_headless."""
import ctypes as C
import struct
import subprocess

import numpy as np
import pytest

from gp1_raytracer_2223_amd import abi

QUIT, KEYDOWN, KEYUP = 0x100, 0x300, 0x301
X, F2, F3, F6 = 27, 59, 60, 63   # SDL scancodes


class State(C.Structure):
    _fields_ = [("lighting_mode", C.c_int32), ("shadows_enabled", C.c_int32), ("looping", C.c_int32),
                ("take_screenshot", C.c_int32), ("start_benchmark", C.c_int32)]


@pytest.fixture(scope="module")
def lib():
    lib = abi.load_host()
    lib.rtx_view_init.argtypes = [C.POINTER(State)]
    lib.rtx_view_on_event.argtypes = [C.POINTER(State), C.c_uint32, C.c_int32]
    lib.rtx_view_on_event.restype = C.c_int
    lib.rtx_view_params.argtypes = [C.POINTER(State), C.c_uint32, C.c_uint32, C.POINTER(abi.PixelFormat),
                                    C.POINTER(abi.RenderParams)]
    lib.rtx_view_save_bmp.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32]
    lib.rtx_view_save_bmp.restype = C.c_int
    return lib


def _run(lib, events):
    st = State()
    lib.rtx_view_init(C.byref(st))
    for ev in events:
        lib.rtx_view_on_event(C.byref(st), *ev)
    return st


def test_initial_state(lib):
    st = _run(lib, [])
    # Renderer.h:49-50 (Combined, shadows on); main.cpp:56 isLooping
    assert (st.lighting_mode, st.shadows_enabled, st.looping, st.take_screenshot, st.start_benchmark) == (3, 1, 1, 0, 0)


def test_f3_cycles_modes_in_enum_order(lib):
    modes = [_run(lib, [(KEYUP, F3)] * k).lighting_mode for k in range(6)]
    # CycleLightingMode: (mode + 1) % Count from Combined (Renderer.cpp:189-193, Renderer.h:40-48)
    assert modes == [3, 0, 1, 2, 3, 0]


def test_keys_act_on_release_only(lib):
    st = _run(lib, [(KEYDOWN, F3), (KEYDOWN, F2), (KEYDOWN, X), (KEYDOWN, F6), (KEYUP, 4), (KEYUP, 58)])
    assert (st.lighting_mode, st.shadows_enabled, st.take_screenshot, st.start_benchmark) == (3, 1, 0, 0)


def test_sequence_to_render_params(lib):
    """A key sequence and the rtx_render_params Renderer::Render then reads."""
    st = _run(lib, [(KEYUP, F2), (KEYUP, F3), (KEYUP, F3), (KEYUP, X), (KEYUP, F6), (KEYUP, F2), (KEYUP, F2)])
    assert st.shadows_enabled == 0 and st.lighting_mode == 1 and st.take_screenshot == 1 and st.start_benchmark == 1
    p = abi.RenderParams()
    fmt = abi.PixelFormat(0, 8, 16, 0xFF000000)   # an ABGR8888 surface: SDL_MapRGB's shifts + alpha
    lib.rtx_view_params(C.byref(st), 640, 480, C.byref(fmt), C.byref(p))
    assert (p.width, p.height, p.lighting_mode, p.shadows_enabled) == (640, 480, 1, 0)
    assert (p.format.rshift, p.format.gshift, p.format.bshift, p.format.amask) == (0, 8, 16, 0xFF000000)
    assert (p.stripe_rows, p.stripe_step) == (0, 1)
    lib.rtx_view_params(C.byref(st), 64, 48, None, C.byref(p))   # NULL: XRGB8888
    assert (p.format.rshift, p.format.gshift, p.format.bshift, p.format.amask) == (16, 8, 0, 0)
    assert lib.rtx_view_on_event(C.byref(st), QUIT, 0) == 1 and st.looping == 0


def test_screenshot_bytes(lib, tmp_path):
    W, H = 5, 3
    px = np.arange(W * H, dtype=np.uint32) * 0x010203 + 0x00102030
    f = tmp_path / "RayTracing_Buffer.bmp"
    assert lib.rtx_view_save_bmp(str(f).encode(), px.ctypes.data_as(C.POINTER(C.c_uint32)), W, H) == 0
    b = f.read_bytes()
    assert len(b) == 54 + 4 * W * H
    magic, size, _, off, hsz, w, h, planes, bpp, comp, img = struct.unpack_from("<2sIIIIiiHHII", b, 0)
    assert (magic, size, off, hsz, w, h, planes, bpp, comp, img) == (b"BM", 54 + 4 * W * H, 54, 40, W, H, 1, 32, 0,
                                                                      4 * W * H)
    rows = np.frombuffer(b, np.uint32, W * H, 54).reshape(H, W)
    assert np.array_equal(rows[::-1].ravel(), px)   # bottom-up rows of the surface's own 32-bit pixels
    assert lib.rtx_view_save_bmp(str(tmp_path / "no" / "dir.bmp").encode(), px.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 W, H) != 0


def test_viewer_without_sdl_exits_cleanly():
    exe = abi.LIB_DIR / "rtx_view"
    if not exe.exists():
        from gp1_raytracer_2223_amd import build
        build.build_view()
    try:
        import ctypes.util
        has_sdl = ctypes.util.find_library("SDL2-2.0") or ctypes.util.find_library("SDL2")
    except Exception:   # noqa: BLE001
        has_sdl = None
    if has_sdl:
        pytest.skip("SDL2 is installed here: the viewer would open a window")
    r = subprocess.run([str(exe), "W4_Bunny", "320", "240"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "libSDL2" in r.stdout
