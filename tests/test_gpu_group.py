"""One frame tiled over several render contexts and gathered on the host,
through the HIP path.  This box has one GPU, so G contexts share device 0 — the same code
path as G devices (one host thread + stream per context, each gathering its 16-row stripes
with hipMemcpy2DAsync into the caller's frame).  The stitched frame must equal one
context's render bit for bit, and at full resolution the reference's own frame."""
import ctypes as C
import hashlib
import os
from pathlib import Path

import numpy as np
import pytest

from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext, DeviceGroup
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu

G = Path(__file__).resolve().parent / "golden"
DEV = int(os.environ.get("RTX_TEST_DEVICE", "0"))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["W4_Bunny", "W3"])
def test_group_equals_single_context(gpu_ctx, name):
    hs = HostScene(name)
    s, cam = hs.view()
    W, H = 1000, 701   # 43.8 stripes: a partial last stripe, uneven ownership
    gpu_ctx.upload(s)
    ref_px, ref_rgb = gpu_ctx.render(cam, abi.make_params(W, H))
    for n in (1, 2, 3, 4, 8):
        grp = DeviceGroup([DEV] * n)
        try:
            grp.upload(s)
            for frame in range(2):
                px, rgb = grp.render(cam, abi.make_params(W, H))
                assert np.array_equal(px, ref_px), f"{name} n={n} frame {frame}"
                assert np.array_equal(rgb.view(np.uint32), ref_rgb.view(np.uint32)), f"{name} n={n} rgb"
        finally:
            grp.close()


@pytest.mark.parametrize("stripe_rows", [32, 48])
def test_group_stripe_heights(gpu_ctx, stripe_rows):
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    W, H = 640, 480
    gpu_ctx.upload(s)
    ref, _ = gpu_ctx.render(cam, abi.make_params(W, H), want_rgb=False)
    grp = DeviceGroup([DEV] * 3)
    try:
        grp.upload(s)
        px, _ = grp.render(cam, abi.make_params(W, H, stripe_rows=stripe_rows), want_rgb=False)
        assert np.array_equal(px, ref)
    finally:
        grp.close()


@pytest.mark.parametrize("name,W,H", [("Synthetic100k", 1920, 1080), ("Bunny8Lights", 3840, 2160)])
def test_group_full_resolution_matches_reference(name, W, H):
    """The north star's multi-GPU configs, tiled over 4 contexts into a page-locked host
    frame: the gathered frame is the reference's (SHA-256 of tests/golden/config_*)."""
    g = np.load(G / f"config_{name}_{W}x{H}.npz")
    hs = HostScene(name)
    s, cam = hs.view()
    grp = DeviceGroup([DEV] * 4)
    lib = grp.lib
    frame = np.zeros(W * H, np.uint32)
    c0 = lib.rtx_group_context(grp.h, 0)
    assert lib.rtx_host_register(c0, frame.ctypes.data_as(C.c_void_p), frame.nbytes) == abi.RTX_OK
    try:
        grp.upload(s)
        for f in range(3):   # frame 1 measures tile costs, the rest run cost-ordered / split
            frame[:] = 0
            grp.render(cam, abi.make_params(W, H), want_rgb=False, out_px=frame)
            assert _sha(frame) == str(g["sha_pixels"][0]), f"{name} frame {f + 1}"
    finally:
        lib.rtx_host_unregister(c0, frame.ctypes.data_as(C.c_void_p))
        grp.close()


def test_group_rejects_caller_stripes():
    hs = HostScene("W3")
    s, cam = hs.view()
    grp = DeviceGroup([DEV, DEV])
    try:
        grp.upload(s)
        with pytest.raises(RuntimeError, match="stripe_step"):
            grp.render(cam, abi.make_params(64, 64, stripe_rows=16, stripe_first=0, stripe_step=2))
        with pytest.raises(RuntimeError, match="multiple of 16"):
            grp.render(cam, abi.make_params(64, 64, stripe_rows=8))
    finally:
        grp.close()


def test_gather_async_leaves_foreign_rows_untouched(gpu_ctx):
    """rtx_gather_async writes exactly the owned stripes (the contract processes sharing one
    host frame rely on)."""
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    W, H = 320, 200
    gpu_ctx.upload(s)
    full, _ = gpu_ctx.render(cam, abi.make_params(W, H), want_rgb=False)
    out = np.full(W * H, 0xDEADBEEF, np.uint32)
    gpu_ctx.render_async(cam, abi.make_params(W, H, stripe_rows=16, stripe_first=1, stripe_step=3))
    gpu_ctx.gather_async(out)
    gpu_ctx.synchronize()
    rows = (np.arange(H) // 16) % 3 == 1
    img, ref = out.reshape(H, W), full.reshape(H, W)
    assert np.array_equal(img[rows], ref[rows])
    assert (img[~rows] == 0xDEADBEEF).all()
