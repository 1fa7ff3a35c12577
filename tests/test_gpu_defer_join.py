"""Deferred join of the split chain (rtx_ctx::join_pending): a frame that repeats the last
one (parameters, cameras, scene image, heavy set) starts its main kernel beside the last frame's split
chain (they write disjoint tiles); anything else joins first.  A sequence that mixes repeats with
every kind of change — lighting mode, camera, a new scene, stripes — must read back, after each
stage, exactly the frame of a context that never splits."""
import ctypes as C
import os

import numpy as np
import pytest

from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu

DEV = int(os.environ.get("RTX_TEST_DEVICE", "0"))
W, H = 1920, 1080


def _ctx(**env):
    saved = {k: os.environ.pop(k, None) for k in ("RTX_SPLIT", "RTX_DEFER_JOIN")}
    os.environ.update(env)
    try:
        return DeviceContext(DEV)
    finally:
        for k in ("RTX_SPLIT", "RTX_DEFER_JOIN"):
            os.environ.pop(k, None)
            if saved[k] is not None:
                os.environ[k] = saved[k]


def _gather(ctx):
    out = np.zeros(W * H, np.uint32)
    abi.check(ctx.lib.rtx_gather_async(ctx.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), None), "gather", ctx.h)
    ctx.synchronize()
    return out


def _frames(ctx, cam, p, n):
    for _ in range(n):
        abi.check(ctx.lib.rtx_render_async(ctx.h, C.byref(cam), C.byref(p), 0), "render", ctx.h)


def _moved(cam, dx):
    c = abi.Camera()
    C.memmove(C.byref(c), C.byref(cam), C.sizeof(abi.Camera))
    c.origin[0] += dx
    return c


def test_deferred_join_sequence():
    ctx, ref = _ctx(), _ctx(RTX_SPLIT="0")
    try:
        s_opt, cam_opt = HostScene("W4_Optional").view()
        s_b8, cam_b8 = HostScene("Bunny8Lights").view()
        share = dict(stripe_rows=16, stripe_first=0, stripe_step=8)
        stages = [  # (scene, camera, params, frames)
            (s_opt, cam_opt, abi.make_params(W, H, **share), 60),
            (s_opt, cam_opt, abi.make_params(W, H, 1, 1, **share), 1),     # lighting mode
            (s_opt, cam_opt, abi.make_params(W, H, **share), 30),
            (s_opt, _moved(cam_opt, 0.25), abi.make_params(W, H, **share), 20),   # camera
            (s_opt, cam_opt, abi.make_params(W, H, stripe_rows=16, stripe_first=3, stripe_step=8), 20),  # share
            (s_b8, cam_b8, abi.make_params(W, H, **share), 40),             # another scene
            (s_b8, cam_b8, abi.make_params(W, H, **share), 1),
        ]
        uploaded = None
        deferred = 0
        for i, (sc, cam, p, n) in enumerate(stages):
            if sc is not uploaded:
                ctx.upload(sc)
                ref.upload(sc)
                uploaded = sc
            _frames(ctx, cam, p, n)
            deferred += ctx.split_info()[0] > 0
            got = _gather(ctx)
            _frames(ref, cam, p, 1)
            want = _gather(ref)
            assert np.array_equal(got, want), f"stage {i}: {(got != want).sum()} pixels differ"
        assert deferred >= 3, "the sequence never split"
    finally:
        ctx.close()
        ref.close()
