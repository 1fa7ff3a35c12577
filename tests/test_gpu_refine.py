"""Frontier refinement (rtx_ctx::refine_*): after kRefineQuiet frames of a static scene
the split frame is measured per BVH frontier part and the heaviest parts are cut into their children.
Parts still partition the triangles, so every frame before, during and after the rounds is the
reference's: compared with a context that never refines (RTX_REFINE=0)."""
import ctypes as C
import os

import numpy as np
import pytest

from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu

DEV = int(os.environ.get("RTX_TEST_DEVICE", "0"))


def _ctx(**env):
    saved = os.environ.pop("RTX_REFINE", None)
    os.environ.update(env)
    try:
        return DeviceContext(DEV)
    finally:
        os.environ.pop("RTX_REFINE", None)
        if saved is not None:
            os.environ["RTX_REFINE"] = saved


def _frame(ctx, cam, p, W, H):
    out = np.zeros(W * H, np.uint32)
    ctx.synchronize()
    abi.check(ctx.lib.rtx_gather_async(ctx.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), None), "gather", ctx.h)
    ctx.synchronize()
    return out


@pytest.mark.parametrize("s_", [4, 8])
def test_refined_frontier_frames_equal_unrefined(s_):
    """Synthetic100k 1080p, rank 0's share of s (its chain outlasts its main kernel, so it refines):
    120 frames (the rounds run), the parts grow, and the frames of every stage equal an unrefined
    context's."""
    W, H = 1920, 1080
    hs = HostScene("Synthetic100k")
    s, cam = hs.view()
    p = abi.make_params(W, H, stripe_rows=16 if s_ > 1 else 0, stripe_first=0, stripe_step=s_)
    ref_ctx, ctx = _ctx(RTX_REFINE="0"), _ctx()
    try:
        ref_ctx.upload(s)
        ctx.upload(s)
        parts0 = ctx.split_info()[1]
        for _ in range(3):
            abi.check(ref_ctx.lib.rtx_render_async(ref_ctx.h, C.byref(cam), C.byref(p), 0), "render", ref_ctx.h)
        ref = _frame(ref_ctx, cam, p, W, H)
        seen_parts = {parts0}
        for f in range(120):
            abi.check(ctx.lib.rtx_render_async(ctx.h, C.byref(cam), C.byref(p), 0), "render", ctx.h)
            if f % 10 == 9:
                got = _frame(ctx, cam, p, W, H)
                assert np.array_equal(got, ref), f"frame {f}: {(got != ref).sum()} pixels differ"
                seen_parts.add(ctx.split_info()[1])
        assert max(seen_parts) > parts0, f"no refinement: parts {sorted(seen_parts)}"
        assert ref_ctx.split_info()[1] == parts0
    finally:
        ref_ctx.close()
        ctx.close()
