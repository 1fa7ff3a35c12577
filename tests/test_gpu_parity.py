"""HIP render path vs the oracle (CPU restatement, pinned to the reference goldens) on
identical inputs.  Tolerance (BASELINE.json north_star): per-channel max-abs <= 1e-4 on
the post-MaxToOne float colour, and the uint32 buffer within 1 LSB per channel.  Paths
without powf (Lambert / SolidColor scenes) are required bit-exact."""
from pathlib import Path

import numpy as np
import pytest

import oracle_bind
from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.scene import HostScene, RENDERABLE

pytestmark = pytest.mark.gpu

TOL = 1e-4
POW_FREE = {"W1", "W2", "W4_Bunny", "Synthetic100k", "Bunny8Lights"}


def _channels(px):
    return np.stack([(px >> 16) & 255, (px >> 8) & 255, px & 255], -1).astype(np.int32)


def _compare(name, gpu_px, gpu_rgb, ref_px, ref_rgb, exact):
    d = np.abs(gpu_rgb - ref_rgb)
    assert not np.isnan(gpu_rgb).any()
    assert float(d.max(initial=0.0)) <= TOL, f"{name}: max-abs {d.max()} at {np.argmax(d)}"
    lsb = np.abs(_channels(gpu_px) - _channels(ref_px)).max(initial=0)
    assert lsb <= 1, f"{name}: {lsb} LSB"
    if exact:
        assert np.array_equal(gpu_px, ref_px), f"{name}: {(gpu_px != ref_px).sum()} pixels differ"
        assert np.array_equal(gpu_rgb.view(np.uint32), ref_rgb.view(np.uint32)), \
            f"{name}: {(gpu_rgb != ref_rgb).sum()} colour values differ"


@pytest.mark.parametrize("name", RENDERABLE)
@pytest.mark.parametrize("t", [-1.0, 1.3])
def test_scene_parity(gpu_ctx, name, t):
    hs = HostScene(name)
    if t >= 0:
        hs.update(t)
    s, cam = hs.view()
    p = abi.make_params(320, 180)
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(name, gpx, grgb, rpx, rrgb, exact=name in POW_FREE)


@pytest.mark.parametrize("name", ["W3", "W3_Test", "W4_Reference", "W2"])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("shadows", [0, 1])
def test_modes(gpu_ctx, name, mode, shadows):
    hs = HostScene(name)
    s, cam = hs.view()
    p = abi.make_params(200, 150, mode, shadows)
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(f"{name}/m{mode}/s{shadows}", gpx, grgb, rpx, rrgb, exact=(mode in (0, 1)) or name == "W2")


@pytest.mark.parametrize("name", ["W4_Bunny", "W3"])
def test_stripes_stitch_bit_identical(gpu_ctx, name):
    """Image tiled over N logical devices (16-row stripes, round robin) == 1 device."""
    hs = HostScene(name)
    s, cam = hs.view()
    W, H = 256, 200
    gpu_ctx.upload(s)
    full, _ = gpu_ctx.render(cam, abi.make_params(W, H), want_rgb=False)
    for n in (2, 3, 4, 8):
        stitched = np.full(W * H, 0xDEADBEEF, np.uint32)
        for r in range(n):
            px, _ = gpu_ctx.render(cam, abi.make_params(W, H, stripe_rows=16, stripe_first=r, stripe_step=n),
                                   want_rgb=False)
            rows = np.zeros(H, bool)
            for y in range(H):
                rows[y] = (y // 16) % n == r
            stitched.reshape(H, W)[rows] = px.reshape(H, W)[rows]
        assert np.array_equal(stitched, full), f"{name} n={n}"


@pytest.mark.parametrize("name", ["W4_Bunny", "W3", "W4_Optional", "W4_Reference"])
def test_work_counters_match_oracle(gpu_ctx, name):
    hs = HostScene(name)
    s, cam = hs.view()
    p = abi.make_params(160, 120)
    gpu_ctx.upload(s)
    g = gpu_ctx.count_work(cam, p)
    o = oracle_bind.count(s, cam, p)
    assert np.array_equal(g, o), dict(zip(oracle_bind.COUNTER_NAMES, zip(g.tolist(), o.tolist())))


@pytest.mark.parametrize("name", ["W4_Bunny", "W3", "W4_Optional"])
def test_cost_ordered_dispatch_is_output_invariant(gpu_ctx, name):
    """Frames 2..n run with the tile order derived from the previous frame's measured
    cost; the pixels must not change."""
    hs = HostScene(name)
    s, cam = hs.view()
    p = abi.make_params(320, 180)
    gpu_ctx.upload(s)
    first, first_rgb = gpu_ctx.render(cam, p)
    for _ in range(3):
        px, rgb = gpu_ctx.render(cam, p)
        assert np.array_equal(px, first)
        assert np.array_equal(rgb.view(np.uint32), first_rgb.view(np.uint32))


@pytest.fixture(scope="module")
def split_ctx():
    """A context that splits EVERY tile (RTX_SPLIT=force) from its second frame on."""
    import os
    from gp1_raytracer_2223_amd.renderer import DeviceContext
    os.environ["RTX_SPLIT"] = "force"
    try:
        ctx = DeviceContext(int(os.environ.get("RTX_TEST_DEVICE", "0")))
    finally:
        del os.environ["RTX_SPLIT"]
    yield ctx
    ctx.close()


SPLIT_CASES = [("W4_Bunny", -1.0), ("W4_Bunny", 1.3), ("W4_Reference", -1.0), ("W4_Optional", -1.0),
               ("Synthetic100k", -1.0), ("Bunny8Lights", -1.0), ("W4_Optional", 1.3)]


@pytest.mark.parametrize("name,t", SPLIT_CASES)
@pytest.mark.parametrize("mode,shadows", [(3, 1), (3, 0), (2, 1), (0, 1)])
def test_split_rendering(split_ctx, gpu_ctx, name, t, mode, shadows):
    """Heavy-tile split rendering (closest hit = min key over BVH frontier parts, occlusion
    = OR over parts) gives the same pixels as the one-piece kernel and the oracle."""
    hs = HostScene(name)
    if t >= 0:
        hs.update(t)
    s, cam = hs.view()
    p = abi.make_params(256, 144, mode, shadows)
    split_ctx.upload(s)
    split_ctx.render(cam, p)                      # measured frame: selects the heavy set
    heavy, parts = split_ctx.split_info()
    assert parts > 1 and heavy == 32 * 18, (heavy, parts)   # every 8x8 wave tile
    spx, srgb = split_ctx.render(cam, p)          # rendered by the split launches
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    assert np.array_equal(spx, gpx), f"{name}: {(spx != gpx).sum()} pixels differ from the one-piece kernel"
    assert np.array_equal(srgb.view(np.uint32), grgb.view(np.uint32))
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(f"{name}/split", spx, srgb, rpx, rrgb, exact=(name in POW_FREE) or mode in (0, 1))


def test_split_rendering_views_and_stripes(split_ctx, gpu_ctx):
    """Split tiles under the multi-view launch with stripe ownership (the bench's layout)."""
    import ctypes as C
    hs = HostScene("W4_Optional")
    s, cam = hs.view()
    W, H, N = 192, 160, 3
    views = (abi.Camera * N)()
    for f in range(N):
        C.memmove(C.byref(views[f]), C.byref(cam), C.sizeof(abi.Camera))
        views[f].origin[0] = cam.origin[0] + 0.05 * f
    for ctx in (split_ctx, gpu_ctx):
        ctx.upload(s)
    for r in range(N):
        p = abi.make_params(W, H, stripe_rows=16, stripe_first=r, stripe_step=N)
        out = []
        for ctx in (split_ctx, gpu_ctx):
            for _ in range(2):   # frame 1 measures, frame 2 splits (split_ctx)
                abi.check(ctx.lib.rtx_render_views_async(ctx.h, views, N, C.byref(p), 0), "views", ctx.h)
            abi.check(ctx.lib.rtx_synchronize(ctx.h), "sync", ctx.h)
            buf = np.zeros(N * W * H, np.uint32)
            abi.check(ctx.lib.rtx_download(ctx.h, buf.ctypes.data_as(C.POINTER(C.c_uint32)), None), "dl", ctx.h)
            out.append(buf)
        assert split_ctx.split_info()[0] > 0
        assert np.array_equal(out[0], out[1]), f"rank {r}: {(out[0] != out[1]).sum()} pixels differ"


SCENE_FILES = sorted((Path(__file__).resolve().parents[1] / "scenes").glob("*.rtxscene"))


@pytest.mark.parametrize("path", SCENE_FILES, ids=lambda p: p.stem)
@pytest.mark.parametrize("t", [-1.0, 1.3])
@pytest.mark.parametrize("mode,shadows", [(3, 1), (1, 1), (2, 0)])
def test_scene_file_parity(gpu_ctx, path, t, mode, shadows):
    """Scenes defined by scene files (scenes/*.rtxscene, pinned to the reference by
    tests/golden/*file_*) render on the GPU like the oracle."""
    hs = HostScene(f"file:{path}")
    if t >= 0:
        hs.update(t)
    s, cam = hs.view()
    p = abi.make_params(256, 144, mode, shadows)
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(f"{path.stem}/m{mode}s{shadows}", gpx, grgb, rpx, rrgb, exact=mode in (0, 1) or path.stem == "w4_bunny")


@pytest.mark.parametrize("name", ["W4_Bunny", "W4_Reference", "W4_Optional", "Bunny8Lights", "Synthetic100k"])
@pytest.mark.parametrize("shadows", [0, 1])
def test_octant_slab_path_bit_identical(gpu_ctx, name, shadows, monkeypatch):
    """Wave batches with one direction octant test the mirrored node copy (slab_mask<kSlabOct>):
    the frame must equal the one rendered with the general slab form only (RTX_NO_OCTANT
    uploads no octant copies), bit for bit, and the oracle's."""
    hs = HostScene(name)
    if name.startswith("W4"):
        hs.update(1.3)
    s, cam = hs.view()
    p = abi.make_params(320, 180, 3, shadows)
    gpu_ctx.upload(s)
    opx, orgb = gpu_ctx.render(cam, p)
    monkeypatch.setenv("RTX_NO_OCTANT", "1")
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    monkeypatch.delenv("RTX_NO_OCTANT")
    gpu_ctx.upload(s)
    assert np.array_equal(opx, gpx) and np.array_equal(orgb.view(np.uint32), grgb.view(np.uint32))
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(name, opx, orgb, rpx, rrgb, exact=name in POW_FREE)


@pytest.mark.parametrize("name,W,H", [("W4_Bunny", 640, 360), ("W4_Optional", 480, 270), ("Synthetic100k", 320, 180)])
def test_frames_in_flight_bit_identical(gpu_ctx, name, W, H):
    """Two contexts on one device rendering alternate frames (bench.py --inflight 2) while each
    other's launches are still running — split rendering of heavy tiles included (own split
    stream and buffers per context): every frame equals the single-context frame."""
    import ctypes as C
    from gp1_raytracer_2223_amd.renderer import DeviceContext
    hs = HostScene(name)
    s, cam = hs.view()
    p = abi.make_params(W, H)
    gpu_ctx.upload(s)
    ref, _ = gpu_ctx.render(cam, p, want_rgb=False)
    other = DeviceContext(0)
    try:
        other.upload(s)
        pair = (gpu_ctx, other)
        for i in range(40):   # enqueue without waiting: launches of the two contexts overlap
            c = pair[i % 2]
            abi.check(c.lib.rtx_render_async(c.h, C.byref(cam), C.byref(p), 0), "render", c.h)
        for c in pair:
            px, _ = c.render(cam, p, want_rgb=False)
            assert np.array_equal(px, ref)
    finally:
        other.close()


LIGHTS_ON_PLANES = {
    # a point light exactly on a wall: shadow rays from the other walls reach it at t == tmax
    # on that wall's plane (the near-tie of the shadow-ray plane skip, plane_cand), and rays
    # from the wall itself run parallel to it (den = 0)
    "floor": "light point 0.5 0 3  30 1 1 1",
    "back": "light point 1 2 10  30 1 0.8 0.6",
    "side": "light point -5 3 2  30 0.6 0.8 1",
    # just in front of / just behind the floor (one ulp of 1e-7-ish), and a corner
    "near_floor": "light point 0.5 1e-7 3  30 1 1 1\nlight point 0.5 -1e-7 3.5  30 1 1 1",
    "corner": "light point -5 0 10  40 1 1 1",
}


@pytest.mark.parametrize("case", sorted(LIGHTS_ON_PLANES))
@pytest.mark.parametrize("mode", [3, 1])
def test_lights_on_planes(gpu_ctx, tmp_path, case, mode):
    """Adversarial shadow-ray cases (lights on or one ulp off a plane) render bit-exact like
    the oracle: Lambert-only scene, so no powf anywhere."""
    path = tmp_path / f"{case}.rtxscene"
    path.write_text("\n".join([
        "camera 0 2.5 -8 50",
        "material lambert 0.49 0.57 0.57 1",
        "material lambert 1 1 1 1",
        "plane 0 0 10   0 0 -1  1",
        "plane 0 0 0    0 1 0   1",
        "plane -5 0 0   1 0 0   1",
        "sphere 2 1 2 0.9 2",
        "mesh lowpoly_bunny2 2 back scale 1.5 1.5 1.5 translate 0 0 0.5",
        LIGHTS_ON_PLANES[case],
    ]) + "\n")
    hs = HostScene(f"file:{path}")
    s, cam = hs.view()
    p = abi.make_params(256, 144, mode, 1)
    gpu_ctx.upload(s)
    gpx, grgb = gpu_ctx.render(cam, p)
    rpx, rrgb = oracle_bind.render(s, cam, p)
    _compare(f"{case}/m{mode}", gpx, grgb, rpx, rrgb, exact=True)
