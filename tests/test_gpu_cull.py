"""The exact cull (rtx_cull.h): nodes skipped because the ray's line misses their
tight box widened by the proven Möller–Trumbore margin.  A skipped node must never change a pixel:
every frame here is compared bit for bit with a context created under RTX_NO_CULL=1 (the
reference's traversal, unpruned) and with the oracle.  Cameras are chosen to stress the bound:
in the plane of a triangle (its margin is then infinite), at a vertex, inside and under the
height field, far away, several views per launch with different anchors, and a camera that
moves between frames of one context (the anchor's records are rebuilt)."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle_bind
from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu

MESH_SCENES = ["W4_Bunny", "W4_Reference", "W4_Optional", "Synthetic100k", "Bunny8Lights"]
POW_FREE = {"W4_Bunny", "Synthetic100k", "Bunny8Lights"}


def _ctx_env(**env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return DeviceContext(int(os.environ.get("RTX_TEST_DEVICE", "0")))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def cull_ctx():
    """A context that culls every scene (the product enables the cull only where the SAH estimate
    says it pays, RTX_CULL_MIN_SA) and tests every record (RTX_CULL_RATIO=0)."""
    ctx = _ctx_env(RTX_CULL_MIN_SA="0", RTX_CULL_RATIO="0", RTX_CULL_ANIMATED="1")
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def product_ctx():
    """The product's cull decision, independent of the upload history (RTX_CULL_ANIMATED=1)."""
    ctx = _ctx_env(RTX_CULL_ANIMATED="1")
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def plain_ctx():
    """A context without the cull: the reference's full traversal."""
    ctx = _ctx_env(RTX_NO_CULL="1")
    yield ctx
    ctx.close()


def _same(a, b, what):
    """uint32 frames equal, colour planes equal bit for bit (a NaN equal to any NaN: the light on
    a shadow-ray origin gives 0/0 directions, whose NaN payload is the CPU's or the GPU's own)."""
    assert np.array_equal(a[0], b[0]), f"{what}: {(a[0] != b[0]).sum()} pixels differ"
    na, nb = np.isnan(a[1]), np.isnan(b[1])
    assert np.array_equal(na, nb), f"{what}: NaN positions differ"
    assert np.array_equal(a[1].view(np.uint32)[~na], b[1].view(np.uint32)[~nb]), f"{what}: colour planes differ"


def _check(gpu_ctx, plain_ctx, s, cam, p, what, exact_oracle):
    gpu_ctx.upload(s)
    plain_ctx.upload(s)
    for _ in range(3):   # the cost-ordered / split frames too
        g = gpu_ctx.render(cam, p)
    q = plain_ctx.render(cam, p)
    _same(g, q, f"{what} cull vs no cull")
    r = oracle_bind.render(s, cam, p)
    assert np.array_equal(np.isnan(g[1]), np.isnan(r[1])), f"{what}: NaN positions differ from the oracle's"
    ok = ~np.isnan(r[1])
    d = float(np.abs(g[1][ok] - r[1][ok]).max(initial=0.0))
    assert d <= 1e-4, f"{what}: max-abs {d} vs the oracle"
    if exact_oracle:
        _same(g, r, f"{what} vs oracle")


@pytest.mark.parametrize("name", MESH_SCENES)
@pytest.mark.parametrize("t", [-1.0, 1.3])
@pytest.mark.parametrize("mode,shadows", [(3, 1), (0, 1), (3, 0)])
def test_cull_equals_full_traversal(cull_ctx, gpu_ctx, plain_ctx, name, t, mode, shadows):
    hs = HostScene(name)
    if t >= 0:
        hs.update(t)
    s, cam = hs.view()
    for ctx in (cull_ctx, gpu_ctx):   # forced on, and the product's choice
        _check(ctx, plain_ctx, s, cam, abi.make_params(320, 180, mode, shadows), f"{name}@{t}/m{mode}s{shadows}",
               name in POW_FREE or mode in (0, 1))


def _synthetic_triangle(hs, k):
    a = hs.arrays()["meshes"][0]
    P = a["tpositions"].reshape(-1, 3)
    I = a["indices"].reshape(-1, 3)
    return P[I[k, 0]], P[I[k, 1]], P[I[k, 2]]


def _cameras():
    hs = HostScene("Synthetic100k")
    v0, v1, v2 = _synthetic_triangle(hs, 777)
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    in_plane = (v0 + np.float32(3.0) * e1 - np.float32(2.0) * e2).astype(np.float32)
    w0, w1, _ = _synthetic_triangle(hs, 40000)
    far_in_plane = (w0 + np.float32(40.0) * (w1 - w0)).astype(np.float32)
    return [
        ("reference", (0.0, 3.0, -9.0), 45.0, 0.0, 0.0),
        ("in_a_triangle_plane", tuple(float(x) for x in in_plane), 60.0, -0.5, 0.3),
        ("in_a_plane_far", tuple(float(x) for x in far_in_plane), 45.0, -0.3, 0.0),
        ("at_a_vertex", tuple(float(x) for x in v0), 70.0, -0.4, 0.8),
        ("inside_the_field", (0.01, 0.55, 1.0), 90.0, 0.0, 0.0),
        ("under_the_field", (0.5, 0.1, 0.5), 90.0, 0.6, 0.2),
        ("grazing_the_top", (-2.9, 0.81, -1.5), 50.0, -0.02, 0.0),
        ("far_away", (30.0, 40.0, -60.0), 20.0, -0.55, -0.45),
    ]


@pytest.mark.parametrize("cam_case", _cameras(), ids=lambda c: c[0])
def test_cull_adversarial_cameras(cull_ctx, plain_ctx, cam_case):
    what, origin, fov, pitch, yaw = cam_case
    hs = HostScene("Synthetic100k")
    hs.set_camera(origin, fov, pitch, yaw)
    s, cam = hs.view()
    _check(cull_ctx, plain_ctx, s, cam, abi.make_params(240, 160), what, True)


def test_cull_views_with_different_anchors(cull_ctx, plain_ctx):
    """One launch, several views: each view's rays use that view's camera anchor."""
    hs = HostScene("Synthetic100k")
    s, cam = hs.view()
    W, H, N = 192, 128, 4
    views = (abi.Camera * N)()
    for f in range(N):
        C.memmove(C.byref(views[f]), C.byref(cam), C.sizeof(abi.Camera))
        views[f].origin[0] = cam.origin[0] + 0.75 * f
        views[f].origin[1] = cam.origin[1] - 0.4 * f
    p = abi.make_params(W, H)
    out = []
    for ctx in (cull_ctx, plain_ctx):
        ctx.upload(s)
        for _ in range(2):
            abi.check(ctx.lib.rtx_render_views_async(ctx.h, views, N, C.byref(p), 1), "views", ctx.h)
        abi.check(ctx.lib.rtx_synchronize(ctx.h), "sync", ctx.h)
        px = np.zeros(N * W * H, np.uint32)
        rgb = np.zeros(3 * N * W * H, np.float32)
        abi.check(ctx.lib.rtx_download(ctx.h, px.ctypes.data_as(C.POINTER(C.c_uint32)),
                                       rgb.ctypes.data_as(C.POINTER(C.c_float))), "dl", ctx.h)
        out.append((px, rgb))
    _same(out[0], out[1], "views")
    for f in range(N):
        r = oracle_bind.render(s, views[f], p)
        g = (out[0][0][f * W * H:(f + 1) * W * H], out[0][1][3 * f * W * H:3 * (f + 1) * W * H])
        _same(g, r, f"view {f} vs oracle")


def test_cull_camera_moves_between_frames(cull_ctx):
    """One context, the camera moved between frames (and back): the anchor's records follow."""
    hs = HostScene("Synthetic100k")
    s, cam0 = hs.view()
    p = abi.make_params(200, 120)
    cull_ctx.upload(s)
    cams = []
    for dx in (0.0, 1.5, -2.0, 0.0):
        c = abi.Camera()
        C.memmove(C.byref(c), C.byref(cam0), C.sizeof(abi.Camera))
        c.origin[0] = cam0.origin[0] + dx
        cams.append(c)
    for c in cams:
        g = cull_ctx.render(c, p)
        _same(g, oracle_bind.render(s, c, p), f"camera x+{c.origin[0] - cam0.origin[0]}")


@pytest.mark.parametrize("name,on", [("Synthetic100k", True), ("W4_Optional", True), ("W4_Bunny", False),
                                     ("Bunny8Lights", False), ("W3", False)])
def test_cull_enabled_where_it_pays(product_ctx, name, on):
    """The product enables the cull where the reference's boxes are inflated enough (the SAH
    estimate of upload_scene: W4_Bunny 1.19, W4_Optional 2.40, Synthetic100k 9.26)."""
    hs = HostScene(name)   # (the scene's arrays live as long as hs)
    s, cam = hs.view()
    product_ctx.upload(s)
    assert product_ctx.cull_info()[0] == on


def _animated_loop(ctx, plain_ctx, renders_per_upload):
    hs = HostScene("W4_Optional")
    p = abi.make_params(96, 64)
    seen = []
    for k, renders in enumerate(renders_per_upload):
        hs.update(0.05 * k)
        s, cam = hs.view()
        ctx.upload(s)
        seen.append(ctx.cull_info()[0])
        for _ in range(renders):
            px, rgb = ctx.render(cam, p)
        plain_ctx.upload(s)
        _same((px, rgb), plain_ctx.render(cam, p), f"upload {k + 1}")   # bit for bit, both planes
        assert np.array_equal(px, oracle_bind.render(s, cam, p)[0]), k   # (Cook-Torrance: powf in rgb)
    return seen


def test_cull_records_built_for_animated_uploads(plain_ctx):
    """An animated loop re-uploads every frame and renders it once; the segment-tree records
    cost tens of microseconds, so every upload gets them (round 4 skipped them after two such
    uploads).  Every frame equals the unculled walk's and the reference's."""
    ctx = _ctx_env()
    try:
        assert _animated_loop(ctx, plain_ctx, [1, 1, 1, 1, 3, 1, 1]) == [True] * 7
    finally:
        ctx.close()


def test_cull_animated_skip_rule_opt_in(plain_ctx):
    """RTX_CULL_ANIMATED=0 keeps round 4's rule: after two consecutive uploads rendered at most
    once each the records are not built, and an upload rendered twice or more turns them back on."""
    ctx = _ctx_env(RTX_CULL_ANIMATED="0")
    try:
        seen = _animated_loop(ctx, plain_ctx, [1, 1, 1, 1, 3, 1, 1])
        # uploads 1-2 follow at most one short upload, 3-5 two or more; 6 follows an upload rendered
        # three times, 7 one short upload
        assert seen == [True, True, False, False, False, True, True], seen
    finally:
        ctx.close()


# ---------------------------------------------------------------- the records themselves
_REF = None


def _records_ref():
    global _REF
    if _REF is None:
        from pathlib import Path
        so = Path(__file__).resolve().parents[1] / "tools" / "bin" / "libcull_records_ref.so"
        if not so.exists():
            pytest.fail(f"{so} missing: run __graft_entry__.build()")
        _REF = C.CDLL(str(so))
        VP = C.c_void_p
        _REF.cull_records_ref.argtypes = [C.c_uint32, C.c_uint32, VP, VP, VP, VP, C.c_float, C.c_int, VP]
        _REF.cull_records_ref.restype = C.c_int
    return _REF


def _dump(ctx, anchor):
    ns, nt = C.c_uint32(), C.c_uint32()
    abi.check(ctx.lib.rtx_cull_dump(ctx.h, anchor, C.byref(ns), C.byref(nt), None, None, None, None, None), "dump",
              ctx.h)
    a = np.zeros(5, np.float32)
    rec = np.zeros(8 * ns.value, np.float32)
    rng = np.zeros(2 * ns.value, np.uint32)
    nodes = np.zeros(8 * ns.value, np.float32)
    tris = np.zeros(16 * nt.value, np.float32)
    abi.check(ctx.lib.rtx_cull_dump(ctx.h, anchor, C.byref(ns), C.byref(nt), a.ctypes.data, rec.ctypes.data,
                                    rng.ctypes.data, nodes.ctypes.data, tris.ctypes.data), "dump", ctx.h)
    return a, rec, rng, nodes, tris, nt.value


@pytest.mark.parametrize("name", ["Synthetic100k", "W4_Optional"])
@pytest.mark.parametrize("top", ["lds", "global"])
def test_cull_records_equal_brute_force(name, top):
    """Every record of the segment-tree build (rtx_cull_tris, rtx_cull_nodes) equals, value for
    value, the direct fold of every triangle of the slot's range (tools/cull_records_ref.c, the
    same double-precision bound, rtx_cull.h): camera anchors of two views, at upload and after a
    camera move, and every light anchor.  "global": the trees' top levels built in global memory
    (RTX_CULL_TOP_LDS=0) instead of LDS."""
    env = {"RTX_CULL_MIN_SA": "0"}
    if top == "global":
        env["RTX_CULL_TOP_LDS"] = "0"
    ctx = _ctx_env(**env)
    try:
        hs = HostScene(name)
        s, cam = hs.view()
        ctx.upload(s)
        W, H = 64, 48
        views = (abi.Camera * 2)()
        for f in range(2):
            C.memmove(C.byref(views[f]), C.byref(cam), C.sizeof(abi.Camera))
            views[f].origin[0] = cam.origin[0] + 0.6 * f
        p = abi.make_params(W, H)
        abi.check(ctx.lib.rtx_render_views_async(ctx.h, views, 2, C.byref(p), 0), "views", ctx.h)
        ref = _records_ref()
        anchors = [0, 1] + [8 + l for l in range(s.n_lights)]
        checked = 0
        for step in range(2):
            if step == 1:   # move view 0's camera: its records are rebuilt alone
                views[0].origin[2] = cam.origin[2] + 0.7
                abi.check(ctx.lib.rtx_render_views_async(ctx.h, views, 2, C.byref(p), 0), "views", ctx.h)
                anchors = [0]
            for j in anchors:
                a, rec, rng, nodes, tris, nt = _dump(ctx, j)
                if j < 8:
                    assert tuple(a[:3]) == tuple(np.float32(x) for x in views[j].origin), j
                want = np.zeros_like(rec)
                ref.cull_records_ref(len(rng) // 2, nt, rng.ctypes.data, nodes.ctypes.data, tris.ctypes.data,
                                     a.ctypes.data, 1.5, 0, want.ctypes.data)
                r8, w8 = rec.reshape(-1, 8), want.reshape(-1, 8)
                bad = np.nonzero(~np.all((r8[:, :7] == w8[:, :7]) & (r8[:, 7:].view(np.uint32) ==
                                                                     w8[:, 7:].view(np.uint32)), axis=1))[0]
                assert bad.size == 0, (f"{name} anchor {j} step {step}: {bad.size} of {len(r8)} records differ, "
                                       f"first slot {bad[0]}: {r8[bad[0]]} vs {w8[bad[0]]}")
                checked += 1
        assert checked == 3 + s.n_lights
    finally:
        ctx.close()


def test_cull_records_follow_the_camera(cull_ctx):
    """A view's records are rebuilt only when its camera origin changes."""
    hs = HostScene("Synthetic100k")
    s, cam = hs.view()
    p = abi.make_params(64, 64)
    cull_ctx.upload(s)
    n0 = cull_ctx.cull_info()[1]
    cull_ctx.render(cam, p)
    cull_ctx.render(cam, p)
    assert cull_ctx.cull_info()[1] == n0 + 1
    c = abi.Camera()
    C.memmove(C.byref(c), C.byref(cam), C.sizeof(abi.Camera))
    c.origin[2] = cam.origin[2] - 0.5
    cull_ctx.render(c, p)
    assert cull_ctx.cull_info()[1] == n0 + 2


def test_cull_ordered_walk_ties(cull_ctx, plain_ctx, tmp_path):
    """The ordered walk replaces the scratch hit on a tie of t only by a LOWER triangle index —
    the reference's first-found winner.  A mesh whose every face appears twice (the copy right
    after the original, so both land in one leaf or in neighbouring subtrees) makes every hit a
    tie between two triangles; the frames must equal the unculled walk's and the oracle's."""
    rng = np.random.default_rng(7)
    n = 24
    lines = []
    for j in range(n + 1):
        for i in range(n + 1):
            lines.append(f"v {-2 + 4 * i / n:.6f} {0.2 + 0.6 * rng.random():.6f} {-1 + 3 * j / n:.6f}")
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i + 1, j * (n + 1) + i + 2, (j + 1) * (n + 1) + i + 1, (j + 1) * (n + 1) + i + 2
            for tri in ((a, c, b), (b, c, d)):
                lines.append("f %d %d %d" % tri)
                lines.append("f %d %d %d" % tri)   # the duplicate
    (tmp_path / "dup_grid.obj").write_text("\n".join(lines) + "\n")
    scene = tmp_path / "dup.rtxscene"
    scene.write_text("camera 0 3 -7 45\nmaterial lambert 1 1 1 1\nmaterial lambert 0.49 0.57 0.57 1\n"
                     "mesh dup_grid 1 back\nplane 0 0 0 0 1 0 2\nlight point 0 5 -2 50 1 0.61 0.45\n"
                     "light point -3 4 1 40 1 0.8 0.45\n")
    hs = HostScene(f"file:{scene}", asset_dir=str(tmp_path))
    s, cam = hs.view()
    for mode in (3, 0):
        _check(cull_ctx, plain_ctx, s, cam, abi.make_params(256, 192, mode, 1), f"dup/m{mode}", True)


# ---------------------------------------------------------------- W4_Optional and light anchors
def _optional_geometry():
    hs = HostScene("W4_Optional")
    a = hs.arrays()["meshes"][0]
    P = a["tpositions"].reshape(-1, 3)
    I = a["indices"].reshape(-1, 3)
    N = a["tnormals"].reshape(-1, 3)
    return P, I, N


def _optional_cameras():
    P, I, _ = _optional_geometry()
    v0, v1, v2 = P[I[1234, 0]], P[I[1234, 1]], P[I[1234, 2]]
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    in_plane = (v0 + np.float32(3.0) * e1 - np.float32(2.0) * e2).astype(np.float32)
    lo, hi = P.min(0), P.max(0)
    mid = (0.5 * (lo + hi)).astype(np.float32)
    return [
        ("reference", (0.0, 2.0, -9.0), 45.0, 0.0, 0.0),
        ("in_a_triangle_plane", tuple(float(x) for x in in_plane), 60.0, -0.3, 0.4),
        ("at_a_vertex", tuple(float(x) for x in v0), 70.0, -0.2, 0.5),
        ("inside_the_mesh", tuple(float(x) for x in mid), 90.0, 0.1, 0.0),
        ("grazing_the_top", (float(mid[0]), float(hi[1]) + 1e-3, float(lo[2]) - 2.0), 40.0, -0.0005, 0.0),
        ("grazing_a_side", (float(hi[0]) + 1e-3, float(mid[1]), float(lo[2]) - 2.0), 40.0, 0.0, 0.0005),
    ]


@pytest.mark.parametrize("cam_case", _optional_cameras(), ids=lambda c: c[0])
def test_cull_adversarial_cameras_optional(cull_ctx, plain_ctx, cam_case):
    """W4_Optional (the other scene the product culls: Cook-Torrance, the irregular Assignment3D1
    mesh with slivers) from cameras in a triangle's plane, at a vertex, inside the mesh and
    grazing it.  Combined mode: bit for bit against the unculled walk, within 1e-4 of the oracle;
    ObservedArea (no powf): bit for bit against the oracle too."""
    what, origin, fov, pitch, yaw = cam_case
    hs = HostScene("W4_Optional")
    hs.set_camera(origin, fov, pitch, yaw)
    s, cam = hs.view()
    _check(cull_ctx, plain_ctx, s, cam, abi.make_params(240, 160), what, False)
    _check(cull_ctx, plain_ctx, s, cam, abi.make_params(240, 160, 0, 1), what + "/observed", True)


def _light_cases():
    P, I, N = _optional_geometry()
    k = 2021
    v0, v1, v2 = P[I[k, 0]], P[I[k, 1]], P[I[k, 2]]
    e1, e2 = (v1 - v0).astype(np.float32), (v2 - v0).astype(np.float32)
    n = N[k] / np.linalg.norm(N[k])
    cen = ((v0 + v1 + v2) / np.float32(3)).astype(np.float32)
    # the centre pixel's shadow-ray origin for a camera at (0, 6, -5) looking along +z: the back
    # wall (z = 10, normal -z) hit at (0, 6, 10), offset by 0.0001f along the normal
    on_origin = (0.0, 6.0, float(np.float32(10.0) - np.float32(0.0001)))
    return [
        ("in_a_triangle_plane", tuple(float(x) for x in (v0 + np.float32(3) * e1 - np.float32(2) * e2))),
        ("1e-3_from_a_face", tuple(float(x) for x in (cen + np.float32(1e-3) * n.astype(np.float32)))),
        ("on_a_vertex", tuple(float(x) for x in v0)),
        ("next_to_the_mesh", tuple(float(x) for x in (cen + np.float32(0.05) * n.astype(np.float32)))),
        ("on_a_shadow_origin", on_origin),
    ]


@pytest.mark.parametrize("light_case", _light_cases(), ids=lambda c: c[0])
def test_cull_adversarial_lights(cull_ctx, plain_ctx, light_case):
    """The light-anchor bound (rtx_cull_light_bounds) at its edges: a point light in a mesh
    triangle's plane, 1e-3 from a face, on a vertex, next to the mesh (its cull bound T = 4 x the
    farthest mesh-box corner + 1 is small, so shadow rays from the walls are longer than T and must
    pass unculled), and exactly on the centre pixel's shadow-ray origin (|L - o| = 0, outside the
    bound's domain).  Light 0 of W4_Optional moves there; the camera looks at the mesh (and, for
    the last case, at the back wall along +z with an odd-sized frame so the centre ray is exactly
    +z).  Bit for bit against the unculled walk, ObservedArea bit for bit against the oracle."""
    what, L = light_case
    hs = HostScene("W4_Optional")
    if what == "on_a_shadow_origin":
        hs.set_camera((0.0, 6.0, -5.0), 45.0, 0.0, 0.0)
        W, H = 161, 121
    else:
        W, H = 240, 160
    s, cam = hs.view()
    for k in range(3):
        s.lights[0].origin[k] = L[k]
    if what == "on_a_shadow_origin":
        assert tuple(cam.forward) == (0.0, 0.0, 1.0)
    _check(cull_ctx, plain_ctx, s, cam, abi.make_params(W, H), what, False)
    _check(cull_ctx, plain_ctx, s, cam, abi.make_params(W, H, 0, 1), what + "/observed", True)
    ok = C.c_uint32()
    abi.check(cull_ctx.lib.rtx_cull_info(cull_ctx.h, C.byref(ok), None), "info", cull_ctx.h)
    assert ok.value == 1


@pytest.fixture(scope="module")
def split_cull_ctx():
    """The cull with every tile split (RTX_SPLIT=force) into few parts: the closest hit is the
    minimum of the parts' (t, triangle) keys (PHASE 1)."""
    ctx = _ctx_env(RTX_CULL_MIN_SA="0", RTX_CULL_RATIO="0", RTX_SPLIT="force", RTX_SPLIT_PARTS="8")
    yield ctx
    ctx.close()


@pytest.mark.parametrize("split", [False, True])
def test_cull_ordered_walk_tie_break_is_observable(cull_ctx, split_cull_ctx, plain_ctx, tmp_path, split):
    """The tie test above cannot see a wrong tie-break: duplicate faces shade identically.  Here
    each duplicate pair gets DIFFERENT normals (the stored per-triangle normals are a separate
    input; the copy's is tilted, same side as the original's so back-face culling is unchanged
    for the view), so the pixel shows which triangle won.  The frame must equal the unculled walk's
    and the oracle's, and must differ from the oracle's frame with each pair's normals swapped —
    what a walk resolving ties to the higher index would show."""
    rng = np.random.default_rng(11)
    n = 20
    lines = []
    for j in range(n + 1):
        for i in range(n + 1):
            lines.append(f"v {-2 + 4 * i / n:.6f} {0.2 + 0.6 * rng.random():.6f} {-1 + 3 * j / n:.6f}")
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i + 1, j * (n + 1) + i + 2, (j + 1) * (n + 1) + i + 1, (j + 1) * (n + 1) + i + 2
            for tri in ((a, c, b), (b, c, d)):
                lines.append("f %d %d %d" % tri)
                lines.append("f %d %d %d" % tri)
    (tmp_path / "dup_grid.obj").write_text("\n".join(lines) + "\n")
    scene = tmp_path / "dup.rtxscene"
    scene.write_text("camera 0 3 -7 45\nmaterial lambert 1 1 1 1\nmaterial lambert 0.49 0.57 0.57 1\n"
                     "mesh dup_grid 1 back\nplane 0 0 0 0 1 0 2\nlight point 0 5 -2 50 1 0.61 0.45\n"
                     "light point -3 4 1 40 1 0.8 0.45\n")
    hs = HostScene(f"file:{scene}", asset_dir=str(tmp_path))
    s, cam = hs.view()
    m = s.meshes[0]
    nt = m.n_indices // 3
    idx = np.ctypeslib.as_array(m.indices, shape=(3 * nt,)).reshape(-1, 3)
    nrm = np.ctypeslib.as_array(m.normals, shape=(3 * nt,)).reshape(-1, 3).copy()
    # duplicate pairs in the BVH's (permuted) triangle order
    first = {}
    pairs = []
    for t in range(nt):
        key = tuple(idx[t])
        if key in first:
            pairs.append((first.pop(key), t))
        else:
            first[key] = t
    assert len(pairs) == nt // 2
    tilted = nrm.copy()
    for lo, hi in pairs:   # the later copy's normal tilted ~25 degrees about x
        x, y, z = nrm[hi]
        c, sn = np.float32(0.906), np.float32(0.423)
        tilted[hi] = (x, y * c - z * sn, y * sn + z * c)

    def with_normals(arr):
        buf = np.ascontiguousarray(arr.astype(np.float32).reshape(-1))
        mm = abi.Mesh()
        C.memmove(C.byref(mm), C.byref(m), C.sizeof(abi.Mesh))
        mm.normals = buf.ctypes.data_as(C.POINTER(C.c_float))
        sc = abi.Scene()
        C.memmove(C.byref(sc), C.byref(s), C.sizeof(abi.Scene))
        marr = (abi.Mesh * 1)(mm)
        sc.meshes = C.cast(marr, C.POINTER(abi.Mesh))
        sc._keep = (buf, marr, s)
        return sc

    sA = with_normals(tilted)
    swapped = tilted.copy()
    for lo, hi in pairs:
        swapped[[lo, hi]] = swapped[[hi, lo]]
    sB = with_normals(swapped)
    p = abi.make_params(256, 192, 0, 1)   # ObservedArea: the normal shows directly
    _check(split_cull_ctx if split else cull_ctx, plain_ctx, sA, cam, p, "tilted duplicates", True)
    if split:
        assert split_cull_ctx.split_info()[0] > 0, "the split frames must have run"
    ra = oracle_bind.render(sA, cam, p)[0]
    rb = oracle_bind.render(sB, cam, p)[0]
    assert (ra != rb).sum() > 1000, "the swapped tie-break must be visible"


# ---------------------------------------------------------------- executed work (rtx_count_work_culled)
def _counts(ctx, s, cam, p, culled):
    ctx.upload(s)
    fn = ctx.lib.rtx_count_work_culled if culled else ctx.lib.rtx_count_work_ex
    out = (C.c_uint64 * 15)()
    abi.check(fn(ctx.h, C.byref(cam), C.byref(p), out, 15), "count", ctx.h)
    return np.array(list(out), np.uint64)


@pytest.mark.parametrize("name", ["Synthetic100k", "W4_Optional", "W4_Bunny"])
def test_executed_work_counts(product_ctx, name):
    """The culled walk's counting variant (bench.py's roofline.frac on the culled lines): every counter
    outside the BVH walk equals the reference traversal's count (same rays, hits, shadows,
    shading), the culled walk tests at most the reference's triangles, and for Synthetic100k it
    executes a small fraction of the reference's slab and triangle tests (the CPU cost model,
    tools/cull_probe.c: 0.066 and 0.015).  A scene without records counts exactly as
    rtx_count_work_ex."""
    hs = HostScene(name)
    s, cam = hs.view()
    p = abi.make_params(320, 180)
    ref = _counts(product_ctx, s, cam, p, False)
    got = _counts(product_ctx, s, cam, p, True)
    walk = [3, 4, 12, 13, 14]   # slab, tri, per-wave steps, cull tests
    same = [k for k in range(12) if k not in walk]
    assert np.array_equal(got[same], ref[same]), (got, ref)
    if not product_ctx.cull_info()[0]:
        assert np.array_equal(got, ref)
        return
    assert got[14] > 0 and got[4] <= ref[4], (got, ref)
    if name == "Synthetic100k":
        assert got[3] < 0.25 * ref[3] and got[4] < 0.1 * ref[4], (got[3] / ref[3], got[4] / ref[4])


@pytest.mark.parametrize("top", ["lds", "global"])
def test_cull_records_across_uploads(top):
    """The record trees hand their workgroup roots to the last workgroup inside the launch, across
    XCDs whose L2s are not coherent; a stale line shows only with warm caches and uneven load.  One
    context alternates uploads of different scenes and states (the same tree scratch rewritten
    each time, frames rendered in between) and after every upload the camera and light records
    must equal the brute-force fold (tools/cull_records_ref.c)."""
    env = {"RTX_CULL_MIN_SA": "0"}
    if top == "global":
        env["RTX_CULL_TOP_LDS"] = "0"
    ctx = _ctx_env(**env)
    ref = _records_ref()
    try:
        seq = [("W4_Optional", -1.0), ("Synthetic100k", -1.0), ("W4_Optional", 1.3), ("W4_Optional", 2.9),
               ("Synthetic100k", -1.0), ("W4_Optional", 0.4)]
        for k, (name, t) in enumerate(seq):
            hs = HostScene(name)
            if t >= 0:
                hs.update(t)
            s, cam = hs.view()
            ctx.upload(s)
            p = abi.make_params(320, 180)
            for _ in range(2):
                ctx.render_async(cam, p)
            ctx.synchronize()
            for j in (0, 8 + k % s.n_lights):
                a, rec, rng, nodes, tris, nt = _dump(ctx, j)
                want = np.zeros_like(rec)
                ref.cull_records_ref(len(rng) // 2, nt, rng.ctypes.data, nodes.ctypes.data, tris.ctypes.data,
                                     a.ctypes.data, 1.5, 0, want.ctypes.data)
                r8, w8 = rec.reshape(-1, 8), want.reshape(-1, 8)
                bad = np.nonzero(~np.all((r8[:, :7] == w8[:, :7]) & (r8[:, 7:].view(np.uint32) ==
                                                                     w8[:, 7:].view(np.uint32)), axis=1))[0]
                assert bad.size == 0, f"upload {k} ({name}@{t}) anchor {j}: {bad.size} records differ, slot {bad[0]}"
    finally:
        ctx.close()


@pytest.mark.parametrize("fail_at", ["1", "2"])
def test_failed_record_build_renders_unculled(plain_ctx, fail_at):
    """A record build that fails (RTX_CULL_FAIL=k injects the k-th build's failure: an allocation in a
    real run) turns the cull off for the image before any frame can read records that were never
    written: that frame and every later one render the reference's full traversal.
    k = 1: the upload's build (boxes, lights, camera); k = 2: a camera move's rebuild."""
    ctx = _ctx_env(RTX_CULL_FAIL=fail_at, RTX_CULL_ANIMATED="1")
    try:
        hs = HostScene("Synthetic100k")
        s, cam = hs.view()
        p = abi.make_params(320, 180)
        ctx.upload(s)
        plain_ctx.upload(s)
        assert ctx.cull_info()[0]
        frames = []
        for k in range(4):
            c2 = abi.Camera()
            C.memmove(C.byref(c2), C.byref(cam), C.sizeof(abi.Camera))
            c2.origin[0] = cam.origin[0] + (0.05 if k >= 2 else 0.0)   # frame 3: a camera move
            frames.append((c2, ctx.render(c2, p)))
        assert not ctx.cull_info()[0], "the failed build must turn the cull off for the image"
        for k, (c2, g) in enumerate(frames):
            _same(g, plain_ctx.render(c2, p), f"frame {k} after an injected failure at build {fail_at}")
    finally:
        ctx.close()
