"""Error paths of the C-ABI on a device (include/rtx.h error convention): a malformed scene is
rejected by rtx_upload_scene with RTX_E_INVALID and a reason in rtx_last_error, the context
stays usable (the previous scene keeps rendering), and calls out of order are state errors.
The BVH checks guard the kernel: an out-of-range child or a cycle would walk off the node
array (rtx_hip.hip bvh_depth_check); a tree of any depth is accepted, the kernel variant
chosen by its depth (LDS stacks of 64 or 1,024 entries, or stacks in HBM)."""
import ctypes as C

import numpy as np
import pytest

from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.renderer import DeviceContext
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu


class _Arrays:
    """Keeps the ctypes arrays of a hand-built scene alive."""


def _scene(nodes, n_tris=1, material=0, indices=None, n_materials=1):
    keep = _Arrays()
    pos = [0, 0, 5, 1, 0, 5, 0, 1, 5]
    keep.pos = (C.c_float * len(pos))(*pos)
    idx = indices if indices is not None else [0, 1, 2] * n_tris
    keep.idx = (C.c_int32 * len(idx))(*idx)
    nrm = [0.0, 0.0, -1.0] * (len(idx) // 3)
    keep.nrm = (C.c_float * len(nrm))(*nrm)
    keep.nodes = (abi.BVHNode * len(nodes))()
    for k, (first, count, left) in enumerate(nodes):
        n = keep.nodes[k]
        n.min[:] = [0.0, 0.0, 5.0]
        n.max[:] = [1.0, 1.0, 5.0]
        n.first_idx, n.idx_count, n.left_node = first, count, left
    keep.mesh = (abi.Mesh * 1)()
    m = keep.mesh[0]
    m.positions, m.n_positions = keep.pos, 3
    m.indices, m.n_indices = keep.idx, len(idx)
    m.normals = keep.nrm
    m.nodes, m.n_nodes = keep.nodes, len(nodes)
    m.cull_mode, m.material = abi.RTX_CULL_NONE, material
    keep.light = (abi.Light * 1)()
    keep.light[0].origin[:] = [0.0, 3.0, 0.0]
    keep.light[0].color[:] = [1.0, 1.0, 1.0]
    keep.light[0].intensity = 10.0
    keep.mat = (abi.Material * n_materials)()
    for k in range(n_materials):
        keep.mat[k].kind = abi.RTX_MAT_LAMBERT
        keep.mat[k].color[:] = [1.0, 1.0, 1.0]
        keep.mat[k].kd = 1.0
    s = abi.Scene()
    s.meshes, s.n_meshes = keep.mesh, 1
    s.lights, s.n_lights = keep.light, 1
    s.materials, s.n_materials = keep.mat, n_materials
    s._keep = keep
    return s


def _upload_rc(ctx, s):
    return ctx.lib.rtx_upload_scene(ctx.h, C.byref(s))


def _reason(ctx):
    return (ctx.lib.rtx_last_error(ctx.h) or b"").decode()


@pytest.fixture()
def ctx():
    c = DeviceContext(0)
    yield c
    c.close()


def test_valid_hand_built_scene_uploads(ctx):
    # one leaf holding the triangle: the fixture itself is a valid scene
    assert _upload_rc(ctx, _scene([(0, 3, 0)])) == abi.RTX_OK


@pytest.mark.parametrize("nodes,why", [
    ([(0, 0, 5), (0, 3, 0), (0, 3, 0)], "out of range"),   # children past the node array
    ([(0, 0, 0), (0, 3, 0)], "out of range"),               # child index 0 (the root): a cycle
])
def test_bad_bvh_links_are_rejected(ctx, nodes, why):
    assert _upload_rc(ctx, _scene(nodes)) == abi.RTX_E_INVALID
    assert why in _reason(ctx)


def _chain(depth):
    # a chain: inner node 2k has children 2k+1 (a leaf) and 2k+2 (the next inner node, a leaf
    # at the bottom), so the pending-sibling depth grows by one per level
    nodes = []
    for _ in range(depth):
        nodes.append((0, 0, len(nodes) + 1))   # inner at 2k: children 2k+1, 2k+2
        nodes.append((0, 3, 0))                # leaf at 2k+1
    nodes.append((0, 3, 0))                    # bottom leaf
    return nodes


def test_bvh_deeper_than_the_default_stack_uses_the_deep_variant(ctx):
    # 70 levels > the 64-entry LDS stack: accepted (deep-stack kernel; rendering parity in
    # tests/test_gpu_deep_bvh.py)
    assert _upload_rc(ctx, _scene(_chain(70))) == abi.RTX_OK


def test_bvh_deeper_than_the_deep_stack_uses_hbm_stacks(ctx):
    # 1,030 levels >= the 1,024-entry LDS stack of the deep variant: accepted (stacks in HBM;
    # rendering parity in tests/test_gpu_deep_bvh.py)
    assert _upload_rc(ctx, _scene(_chain(1030))) == abi.RTX_OK, _reason(ctx)
    # a 60-level chain (the default stack) uploads
    assert _upload_rc(ctx, _scene(_chain(60))) == abi.RTX_OK, _reason(ctx)


@pytest.mark.parametrize("kw,why", [
    (dict(material=3), "material out of range"),
    (dict(indices=[0, 1, 7]), "index out of range"),
    (dict(indices=[0, 1]), "multiple of 3"),
])
def test_bad_mesh_records_are_rejected(ctx, kw, why):
    assert _upload_rc(ctx, _scene([(0, 3, 0)], **kw)) == abi.RTX_E_INVALID
    assert why in _reason(ctx)


def test_rejected_upload_keeps_the_previous_scene(ctx):
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    p = abi.make_params(128, 72)
    ctx.upload(s)
    px0, _ = ctx.render(cam, p)
    assert _upload_rc(ctx, _scene([(0, 0, 5), (0, 3, 0), (0, 3, 0)])) == abi.RTX_E_INVALID
    px1, _ = ctx.render(cam, p)
    assert np.array_equal(px0, px1)


def test_calls_out_of_order_are_state_errors(ctx):
    cam = abi.Camera()
    p = abi.make_params(64, 64)
    px = np.zeros(64 * 64, np.uint32)
    out = px.ctypes.data_as(C.POINTER(C.c_uint32))
    assert ctx.lib.rtx_render(ctx.h, C.byref(cam), C.byref(p), out, None) == abi.RTX_E_STATE
    assert "no scene" in _reason(ctx)
    assert ctx.lib.rtx_download(ctx.h, out, None) == abi.RTX_E_STATE
