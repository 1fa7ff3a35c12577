"""BVHs deeper than the default per-wave DFS stack (kStackDepth = 64 entries in LDS) render
with the deep-stack kernel variant (kStackDepthDeep = 1024 entries), and deeper ones with the
variant whose stacks are in HBM (any depth), bit-exact against the oracle.

The reference traverses recursively (Utils.h:246-288) and has no depth limit.  The scenes
here are the Bunny scene's room, lights and camera with the bunny replaced by a mesh whose
hand-built BVH is a chain: every inner node's left child is a one-triangle leaf and its
right child the rest of the chain, so a mesh of T triangles is T-1 levels deep."""
import ctypes as C

import numpy as np
import pytest

import oracle_bind
from gp1_raytracer_2223_amd import abi
from gp1_raytracer_2223_amd.scene import HostScene

pytestmark = pytest.mark.gpu


def chain_mesh(T: int):
    """T small triangles on a staircase in the plane z = 0.5 facing the camera (-z), and a
    chain BVH over them in the reference's node layout (left = leaf k, right = rest)."""
    pos, idx, nrm = [], [], []
    for k in range(T):
        x = -2.0 + 4.0 * k / T
        y = 0.6 + 1.8 * ((k * 37) % T) / T
        s = 4.0 / T + 0.05
        b = len(pos)
        pos += [(x, y, 0.5), (x + s, y, 0.5), (x, y + s, 0.5)]
        idx += [b, b + 2, b + 1]
        nrm.append((0.0, 0.0, -1.0))
    pos = np.array(pos, np.float32)
    idx = np.array(idx, np.int32)
    nrm = np.array(nrm, np.float32)
    tri_lo = pos[idx.reshape(-1, 3)].min(axis=1)
    tri_hi = pos[idx.reshape(-1, 3)].max(axis=1)
    nodes = (abi.BVHNode * (2 * T - 1))()

    def setbox(n, lo, hi):
        for a in range(3):
            nodes[n].min[a] = float(lo[a])
            nodes[n].max[a] = float(hi[a])

    # inner node i (i = 0, 2, 4, ...) covers triangles k..T-1 with k = i / 2
    for k in range(T - 1):
        inner = 2 * k
        setbox(inner, tri_lo[k:].min(axis=0), tri_hi[k:].max(axis=0))
        nodes[inner].first_idx, nodes[inner].idx_count, nodes[inner].left_node = 0, 0, inner + 1
        leaf = inner + 1
        setbox(leaf, tri_lo[k], tri_hi[k])
        nodes[leaf].first_idx, nodes[leaf].idx_count, nodes[leaf].left_node = 3 * k, 3, 0
    last = 2 * (T - 1)   # the chain's last right child: a leaf with the last triangle
    setbox(last, tri_lo[T - 1], tri_hi[T - 1])
    nodes[last].first_idx, nodes[last].idx_count, nodes[last].left_node = 3 * (T - 1), 3, 0
    return pos, idx, nrm, nodes


def deep_scene(T: int):
    hs = HostScene("W4_Bunny")
    base, cam = hs.view()
    pos, idx, nrm, nodes = chain_mesh(T)
    m = abi.Mesh()
    m.positions = pos.ctypes.data_as(C.POINTER(C.c_float))
    m.n_positions = len(pos)
    m.indices = idx.ctypes.data_as(C.POINTER(C.c_int32))
    m.n_indices = len(idx)
    m.normals = nrm.ctypes.data_as(C.POINTER(C.c_float))
    m.nodes = nodes
    m.n_nodes = len(nodes)
    m.cull_mode = abi.RTX_CULL_NONE
    m.material = 2
    meshes = (abi.Mesh * 1)(m)
    s = abi.Scene()
    s.spheres, s.n_spheres = base.spheres, base.n_spheres
    s.planes, s.n_planes = base.planes, base.n_planes
    s.lights, s.n_lights = base.lights, base.n_lights
    s.materials, s.n_materials = base.materials, base.n_materials
    s.meshes, s.n_meshes = meshes, 1
    keep = (hs, pos, idx, nrm, nodes, meshes)   # everything the pointers refer to
    return s, cam, keep


@pytest.mark.parametrize("T", [40, 65, 300, 1000, 1100, 2500])
def test_deep_bvh_renders_bit_exact(gpu_ctx, T):
    s, cam, keep = deep_scene(T)
    gpu_ctx.upload(s)
    for mode, sh in [(3, 1), (0, 1)]:
        p = abi.make_params(320, 180, mode, sh)
        gpx, grgb = gpu_ctx.render(cam, p)
        rpx, rrgb = oracle_bind.render(s, cam, p)
        assert np.array_equal(gpx, rpx), f"T={T}: {(gpx != rpx).sum()} pixels differ"
        assert np.array_equal(grgb.view(np.uint32), rrgb.view(np.uint32))
    assert (gpx != gpx[0]).any()   # the mesh is in view
    p = abi.make_params(160, 90)
    assert np.array_equal(gpu_ctx.count_work(cam, p), oracle_bind.count(s, cam, p))
    del keep


def test_hbm_stack_variant_serves_frames_of_any_size(gpu_ctx):
    """The HBM stacks grow with the frame (one stack per wave of the launch): a larger frame
    after a smaller one, and the smaller one again, both equal the oracle."""
    s, cam, keep = deep_scene(1500)
    gpu_ctx.upload(s)
    for w, h in [(96, 64), (400, 224), (96, 64)]:
        p = abi.make_params(w, h)
        gpx, _ = gpu_ctx.render(cam, p)
        rpx, _ = oracle_bind.render(s, cam, p)
        assert np.array_equal(gpx, rpx), f"{w}x{h}"
    del keep


def test_hbm_stack_limit_is_frame_size_times_depth(gpu_ctx):
    """The HBM stacks take (depth + 1) x 24 B for every wave of the launch:
    a 25,000-level chain needs 0.6 GB at 64 x 32 but 77.8 GB at 3840 x 2160, past the 64 GiB cap,
    so the 4K frame is refused with RTX_E_UNSUPPORTED before anything is allocated, and the
    context still renders the small frame bit-exact afterwards."""
    s, cam, keep = deep_scene(25000)
    gpu_ctx.upload(s)
    small = abi.make_params(64, 32)
    rpx, _ = oracle_bind.render(s, cam, small)
    gpx, _ = gpu_ctx.render(cam, small)
    assert np.array_equal(gpx, rpx)
    px = np.zeros(3840 * 2160, np.uint32)
    rc = gpu_ctx.lib.rtx_render(gpu_ctx.h, C.byref(cam), C.byref(abi.make_params(3840, 2160)),
                                px.ctypes.data_as(C.POINTER(C.c_uint32)), None)
    assert rc == abi.RTX_E_UNSUPPORTED
    assert b"exceed 64 GB" in gpu_ctx.lib.rtx_last_error(gpu_ctx.h)
    gpx, _ = gpu_ctx.render(cam, small)
    assert np.array_equal(gpx, rpx)
    del keep
