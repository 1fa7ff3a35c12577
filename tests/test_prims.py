"""Known-answer vectors of the reference's primitive functions (GeometryUtils::HitTest_*,
SlabTest_BVH, Material::Shade), captured from the reference build, against the oracle."""
from pathlib import Path

import ctypes as C
import numpy as np

import oracle_bind
from gp1_raytracer_2223_amd import abi

G = np.load(Path(__file__).resolve().parent / "golden" / "prims.npz")
F = oracle_bind.fptr


def _rows(name, w):
    return G[name].reshape(-1, w).astype(np.float32)


def _eq(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_sphere_plane_triangle_slab():
    L = oracle_bind.lib()
    rays, sph, pl, tri = _rows("rays", 8), _rows("spheres", 4), _rows("planes", 6), _rows("triangles", 12)
    cull, aabb = G["tri_cull"], _rows("aabbs", 6)
    exp_s, exp_p, exp_t = _rows("sphere_hit", 8), _rows("plane_hit", 8), _rows("tri_hit", 8)
    out = np.zeros(8, np.float32)
    bad = []
    for i in range(len(rays)):
        r = np.ascontiguousarray(rays[i])
        for fn, prim, exp, anyv in ((L.rtx_oracle_hit_sphere, sph, exp_s, G["sphere_any"]),
                                    (L.rtx_oracle_hit_plane, pl, exp_p, G["plane_any"])):
            hit = fn(F(r), F(np.ascontiguousarray(prim[i])), 0, F(out))
            if hit and not _eq(out, exp[i]) or bool(hit) != bool(exp[i, 0]):
                bad.append((fn.__name__, i))
            if bool(fn(F(r), F(np.ascontiguousarray(prim[i])), 1, F(out))) != bool(anyv[i]):
                bad.append((fn.__name__ + "/any", i))
        hit = L.rtx_oracle_hit_triangle(F(r), F(np.ascontiguousarray(tri[i])), int(cull[i]), 0, F(out))
        if bool(hit) != bool(exp_t[i, 0]) or (hit and not _eq(out, exp_t[i])):
            bad.append(("tri", i))
        if bool(L.rtx_oracle_hit_triangle(F(r), F(np.ascontiguousarray(tri[i])), int(cull[i]), 1, F(out))) != \
                bool(G["tri_any"][i]):
            bad.append(("tri/any", i))
        if bool(L.rtx_oracle_slab(F(r), F(np.ascontiguousarray(aabb[i])))) != bool(G["slab"][i]):
            bad.append(("slab", i))
    assert not bad, bad[:10]
    # the vectors exercise both outcomes of every test
    for k in ("sphere_any", "plane_any", "tri_any", "slab"):
        assert 0 < G[k].sum() < len(G[k]), k


def test_shade_materials():
    L = oracle_bind.lib()
    kinds, ins, outs = G["shade_kind"], _rows("shade_in", 17), _rows("shade_out", 3)
    o = np.zeros(3, np.float32)
    bad = []
    for i in range(len(kinds)):
        n, l, v = ins[i, 0:3].copy(), ins[i, 3:6].copy(), ins[i, 6:9].copy()
        m = abi.Material()
        m.kind = int(kinds[i])
        m.color[0], m.color[1], m.color[2] = map(float, ins[i, 9:12])
        m.kd, m.ks, m.exponent, m.metalness, m.roughness = map(float, ins[i, 12:17])
        L.rtx_oracle_shade(C.byref(m), F(n), F(l), F(v), F(o))
        if not _eq(o, outs[i]):
            bad.append((i, int(kinds[i]), o.tolist(), outs[i].tolist()))
    assert not bad, bad[:5]
