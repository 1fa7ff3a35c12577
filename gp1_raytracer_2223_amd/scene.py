"""Python handle on the C++ host scene layer (include/rtx_host.h).

`HostScene("W4_Bunny")` is Scene_W4_BunnyScene::Initialize() (source/Scene.cpp:402-430);
`.update(t)` is its Update without SDL input; `.view()` returns the flat rtx_scene
(pointers into the C++ object, valid until the next update) and the camera after
CalculateCameraToWorld (source/Camera.h:43-53).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi

SCENES = ["W1", "W2", "W3", "W3_Test", "W4_Test", "W4_Reference", "W4_Bunny", "W4_Optional",
          "Synthetic100k", "Bunny8Lights"]
RENDERABLE = [s for s in SCENES if s != "W4_Test"]
ANIMATED = ["W4_Reference", "W4_Bunny", "W4_Optional", "Bunny8Lights"]


class HostScene:
    def __init__(self, name: str, asset_dir: str | None = None):
        self._lib = abi.load_host()
        self.name = name
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        ad = str(asset_dir if asset_dir is not None else abi.ASSET_DIR).encode()
        rc = self._lib.rtx_host_scene_create(name.encode(), ad, C.byref(h), err, len(err))
        if rc != abi.RTX_OK:
            raise RuntimeError(f"scene {name!r}: {err.value.decode()} (code {rc})")
        self._h = h
        # bumped by every update(): a Renderer re-uploads when the generation it uploaded
        # differs (value comparison, so a recycled id() can never alias another scene)
        self.generation = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.rtx_host_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, total_time: float) -> None:
        abi.check(self._lib.rtx_host_scene_update(self._h, float(total_time)), "rtx_host_scene_update")
        self.generation += 1

    def copy_state(self, src: "HostScene") -> None:
        """The state src's Updates left (rtx_host_scene_copy_state): a snapshot of ONE Update
        history, as the pipelined frame loop uploads them."""
        abi.check(self._lib.rtx_host_scene_copy_state(self._h, src._h), "rtx_host_scene_copy_state")
        self.generation += 1

    @property
    def animated(self) -> bool:
        """Update(t) moves geometry (re-upload after it)."""
        r = self._lib.rtx_host_scene_animated(self._h)
        if r < 0:
            abi.check(r, "rtx_host_scene_animated")
        return bool(r)

    # ---- device-side Update (rtx_anim_*) ------------------------------------------
    def spinning(self) -> list[int]:
        """Indices of the meshes Update(t) turns."""
        ids = (C.c_int32 * 64)()
        n = self._lib.rtx_host_scene_spinning(self._h, ids, 64)
        if n < 0:
            abi.check(n, "rtx_host_scene_spinning")
        return [int(ids[i]) for i in range(min(n, 64))]

    def mesh_source(self, mesh: int) -> abi.MeshSource:
        """Object-space state of a mesh (pointers into the scene, valid until its next update)."""
        src = abi.MeshSource()
        abi.check(self._lib.rtx_host_scene_mesh_source(self._h, mesh, C.byref(src)), "rtx_host_scene_mesh_source")
        return src

    def transforms(self, total_time: float) -> np.ndarray:
        """Update(t)'s finalTransform per turning mesh (16 floats each) without rebuilding."""
        cap = 64
        out = np.zeros(16 * cap, np.float32)
        n = self._lib.rtx_host_scene_transforms(self._h, float(total_time), out.ctypes.data_as(C.POINTER(C.c_float)),
                                                cap)
        if n < 0:
            abi.check(n, "rtx_host_scene_transforms")
        if n > cap:
            raise RuntimeError(f"{n} turning meshes, more than the {cap} this wrapper holds")
        return out[: 16 * n].copy()

    def set_camera(self, origin, fov_degrees: float = 45.0, pitch: float = 0.0, yaw: float = 0.0) -> None:
        o = (C.c_float * 3)(*origin)
        abi.check(self._lib.rtx_host_camera_set(self._h, o, fov_degrees, pitch, yaw), "rtx_host_camera_set")

    def view(self) -> tuple[abi.Scene, abi.Camera]:
        """The flat scene (pointers into this object's arrays, valid until its next update) and
        the camera.  Both hold a reference to this HostScene, so `HostScene(name).view()` keeps the
        arrays alive as long as the returned Scene (the reference's Scene owns its vectors,
        Scene.h:36-43)."""
        s, cam = abi.Scene(), abi.Camera()
        abi.check(self._lib.rtx_host_scene_view(self._h, C.byref(s), C.byref(cam)), "rtx_host_scene_view")
        s._owner = self
        cam._owner = self
        return s, cam

    # ---- inspection helpers (tests) -----------------------------------------------
    def arrays(self) -> dict:
        """Copy the flattened scene into numpy arrays (same names as the oracle dumps)."""
        s, cam = self.view()
        out: dict = {"camera": np.array(list(cam.origin) + list(cam.right) + list(cam.up) + list(cam.forward)
                                        + [cam.fov], dtype=np.float32)}
        out["spheres"] = np.array([[*s.spheres[i].origin, s.spheres[i].radius] for i in range(s.n_spheres)],
                                  dtype=np.float32).reshape(-1)
        out["sphere_mat"] = np.array([s.spheres[i].material for i in range(s.n_spheres)], dtype=np.uint8)
        out["planes"] = np.array([[*s.planes[i].origin, *s.planes[i].normal] for i in range(s.n_planes)],
                                 dtype=np.float32).reshape(-1)
        out["plane_mat"] = np.array([s.planes[i].material for i in range(s.n_planes)], dtype=np.uint8)
        meshes = []
        for i in range(s.n_meshes):
            m = s.meshes[i]
            nI = m.n_indices
            nodes = np.ctypeslib.as_array(C.cast(m.nodes, C.POINTER(C.c_uint32)), shape=(m.n_nodes * 9,)).copy() \
                if m.n_nodes else np.zeros(0, np.uint32)
            nodes = nodes.reshape(-1, 9)
            meshes.append({
                "tpositions": np.ctypeslib.as_array(m.positions, shape=(m.n_positions * 3,)).copy(),
                "indices": np.ctypeslib.as_array(m.indices, shape=(nI,)).copy(),
                "tnormals": np.ctypeslib.as_array(m.normals, shape=(nI,)).copy(),
                "node_bounds": nodes[:, :6].copy().view(np.float32).reshape(-1),
                "node_links": nodes[:, 6:].copy().reshape(-1),
                "cull": m.cull_mode, "material": m.material,
            })
        out["meshes"] = meshes
        out["lights"] = np.array([[*s.lights[i].origin, *s.lights[i].direction, *s.lights[i].color,
                                   s.lights[i].intensity] for i in range(s.n_lights)], dtype=np.float32).reshape(-1)
        out["light_type"] = np.array([s.lights[i].type for i in range(s.n_lights)], dtype=np.int32)
        out["material_kind"] = np.array([s.materials[i].kind for i in range(s.n_materials)], dtype=np.int32)
        out["material_params"] = np.array([[*s.materials[i].color, s.materials[i].kd, s.materials[i].ks,
                                            s.materials[i].exponent, s.materials[i].metalness,
                                            s.materials[i].roughness] for i in range(s.n_materials)],
                                          dtype=np.float32).reshape(-1)
        return out


def parse_obj(path: str) -> dict:
    """Utils::ParseOBJ through the host library."""
    lib = abi.load_host()
    nv, ni = C.c_uint32(), C.c_uint32()
    rc = lib.rtx_host_parse_obj(str(path).encode(), None, C.byref(nv), None, None, C.byref(ni), 0, 0)
    abi.check(rc, "rtx_host_parse_obj")
    p = np.zeros(nv.value * 3, np.float32)
    n = np.zeros(ni.value, np.float32)
    idx = np.zeros(ni.value, np.int32)
    rc = lib.rtx_host_parse_obj(str(path).encode(), p.ctypes.data_as(C.POINTER(C.c_float)), C.byref(nv),
                                n.ctypes.data_as(C.POINTER(C.c_float)), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                C.byref(ni), nv.value, ni.value)
    abi.check(rc, "rtx_host_parse_obj")
    return {"positions": p, "normals": n, "indices": idx}
