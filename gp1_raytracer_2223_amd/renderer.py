"""Python mirror of dae::Renderer (source/Renderer.h:17-61) over the HIP C-ABI.

    r = Renderer(1920, 1080)            # Renderer(SDL_Window*): width/height of the surface
    r.Render(scene)                     # Renderer::Render(Scene*) -> fills r.buffer (uint32 XRGB)
    r.CycleLightingMode(); r.ToggleShadows(); r.SaveBufferToImage("out.bmp")

Multi-GPU: `Renderer(..., device=rank, stripe=(16, rank, world))` renders only the
16-row stripes this rank owns (rows of stripe s with s % world == rank); stitching the
ranks' buffers gives the single-GPU image bit for bit.

There is no CPU fallback: if librtx_hip.so or the GPU is missing this raises.
"""
from __future__ import annotations

import ctypes as C
import struct
import weakref

import numpy as np

from . import abi
from .scene import HostScene


class LightingMode:
    ObservedArea, Radiance, BRDF, Combined, Count = 0, 1, 2, 3, 4


class DeviceContext:
    """Owns one rtx_ctx (one GPU) and its uploaded scene."""

    def __init__(self, device: int = 0):
        self.lib = abi.load_hip()
        h = C.c_void_p()
        rc = self.lib.rtx_create(C.byref(h), int(device))
        if rc != abi.RTX_OK:
            why = (self.lib.rtx_last_error(None) or b"").decode(errors="replace")
            raise RuntimeError(f"rtx_create(device={device}) failed with code {rc}: {why or 'no usable HIP device?'}")
        self.h = h
        self.device = device
        self._uploaded = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.rtx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: abi.Scene) -> None:
        abi.check(self.lib.rtx_upload_scene(self.h, C.byref(scene)), "rtx_upload_scene", self.h)

    def render(self, cam: abi.Camera, params: abi.RenderParams, want_rgb: bool = True):
        n = params.width * params.height
        px = np.zeros(n, np.uint32)
        rgb = np.zeros(3 * n, np.float32) if want_rgb else None
        rc = self.lib.rtx_render(self.h, C.byref(cam), C.byref(params),
                                 px.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 rgb.ctypes.data_as(C.POINTER(C.c_float)) if want_rgb else None)
        abi.check(rc, "rtx_render", self.h)
        return px, rgb

    def render_async(self, cam, params, want_rgb=False):
        abi.check(self.lib.rtx_render_async(self.h, C.byref(cam), C.byref(params), int(want_rgb)),
                  "rtx_render_async", self.h)

    def synchronize(self):
        abi.check(self.lib.rtx_synchronize(self.h), "rtx_synchronize", self.h)

    def gather_async(self, out_px: np.ndarray, out_rgb: np.ndarray | None = None) -> None:
        """Queue the D2H copy of the rows the last render owns into full-frame host arrays
        (rtx_gather_async); complete after synchronize()."""
        assert out_px.dtype == np.uint32 and out_px.flags.c_contiguous
        rgbp = None
        if out_rgb is not None:
            assert out_rgb.dtype == np.float32 and out_rgb.flags.c_contiguous
            rgbp = out_rgb.ctypes.data_as(C.POINTER(C.c_float))
        abi.check(self.lib.rtx_gather_async(self.h, out_px.ctypes.data_as(C.POINTER(C.c_uint32)), rgbp),
                  "rtx_gather_async", self.h)

    def time_frames(self, cam, params, iters: int) -> float:
        ms = C.c_float()
        abi.check(self.lib.rtx_time_frames(self.h, C.byref(cam), C.byref(params), int(iters), C.byref(ms)),
                  "rtx_time_frames", self.h)
        return ms.value

    def split_info(self) -> tuple[int, int]:
        """(heavy tiles the next frame splits, BVH frontier parts of the scene)."""
        h, p = C.c_uint32(), C.c_uint32()
        abi.check(self.lib.rtx_split_info(self.h, C.byref(h), C.byref(p)), "rtx_split_info", self.h)
        return h.value, p.value

    def split_tune_info(self) -> dict:
        """The split threshold's tuner: factor, last timed main kernel / split chain (ms), state."""
        f, m, ch, d = C.c_float(), C.c_float(), C.c_float(), C.c_uint32()
        abi.check(self.lib.rtx_split_tune_info(self.h, C.byref(f), C.byref(m), C.byref(ch), C.byref(d)),
                  "rtx_split_tune_info", self.h)
        return {"factor": round(f.value, 4), "main_ms": round(m.value, 5), "chain_ms": round(ch.value, 5),
                "state": ["tuning", "converged", "off"][d.value]}

    def inflight_info(self) -> dict:
        """Frames in flight: the last frame saw another context's frame in flight / rendered one piece
        for it; the heaviest tile's serialized time over the split frame's serialized span, the
        threshold, and the split frames' interval in flight on this context's stream (ms)."""
        a, b, r, t, w = C.c_uint32(), C.c_uint32(), C.c_float(), C.c_float(), C.c_float()
        abi.check(self.lib.rtx_inflight_info(self.h, C.byref(a), C.byref(b), C.byref(r), C.byref(t), C.byref(w)),
                  "rtx_inflight_info", self.h)
        return {"concurrent": bool(a.value), "onepiece": bool(b.value), "crit": round(r.value, 3),
                "threshold": round(t.value, 3), "split_interval_ms": round(w.value, 5)}

    def light_major_info(self) -> tuple[bool, int]:
        """(the last prepared frame was light-major, the largest light-major launch in wave tiles)."""
        a, b = C.c_uint32(), C.c_uint32()
        abi.check(self.lib.rtx_light_major_info(self.h, C.byref(a), C.byref(b)), "rtx_light_major_info", self.h)
        return bool(a.value), int(b.value)

    def cull_info(self) -> tuple[bool, int]:
        """(the uploaded scene renders with the exact cull, camera-record rebuilds so far)."""
        on, n = C.c_uint32(), C.c_uint64()
        abi.check(self.lib.rtx_cull_info(self.h, C.byref(on), C.byref(n)), "rtx_cull_info", self.h)
        return bool(on.value), n.value

    def count_work(self, cam, params) -> np.ndarray:
        out = (C.c_uint64 * 12)()
        abi.check(self.lib.rtx_count_work(self.h, C.byref(cam), C.byref(params), out), "rtx_count_work", self.h)
        return np.array(list(out), dtype=np.uint64)

    def count_work_culled(self, cam, params) -> np.ndarray:
        """The 15 counters of the walk the product executes (rtx_count_work_culled): the 12 model
        counters, per-wave node-pair and triangle steps, exact-cull box tests."""
        out = (C.c_uint64 * 15)()
        abi.check(self.lib.rtx_count_work_culled(self.h, C.byref(cam), C.byref(params), out, 15),
                  "rtx_count_work_culled", self.h)
        return np.array(list(out), dtype=np.uint64)


class DeviceGroup:
    """Owns one rtx_group: one frame tiled over several contexts (GPUs) by this process,
    each member with its own host thread and stream gathering its 16-row stripes into
    one host frame (include/rtx.h)."""

    def __init__(self, devices):
        self.lib = abi.load_hip()
        ids = (C.c_int * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        rc = self.lib.rtx_group_create(C.byref(h), ids, len(devices))
        if rc != abi.RTX_OK:
            why = (self.lib.rtx_group_last_error(None) or b"").decode(errors="replace")
            raise RuntimeError(f"rtx_group_create({list(devices)}) failed with code {rc}: {why}")
        self.h = h
        self.devices = list(devices)

    def _check(self, rc, what):
        if rc != abi.RTX_OK:
            why = (self.lib.rtx_group_last_error(self.h) or b"").decode(errors="replace")
            raise RuntimeError(f"{what} failed with code {rc}: {why}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.rtx_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: abi.Scene) -> None:
        self._check(self.lib.rtx_group_upload_scene(self.h, C.byref(scene)), "rtx_group_upload_scene")

    def render(self, cam: abi.Camera, params: abi.RenderParams, want_rgb: bool = True, out_px=None):
        n = params.width * params.height
        px = np.zeros(n, np.uint32) if out_px is None else out_px
        rgb = np.zeros(3 * n, np.float32) if want_rgb else None
        rc = self.lib.rtx_group_render(self.h, C.byref(cam), C.byref(params),
                                       px.ctypes.data_as(C.POINTER(C.c_uint32)),
                                       rgb.ctypes.data_as(C.POINTER(C.c_float)) if want_rgb else None)
        self._check(rc, "rtx_group_render")
        return px, rgb


class DeviceAnimation:
    """Owns one rtx_anim: Scene::Update of a host scene's turning meshes done on the device
    (transform, the reference's binned-SAH rebuild, scene image) — SURVEY §8(f)1.
    `DeviceAnimation(scene, ctx)` registers the scene's current state and uploads it to
    `ctx`; `update(t, ctx)` queues Update(t) into `ctx`'s scene image."""

    def __init__(self, scene, ctx: DeviceContext):
        self.lib = abi.load_hip()
        self.scene = scene
        ids = scene.spinning()
        if not ids:
            raise ValueError(f"scene {scene.name!r} has no turning mesh")
        s, _ = scene.view()
        srcs = (abi.MeshSource * len(ids))(*[scene.mesh_source(i) for i in ids])
        cids = (C.c_int32 * len(ids))(*ids)
        h = C.c_void_p()
        rc = self.lib.rtx_anim_create(C.byref(h), ctx.h, C.byref(s), cids, srcs, len(ids))
        if rc != abi.RTX_OK:
            why = (self.lib.rtx_anim_last_error(None) or b"").decode(errors="replace")
            raise RuntimeError(f"rtx_anim_create failed with code {rc}: {why}")
        self.h = h
        self.mesh_ids = list(ids)
        self.n_tris = [s.meshes[i].n_indices // 3 for i in ids]
        self.n_positions = [s.meshes[i].n_positions for i in ids]

    def _check(self, rc, what):
        if rc != abi.RTX_OK:
            why = (self.lib.rtx_anim_last_error(self.h) or b"").decode(errors="replace")
            raise RuntimeError(f"{what} failed with code {rc}: {why}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.rtx_anim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, total_time: float, ctx: DeviceContext) -> None:
        m = self.scene.transforms(total_time)
        self._check(self.lib.rtx_anim_update(self.h, ctx.h, m.ctypes.data_as(C.POINTER(C.c_float))),
                    "rtx_anim_update")

    def status(self, i: int = 0) -> np.ndarray:
        st = (C.c_uint32 * 4)()
        self._check(self.lib.rtx_anim_status(self.h, i, st), "rtx_anim_status")
        return np.array(list(st), np.uint32)

    def stamps(self, i: int = 0) -> np.ndarray:
        """The last update's 128 status words of registered mesh i (rtx_anim.h: errors, counts,
        phase stamps, completeness word 28); no error check."""
        out = (C.c_uint32 * 128)()
        self._check(self.lib.rtx_anim_stamps(self.h, i, out), "rtx_anim_stamps")
        return np.array(list(out), np.uint32)

    def download(self, i: int = 0) -> dict:
        """Registered mesh i in the reference's form (TriangleMesh after UpdateTransforms)."""
        T, V = self.n_tris[i], self.n_positions[i]
        pos = np.zeros(3 * V, np.float32)
        idx = np.zeros(3 * T, np.int32)
        nrm = np.zeros(3 * T, np.float32)
        tn = np.zeros(3 * T, np.float32)
        nodes = (abi.BVHNode * (3 * T))()
        f = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        self._check(self.lib.rtx_anim_download(self.h, i, f(pos), idx.ctypes.data_as(C.POINTER(C.c_int32)), f(nrm),
                                               f(tn), nodes), "rtx_anim_download")
        raw = np.ctypeslib.as_array(C.cast(nodes, C.POINTER(C.c_uint32)), shape=(3 * T * 9,)).copy().reshape(-1, 9)
        return {"tpositions": pos, "indices": idx, "normals": nrm, "tnormals": tn, "nodes": raw}


class Renderer:
    def __init__(self, width: int, height: int, device: int = 0, stripe: tuple[int, int, int] | None = None,
                 pixel_format=abi.XRGB8888):
        self.m_Width, self.m_Height = int(width), int(height)
        self.m_AspectRatio = self.m_Width / float(self.m_Height)
        self.m_CurrentLightingMode = LightingMode.Combined
        self.m_ShadowsEnabled = True
        self.stripe = stripe
        self.format = pixel_format
        self.ctx = DeviceContext(device)
        self._scene_ref = None    # weakref to the uploaded HostScene
        self._scene_gen = -1      # its generation at upload
        self.buffer = np.zeros(self.m_Width * self.m_Height, np.uint32)
        self.rgb = None

    def params(self) -> abi.RenderParams:
        sr, first, step = self.stripe if self.stripe else (0, 0, 1)
        return abi.make_params(self.m_Width, self.m_Height, self.m_CurrentLightingMode, self.m_ShadowsEnabled,
                               self.format, sr, first, step)

    def Render(self, scene: HostScene, upload: bool = True, want_rgb: bool = False) -> np.ndarray:
        """Renderer::Render (Renderer.cpp:34-98): blocking; fills self.buffer."""
        s, cam = scene.view()
        same = self._scene_ref is not None and self._scene_ref() is scene and self._scene_gen == scene.generation
        if upload or not same:
            self.ctx.upload(s)
            self._scene_ref = weakref.ref(scene)
            self._scene_gen = scene.generation
        n = self.m_Width * self.m_Height
        rgb = np.zeros(3 * n, np.float32) if want_rgb else None
        rc = self.ctx.lib.rtx_render(self.ctx.h, C.byref(cam), C.byref(self.params()),
                                     self.buffer.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     rgb.ctypes.data_as(C.POINTER(C.c_float)) if want_rgb else None)
        abi.check(rc, "rtx_render", self.ctx.h)
        self.rgb = rgb
        return self.buffer

    def CycleLightingMode(self) -> None:   # Renderer.cpp:189-193
        self.m_CurrentLightingMode = (self.m_CurrentLightingMode + 1) % LightingMode.Count

    def ToggleShadows(self) -> None:       # Renderer.h:34-36
        self.m_ShadowsEnabled = not self.m_ShadowsEnabled

    def SaveBufferToImage(self, path: str = "RayTracing_Buffer.bmp") -> bool:
        """SDL_SaveBMP of the XRGB8888 surface (Renderer.cpp:184-187): 32-bit BI_RGB BMP."""
        return save_bmp(path, self.buffer, self.m_Width, self.m_Height)


def save_bmp(path: str, pixels: np.ndarray, width: int, height: int) -> bool:
    img = np.asarray(pixels, dtype=np.uint32).reshape(height, width)[::-1]   # bottom-up rows
    data = img.astype("<u4").tobytes()
    header = struct.pack("<2sIHHI", b"BM", 14 + 40 + len(data), 0, 0, 54)
    info = struct.pack("<IiiHHIIiiII", 40, width, height, 1, 32, 0, len(data), 2835, 2835, 0, 0)
    with open(path, "wb") as f:
        f.write(header + info + data)
    return True
