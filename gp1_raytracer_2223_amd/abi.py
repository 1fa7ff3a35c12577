"""ctypes mirror of the C-ABI in include/rtx.h and include/rtx_host.h.

Struct layouts match the C headers field-for-field (checked against the C compiler's
sizeof/offsetof in tests/test_abi.py).  Nothing here computes anything: it only loads
the native libraries and declares the entry points.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"
ASSET_DIR = PKG_DIR / "assets"

RTX_OK = 0
RTX_E_INVALID = -1
RTX_E_DEVICE = -2
RTX_E_NOMEM = -3
RTX_E_STATE = -4
RTX_E_UNSUPPORTED = -5

RTX_CULL_FRONT, RTX_CULL_BACK, RTX_CULL_NONE = 0, 1, 2
RTX_LIGHT_POINT, RTX_LIGHT_DIRECTIONAL = 0, 1
RTX_MODE_OBSERVED_AREA, RTX_MODE_RADIANCE, RTX_MODE_BRDF, RTX_MODE_COMBINED = 0, 1, 2, 3
RTX_MAT_SOLID_COLOR, RTX_MAT_LAMBERT, RTX_MAT_LAMBERT_PHONG, RTX_MAT_COOK_TORRANCE = 0, 1, 2, 3

F3 = C.c_float * 3


class Sphere(C.Structure):
    _fields_ = [("origin", F3), ("radius", C.c_float), ("material", C.c_uint8), ("_pad", C.c_uint8 * 3)]


class Plane(C.Structure):
    _fields_ = [("origin", F3), ("normal", F3), ("material", C.c_uint8), ("_pad", C.c_uint8 * 3)]


class BVHNode(C.Structure):
    _fields_ = [("min", F3), ("max", F3), ("first_idx", C.c_uint32), ("idx_count", C.c_uint32),
                ("left_node", C.c_uint32)]


class Mesh(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("n_positions", C.c_uint32),
                ("indices", C.POINTER(C.c_int32)), ("n_indices", C.c_uint32),
                ("normals", C.POINTER(C.c_float)), ("nodes", C.POINTER(BVHNode)), ("n_nodes", C.c_uint32),
                ("cull_mode", C.c_int32), ("material", C.c_uint8), ("_pad", C.c_uint8 * 3)]


class Light(C.Structure):
    _fields_ = [("origin", F3), ("direction", F3), ("color", F3), ("intensity", C.c_float), ("type", C.c_int32)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("color", F3), ("kd", C.c_float), ("ks", C.c_float),
                ("exponent", C.c_float), ("metalness", C.c_float), ("roughness", C.c_float)]


class MeshSource(C.Structure):   # rtx_mesh_source (rtx.h): object-space state of an animated mesh
    _fields_ = [("positions", C.POINTER(C.c_float)), ("n_positions", C.c_uint32),
                ("normals", C.POINTER(C.c_float)), ("indices", C.POINTER(C.c_int32)), ("n_indices", C.c_uint32)]


class Scene(C.Structure):
    _fields_ = [("spheres", C.POINTER(Sphere)), ("n_spheres", C.c_uint32),
                ("planes", C.POINTER(Plane)), ("n_planes", C.c_uint32),
                ("meshes", C.POINTER(Mesh)), ("n_meshes", C.c_uint32),
                ("lights", C.POINTER(Light)), ("n_lights", C.c_uint32),
                ("materials", C.POINTER(Material)), ("n_materials", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("origin", F3), ("right", F3), ("up", F3), ("forward", F3), ("fov", C.c_float)]


class PixelFormat(C.Structure):
    _fields_ = [("rshift", C.c_uint32), ("gshift", C.c_uint32), ("bshift", C.c_uint32), ("amask", C.c_uint32)]


XRGB8888 = (16, 8, 0, 0)


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("lighting_mode", C.c_int32),
                ("shadows_enabled", C.c_int32), ("format", PixelFormat), ("stripe_rows", C.c_uint32),
                ("stripe_first", C.c_uint32), ("stripe_step", C.c_uint32)]


def make_params(width, height, mode=RTX_MODE_COMBINED, shadows=True, fmt=XRGB8888,
                stripe_rows=0, stripe_first=0, stripe_step=1) -> RenderParams:
    p = RenderParams()
    p.width, p.height = int(width), int(height)
    p.lighting_mode, p.shadows_enabled = int(mode), int(bool(shadows))
    p.format = PixelFormat(*fmt)
    p.stripe_rows, p.stripe_first, p.stripe_step = int(stripe_rows), int(stripe_first), int(stripe_step)
    return p


def _lib_path(name: str) -> Path:
    return LIB_DIR / name


_host = None
_hip = None


def load_host() -> C.CDLL:
    """librtx_host.so: the C++ scene layer (pure host code; loads without a GPU)."""
    global _host
    if _host is None:
        path = _lib_path("librtx_host.so")
        if not path.exists():
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build() first")
        lib = C.CDLL(str(path))
        VP = C.c_void_p
        lib.rtx_host_scene_create.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(VP), C.c_char_p, C.c_size_t]
        lib.rtx_host_scene_create.restype = C.c_int
        lib.rtx_host_scene_destroy.argtypes = [VP]
        lib.rtx_host_scene_destroy.restype = None
        lib.rtx_host_scene_update.argtypes = [VP, C.c_float]
        lib.rtx_host_scene_update.restype = C.c_int
        lib.rtx_host_scene_copy_state.argtypes = [VP, VP]
        lib.rtx_host_scene_copy_state.restype = C.c_int
        lib.rtx_host_scene_view.argtypes = [VP, C.POINTER(Scene), C.POINTER(Camera)]
        lib.rtx_host_scene_view.restype = C.c_int
        lib.rtx_host_scene_animated.argtypes = [VP]
        lib.rtx_host_scene_animated.restype = C.c_int
        lib.rtx_host_camera_set.argtypes = [VP, C.POINTER(C.c_float), C.c_float, C.c_float, C.c_float]
        lib.rtx_host_camera_set.restype = C.c_int
        lib.rtx_host_parse_obj.argtypes = [C.c_char_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32),
                                           C.POINTER(C.c_float), C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                           C.c_uint32, C.c_uint32]
        lib.rtx_host_parse_obj.restype = C.c_int
        lib.rtx_host_obj_to_asset.argtypes = [C.c_char_p, C.c_char_p]
        lib.rtx_host_obj_to_asset.restype = C.c_int
        lib.rtx_host_scene_spinning.argtypes = [VP, C.POINTER(C.c_int32), C.c_uint32]
        lib.rtx_host_scene_spinning.restype = C.c_int
        lib.rtx_host_scene_mesh_source.argtypes = [VP, C.c_uint32, C.POINTER(MeshSource)]
        lib.rtx_host_scene_mesh_source.restype = C.c_int
        lib.rtx_host_scene_transforms.argtypes = [VP, C.c_float, C.POINTER(C.c_float), C.c_uint32]
        lib.rtx_host_scene_transforms.restype = C.c_int
        _host = lib
    return _host


HIP_SYMBOLS = ["rtx_abi_version", "rtx_create", "rtx_destroy", "rtx_last_error", "rtx_upload_scene",
               "rtx_render", "rtx_render_async", "rtx_synchronize", "rtx_download", "rtx_device_buffers",
               "rtx_time_frames", "rtx_scene_bytes", "rtx_count_work",
               "rtx_render_views_async", "rtx_time_views", "rtx_count_work_ex", "rtx_count_work_culled", "rtx_split_info",
               "rtx_split_tune_info",
               "rtx_gather_async", "rtx_host_register", "rtx_host_unregister",
               "rtx_group_create", "rtx_group_destroy", "rtx_group_last_error", "rtx_group_size",
               "rtx_group_context", "rtx_group_upload_scene", "rtx_group_render", "rtx_schedule_state",
               "rtx_anim_create", "rtx_anim_destroy", "rtx_anim_last_error", "rtx_anim_update", "rtx_anim_status",
               "rtx_anim_download", "rtx_scene_image", "rtx_anim_stamps", "rtx_cull_info", "rtx_cull_dump", "rtx_light_major_info",
               "rtx_inflight_info"]


def load_hip() -> C.CDLL:
    """librtx_hip.so: the HIP render path.  There is no fallback: if the library is
    missing the product path fails loudly."""
    global _hip
    if _hip is None:
        # RTX_HIP_LIB selects an alternative in-tree build (kernel experiments only)
        path = Path(os.environ.get("RTX_HIP_LIB", str(_lib_path("librtx_hip.so"))))
        if not path.exists():
            raise RuntimeError(f"{path} is missing: the HIP render path is not built (run __graft_entry__.build())")
        lib = C.CDLL(str(path))
        VP = C.c_void_p
        lib.rtx_abi_version.argtypes = []
        lib.rtx_abi_version.restype = C.c_int
        lib.rtx_create.argtypes = [C.POINTER(VP), C.c_int]
        lib.rtx_create.restype = C.c_int
        lib.rtx_destroy.argtypes = [VP]
        lib.rtx_destroy.restype = None
        lib.rtx_last_error.argtypes = [VP]
        lib.rtx_last_error.restype = C.c_char_p
        lib.rtx_upload_scene.argtypes = [VP, C.POINTER(Scene)]
        lib.rtx_upload_scene.restype = C.c_int
        lib.rtx_render.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_float)]
        lib.rtx_render.restype = C.c_int
        lib.rtx_render_async.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.c_int]
        lib.rtx_render_async.restype = C.c_int
        lib.rtx_render_views_async.argtypes = [VP, C.POINTER(Camera), C.c_int, C.POINTER(RenderParams), C.c_int]
        lib.rtx_render_views_async.restype = C.c_int
        lib.rtx_time_views.argtypes = [VP, C.POINTER(Camera), C.c_int, C.POINTER(RenderParams), C.c_int,
                                       C.POINTER(C.c_float)]
        lib.rtx_time_views.restype = C.c_int
        lib.rtx_synchronize.argtypes = [VP]
        lib.rtx_synchronize.restype = C.c_int
        lib.rtx_download.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_float)]
        lib.rtx_download.restype = C.c_int
        lib.rtx_device_buffers.argtypes = [VP, C.POINTER(VP), C.POINTER(VP)]
        lib.rtx_device_buffers.restype = C.c_int
        lib.rtx_time_frames.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.c_int,
                                        C.POINTER(C.c_float)]
        lib.rtx_time_frames.restype = C.c_int
        lib.rtx_scene_bytes.argtypes = [VP, C.POINTER(C.c_uint64)]
        lib.rtx_scene_bytes.restype = C.c_int
        lib.rtx_count_work.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(C.c_uint64)]
        lib.rtx_count_work.restype = C.c_int
        lib.rtx_count_work_ex.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(C.c_uint64),
                                          C.c_int]
        lib.rtx_count_work_ex.restype = C.c_int
        if hasattr(lib, "rtx_count_work_culled"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_count_work_culled.argtypes = lib.rtx_count_work_ex.argtypes
            lib.rtx_count_work_culled.restype = C.c_int
        if hasattr(lib, "rtx_cull_info"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_cull_info.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
            lib.rtx_cull_info.restype = C.c_int
        if hasattr(lib, "rtx_cull_dump"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_cull_dump.argtypes = [VP, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), VP, VP, VP,
                                          VP, VP]
            lib.rtx_cull_dump.restype = C.c_int
        if hasattr(lib, "rtx_split_tune_info"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_split_tune_info.argtypes = [VP, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                                C.POINTER(C.c_uint32)]
            lib.rtx_split_tune_info.restype = C.c_int
        if hasattr(lib, "rtx_light_major_info"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_light_major_info.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
            lib.rtx_light_major_info.restype = C.c_int
        if hasattr(lib, "rtx_inflight_info"):
            lib.rtx_inflight_info.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                              C.POINTER(C.c_float), C.POINTER(C.c_float)]
            lib.rtx_inflight_info.restype = C.c_int
        if hasattr(lib, "rtx_split_info"):   # absent only in older experiment builds (RTX_HIP_LIB)
            lib.rtx_split_info.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
            lib.rtx_split_info.restype = C.c_int
        if hasattr(lib, "rtx_schedule_state"):
            lib.rtx_schedule_state.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32,
                                               C.POINTER(C.c_uint32)]
            lib.rtx_schedule_state.restype = C.c_int
        if hasattr(lib, "rtx_group_create"):   # absent only in older experiment builds
            lib.rtx_gather_async.argtypes = [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_float)]
            lib.rtx_gather_async.restype = C.c_int
            lib.rtx_host_register.argtypes = [VP, VP, C.c_size_t]
            lib.rtx_host_register.restype = C.c_int
            lib.rtx_host_unregister.argtypes = [VP, VP]
            lib.rtx_host_unregister.restype = C.c_int
            lib.rtx_group_create.argtypes = [C.POINTER(VP), C.POINTER(C.c_int), C.c_int]
            lib.rtx_group_create.restype = C.c_int
            lib.rtx_group_destroy.argtypes = [VP]
            lib.rtx_group_destroy.restype = None
            lib.rtx_group_last_error.argtypes = [VP]
            lib.rtx_group_last_error.restype = C.c_char_p
            lib.rtx_group_size.argtypes = [VP]
            lib.rtx_group_size.restype = C.c_int
            lib.rtx_group_context.argtypes = [VP, C.c_int]
            lib.rtx_group_context.restype = VP
            lib.rtx_group_upload_scene.argtypes = [VP, C.POINTER(Scene)]
            lib.rtx_group_upload_scene.restype = C.c_int
            lib.rtx_group_render.argtypes = [VP, C.POINTER(Camera), C.POINTER(RenderParams), C.POINTER(C.c_uint32),
                                             C.POINTER(C.c_float)]
            lib.rtx_group_render.restype = C.c_int
        if hasattr(lib, "rtx_scene_image"):
            lib.rtx_scene_image.argtypes = [VP, VP, C.c_size_t, C.POINTER(C.c_size_t)]
            lib.rtx_scene_image.restype = C.c_int
        if hasattr(lib, "rtx_anim_create"):   # absent only in older experiment builds
            lib.rtx_anim_create.argtypes = [C.POINTER(VP), VP, C.POINTER(Scene), C.POINTER(C.c_int32),
                                            C.POINTER(MeshSource), C.c_uint32]
            lib.rtx_anim_create.restype = C.c_int
            lib.rtx_anim_destroy.argtypes = [VP]
            lib.rtx_anim_destroy.restype = None
            lib.rtx_anim_last_error.argtypes = [VP]
            lib.rtx_anim_last_error.restype = C.c_char_p
            lib.rtx_anim_update.argtypes = [VP, VP, C.POINTER(C.c_float)]
            lib.rtx_anim_update.restype = C.c_int
            lib.rtx_anim_status.argtypes = [VP, C.c_uint32, C.POINTER(C.c_uint32)]
            lib.rtx_anim_status.restype = C.c_int
            lib.rtx_anim_download.argtypes = [VP, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_int32),
                                              C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(BVHNode)]
            lib.rtx_anim_download.restype = C.c_int
            lib.rtx_anim_stamps.argtypes = [VP, C.c_uint32, C.POINTER(C.c_uint32)]
            lib.rtx_anim_stamps.restype = C.c_int
        _hip = lib
    return _hip


def check(rc: int, what: str, ctx=None) -> None:
    if rc != RTX_OK:
        msg = ""
        if ctx is not None and _hip is not None:
            m = _hip.rtx_last_error(ctx)
            msg = m.decode() if m else ""
        raise RuntimeError(f"{what} failed with code {rc}: {msg}")


def env_flag(name: str) -> bool:
    return os.environ.get(name, "") not in ("", "0")
