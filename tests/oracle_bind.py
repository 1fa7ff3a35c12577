"""ctypes binding of oracle/_build/librtx_oracle.so — TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from gp1_raytracer_2223_amd import abi

ORACLE_SO = Path(__file__).resolve().parents[1] / "oracle" / "_build" / "librtx_oracle.so"
REF_HARNESS = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "ref_harness"
_lib = None

COUNTER_NAMES = ["pixels", "sphere", "plane", "slab", "tri", "hit", "shadow", "occluded",
                 "shade_base", "shade_lambert", "shade_phong", "shade_ct"]
# SURVEY.md §8(d) cost model (FLOP per event)
FLOP_COST = {"pixels": 41, "sphere": 19, "plane": 14, "slab": 12, "tri": 63, "hit": 9, "shadow": 15,
             "occluded": 1, "shade_base": 26, "shade_lambert": 6, "shade_phong": 31, "shade_ct": 103}


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not ORACLE_SO.exists():
            from gp1_raytracer_2223_amd.build import build_oracle
            build_oracle()
        L = C.CDLL(str(ORACLE_SO))
        P = C.POINTER
        L.rtx_oracle_render.argtypes = [P(abi.Scene), P(abi.Camera), P(abi.RenderParams), P(C.c_uint32),
                                        P(C.c_float), C.c_int]
        L.rtx_oracle_count.argtypes = [P(abi.Scene), P(abi.Camera), P(abi.RenderParams), P(C.c_uint32), C.c_int,
                                       P(C.c_uint64)]
        for n in ("rtx_oracle_hit_sphere", "rtx_oracle_hit_plane"):
            getattr(L, n).argtypes = [P(C.c_float), P(C.c_float), C.c_int, P(C.c_float)]
        L.rtx_oracle_hit_triangle.argtypes = [P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_float)]
        L.rtx_oracle_slab.argtypes = [P(C.c_float), P(C.c_float)]
        L.rtx_oracle_shade.argtypes = [P(abi.Material), P(C.c_float), P(C.c_float), P(C.c_float), P(C.c_float)]
        L.rtx_oracle_shade.restype = None
        _lib = L
    return _lib


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def render(scene: abi.Scene, cam: abi.Camera, params: abi.RenderParams, threads: int = 8, want_rgb: bool = True,
           out_px: np.ndarray | None = None, out_rgb: np.ndarray | None = None):
    n = params.width * params.height
    px = np.zeros(n, np.uint32) if out_px is None else out_px
    rgb = (np.zeros(3 * n, np.float32) if out_rgb is None else out_rgb) if want_rgb else None
    rc = lib().rtx_oracle_render(C.byref(scene), C.byref(cam), C.byref(params),
                                 px.ctypes.data_as(C.POINTER(C.c_uint32)), fptr(rgb) if want_rgb else None, threads)
    abi.check(rc, "rtx_oracle_render")
    return px, rgb


def count(scene, cam, params, threads: int = 8) -> np.ndarray:
    n = params.width * params.height
    px = np.zeros(n, np.uint32)
    out = (C.c_uint64 * 12)()
    rc = lib().rtx_oracle_count(C.byref(scene), C.byref(cam), C.byref(params),
                                px.ctypes.data_as(C.POINTER(C.c_uint32)), threads, out)
    abi.check(rc, "rtx_oracle_count")
    return np.array(list(out), dtype=np.uint64)


def flops(counts) -> int:
    return int(sum(int(counts[i]) * FLOP_COST[n] for i, n in enumerate(COUNTER_NAMES)))
