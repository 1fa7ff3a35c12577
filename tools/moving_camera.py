"""Moving-camera frame loop: the camera origin changes every frame, so the
exact cull's camera-anchor records are rebuilt before every frame.  Per setting
(product default, RTX_NO_CULL=1, and any extra NAME=VAR:value,... arguments) one context renders
K frames of a scene along a fixed camera path (render_async back to back on the context stream,
HIP-serialized like the reference's loop), wall-clock timed; the last frame of every setting is
checked bit for bit against the unculled one.  Prints one JSON line per (scene, setting).

Usage (GPU box): python tools/moving_camera.py [K] [scene,...] [setting ...]
"""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

SIZES = {"Synthetic100k": (1920, 1080), "W4_Optional": (1920, 1080), "W4_Bunny": (1920, 1080)}
KNOBS = ("RTX_NO_CULL", "RTX_CULL_ANIMATED", "RTX_CULL_MIN_SA", "RTX_CULL_RATIO", "RTX_CULL_TOP_LDS", "RTX_SCHED_PERIOD",
         "RTX_SPLIT", "RTX_SPLIT_FACTOR")


def ctx_with(env: dict) -> DeviceContext:
    saved = {k: os.environ.pop(k, None) for k in KNOBS}
    os.environ.update(env)
    try:
        return DeviceContext(0)
    finally:
        for k in KNOBS:
            os.environ.pop(k, None)
            if saved[k] is not None:
                os.environ[k] = saved[k]


def path(cam0: abi.Camera, k: int) -> abi.Camera:
    """Frame k's camera: the reference camera swaying on a small loop (a few cm per frame)."""
    c = abi.Camera()
    C.memmove(C.byref(c), C.byref(cam0), C.sizeof(abi.Camera))
    a = 0.05 * k
    c.origin[0] = cam0.origin[0] + 0.6 * np.sin(a)
    c.origin[1] = cam0.origin[1] + 0.2 * np.sin(0.5 * a)
    c.origin[2] = cam0.origin[2] + 0.4 * (1.0 - np.cos(a))
    return c


def run(name: str, K: int, settings) -> None:
    W, H = SIZES[name]
    hs = HostScene(name)
    s, cam0 = hs.view()
    p = abi.make_params(W, H)
    cams = [path(cam0, k) for k in range(K)]
    base = None
    for tag, env in settings:
        ctx = ctx_with(env)
        ctx.upload(s)
        for k in range(8):   # warm-up: cost-ordered and split state live
            ctx.render_async(cams[k], p)
        ctx.synchronize()
        n0 = ctx.cull_info()[1]
        t0 = time.perf_counter()
        for k in range(K):
            ctx.render_async(cams[k], p)
        ctx.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        rebuilds = ctx.cull_info()[1] - n0
        px, rgb = ctx.render(cams[K - 1], p)
        ctx.close()
        row = {"scene": f"{name} {W}x{H}", "setting": tag, "frames": K, "ms_per_frame": round(ms, 4),
               "camera_record_rebuilds": rebuilds, "cull": ctx_cull_flag(env)}
        if base is None:
            base = (px, rgb, ms)
        else:
            row["bit_identical_to_" + settings[0][0]] = bool(
                np.array_equal(px, base[0]) and np.array_equal(rgb.view(np.uint32), base[1].view(np.uint32)))
            row["speedup"] = round(base[2] / ms, 4)
        print(json.dumps(row), flush=True)


def ctx_cull_flag(env: dict) -> bool:
    return env.get("RTX_NO_CULL") != "1"


def main() -> None:
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    scenes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["Synthetic100k", "W4_Optional"]
    extra = []
    for a in sys.argv[3:]:
        tag, _, rest = a.partition("=")
        extra.append((tag, dict(kv.split(":", 1) for kv in rest.split(",") if kv)))
    settings = [("no_cull", {"RTX_NO_CULL": "1"}), ("cull", {})] + extra
    for name in scenes:
        run(name, K, settings)


if __name__ == "__main__":
    main()
