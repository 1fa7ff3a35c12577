"""Moving-camera frame loop: the camera origin changes every frame, so the
exact cull's camera-anchor records are rebuilt before every frame and the tile
schedule runs in motion mode (rtx_hip.hip, kMotionFrames).  Per setting (product default,
RTX_NO_CULL=1, and any extra NAME=VAR:value,... arguments) K frames of a scene along a fixed camera
path, wall-clock timed, with F frames in flight (MC_INFLIGHT, default 2: frame k on context k mod F,
which first waits for its previous frame — the bench's and the CLI's frame loop; 1 = the
reference's serial loop, each frame complete before the next is queued).  The last frame of every
setting is checked bit for bit against the unculled one.  One JSON line per (scene, setting).

Usage (GPU box): [MC_INFLIGHT=F] python tools/moving_camera.py [K] [scene,...] [setting ...]
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
         "RTX_SPLIT", "RTX_SPLIT_FACTOR", "RTX_MOTION")


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
    nf = int(os.environ.get("MC_INFLIGHT", "2"))
    for tag, env in settings:
        ctxs = [ctx_with(env) for _ in range(nf)]
        for ctx in ctxs:
            ctx.upload(s)
        for k in range(8 * nf):   # warm-up: cost-ordered and split state live
            ctxs[k % nf].render_async(cams[k // nf], p)
        for ctx in ctxs:
            ctx.synchronize()
        n0 = sum(ctx.cull_info()[1] for ctx in ctxs)
        t0 = time.perf_counter()
        still = tag.startswith("static")   # the same loop with the camera standing still
        for k in range(K):
            ctx = ctxs[k % nf]
            ctx.synchronize()   # its previous frame (k - nf) is complete
            ctx.render_async(cams[0] if still else cams[k], p)
        for ctx in ctxs:
            ctx.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / K
        rebuilds = sum(ctx.cull_info()[1] for ctx in ctxs) - n0
        heavy = ctxs[(K - 1) % nf].split_info()[0]
        px, rgb = ctxs[0].render(cams[K - 1], p)   # (the check frame: the path's last camera for every setting)
        for ctx in ctxs:
            ctx.close()
        row = {"scene": f"{name} {W}x{H}", "setting": tag, "frames": K, "inflight": nf, "ms_per_frame": round(ms, 4),
               "camera_record_rebuilds": rebuilds, "heavy_tiles_last": heavy, "cull": ctx_cull_flag(env)}
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
    settings = [("no_cull", {"RTX_NO_CULL": "1"}), ("cull", {}), ("static_cull", {})] + extra
    for name in scenes:
        run(name, K, settings)


if __name__ == "__main__":
    main()
